"""G1 golden vectors: raw adapterAlignment result strings produced by the REFERENCE itself
(oracle/_ref/cpp_functions.so, compiled in place from /root/reference sources by
`make -C oracle ref`). Container-only generator; the output is committed as data:
tests/golden/g1_alignments.tsv.gz  (scheme, read, adapter, result).

Cases: random and tie-heavy alphabets (A, AT, AC, ACGT, ACGTN, with '-'),
embedded mutated real adapters from the adapter database, read lengths 0-1200 plus a few 8 kb,
adapter lengths 1-111, four scoring schemes incl. linear gaps, empty inputs.
"""
import ctypes
import gzip
import json
import os
import random

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, 'oracle', '_ref', 'cpp_functions.so')
OUT = os.path.join(ROOT, 'tests', 'golden', 'g1_alignments.tsv.gz')

lib = ctypes.CDLL(REF)
lib.adapterAlignment.argtypes = [ctypes.c_char_p, ctypes.c_char_p] + [ctypes.c_int] * 4
lib.adapterAlignment.restype = ctypes.c_void_p
lib.freeCString.argtypes = [ctypes.c_void_p]


def ref(r, a, sc):
    p = lib.adapterAlignment(r.encode(), a.encode(), *sc)
    s = ctypes.cast(p, ctypes.c_char_p).value.decode()
    lib.freeCString(p)
    return s


def mutate(rng, s, rate):
    o = []
    for c in s:
        x = rng.random()
        if x < rate / 3:
            o.append(rng.choice('ACGT'))
        elif x < 2 * rate / 3:
            pass
        elif x < rate:
            o.append(c + rng.choice('ACGT'))
        else:
            o.append(c)
    return ''.join(o)


def main(n=20000, seed=2024):
    rng = random.Random(seed)
    db = json.load(open(os.path.join(ROOT, 'custom_porechop_abi_amd', 'data', 'adapters.json')))
    real = sorted({x[1] for s in db['sets'] for x in (s['start'], s['end']) if x})
    fl = db['full_barcode_flanks']['make_full_native_barcode_adapter']
    real += [fl[0] + rng.choice(real) + fl[1] for _ in range(20)]           # 60-111 bp adapters
    schemes = [(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (3, -6, -2, -5)]
    alphs = ['A', 'AT', 'AC', 'ACGT', 'ACGT', 'ACGTN', 'ACGT-']
    rows = []
    for k in range(n):
        sc = schemes[k % len(schemes)]
        if rng.random() < 0.5:
            a = rng.choice(real)
        else:
            a = ''.join(rng.choice('ACGT') for _ in range(rng.choice([1, 2, 3, 5, 8, 13, rng.randint(1, 111)])))
        al = rng.choice(alphs)
        nlen = rng.choice([0, 1, 2, 5, 20, 75, 150, 150, 150, rng.randint(0, 1200)]) if k % 500 else 8000
        r = ''.join(rng.choice(al) for _ in range(nlen))
        if nlen > 10 and rng.random() < 0.6:
            m = mutate(rng, a, rng.choice([0.0, 0.05, 0.1, 0.2]))
            p = rng.randint(0, max(0, nlen - len(m)))
            r = r[:p] + m + r[p + len(m):]
        if k % 997 == 0:
            a = '' if k % 2 else a
            r = r if k % 2 else ''
        rows.append('%d,%d,%d,%d\t%s\t%s\t%s' % (sc + (r, a, ref(r, a, sc))))
    with gzip.open(OUT, 'wt') as f:
        f.write('\n'.join(rows) + '\n')
    print('wrote', OUT, len(rows))


if __name__ == '__main__':
    main()

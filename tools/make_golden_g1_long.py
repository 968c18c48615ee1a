"""G1-long golden vectors: raw adapterAlignment result strings from the REFERENCE itself
(oracle/_ref/cpp_functions.so, compiled in place from /root/reference sources by
`make -C oracle ref`) for adapters LONGER than 128 bp -- the striped core's range (the reference
bounds neither sequence, porechop_abi/src/adapter_align.cpp:11-31). Container-only generator;
the output is committed as data: tests/golden/g1_long.tsv.gz (scheme, read, adapter, result).

Cases: adapter lengths 129-1200 (129, 200, 255, 256, 512, 1000 always present), random and
tie-heavy alphabets, reads of 0-2000 bases (end windows of 150 among them) carrying mutated copies
(whole, cut at either read end), five scoring schemes (linear gaps, open cheaper than extend),
empty inputs.
"""
import ctypes
import gzip
import os
import random

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, 'oracle', '_ref', 'cpp_functions.so')
OUT = os.path.join(ROOT, 'tests', 'golden', 'g1_long.tsv.gz')

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


def main(n=1500, seed=4096):
    rng = random.Random(seed)
    schemes = [(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (3, -6, -2, -5), (5, -4, -8, -6)]
    fixed = [129, 200, 255, 256, 512, 1000]
    rows = []
    for k in range(n):
        sc = schemes[k % len(schemes)]
        L = fixed[k % len(fixed)] if k % 3 else rng.randint(129, 1200)
        aal = rng.choice(['ACGT', 'ACGT', 'ACGT', 'AT', 'ACGTN'])
        a = ''.join(rng.choice(aal) for _ in range(L))
        al = rng.choice(['ACGT', 'ACGT', 'AT', 'A', 'ACGTN', 'ACGT-'])
        nlen = rng.choice([0, 1, 5, 60, 150, 150, rng.randint(0, 600), rng.randint(600, 2000)])
        r = ''.join(rng.choice(al) for _ in range(nlen))
        if nlen > 10 and rng.random() < 0.7:
            m = mutate(rng, a, rng.choice([0.0, 0.05, 0.1, 0.2]))
            w = rng.random()
            if w < 0.2:
                r = m[rng.randint(0, len(m) - 1):] + r
            elif w < 0.4:
                r = r + m[:rng.randint(1, len(m))]
            else:
                p = rng.randint(0, nlen)
                r = r[:p] + m + r[p:]
        if k % 250 == 0:
            a = '' if k % 500 else a
            r = r if k % 500 else ''
        rows.append('%d,%d,%d,%d\t%s\t%s\t%s' % (sc + (r, a, ref(r, a, sc))))
    with gzip.open(OUT, 'wt') as f:
        f.write('\n'.join(rows) + '\n')
    print('wrote', OUT, len(rows))


if __name__ == '__main__':
    main()

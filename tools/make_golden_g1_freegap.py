"""G1-freegap golden vectors: raw adapterAlignment result strings from the REFERENCE itself
(oracle/_ref/cpp_functions.so, compiled in place from /root/reference sources by
`make -C oracle ref`) under the scoring schemes the other fixtures never use: gap costs >= 0,
match <= 0, all-zero. The reference accepts any four integers as --scoring_scheme
(porechop_abi/arg_parser.py:229-236) and aligns reads of any length under them
(porechop_abi/src/adapter_align.cpp:11-31). Container-only generator; the output is committed as
data: tests/golden/g1_freegap.tsv.gz (scheme, read, adapter, result), one row per line.

Cases (>= 2,400 rows over the eight schemes):
  * adapters of 1-140 bp (the register cores up to 128, the striped core past it), random and
    tie-heavy alphabets, reads of 0-2,000 bases carrying whole, cut and mutated copies;
  * 40 reads of 33-70 kb (past the register cores' 32 k start-column field) with a planted
    copy past the 32 k mark, against 22-50 bp adapters -- the whole-read middle-scan shape;
  * empty inputs.
"""
import ctypes
import gzip
import os
import random

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, 'oracle', '_ref', 'cpp_functions.so')
OUT = os.path.join(ROOT, 'tests', 'golden', 'g1_freegap.tsv.gz')

SCHEMES = [(2, -1, 0, 0), (3, -6, 0, -2), (1, -1, 1, 1), (0, 0, 0, 0), (-1, -1, -1, -1), (3, -6, 2, -1),
           (5, -4, -1, 0), (3, -6, -8, 0)]   # the last two: free gap extension (a run costs its open only)

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


def main(n=2400, n_long=40, seed=8191):
    rng = random.Random(seed)
    rows = []
    for k in range(n):
        sc = SCHEMES[k % len(SCHEMES)]
        L = rng.choice([1, 2, 5, 8, 22, 24, 28, 33, 50, 64, 68, 111, 128, rng.randint(1, 140)])
        aal = rng.choice(['ACGT', 'ACGT', 'ACGT', 'AT', 'ACGTN'])
        a = ''.join(rng.choice(aal) for _ in range(L))
        al = rng.choice(['ACGT', 'ACGT', 'AT', 'A', 'ACGTN', 'ACGT-'])
        nlen = rng.choice([0, 1, 5, 60, 150, 150, rng.randint(0, 600), rng.randint(600, 2000)])
        r = ''.join(rng.choice(al) for _ in range(nlen))
        if nlen > 10 and rng.random() < 0.7:
            m = mutate(rng, a, rng.choice([0.0, 0.05, 0.1, 0.2])) or a
            w = rng.random()
            if w < 0.2:
                r = m[rng.randint(0, len(m) - 1):] + r
            elif w < 0.4:
                r = r + m[:rng.randint(1, len(m))]
            else:
                p = rng.randint(0, nlen)
                r = r[:p] + m + r[p:]
        if k % 300 == 0:
            a = '' if k % 600 else a
            r = r if k % 600 else ''
        rows.append('%d,%d,%d,%d\t%s\t%s\t%s' % (sc + (r, a, ref(r, a, sc))))
    for k in range(n_long):
        sc = SCHEMES[k % len(SCHEMES)]
        a = ''.join(rng.choice('ACGT') for _ in range(rng.choice([22, 24, 28, 33, 50])))
        nlen = rng.randint(33000, 70000)
        r = ''.join(rng.choice('ACGT') for _ in range(nlen))
        p = rng.randint(32800, nlen - len(a))
        r = r[:p] + mutate(rng, a, 0.05) + r[p:]
        rows.append('%d,%d,%d,%d\t%s\t%s\t%s' % (sc + (r, a, ref(r, a, sc))))
    with gzip.open(OUT, 'wt') as f:
        f.write('\n'.join(rows) + '\n')
    print('wrote', OUT, len(rows))


if __name__ == '__main__':
    main()

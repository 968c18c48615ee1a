"""G4 golden vectors: check_compatibility flags from the REFERENCE ITSELF
(oracle/_ref/compatibility.so, compiled by `make -C oracle ref` from
porechop_abi/ab_initio_src/compatibility.cpp and the vendored SeqAn), for the ab-initio
clustering's all-vs-all link test (porechop_abi/consensus.py:72-100).

Container-only generator. `--long` writes tests/golden/g4_compat_long.json.gz instead: the same
pair kinds over 129-600 bp sequences (both longer than the register-resident cores' 128 rows,
so the shorter one runs on the striped core). Pairs: adapter-like sequences of 4-120 bp and their mutated copies
(substitutions / insertions / deletions at 0-25%), contained substrings, prefix / suffix
overlaps, unrelated pairs, equal lengths (row-order ties), lower case, U, N and IUPAC letters
(SeqAn String<Dna> maps them to A). Pairs whose Dna letters share nothing are skipped: with no
overlap the reference divides by zero. Also checks the C restatement (oracle/pcabi_oracle.c
pcabi_oracle_compat) against every vector. Writes tests/golden/g4_compat.json.gz.
"""
import ctypes
import gzip
import json
import os
import random

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, 'tests', 'golden', 'g4_compat.json.gz')


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


def dna(c):
    c = c.upper()
    return c if c in 'CGT' else ('T' if c == 'U' else 'A')


def main(long=False):
    ref = ctypes.CDLL(os.path.join(ROOT, 'oracle', '_ref', 'compatibility.so'))
    ref.check_compatibility.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    ref.check_compatibility.restype = ctypes.c_int
    orc = ctypes.CDLL(os.path.join(ROOT, 'oracle', 'liboracle.so'))
    orc.pcabi_oracle_compat.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    orc.pcabi_oracle_compat.restype = ctypes.c_int
    rng = random.Random(4243 if long else 4242)
    out = OUT.replace('g4_compat', 'g4_compat_long') if long else OUT
    pairs = []
    while len(pairs) < (2000 if long else 20000):
        if long:
            L = rng.choice([129, 150, 200, 255, 300, 400, 600, rng.randint(129, 600)])
        else:
            L = rng.choice([4, 8, 12, 16, 20, 22, 24, 28, 32, 40, 50, 64, 80, 100, 120, rng.randint(4, 120)])
        alph = rng.choice(['ACGT'] * 6 + ['acgt', 'ACGTN', 'ACGU', 'AT', 'ACGTRYKM'])
        a = ''.join(rng.choice(alph) for _ in range(L))
        kind = rng.random()
        if kind < 0.35:
            b = mutate(rng, a, rng.choice([0.0, 0.02, 0.05, 0.1, 0.15, 0.25]))
        elif kind < 0.5:
            i = rng.randint(0, L - 1)
            b = a[i:i + rng.randint(1, L - i)]
            b = mutate(rng, b, rng.choice([0.0, 0.05]))
        elif kind < 0.7:
            k = rng.randint(1, L)
            tail = ''.join(rng.choice('ACGT') for _ in range(rng.randint(0, 30)))
            b = (a[-k:] + tail) if rng.random() < 0.5 else (tail + a[:k])
        elif kind < 0.8:
            b = mutate(rng, a, 0.05)
            b = b[:L] if len(b) >= L else b + a[len(b):]          # equal lengths
        else:
            b = ''.join(rng.choice(alph) for _ in range(rng.randint(129, 600) if long else rng.randint(4, 120)))
        if long and min(len(a), len(b)) <= 128:
            continue
        if not b:
            continue
        if not (set(map(dna, a)) & set(map(dna, b))):
            continue
        if rng.random() < 0.5:
            a, b = b, a
        f = ref.check_compatibility(a.encode(), b.encode())
        o = orc.pcabi_oracle_compat(a.encode(), b.encode())
        if o != f:
            raise SystemExit('oracle restatement differs: %r %r ref=%d oracle=%d' % (a, b, f, o))
        pairs.append([a, b, f])
    with gzip.open(out, 'wt') as fh:
        json.dump({'generator': 'tools/make_golden_g4.py' + (' --long' if long else ''), 'pairs': pairs}, fh)
    counts = [sum(1 for p in pairs if p[2] == k) for k in range(3)]
    print('wrote', out, len(pairs), 'pairs; flags 0/1/2:', counts)


if __name__ == '__main__':
    import sys
    main(long='--long' in sys.argv[1:])

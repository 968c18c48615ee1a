#!/usr/bin/env python3
"""GPU fuzz parity: random cases through libpcabi.so vs the CPU oracle, for a time budget.

    python tools/gpu_fuzz.py [seconds] [seed]

Each iteration draws a scoring scheme (tests/test_gpu_parity.SCHEMES: gap costs >= 0, match <= 0
and all-zero schemes among them), adapters (1..40 bp mostly, some up to 140, a few past
128 -- the striped core) and windows (empty to 3 kb, ACGT / ACGTN / low-complexity alphabets,
planted mutated adapter copies), then checks
  * the cross product (engine.align) and a random pairs subset, all 8 fields;
  * the middle scan (engine.middle_scan) with a random threshold and seed / plan mode,
    against the oracle's masked loop (C, threaded).
Mismatches are printed with the case seed; the exit status is the number of failing cases.
"""
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401  (one HIP runtime)
from custom_porechop_abi_amd import engine
from tests import oracle_lib
from tests.test_gpu_parity import SCHEMES, _mutate, _rand_seq


def case(rng):
    alph = rng.choice(['ACGT', 'ACGT', 'ACGTN', 'AT', 'AAAC'])
    n_adp = rng.randint(1, 12)
    adps = []
    for _ in range(n_adp):
        r = rng.random()
        L = rng.randint(1, 40) if r < 0.7 else (rng.randint(41, 140) if r < 0.93 else rng.randint(129, 300))
        adps.append(_rand_seq(rng, L, 'ACGT'))
    reads = []
    for _ in range(rng.randint(1, 200)):
        n = rng.choice([0, 1, 7, 150, rng.randint(0, 600), rng.randint(0, 3000)])
        s = _rand_seq(rng, n, alph)
        for _ in range(rng.choice([0, 1, 1, 2])):
            a = _mutate(rng, rng.choice(adps), rng.choice([0.0, 0.03, 0.1]))
            p = rng.randint(0, len(s))
            s = s[:p] + a + s[p:]
        reads.append(s)
    return reads, adps


def sort_hits(h):
    return h[:, np.lexsort((np.arange(h.shape[1]), h[0]))] if h.size else h


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 120.0
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    t_end = time.time() + budget
    fails = 0
    it = 0
    stats = {'alignments': 0, 'middle_reads': 0}
    t_last = time.time()
    while time.time() < t_end:
        seed = seed0 * 1000003 + it
        it += 1
        rng = random.Random(seed)
        reads, adps = case(rng)
        sc = rng.choice(SCHEMES)
        pack = engine.SeqPack(reads)
        views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
        # cross product
        got = engine.align(views, adps, sc)
        exp = oracle_lib.align_windows(views, adps, sc)
        ok = exp[0] != -1
        stats['alignments'] += exp.shape[1]
        if not (np.array_equal(got[0], exp[0]) and np.array_equal(got[:, ok], exp[:, ok])):
            bad = np.nonzero((got != exp).any(axis=0) & (ok | (got[0] != exp[0])))[0]
            j = int(bad[0])
            print('CROSS MISMATCH seed %d scheme %s: %d pairs; first (window %d, adapter %d len %d, read len %d) got %s '
                  'exp %s' % (seed, sc, len(bad), j % len(reads), j // len(reads), len(adps[j // len(reads)]),
                              len(reads[j % len(reads)]), got[:, j].tolist(), exp[:, j].tolist()), flush=True)
            fails += 1
        # pairs subset
        m = rng.randint(1, 300)
        pr = np.array([rng.randrange(len(reads)) for _ in range(m)])
        pa = np.array([rng.randrange(len(adps)) for _ in range(m)])
        got = engine.align(views, adps, sc, pairs=(pr, pa))
        exp = oracle_lib.align_windows(views, adps, sc, pairs=(pr, pa))
        ok = exp[0] != -1
        if not (np.array_equal(got[0], exp[0]) and np.array_equal(got[:, ok], exp[:, ok])):
            print('PAIRS MISMATCH seed %d scheme %s' % (seed, sc), flush=True)
            fails += 1
        # middle scan (the reference's masked loop), a random threshold and mode
        if rng.random() < 0.5:
            th = rng.choice([80.0, 85.0, 88.0, 90.0, 95.0])
            # adapters of a few bases hit almost every base, and the reference's masked loop then runs
            # one round per hit (thousands per read): the middle scan takes adapters of >= 8 bp
            adps = [a for a in adps if len(a) >= 8] or [max(adps, key=len) + 'ACGTACGT']
            mode = rng.choice([('PCABI_MIDDLE_SEEDS', '2'), ('PCABI_MIDDLE_SEEDS', '1'),
                               ('PCABI_MIDDLE_DEVPLAN', '0'), ('PCABI_MIDDLE_PLAN_WAVES', '1'),
                               ('PCABI_MIDDLE_PLAN_WAVES', '100000000'), ('PCABI_MIDDLE_FILTER', '0')])
            os.environ[mode[0]] = mode[1]
            if os.environ.get('FUZZ_VERBOSE'):
                print('case %d: scheme %s threshold %s mode %s, %d reads (longest %d), adapters %s' %
                      (seed, sc, th, mode, len(reads), max(map(len, reads)), [len(a) for a in adps]), flush=True)
            try:
                got = engine.middle_scan(views, adps, sc, th)
            finally:
                del os.environ[mode[0]]
            exp = oracle_lib.middle_scan_threaded(views, adps, sc, th)
            stats['middle_reads'] += len(reads)
            if got.shape != exp.shape or not np.array_equal(sort_hits(got), sort_hits(exp)):
                print('MIDDLE MISMATCH seed %d scheme %s threshold %s mode %s: got %d hits, exp %d' %
                      (seed, sc, th, mode, got.shape[1], exp.shape[1]), flush=True)
                fails += 1
        if time.time() - t_last >= 20.0:             # a line at least every ~20 s (gpurun's hang check)
            t_last = time.time()
            print('iteration %d: %d failing cases, %s' % (it, fails, stats), flush=True)
    print('done: %d iterations, %d failing cases, %s' % (it, fails, stats), flush=True)
    return min(fails, 100)


if __name__ == '__main__':
    sys.exit(main())

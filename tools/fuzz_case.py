#!/usr/bin/env python3
"""Re-run one tools/gpu_fuzz.py case (its seed) on the GPU with timing: the middle scan with the
case's threshold and mode, then the oracle; or ('align') three cross products of the case.
Debugging aid: python tools/fuzz_case.py SEED [THRESHOLD MODE_VAR VALUE | align]"""
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
from custom_porechop_abi_amd import engine  # noqa: E402
from tests import oracle_lib  # noqa: E402
from tests.test_gpu_parity import SCHEMES  # noqa: E402
from tools.gpu_fuzz import case  # noqa: E402


def main():
    seed = int(sys.argv[1])
    rng = random.Random(seed)
    reads, adps = case(rng)
    sc = rng.choice(SCHEMES)
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    rng.randint(1, 300)
    m = None  # the pairs draws of the fuzz loop
    rng2 = rng
    del m, rng2
    if len(sys.argv) > 2 and sys.argv[2] == 'align':
        for _ in range(3):
            t = time.time()
            engine.align(views, adps, sc)
            print('cross product: %.1f ms' % (1e3 * (time.time() - t)), flush=True)
        return
    th = float(sys.argv[2]) if len(sys.argv) > 2 else 95.0
    mode = (sys.argv[3], sys.argv[4]) if len(sys.argv) > 4 else None
    if mode:
        os.environ[mode[0]] = mode[1]
    t = time.time()
    got = engine.middle_scan(views, adps, sc, th)
    print('gpu: %d hits in %.2f s' % (got.shape[1], time.time() - t), flush=True)
    t = time.time()
    exp = oracle_lib.middle_scan_threaded(views, adps, sc, th)
    print('oracle: %d hits in %.2f s, equal %s' % (exp.shape[1], time.time() - t,
                                                   got.shape == exp.shape and bool((got == exp).all())), flush=True)


if __name__ == '__main__':
    main()

#!/usr/bin/env python3
"""Perf probe: one cross product of 100k synthetic 150-bp windows against a given adapter list,
launched alone (no other bucket beside it), timed with HIP events. Used to see how a register
bucket with few adapters (a small grid) runs on its own.
usage: python tools/bucket_micro.py L1,L2,... [reps]"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401
from custom_porechop_abi_amd import _lib, synth
from custom_porechop_abi_amd.engine import encode_adapters


def main():
    lens = [int(x) for x in sys.argv[1].split(',')]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    L = _lib.lib()
    vp = ctypes.c_void_p
    rng = np.random.default_rng(5)
    adps = [''.join('ACGT'[c] for c in rng.integers(0, 4, l)) for l in lens]
    n, E = 100000, 150
    codes = rng.integers(0, 4, n * E + 64).astype(np.uint8)
    off = np.arange(n, dtype=np.int64) * E
    ln = np.full(n, E, np.int32)

    def h2d(a):
        a = np.ascontiguousarray(a)
        p = vp()
        _lib.check(L.pcabi_dev_malloc(ctypes.byref(p), max(a.nbytes, 16)), 'malloc')
        _lib.check(L.pcabi_dev_h2d(p, a.ctypes.data_as(vp), a.nbytes), 'h2d')
        return p
    d_codes, d_off, d_len = h2d(codes), h2d(off), h2d(ln)
    toff = np.zeros((n + 255) // 256 + 1, np.int64)
    nd = L.pcabi_tile_layout(ln.ctypes.data_as(vp), n, toff.ctypes.data_as(vp))
    d_toff = h2d(toff)
    d_tiles = vp()
    _lib.check(L.pcabi_dev_malloc(ctypes.byref(d_tiles), 4 * nd), 'malloc')
    stream = vp()
    _lib.check(L.pcabi_stream_create(ctypes.byref(stream)), 'stream')
    _lib.check(L.pcabi_tile_windows_dev(d_codes, d_off, d_len, n, d_toff, int(np.diff(toff).max() // 256), d_tiles,
                                        stream), 'tile')
    c, o, l = encode_adapters(adps)
    tab = vp()
    _lib.check(L.pcabi_adapters_create_scored(c.ctypes.data_as(vp), o.ctypes.data_as(vp), l.ctypes.data_as(vp),
                                              len(adps), 3, -6, -5, -2, ctypes.byref(tab)), 'tab')
    d_res = vp()
    _lib.check(L.pcabi_dev_malloc(ctypes.byref(d_res), 4 * 8 * n * len(adps)), 'malloc')
    e0, e1 = vp(), vp()
    L.pcabi_event_create(ctypes.byref(e0)); L.pcabi_event_create(ctypes.byref(e1))
    ms = []
    for r in range(reps + 2):
        L.pcabi_event_record(e0, stream)
        _lib.check(L.pcabi_align_cross_dev(d_tiles, d_toff, d_len, n, E, tab, 3, -6, -5, -2, d_res, n * len(adps),
                                           stream), 'align')
        L.pcabi_event_record(e1, stream)
        L.pcabi_stream_sync(stream)
        f = ctypes.c_float()
        L.pcabi_event_elapsed_ms(ctypes.byref(f), e0, e1)
        if r >= 2:
            ms.append(f.value)
    cells = n * E * sum(lens)
    t = float(np.median(ms))
    print('adapters %s: %.3f ms, %.2f T cells/s' % (sys.argv[1], t, cells / t / 1e9))


if __name__ == '__main__':
    main()

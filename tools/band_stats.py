"""Band-class lane statistics of one middle-scan step, from pcabi_scan_profile's counters (the
profiled launches of k_seed_band_pin count their row iterations x 64 lanes, active lane-rows, tasks
and passes): the lanes a pass leaves idle behind its longest task. GPU only.

    python tools/band_stats.py [mean_len]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    mean_len = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    import torch  # noqa: F401
    from custom_porechop_abi_amd import _lib, engine, synth
    from custom_porechop_abi_amd import adapters as A
    from custom_porechop_abi_amd.porechop_abi import middle_adapter_list
    L = _lib.lib()
    vp = ctypes.c_void_p
    sets = [a for a in A.fresh_adapters() if '(full sequence)' not in a.name][:50]
    mid = [x[1] for x in middle_adapter_list(sets)[0]]
    reads = synth.make_reads(20000, mean_len, seed=12345)
    pack = engine.SeqPack([synth.codes_to_str(r) for r in reads])
    codes, offs, lens = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    held = []

    def h2d(arr):
        arr = np.ascontiguousarray(arr)
        p = vp()
        _lib.check(L.pcabi_dev_malloc(ctypes.byref(p), max(arr.nbytes, 16)), 'malloc')
        held.append(p)
        _lib.check(L.pcabi_dev_h2d(p, arr.ctypes.data_as(vp), arr.nbytes), 'h2d')
        return p
    d_codes, d_off, d_len = h2d(codes), h2d(offs.astype(np.int64)), h2d(lens.astype(np.int32))
    c, o, ln = engine.encode_adapters(mid)
    tab, scan = vp(), vp()
    sc = (3, -6, -5, -2)
    _lib.check(L.pcabi_adapters_create_scored(c.ctypes.data_as(vp), o.ctypes.data_as(vp), ln.ctypes.data_as(vp),
                                              len(mid), *sc, ctypes.byref(tab)), 'adapters')
    _lib.check(L.pcabi_scan_create(tab, ctypes.byref(scan)), 'scan')
    h_len = np.ascontiguousarray(lens, np.int32)
    cap = 8 * len(lens) + 1024
    hits = np.zeros((6, cap), np.int32)
    prof = np.zeros(26, np.float64)
    for k in range(2):
        if k == 1:
            assert L.pcabi_scan_profile(scan, 1, None, 0) == 26
        nh = L.pcabi_middle_scan_dev(scan, d_codes, d_off, d_len, h_len.ctypes.data_as(vp), len(lens), *sc, 90.0,
                                     hits.ctypes.data_as(vp), cap, None)
        _lib.check(int(min(nh, 0)), 'scan')
    assert L.pcabi_scan_profile(scan, 0, prof.ctypes.data_as(vp), 26) == 26
    L.pcabi_scan_destroy(scan)
    L.pcabi_adapters_destroy(tab)
    for p in held:
        L.pcabi_dev_free(p)
    print('bands %.3f ms (profiled rounds)' % prof[2])
    for c in range(2):
        it, act, tasks, passes = (int(x) for x in prof[16 + 4 * c:20 + 4 * c])
        if it:
            print('class %d (E %d): lane-rows %d of %d (%.3f active), tasks %d, passes %d, rows/task %.2f, '
                  'iterations/pass %.2f' % (c, int(prof[24 + c]), act, it, act / it, tasks, passes,
                                            act / max(tasks, 1), it / 64 / max(passes, 1)))


if __name__ == '__main__':
    main()

"""Band-class lane statistics of one middle-scan step (experiments: a -DPCABI_BAND_STATS build of
pcabi_seed, tools/build_variant.sh): per class, row iterations x 64 lanes against active lane-rows --
the lanes a pass of k_seed_band_pin leaves idle behind its longest task. GPU only.

    PCABI_LIB=perf_variants/bandstats.so python tools/band_stats.py [mean_len]
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
    sets = [a for a in A.fresh_adapters() if '(full sequence)' not in a.name][:50]
    mid = [x[1] for x in middle_adapter_list(sets)[0]]
    reads = synth.make_reads(20000, mean_len, seed=12345)
    pack = engine.SeqPack([synth.codes_to_str(r) for r in reads])
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    f = L.pcabi_debug_band_stats
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    out = np.zeros(8, np.uint64)
    os.environ.setdefault('PCABI_MIDDLE_SEEDS', '2')
    engine.middle_scan(views, mid, (3, -6, -5, -2), 90.0)
    f(out.ctypes.data, 1)
    engine.middle_scan(views, mid, (3, -6, -5, -2), 90.0)
    rc = f(out.ctypes.data, 1)
    for c, name in ((0, 'class 0 (E small)'), (1, 'class 1 (E large)')):
        it, act, tasks, passes = (int(x) for x in out[4 * c:4 * c + 4])
        if it:
            print('%s: rc %d, lane-rows %d of %d (%.3f active), tasks %d, passes %d, rows/task %.2f, '
                  'iterations/pass %.2f' % (name, rc, act, it, act / it, tasks, passes, act / max(tasks, 1),
                                            it / 64 / max(passes, 1)))


if __name__ == '__main__':
    main()

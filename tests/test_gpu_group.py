"""Grouped cross launches (r06): pcabi_align_cross_multi_dev runs several regions' cross products
with the register buckets of one core family -- the run-tagged core (affine, <= 32 rows) and the
packed core (affine, 36..64 rows) -- grouped across regions into one launch each
(csrc/pcabi_k_group.hip). Results must equal the oracle's, and the per-region
pcabi_align_cross_dev's, bit for bit on every field: end-trim windows of both read ends (the
headline's shape: 150 bp windows, adapters of 1..60 bp, several units per class), ragged windows
over several tiles, a class with a single unit (launched alone), buckets outside both classes
(wide, long, generic) and linear-gap schemes (no grouping at all)."""
import ctypes
import random

import numpy as np
import pytest

from tests import oracle_lib
from tests.test_gpu_parity import SCHEMES, _mutate, _rand_seq


def _region_cases(seed):
    rng = random.Random(seed)
    lens = [1, 5, 8, 21, 22, 23, 24, 24, 24, 25, 27, 28, 30, 33, 37, 38, 44, 50, 52, 57, 60]
    start = [_rand_seq(rng, L, 'ACGT') for L in lens]
    # the end table: a run-tagged pair, one 40-row bucket alone in its class, a wide and a long adapter
    end = [_rand_seq(rng, L, 'ACGT') for L in (24, 24, 30, 38, 70, 100)]
    reads = []
    for k in range(700):
        n = rng.choice([0, 1, 40, 150, 150, 150, rng.randint(150, 2400)])
        r = _rand_seq(rng, n, rng.choice(['ACGT', 'ACGT', 'ACGTN']))
        if n > 60:
            a = _mutate(rng, rng.choice(start + end), 0.08)
            p = rng.randint(0, max(0, n - len(a)))
            r = r[:p] + a + r[p + len(a):]
        reads.append(r)
    return reads, start, end


@pytest.mark.gpu
@pytest.mark.parametrize('scheme', SCHEMES[:6])
@pytest.mark.parametrize('side', [1, 0])
def test_cross_multi_regions(gpu_lib, scheme, side):
    from custom_porechop_abi_amd import _lib, engine
    L, vp = gpu_lib, ctypes.c_void_p
    reads, start, end = _region_cases(hash(scheme) & 0xFFFF)
    n = len(reads)
    # region windows: the start windows (first 150 bases), the end windows (last 150), and the
    # whole reads (ragged: several kb, more than one tile of one length)
    wins = [[r[:150] for r in reads], [r[-150:] if len(r) > 150 else r for r in reads], reads]
    tables = [start, end, start[::3] + end[:2]]
    bufs, tabs = [], []

    def h2d(a):
        a = np.ascontiguousarray(a)
        p = vp()
        _lib.check(L.pcabi_dev_malloc(ctypes.byref(p), max(a.nbytes, 16)), 'malloc')
        _lib.check(L.pcabi_dev_h2d(p, a.ctypes.data_as(vp), a.nbytes), 'h2d')
        bufs.append(p)
        return p

    def dalloc(nbytes):
        p = vp()
        _lib.check(L.pcabi_dev_malloc(ctypes.byref(p), max(nbytes, 16)), 'malloc')
        bufs.append(p)
        return p

    prev = L.pcabi_set_side_streams(side)
    try:
        regions, singles, outs = [], [], []
        for w, adps in zip(wins, tables):
            pack = engine.SeqPack(w)
            lens = pack.lengths.astype(np.int32)
            offs = pack.offsets.astype(np.int64)
            toff = np.zeros((n + 255) // 256 + 1, np.int64)
            nd = L.pcabi_tile_layout(lens.ctypes.data_as(vp), n, toff.ctypes.data_as(vp))
            d_codes, d_off, d_len, d_toff = h2d(pack.codes), h2d(offs), h2d(lens), h2d(toff)
            d_tiles = dalloc(4 * int(nd))
            _lib.check(L.pcabi_tile_windows_dev(d_codes, d_off, d_len, n, d_toff, int(np.diff(toff).max() // 256),
                                                d_tiles, None), 'tile')
            c, o, l = engine.encode_adapters(adps)
            tab = vp()
            _lib.check(L.pcabi_adapters_create_scored(c.ctypes.data_as(vp), o.ctypes.data_as(vp), l.ctypes.data_as(vp),
                                                      len(adps), *scheme, ctypes.byref(tab)), 'adapters_create')
            tabs.append(tab)
            stride = n * len(adps)
            d_out, d_ref = dalloc(4 * 8 * stride), dalloc(4 * 8 * stride)
            _lib.check(L.pcabi_dev_memset(d_out, 0x5A, 4 * 8 * stride), 'memset')
            regions.append((d_tiles, d_toff, d_len, n, max(1, int(lens.max())), tab, d_out, stride))
            singles.append((d_tiles, d_toff, d_len, n, max(1, int(lens.max())), tab, d_ref, stride))
            outs.append((d_out, d_ref, stride, adps, w))
        arr = _lib.cross_regions(regions)
        st, e0, e1 = vp(), vp(), vp()
        _lib.check(L.pcabi_stream_create(ctypes.byref(st)), 'stream')
        _lib.check(L.pcabi_event_create(ctypes.byref(e0)), 'event')
        _lib.check(L.pcabi_event_create(ctypes.byref(e1)), 'event')
        _lib.check(L.pcabi_align_cross_multi_dev(arr, len(regions), *scheme, st, e0, e1), 'multi')
        for r in singles:
            _lib.check(L.pcabi_align_cross_dev(*r[:6], *scheme, r[6], r[7], st), 'align')
        _lib.check(L.pcabi_stream_sync(st), 'sync')
        ms = ctypes.c_float()
        _lib.check(L.pcabi_event_elapsed_ms(ctypes.byref(ms), e0, e1), 'elapsed')
        assert ms.value > 0.0
        for e in (e0, e1):
            L.pcabi_event_destroy(e)
        L.pcabi_stream_destroy(st)
        for d_out, d_ref, stride, adps, w in outs:
            got = np.zeros((8, stride), np.int32)
            ref = np.zeros((8, stride), np.int32)
            _lib.check(L.pcabi_dev_d2h(got.ctypes.data_as(vp), d_out, got.nbytes), 'd2h')
            _lib.check(L.pcabi_dev_d2h(ref.ctypes.data_as(vp), d_ref, ref.nbytes), 'd2h')
            assert np.array_equal(got, ref)
            exp = oracle_lib.align_many(w, adps, (np.tile(np.arange(n), len(adps)), np.repeat(np.arange(len(adps)), n)),
                                        scheme)
            ok = exp[0] != -1
            assert np.array_equal(got[0], exp[0])
            assert np.array_equal(got[:, ok], exp[:, ok])
    finally:
        L.pcabi_set_side_streams(prev)
        for t in tabs:
            L.pcabi_adapters_destroy(t)
        for p in bufs:
            L.pcabi_dev_free(p)


@pytest.mark.gpu
def test_cross_multi_empty_and_bad_args(gpu_lib):
    from custom_porechop_abi_amd import _lib
    L = gpu_lib
    assert L.pcabi_align_cross_multi_dev(None, 0, 3, -6, -5, -2, None, None, None) == 0
    assert L.pcabi_align_cross_multi_dev(None, 1, 3, -6, -5, -2, None, None, None) != 0
    bad = _lib.cross_regions([(0, 0, 0, 5, 150, 0, 0, 0)])
    assert L.pcabi_align_cross_multi_dev(bad, 1, 3, -6, -5, -2, None, None, None) != 0

"""Batches back to back with their memory-bound steps overlapped (bench.py
--overlap-steps): two sets of tiles and results; batch k+1's pcabi_tile_windows_dev and batch k's
pcabi_end_trim_dev run on a second stream while the main stream runs batch k's
pcabi_align_cross_multi_dev, ordered by events only. Every batch holds DIFFERENT reads, so a tile or
result buffer reused too early would hand one batch another's windows or alignments: each batch's
trim amounts must equal the oracle's end decisions for its own reads (nanopore_read.py:175-217's
rules over the reference alignments, tests/oracle_lib.end_decisions_windows)."""
import ctypes
import random

import numpy as np
import pytest

from tests import oracle_lib
from tests.test_gpu_parity import _mutate, _rand_seq

E = 150
SCHEME = (3, -6, -5, -2)


def _batch(rng, n, adps):
    reads = []
    for _ in range(n):
        L = rng.choice([0, 30, 150, 400, rng.randint(150, 3000)])
        r = _rand_seq(rng, L, 'ACGT')
        if L > 60 and rng.random() < 0.7:
            a = _mutate(rng, rng.choice(adps), 0.06)
            p = rng.randint(0, 20) if rng.random() < 0.5 else max(0, L - len(a) - rng.randint(0, 20))
            r = r[:p] + a + r[p + len(a):]
        reads.append(r[:L])
    return reads


@pytest.mark.gpu
def test_overlapped_batches_match_the_oracle(gpu_lib):
    from custom_porechop_abi_amd import _lib, engine
    L, vp = gpu_lib, ctypes.c_void_p
    rng = random.Random(606)
    # both grouped classes (run-tagged <= 32 rows, packed 36..64) and a bucket of one adapter
    start = [_rand_seq(rng, k, 'ACGT') for k in (22, 24, 28, 40, 52)]
    end = [_rand_seq(rng, k, 'ACGT') for k in (24, 26, 44)]
    sizes = [1300, 700, 1500, 900, 1100]
    batches = [_batch(rng, m, start + end) for m in sizes]
    bufs, tabs, streams, events = [], [], [], []

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
        _lib.check(L.pcabi_dev_memset(p, 0x5A, max(nbytes, 16)), 'memset')
        bufs.append(p)
        return p

    try:
        for adps in (start, end):
            c, o, l = engine.encode_adapters(adps)
            t = vp()
            _lib.check(L.pcabi_adapters_create_scored(c.ctypes.data_as(vp), o.ctypes.data_as(vp), l.ctypes.data_as(vp),
                                                      len(adps), *SCHEME, ctypes.byref(t)), 'adapters_create')
            tabs.append(t)
        # per batch: its reads on the device, each side's window offsets / lengths and tile layout,
        # its own trim outputs; the tile and result buffers are the two shared sets
        per, nd_max = [], 0
        for reads in batches:
            n = len(reads)
            pack = engine.SeqPack(reads)
            offs = pack.offsets.astype(np.int64)
            lens = pack.lengths.astype(np.int64)
            s_len = np.minimum(lens, E).astype(np.int32)
            e_len = s_len.copy()
            e_off = offs + lens - e_len
            b = dict(n=n, codes_host=pack.codes, wins=[(offs, s_len), (e_off, e_len)], d_codes=h2d(pack.codes),
                     sides=[], d_st=dalloc(4 * n), d_et=dalloc(4 * n))
            for w_off, w_len in b['wins']:
                toff = np.zeros((n + 255) // 256 + 1, np.int64)
                nd = int(L.pcabi_tile_layout(w_len.ctypes.data_as(vp), n, toff.ctypes.data_as(vp)))
                nd_max = max(nd_max, nd)
                b['sides'].append(dict(d_off=h2d(w_off), d_len=h2d(w_len), d_toff=h2d(toff),
                                       mq=int(np.diff(toff).max() // 256), mx=max(1, int(w_len.max()))))
            per.append(b)
        n_max = max(sizes)
        tiles = [[dalloc(4 * nd_max) for _ in range(2)] for _ in range(2)]          # [set][side]
        res = [[dalloc(4 * 8 * len(adps) * n_max) for adps in (start, end)] for _ in range(2)]
        main, aux = vp(), vp()
        for s_ in (main, aux):
            _lib.check(L.pcabi_stream_create(ctypes.byref(s_)), 'stream')
            streams.append(s_)
        ev = {k: [vp(), vp()] for k in ('tile', 'align', 'trim')}
        used = {k: [False, False] for k in ev}
        for k in ev:
            for e_ in ev[k]:
                _lib.check(L.pcabi_event_create(ctypes.byref(e_)), 'event')
                events.append(e_)

        def record(kind, s_, st):
            L.pcabi_event_record(ev[kind][s_], st)
            used[kind][s_] = True

        def wait(st, kind, s_):
            if used[kind][s_]:
                L.pcabi_stream_wait_event(st, ev[kind][s_])

        def issue_tiles(k, s_):
            b = per[k]
            wait(aux, 'align', s_)
            for side, sd in enumerate(b['sides']):
                _lib.check(L.pcabi_tile_windows_dev(b['d_codes'], sd['d_off'], sd['d_len'], b['n'], sd['d_toff'],
                                                    sd['mq'], tiles[s_][side], aux), 'tile')
            record('tile', s_, aux)

        issue_tiles(0, 0)
        for k, b in enumerate(per):
            s_, n = k % 2, b['n']
            regions = _lib.cross_regions([(tiles[s_][side], sd['d_toff'], sd['d_len'], n, sd['mx'], tabs[side],
                                           res[s_][side], len(adps) * n)
                                          for side, (sd, adps) in enumerate(zip(b['sides'], (start, end)))])
            wait(main, 'tile', s_)
            wait(main, 'trim', s_)
            _lib.check(L.pcabi_align_cross_multi_dev(regions, 2, *SCHEME, main, None, None), 'multi')
            record('align', s_, main)
            if k + 1 < len(per):
                issue_tiles(k + 1, 1 - s_)
            wait(aux, 'align', s_)
            _lib.check(L.pcabi_end_trim_dev(res[s_][0], len(start) * n, len(start), res[s_][1], len(end) * n, len(end),
                                            n, E, 2, 75.0, 4, b['d_st'], b['d_et'], None, None, aux), 'end_trim')
            record('trim', s_, aux)
        for s_ in (aux, main):
            _lib.check(L.pcabi_stream_sync(s_), 'sync')
        for b in per:
            st = np.empty(b['n'], np.int32)
            et = np.empty(b['n'], np.int32)
            _lib.check(L.pcabi_dev_d2h(st.ctypes.data_as(vp), b['d_st'], st.nbytes), 'd2h')
            _lib.check(L.pcabi_dev_d2h(et.ctypes.data_as(vp), b['d_et'], et.nbytes), 'd2h')
            exp_s, exp_e, _, _, _ = oracle_lib.end_decisions_windows(b['codes_host'], b['wins'][0], b['wins'][1], start,
                                                                     end, SCHEME, E, 2, 75.0, 4)
            assert np.array_equal(st, exp_s)
            assert np.array_equal(et, exp_e)
            assert (st > 0).any() and (et > 0).any()   # the planted adapters are found
    finally:
        for e_ in events:
            L.pcabi_event_destroy(e_)
        for s_ in streams:
            L.pcabi_stream_destroy(s_)
        for t in tabs:
            L.pcabi_adapters_destroy(t)
        for p in bufs:
            L.pcabi_dev_free(p)

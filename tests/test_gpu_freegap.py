"""GPU parity under the scoring schemes the other GPU tests never use: gap costs >= 0, match <= 0,
all zero. The reference takes any four integers as --scoring_scheme
(porechop_abi/arg_parser.py:229-236) and aligns reads of any length under them
(porechop_abi/src/adapter_align.cpp:11-31, SeqAn's Score(match, mismatch, gapExtend, gapOpen)).

Under such a scheme no path span is bounded, so the register cores' start-column field (mod 2^16)
cannot serve windows of 32 k and more: the engine routes those to the striped core, whose
attributes never wrap (pcabi_engine.hip needs_striped / adapters_for). Checked here, on the GPU:
  * the reference's own result text (tests/golden/g1_freegap.tsv.gz, from oracle/_ref) through
    the batch ABI (pairs) and the legacy adapterAlignment symbol, reads of 33-70 kb included;
  * cross product and pairs vs the oracle (ragged windows, tie-heavy alphabets);
  * the device table ABI (pcabi_align_cross_dev) with a table laid out for another scoring and
    with a 40 kb window among short ones (the cached alternate layouts);
  * the whole-read middle scan with reads of 40-70 kb, hits past the 32 k mark.
"""
import ctypes
import random

import numpy as np
import pytest

from tests import golden_lib, oracle_lib
from tests.test_gpu_parity import _case_set, _first_diff, _mutate, _rand_seq

FREE_SCHEMES = [(2, -1, 0, 0), (3, -6, 0, -2), (1, -1, 1, 1), (0, 0, 0, 0), (-1, -1, -1, -1), (3, -6, 2, -1),
                (5, -4, -1, 0), (3, -6, -8, 0)]


def _fmt(res):
    rs, re_, as_, ae, score, m, l1, l2 = (int(x) for x in res)
    p1 = '-nan' if l1 == 0 else '%f' % (100.0 * m / l1)
    p2 = '-nan' if l2 == 0 else '%f' % (100.0 * m / l2)
    return '%d,%d,%d,%d,%d,%s,%s' % (rs, re_, as_, ae, score, p1, p2)


def _same_text(got, exp):
    if exp.split(',')[0] == '-1':          # empty input: only field 0 is defined by the reference
        return got.split(',')[0] == '-1'
    return got == exp


@pytest.mark.gpu
def test_freegap_reference_rows_batch_and_legacy(gpu_lib):
    """Every row of the reference's free-gap fixture through pcabi_align_host (explicit pairs; the
    short rows on the register cores, the 33-70 kb reads on the striped core) and a third of them
    -- every long read among them -- through the legacy adapterAlignment text, which no longer
    aborts on these schemes."""
    from custom_porechop_abi_amd import cpp_function_wrappers as w
    from custom_porechop_abi_amd import engine
    rows = golden_lib.g1_freegap_rows()
    n_long = 0
    for sc in FREE_SCHEMES:
        mine = [x for x in rows if x[0] == sc]
        assert len(mine) >= 250
        for long_batch in (False, True):
            part = [x for x in mine if (len(x[1]) >= 32768) == long_batch]
            if not part:
                continue
            reads, adps = [x[1] for x in part], [x[2] or 'A' for x in part]
            pack = engine.SeqPack(reads)
            views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
            idx = np.arange(len(part), dtype=np.int32)
            ok_adp = np.array([bool(x[2]) for x in part])
            got = engine.align(views, adps, sc, pairs=(idx[ok_adp], idx[ok_adp]))
            for k, j in enumerate(np.nonzero(ok_adp)[0].tolist()):
                assert _same_text(_fmt(got[:, k]), part[j][3]), (sc, len(reads[j]), len(adps[j]), part[j][3],
                                                                 got[:, k].tolist())
            n_long += len(part) if long_batch else 0
        for k, (_, r, a, exp) in enumerate(mine):
            if k % 3 == 0 or len(r) >= 32768:
                assert _same_text(w.adapter_alignment(r, a, list(sc)), exp), (sc, len(r), len(a))
    assert n_long >= 30


@pytest.mark.gpu
@pytest.mark.parametrize('scheme', FREE_SCHEMES)
def test_freegap_cross_and_pairs(gpu_lib, scheme):
    """Cross product and explicit pairs vs the oracle: adapters of 1-128 bp (the generic register
    buckets these schemes get) and past 128 (striped), ragged windows over random and tie-heavy
    alphabets, planted mutated copies."""
    from custom_porechop_abi_amd import engine
    for seed in range(2):
        reads, adps = _case_set(500 * seed + abs(hash(scheme)) % 991, 80, 8, 400, 140)
        pack = engine.SeqPack(reads)
        views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
        n = len(reads)
        got = engine.align(views, adps, scheme)
        exp = oracle_lib.align_many(reads, adps, (np.tile(np.arange(n), len(adps)), np.repeat(np.arange(len(adps)), n)),
                                    scheme)
        ok = exp[0] != -1
        assert np.array_equal(got[0], exp[0])
        assert np.array_equal(got[:, ok], exp[:, ok]), _first_diff(got, exp, reads, adps, n)
        rng = random.Random(seed)
        pr = np.array([rng.randrange(n) for _ in range(400)], np.int32)
        pa = np.array([rng.randrange(len(adps)) for _ in range(400)], np.int32)
        got = engine.align(views, adps, scheme, pairs=(pr, pa))
        exp = oracle_lib.align_many(reads, adps, (pr, pa), scheme)
        ok = exp[0] != -1
        assert np.array_equal(got[0], exp[0]) and np.array_equal(got[:, ok], exp[:, ok])


def _device_cross(L, reads, adps, scheme, table_scheme):
    """pcabi_tile_layout -> pcabi_tile_windows_dev -> pcabi_align_cross_dev with a table built for
    table_scheme (None: pcabi_adapters_create, the unscored register layout)."""
    from custom_porechop_abi_amd import _lib, engine
    vp = ctypes.c_void_p
    pack = engine.SeqPack(reads)
    n = len(reads)
    lens = pack.lengths.astype(np.int32)
    offs = pack.offsets.astype(np.int64)
    toff = np.zeros((n + 255) // 256 + 1, np.int64)
    nd = L.pcabi_tile_layout(lens.ctypes.data_as(vp), n, toff.ctypes.data_as(vp))
    bufs = []

    def h2d(a):
        a = np.ascontiguousarray(a)
        p = vp()
        _lib.check(L.pcabi_dev_malloc(ctypes.byref(p), max(a.nbytes, 16)), 'malloc')
        _lib.check(L.pcabi_dev_h2d(p, a.ctypes.data_as(vp), a.nbytes), 'h2d')
        bufs.append(p)
        return p

    d_codes, d_off, d_len, d_toff = h2d(pack.codes), h2d(offs), h2d(lens), h2d(toff)
    d_tiles, d_out = vp(), vp()
    stride = n * len(adps)
    _lib.check(L.pcabi_dev_malloc(ctypes.byref(d_tiles), 4 * int(nd)), 'malloc')
    _lib.check(L.pcabi_dev_malloc(ctypes.byref(d_out), 4 * 8 * stride), 'malloc')
    bufs += [d_tiles, d_out]
    c, o, l = engine.encode_adapters(adps)
    tab = vp()
    if table_scheme is None:
        _lib.check(L.pcabi_adapters_create(c.ctypes.data_as(vp), o.ctypes.data_as(vp), l.ctypes.data_as(vp), len(adps),
                                           ctypes.byref(tab)), 'adapters_create')
    else:
        _lib.check(L.pcabi_adapters_create_scored(c.ctypes.data_as(vp), o.ctypes.data_as(vp), l.ctypes.data_as(vp),
                                                  len(adps), *table_scheme, ctypes.byref(tab)), 'adapters_create')
    try:
        _lib.check(L.pcabi_tile_windows_dev(d_codes, d_off, d_len, n, d_toff, int(np.diff(toff).max() // 256), d_tiles,
                                            None), 'tile')
        _lib.check(L.pcabi_align_cross_dev(d_tiles, d_toff, d_len, n, int(lens.max()), tab, *scheme, d_out, stride,
                                           None), 'align')
        _lib.check(L.pcabi_dev_sync(), 'sync')
        got = np.zeros((8, stride), np.int32)
        _lib.check(L.pcabi_dev_d2h(got.ctypes.data_as(vp), d_out, got.nbytes), 'd2h')
    finally:
        L.pcabi_adapters_destroy(tab)
        for p in bufs:
            L.pcabi_dev_free(p)
    return got


@pytest.mark.gpu
@pytest.mark.parametrize('table', ['unscored', 'other_scoring', 'own_scoring'])
def test_freegap_device_table_abi(gpu_lib, table):
    """The device table ABI serves any scoring on any window: a table laid out without a scoring
    (padded fast buckets), one merged for the default scheme, and one built for the scheme itself,
    each called with free-gap schemes on short windows and on a batch holding a 40 kb window (the
    striped layout); every field vs the oracle."""
    rng = random.Random(77)
    adps = ['AATGTACTTCGTTCAGTTACGTATTGCT', 'GCAATACGTAACTGAACGAAGT', 'ACGTTTAGG', _rand_seq(rng, 50, 'ACGT'),
            _rand_seq(rng, 70, 'ACGT'), _rand_seq(rng, 111, 'ACGT'), _rand_seq(rng, 140, 'ACGT')]
    short = []
    for k in range(150):
        r = _rand_seq(rng, rng.choice([0, 1, 30, 150, rng.randint(1, 900)]), rng.choice(['ACGT', 'ACGTN', 'AT']))
        if len(r) > 20 and rng.random() < 0.6:
            p = rng.randint(0, len(r))
            r = r[:p] + _mutate(rng, rng.choice(adps), 0.05) + r[p:]
        short.append(r)
    big = _rand_seq(rng, 40000, 'ACGT')
    big = big[:33000] + adps[0] + big[33000:]
    for scheme in [(2, -1, 0, 0), (5, -4, -1, 0), (3, -6, 2, -1)]:
        tsc = {'unscored': None, 'other_scoring': (3, -6, -5, -2), 'own_scoring': scheme}[table]
        for reads in (short, short[:40] + [big]):
            got = _device_cross(gpu_lib, reads, adps, scheme, tsc)
            n = len(reads)
            exp = oracle_lib.align_many(reads, adps, (np.tile(np.arange(n), len(adps)),
                                                      np.repeat(np.arange(len(adps)), n)), scheme)
            ok = exp[0] != -1
            assert np.array_equal(got[0], exp[0])
            assert np.array_equal(got[:, ok], exp[:, ok]), (scheme, _first_diff(got, exp, reads, adps, n))


@pytest.mark.gpu
@pytest.mark.parametrize('scheme', [(5, -4, -1, 0), (3, -6, -8, 0), (2, -1, 0, 0), (3, -6, 0, -2)])
def test_freegap_middle_scan_long_reads(gpu_lib, scheme):
    """The whole-read middle scan (the reference's masked loop, nanopore_read.py:219-252) under
    free-gap schemes, reads of 200 bp - 3 kb next to reads of 40-70 kb with copies past the 32 k
    mark: every hit, in every round, vs the oracle's loop."""
    from custom_porechop_abi_amd import engine
    rng = random.Random(9)
    adps = ['AATGTACTTCGTTCAGTTACGTATTGCT', 'GCAATACGTAACTGAACGAAGT', 'ACGTTTAGGCATTGCAGGTA', _rand_seq(rng, 33, 'ACGT'),
            _rand_seq(rng, 50, 'ACGT')]
    reads = []
    for k in range(24):
        n = rng.randint(40000, 70000) if k % 4 == 3 else rng.randint(200, 3000)
        r = _rand_seq(rng, n, 'ACGT')
        for _ in range(rng.choice([1, 2, 3])):
            a = _mutate(rng, rng.choice(adps), rng.choice([0.0, 0.0, 0.03]))
            p = rng.randint(32800, n) if n > 40000 and rng.random() < 0.7 else rng.randint(0, n)
            r = r[:p] + a + r[p:]
        reads.append(r)
    assert sum(len(r) >= 40000 for r in reads) >= 5
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    exp = oracle_lib.middle_scan_threaded(views, adps, scheme, 90.0)
    got = engine.middle_scan(views, adps, scheme, 90.0)
    og = np.lexsort((np.arange(got.shape[1]), got[0]))
    oe = np.lexsort((np.arange(exp.shape[1]), exp[0]))
    assert got.shape == exp.shape and np.array_equal(got[:, og], exp[:, oe])
    if scheme[2] < 0 and scheme[3] == 0:   # opens cost, extensions free: the planted copies hit, long reads' too
        assert exp.shape[1] >= 30 and (exp[2] > 32768).sum() >= 5

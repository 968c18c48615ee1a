"""GPU parity: libpcabi.so (HIP, gfx950) vs the CPU oracle, bit-exact on every integer field.

Oracle = oracle/pcabi_oracle.c, itself pinned to the reference's own outputs by
tests/test_oracle_golden.py. Sizes are chosen so the oracle finishes in seconds.
"""
import ctypes
import random

import numpy as np
import pytest

from tests import oracle_lib

SCHEMES = [(3, -6, -5, -2),   # reference default (arg_parser.py:178-180)
           (2, -1, -1, -1),   # linear gaps (open == extend)
           (1, -1, -3, -1),
           (3, -6, -2, -5),   # open cheaper than extend
           (5, -4, -8, -6),
           (1, 3, -5, -2),    # mismatch outscoring match (any --scoring_scheme is accepted)
           # gap costs >= 0, match <= 0, all zero: no path-span bound (tests/test_gpu_freegap.py
           # covers them on 32 k+ reads and the device table ABI)
           (2, -1, 0, 0), (3, -6, 0, -2), (1, -1, 1, 1), (0, 0, 0, 0), (-1, -1, -1, -1), (3, -6, 2, -1)]


def _rand_seq(rng, n, alph):
    return ''.join(rng.choice(alph) for _ in range(n))


def _mutate(rng, s, rate):
    out = []
    for c in s:
        x = rng.random()
        if x < rate / 3:
            out.append(rng.choice('ACGT'))
        elif x < 2 * rate / 3:
            continue
        elif x < rate:
            out.append(c)
            out.append(rng.choice('ACGT'))
        else:
            out.append(c)
    return ''.join(out)


def _native_full(i):
    """The native barcoding "full sequence" adapters of barcode i (68 bp start, 63 bp end,
    porechop_abi/adapters.py:466-477)."""
    from custom_porechop_abi_amd import adapters as A
    f = A.make_full_native_barcode_adapter(i)
    return [f.start_sequence[1], f.end_sequence[1]]


def _case_set(seed, n_reads, n_adp, max_read, max_adp):
    rng = random.Random(seed)
    alph = rng.choice(['ACGT', 'ACGTN', 'AT', 'A', 'ACGT-'])
    adps = [_rand_seq(rng, rng.choice([1, 2, 5, 8, 22, 24, 28, 32, 33, 50, rng.randint(1, max_adp)]), 'ACGT')
            for _ in range(n_adp)]
    reads = []
    for _ in range(n_reads):
        n = rng.choice([0, 1, 3, 17, 150, rng.randint(0, max_read)])
        r = _rand_seq(rng, n, alph)
        if n > 30 and rng.random() < 0.5:
            a = _mutate(rng, rng.choice(adps), 0.1)
            p = rng.randint(0, max(0, n - len(a)))
            r = r[:p] + a + r[p + len(a):]
        reads.append(r)
    return reads, adps


@pytest.mark.gpu
@pytest.mark.parametrize('scheme', SCHEMES)
def test_cross_product_parity(gpu_lib, scheme):
    from custom_porechop_abi_amd import engine
    for seed in range(3):
        reads, adps = _case_set(1000 * seed + hash(scheme) % 997, 96, 9, 260, 128)
        pack = engine.SeqPack(reads)
        got = engine.align(pack.views(np.zeros(len(reads), np.int64), pack.lengths), adps, scheme)
        n = len(reads)
        pr = np.tile(np.arange(n), len(adps))
        pa = np.repeat(np.arange(len(adps)), n)
        exp = oracle_lib.align_many(reads, adps, (pr, pa), scheme)
        ok = exp[0] != -1
        # rs == -1 (empty input): only field 0 is defined by the reference
        assert np.array_equal(got[0], exp[0])
        assert np.array_equal(got[:, ok], exp[:, ok]), _first_diff(got, exp, reads, adps, n)


def _first_diff(got, exp, reads, adps, n):
    bad = np.nonzero(np.any(got != exp, axis=0))[0]
    k = int(bad[0])
    return 'pair %d read=%r adapter=%r got=%s exp=%s' % (k, reads[k % n], adps[k // n], got[:, k], exp[:, k])


@pytest.mark.gpu
def test_pairs_mode_and_windows(gpu_lib):
    """Explicit pairs + start/end windows of longer reads (the end-trim layout)."""
    from custom_porechop_abi_amd import engine
    rng = random.Random(7)
    reads, adps = _case_set(77, 200, 12, 1200, 64)
    pack = engine.SeqPack(reads)
    sw, ew = engine.start_end_windows(pack, 150)
    sc = (3, -6, -5, -2)
    pr = np.array([rng.randrange(len(reads)) for _ in range(3000)], np.int32)
    pa = np.array([rng.randrange(len(adps)) for _ in range(3000)], np.int32)
    for win, slicer in ((sw, lambda s: s[:150]), (ew, lambda s: s[-150:])):
        got = engine.align(win, adps, sc, pairs=(pr, pa))
        exp = oracle_lib.align_many([slicer(r) for r in reads], adps, (pr, pa), sc)
        ok = exp[0] != -1
        assert np.array_equal(got[0], exp[0])
        assert np.array_equal(got[:, ok], exp[:, ok])


@pytest.mark.gpu
def test_legacy_string_abi(gpu_lib):
    """adapterAlignment()/freeCString() return the reference's exact text."""
    from custom_porechop_abi_amd import cpp_function_wrappers as w
    known = [('ACGTACGTAC', 'GTAC', '2,5,0,3,12,100.000000,100.000000'),
             ('AAAAAAAAAA', 'AAAA', '0,3,0,3,12,100.000000,100.000000'),
             ('AAAA', 'AAAAAAAAAA', '0,3,0,3,12,100.000000,40.000000'),
             ('GGGGGGGG', 'TTTT', '0,0,4,3,0,-nan,0.000000'),
             ('A', 'C', '0,0,1,0,0,-nan,0.000000'),
             ('AC--GT', 'ACGT', '0,5,0,3,5,66.666667,66.666667')]
    for r, a, s in known:
        assert w.adapter_alignment(r, a, [3, -6, -5, -2]) == s
    assert w.adapter_alignment('', 'ACGT', [3, -6, -5, -2]).split(',')[0] == '-1'
    rng = random.Random(3)
    for _ in range(60):
        sc = rng.choice(SCHEMES)
        r = _rand_seq(rng, rng.randint(1, 400), 'ACGTN')
        a = _rand_seq(rng, rng.randint(1, 100), 'ACGT')
        assert w.adapter_alignment(r, a, list(sc)) == oracle_lib.result_string(r, a, sc)


@pytest.mark.gpu
def test_long_reads_middle_shape(gpu_lib):
    """Whole-read alignments (the middle-adapter scan shape): reads of several kb."""
    from custom_porechop_abi_amd import engine
    rng = random.Random(11)
    adps = ['AATGTACTTCGTTCAGTTACGTATTGCT', 'GCAATACGTAACTGAACGAAGT', 'ACGTTTAGGCAT']
    reads = []
    for k in range(70):
        n = rng.randint(1000, 9000)
        r = _rand_seq(rng, n, 'ACGT')
        if k % 3 == 0:
            a = _mutate(rng, adps[k % 2], 0.05)
            p = rng.randint(0, n - len(a))
            r = r[:p] + a + r[p + len(a):]
        reads.append(r)
    pack = engine.SeqPack(reads)
    sc = (3, -6, -5, -2)
    got = engine.align(pack.views(np.zeros(len(reads), np.int64), pack.lengths), adps, sc)
    n = len(reads)
    exp = oracle_lib.align_many(reads, adps, (np.tile(np.arange(n), 3), np.repeat(np.arange(3), n)), sc)
    assert np.array_equal(got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize('side', [1, 0])
@pytest.mark.parametrize('scored', [False, True])
@pytest.mark.parametrize('scheme', [(3, -6, -5, -2), (2, -1, -1, -1)])
def test_device_abi_tiled_cross(gpu_lib, scheme, scored, side):
    """Device-pointer ABI: pcabi_tile_layout -> pcabi_tile_windows_dev -> pcabi_align_cross_dev,
    with ragged windows (empty, 1 bp, several kb) and more than one tile. scored: the table is
    built for the scoring, so small register buckets are merged (extra padding rows), and the
    call goes through pcabi_align_cross_dev_marked on a stream of its own (events around the
    largest bucket). side: the buckets side by side on the side streams (1) or one after the
    other on the caller's stream (0, pcabi_set_side_streams)."""
    from custom_porechop_abi_amd import _lib, engine
    L, vp = gpu_lib, ctypes.c_void_p
    side_prev = L.pcabi_set_side_streams(side)
    try:
        _tiled_cross_case(L, _lib, engine, vp, scheme, scored)
    finally:
        L.pcabi_set_side_streams(side_prev)
    assert L.pcabi_set_side_streams(-1) == side_prev


@pytest.mark.gpu
@pytest.mark.parametrize('side', [1, 0])
def test_device_abi_per_stream_side_streams(gpu_lib, side):
    """pcabi_stream_side_streams (r05): the setting of the call's own stream wins over the
    process-wide one (set to the opposite here); the entry reports its previous value and -1
    removes it. Results bit-exact either way."""
    from custom_porechop_abi_amd import _lib, engine
    L, vp = gpu_lib, ctypes.c_void_p
    side_prev = L.pcabi_set_side_streams(1 - side)
    try:
        _tiled_cross_case(L, _lib, engine, vp, (3, -6, -5, -2), True, stream_side=side)
    finally:
        L.pcabi_set_side_streams(side_prev)


def _tiled_cross_case(L, _lib, engine, vp, scheme, scored, stream_side=None):
    reads, adps = _case_set(31, 700, 7, 3000, 64)
    adps = adps + ['ACGTTGCA' * k for k in (1, 2, 3, 4, 5, 6, 7)] + ['GATTACA' * 5 + 'G', 'TTAGGC' * 9]
    # wide register buckets (65..88 bp, packed-key core, pk::Lay<RPL > 64>) and past them (generic)
    adps = adps + _native_full(3) + ['ACGTTGCA' * 9, 'GATTACA' * 12, 'TTAGGCA' * 13]
    pack = engine.SeqPack(reads)
    n = len(reads)
    # windows seq[k:] with random (unaligned) starts k
    rng = random.Random(5)
    starts = np.array([rng.randint(0, min(7, len(r))) for r in reads], np.int64)
    _, offs, lens = pack.views(starts, (pack.lengths - starts).astype(np.int32))
    reads = [r[k:] for r, k in zip(reads, starts.tolist())]
    lens = lens.astype(np.int32)
    toff = np.zeros((n + 255) // 256 + 1, np.int64)
    nd = L.pcabi_tile_layout(lens.ctypes.data_as(vp), n, toff.ctypes.data_as(vp))
    assert nd == toff[-1] > 0
    bufs = []

    def h2d(a):
        a = np.ascontiguousarray(a)
        p = vp()
        _lib.check(L.pcabi_dev_malloc(ctypes.byref(p), max(a.nbytes, 16)), 'malloc')
        _lib.check(L.pcabi_dev_h2d(p, a.ctypes.data_as(vp), a.nbytes), 'h2d')
        bufs.append(p)
        return p

    d_codes, d_off, d_len, d_toff = h2d(pack.codes), h2d(offs), h2d(lens), h2d(toff)
    d_tiles = vp()
    _lib.check(L.pcabi_dev_malloc(ctypes.byref(d_tiles), 4 * int(nd)), 'malloc')
    bufs.append(d_tiles)
    c, o, l = engine.encode_adapters(adps)
    tab = vp()
    if scored:
        _lib.check(L.pcabi_adapters_create_scored(c.ctypes.data_as(vp), o.ctypes.data_as(vp), l.ctypes.data_as(vp),
                                                  len(adps), *scheme, ctypes.byref(tab)), 'adapters_create')
    else:
        _lib.check(L.pcabi_adapters_create(c.ctypes.data_as(vp), o.ctypes.data_as(vp), l.ctypes.data_as(vp),
                                           len(adps), ctypes.byref(tab)), 'adapters_create')
    stride = n * len(adps)
    d_out = vp()
    _lib.check(L.pcabi_dev_malloc(ctypes.byref(d_out), 4 * 8 * stride), 'malloc')
    bufs.append(d_out)
    try:
        mq = int(np.diff(toff).max() // 256)
        _lib.check(L.pcabi_tile_windows_dev(d_codes, d_off, d_len, n, d_toff, mq, d_tiles, None), 'tile')
        if scored:
            # the marked entry point: events around the largest bucket's launch, on the stream
            st, e0, e1 = vp(), vp(), vp()
            _lib.check(L.pcabi_stream_create(ctypes.byref(st)), 'stream')
            _lib.check(L.pcabi_event_create(ctypes.byref(e0)), 'event')
            _lib.check(L.pcabi_event_create(ctypes.byref(e1)), 'event')
            if stream_side is not None:
                assert L.pcabi_stream_side_streams(st, stream_side) == -1       # no entry before
                assert L.pcabi_stream_side_streams(st, stream_side) == stream_side
            _lib.check(L.pcabi_align_cross_dev_marked(d_tiles, d_toff, d_len, n, int(lens.max()), tab, *scheme,
                                                      d_out, stride, st, e0, e1), 'align')
            _lib.check(L.pcabi_stream_sync(st), 'sync')
            if stream_side is not None:
                assert L.pcabi_stream_side_streams(st, -1) == stream_side       # entry removed
                assert L.pcabi_stream_side_streams(st, -1) == -1
            ms = ctypes.c_float()
            _lib.check(L.pcabi_event_elapsed_ms(ctypes.byref(ms), e0, e1), 'elapsed')
            assert ms.value > 0.0
            for e in (e0, e1):
                L.pcabi_event_destroy(e)
            L.pcabi_stream_destroy(st)
        else:
            _lib.check(L.pcabi_align_cross_dev(d_tiles, d_toff, d_len, n, int(lens.max()), tab, *scheme, d_out,
                                               stride, None), 'align')
        _lib.check(L.pcabi_dev_sync(), 'sync')
        got = np.zeros((8, stride), np.int32)
        _lib.check(L.pcabi_dev_d2h(got.ctypes.data_as(vp), d_out, got.nbytes), 'd2h')
    finally:
        L.pcabi_adapters_destroy(tab)
        for p in bufs:
            L.pcabi_dev_free(p)
    exp = oracle_lib.align_many(reads, adps, (np.tile(np.arange(n), len(adps)), np.repeat(np.arange(len(adps)), n)),
                                scheme)
    ok = exp[0] != -1
    assert np.array_equal(got[0], exp[0])
    assert np.array_equal(got[:, ok], exp[:, ok]), _first_diff(got, exp, reads, adps, n)


@pytest.mark.gpu
@pytest.mark.parametrize('threshold', [90.0, 70.0])
def test_first_hits_middle_round1(gpu_lib, threshold):
    """Middle-scan round 1 (k_first_hit over a tiled cross product): first adapter over the
    threshold per whole read, vs the oracle."""
    from custom_porechop_abi_amd import engine
    rng = random.Random(int(threshold))
    adps = ['AATGTACTTCGTTCAGTTACGTATTGCT', 'GCAATACGTAACTGAACGAAGT', 'ACGTTTAGGCATTGCA',
            'TTGGCCAAGGTT' * 3]
    reads = []
    for k in range(300):
        n = rng.choice([0, 5, rng.randint(100, 4000)])
        r = _rand_seq(rng, n, 'ACGT')
        for _ in range(rng.randint(0, 2)):
            if n > 60:
                a = _mutate(rng, rng.choice(adps), rng.choice([0.0, 0.05, 0.15]))
                p = rng.randint(0, n - len(a))
                r = r[:p] + a + r[p + len(a):]
        reads.append(r)
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    sc = (3, -6, -5, -2)
    got = engine.first_hits(views, adps, sc, threshold)
    exp = oracle_lib.first_hits_windows(views, adps, sc, threshold)
    assert (exp[0] >= 0).sum() > 20
    assert np.array_equal(got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize('scheme', [(3, -6, -5, -2), (2, -1, -1, -1)])
def test_middle_scan_rounds(gpu_lib, scheme):
    """The whole masked re-alignment loop on the device (pcabi_middle_scan_host) vs the
    reference's loop restated on the oracle: reads carrying 0-4 adapters, repeats of the same
    adapter (several rounds), adjacent hits, empty and tiny reads."""
    from custom_porechop_abi_amd import engine
    rng = random.Random(sum(scheme) + 100)
    adps = ['AATGTACTTCGTTCAGTTACGTATTGCT', 'GCAATACGTAACTGAACGAAGT', 'ACGTTTAGGCATTGCA'] + _native_full(2)
    reads = []
    for k in range(160):
        n = rng.choice([0, 3, rng.randint(200, 3000)])
        r = _rand_seq(rng, n, 'ACGT')
        for _ in range(rng.choice([0, 0, 1, 2, 4])):
            if len(r) > 80:
                a = _mutate(rng, rng.choice(adps), rng.choice([0.0, 0.03, 0.1]))
                p = rng.randint(0, len(r))
                r = r[:p] + a + (a if rng.random() < 0.2 else '') + r[p:]
        reads.append(r)
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    got = engine.middle_scan(views, adps, scheme, 85.0)
    exp = oracle_lib.middle_scan_windows(views, adps, scheme, 85.0)
    assert exp.shape[1] > 40 and np.bincount(exp[0]).max() >= 3
    # per read, the hits in discovery order
    order_g = np.lexsort((np.arange(got.shape[1]), got[0]))
    order_e = np.lexsort((np.arange(exp.shape[1]), exp[0]))
    assert np.array_equal(got[:, order_g], exp[:, order_e])


def _edit_exactly(rng, s, k):
    """s with exactly k random edits (substitution to another base, deletion, insertion)."""
    s = list(s)
    for _ in range(k):
        op = rng.randrange(3)
        p = rng.randrange(len(s))
        if op == 0:
            s[p] = rng.choice([c for c in 'ACGT' if c != s[p]])
        elif op == 1 and len(s) > 1:
            del s[p]
        else:
            s.insert(p, rng.choice('ACGT'))
    return ''.join(s)


@pytest.mark.gpu
@pytest.mark.parametrize('threshold,scheme', [(90.0, (3, -6, -5, -2)), (88.0, (3, -6, -5, -2)),
                                              (85.0, (2, -1, -1, -1)), (90.0, (1, -1, -3, -1))])
def test_middle_scan_seeds(gpu_lib, monkeypatch, threshold, scheme):
    """Round 1 from exact k-mer seeds (pcabi_seed.hip, PCABI_MIDDLE_SEEDS=2) vs the oracle's
    masked loop: adapter copies with exactly 0 .. e_max + 2 edits (e_max = the most non-matching
    columns an alignment at the threshold can hold), copies cut at either read end (the adapter
    hangs off), repeats, N runs, and adapters of 16..102 bp (both band classes; the 102 bp one
    runs on the generic core, chunked like the packed one)."""
    from custom_porechop_abi_amd import engine
    L = gpu_lib
    rng = random.Random(int(threshold) * 7 + scheme[0])
    adps = ['AATGTACTTCGTTCAGTTACGTATTGCT', 'GCAATACGTAACTGAACGAAGT', 'ACGTTTAGGCATTGCA',
            _rand_seq(rng, 50, 'ACGT'), _rand_seq(rng, 64, 'ACGT'), _rand_seq(rng, 33, 'ACGT'),
            'TTTTTTTTTTAAAAAAAAAACCCCCGGGGG']
    if threshold >= 88.0:   # a long adapter (generic core: 102 bp, as the full rapid sequences)
        adps.append(_rand_seq(rng, 102, 'ACGT'))
    th = threshold / 100.0
    reads = []
    for k in range(240):
        n = rng.choice([0, 7, rng.randint(100, 2500)])
        r = _rand_seq(rng, n, 'ACGT' if rng.random() < 0.8 else 'ACGTN')
        for _ in range(rng.choice([0, 1, 1, 2, 3])):
            a = rng.choice(adps)
            e = int(len(a) * (1 - th) / th)
            a = _edit_exactly(rng, a, rng.randint(0, e + 2))
            where = rng.random()
            if where < 0.15:
                a = a[rng.randint(0, 4):]
                r = a + r
            elif where < 0.3:
                a = a[:len(a) - rng.randint(0, 4)]
                r = r + a
            else:
                p = rng.randint(0, len(r))
                r = r[:p] + a + (a if rng.random() < 0.15 else '') + r[p:]
        reads.append(r)
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    exp = oracle_lib.middle_scan_windows(views, adps, scheme, threshold)
    assert exp.shape[1] > 60
    order_e = np.lexsort((np.arange(exp.shape[1]), exp[0]))
    runs0 = L.pcabi_middle_seed_runs()
    monkeypatch.setenv('PCABI_MIDDLE_SEEDS', '2')
    got = engine.middle_scan(views, adps, scheme, threshold)
    assert L.pcabi_middle_seed_runs() > runs0, 'the seeded round 1 did not run'
    order_g = np.lexsort((np.arange(got.shape[1]), got[0]))
    assert np.array_equal(got[:, order_g], exp[:, order_e])
    # the seeded rounds plan the candidate DP on the device (default) with the chunk length set
    # by the wave target: the longest (512) and the shortest (64) chunks, and the host plan
    for env in (('PCABI_MIDDLE_PLAN_WAVES', '1'), ('PCABI_MIDDLE_PLAN_WAVES', '100000000'),
                ('PCABI_MIDDLE_DEVPLAN', '0')):
        monkeypatch.setenv(*env)
        assert np.array_equal(engine.middle_scan(views, adps, scheme, threshold), got), env
        monkeypatch.delenv(env[0])
    monkeypatch.setenv('PCABI_MIDDLE_SEEDS', '0')
    runs1 = L.pcabi_middle_seed_runs()
    got0 = engine.middle_scan(views, adps, scheme, threshold)
    assert L.pcabi_middle_seed_runs() == runs1
    assert np.array_equal(got0, got)


@pytest.mark.gpu
def test_middle_scan_equal_scores_in_chunks_from_the_read_start(gpu_lib, monkeypatch):
    """Device-planned candidate DP with the shortest chunks (64 owned columns): in a short read
    every chunk starts at offset 0 (the lead-in D covers the read start), and two exact copies of
    the adapter score the same in chunks 0 and 1 -- the merge must take chunk 0 (the full DP's
    first maximum) every time, the later copy is the second round's hit."""
    from custom_porechop_abi_amd import engine
    rng = random.Random(41)
    adp = _rand_seq(rng, 50, 'ACGT')
    reads = []
    for k in range(300):
        pre = _rand_seq(rng, rng.randint(0, 14), 'ACGT')
        mid = _rand_seq(rng, rng.randint(0, 6), 'ACGT')
        reads.append(pre + adp + mid + adp + _rand_seq(rng, rng.randint(0, 20), 'ACGT'))
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    sc = (3, -6, -5, -2)
    exp = oracle_lib.middle_scan_windows(views, [adp], sc, 88.0)
    monkeypatch.setenv('PCABI_MIDDLE_SEEDS', '2')
    monkeypatch.setenv('PCABI_MIDDLE_PLAN_WAVES', '100000000')
    assert exp.shape[1] == 2 * len(reads)
    order_e = np.lexsort((np.arange(exp.shape[1]), exp[0]))
    for _ in range(3):
        got = engine.middle_scan(views, [adp], sc, 88.0)
        order_g = np.lexsort((np.arange(got.shape[1]), got[0]))
        assert np.array_equal(got[:, order_g], exp[:, order_e])


@pytest.mark.gpu
@pytest.mark.parametrize('scheme', SCHEMES)
def test_long_adapters_two_pass(gpu_lib, scheme):
    """89-128 bp adapters (the 102 / 111 bp full rapid-barcode sequences among them) on the
    two-pass long buckets (pk::LayL) in cross mode, vs the oracle: end windows and whole reads
    carrying mutated copies, cut copies at the read ends, N runs."""
    from custom_porechop_abi_amd import adapters as A
    from custom_porechop_abi_amd import engine
    rng = random.Random(sum(scheme) * 13 + 5)
    adps = [A.make_new_full_rapid_barcode_adapter(3).start_sequence[1],
            A.make_old_full_rapid_barcode_adapter(7).start_sequence[1]] + \
        [_rand_seq(rng, L, 'ACGT') for L in (89, 96, 97, 112, 113, 128)]
    reads = []
    for k in range(180):
        n = rng.choice([1, 30, 150, rng.randint(100, 700)])
        r = _rand_seq(rng, n, 'ACGT' if rng.random() < 0.8 else 'ACGTN')
        if rng.random() < 0.7:
            cp = _mutate(rng, rng.choice(adps), rng.choice([0.0, 0.05, 0.15]))
            where = rng.random()
            if where < 0.25:
                r = cp[rng.randint(0, 30):] + r
            elif where < 0.5:
                r = r + cp[:len(cp) - rng.randint(0, 30)]
            else:
                p = rng.randint(0, len(r))
                r = r[:p] + cp + r[p:]
        reads.append(r)
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    got = engine.align(views, adps, scheme)
    n = len(reads)
    exp = oracle_lib.align_many(reads, adps, (np.tile(np.arange(n), len(adps)), np.repeat(np.arange(len(adps)), n)),
                                scheme)
    ok = exp[0] != -1
    assert np.array_equal(got[0], exp[0])
    assert np.array_equal(got[:, ok], exp[:, ok]), _first_diff(got, exp, reads, adps, n)


@pytest.mark.gpu
def test_middle_scan_seed_plan_follows_adapters(gpu_lib, monkeypatch):
    """The seed plan is cached per scan; consecutive host-API scans with different adapters of
    the same lengths (their tables may land at the same address) must each use their own
    probes: every scan equals the oracle."""
    from custom_porechop_abi_amd import engine
    monkeypatch.setenv('PCABI_MIDDLE_SEEDS', '2')
    rng = random.Random(4242)
    sc = (3, -6, -5, -2)
    for trial in range(4):
        adps = [_rand_seq(rng, L, 'ACGT') for L in (24, 24, 22, 28)]
        reads = []
        for k in range(60):
            r = _rand_seq(rng, rng.randint(300, 3000), 'ACGT')
            for _ in range(rng.choice([1, 2, 3])):
                a = _mutate(rng, rng.choice(adps), rng.choice([0.0, 0.04]))
                p = rng.randint(0, len(r))
                r = r[:p] + a + r[p:]
            reads.append(r)
        pack = engine.SeqPack(reads)
        views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
        got = engine.middle_scan(views, adps, sc, 90.0)
        exp = oracle_lib.middle_scan_windows(views, adps, sc, 90.0)
        assert exp.shape[1] > 40
        order_g = np.lexsort((np.arange(got.shape[1]), got[0]))
        order_e = np.lexsort((np.arange(exp.shape[1]), exp[0]))
        assert np.array_equal(got[:, order_g], exp[:, order_e]), trial


@pytest.mark.gpu
@pytest.mark.parametrize('split', ['2', '4', ''])
@pytest.mark.parametrize('scheme', [(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (1, 3, -5, -2)])
def test_row_split_cross_product(gpu_lib, monkeypatch, split, scheme):
    """Cross products of a few adapters over thousands of windows -- the launches the row-split
    core (k_align_split: K lanes per window, DPP row shifts, the last column in K phases) takes
    (PCABI_SPLIT unset: by wave count; 2 / 4 forced) -- vs the oracle on every field: run-tagged
    and packed buckets of 8..64 rows, adapters padded into larger buckets, ragged, empty and
    1-column windows, tie-heavy alphabets, planted mutated copies."""
    from custom_porechop_abi_amd import engine
    monkeypatch.setenv('PCABI_SPLIT', split)
    rng = random.Random(sum(scheme) * 31 + len(split))
    adps = ['AATGTACTTCGTTCAGTTACGTATTGCT', 'GCAATACGTAACTGAACGAAGT', 'CTTCGTTCAGTTACGTATTGCTGGCGTCTGCTT',
            _rand_seq(rng, 7, 'ACGT'), _rand_seq(rng, 45, 'ACGT'), _rand_seq(rng, 63, 'ACGT')]
    reads = []
    for k in range(3000):
        n = rng.choice([0, 1, 2, 150, 150, 150, rng.randint(3, 400)])
        r = _rand_seq(rng, n, rng.choice(['ACGT', 'ACGT', 'AT', 'ACGTN']))
        if n > 40 and rng.random() < 0.6:
            a = _mutate(rng, rng.choice(adps), rng.choice([0.0, 0.05, 0.15]))
            p = rng.randint(0, n)
            r = (r[:p] + a + r[p:])[:max(n, len(a))]
        reads.append(r)
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    n = len(reads)
    for group in ([0], [1], [2], [3], [4], [5], [0, 1], [1, 2, 4]):
        sel = [adps[i] for i in group]
        got = engine.align(views, sel, scheme)
        k = 700                                    # the oracle on the first k windows of every adapter
        exp = oracle_lib.align_many(reads[:k], sel, (np.tile(np.arange(k), len(sel)), np.repeat(np.arange(len(sel)), k)),
                                    scheme)
        g = got.reshape(8, len(sel), n)[:, :, :k].reshape(8, -1)
        ok = exp[0] != -1
        assert np.array_equal(g[0], exp[0])
        assert np.array_equal(g[:, ok], exp[:, ok]), (group, _first_diff(g, exp, reads[:k], sel, k))

"""GPU parity of the middle scan's product paths that the default inputs rarely force, vs the
oracle's masked loop (the reference's find_middle_adapters, porechop_abi/nanopore_read.py:219-252):

  * overflow recovery of the queued device rounds (pcabi_engine.hip middle_device_rounds): a round
    whose raw-hit slabs (flag 1), band task regions (2) or candidate-DP task slots (4) overflow keeps
    nothing, is queued again and the scan still equals the oracle -- forced in round 1 by small
    initial buffers that must grow (PCABI_MIDDLE_INIT_CAPS, a fresh scan through the device ABI),
    and in round 1 and later rounds by buffers shrunk for one run of that round (PCABI_MIDDLE_FAULT);
  * candidate windows (PCABI_MIDDLE_WINDOWS=1: the verified seeds' windows, k_certify, the second
    plan for the candidates the certificate cannot vouch for) on 8 kb and 20 kb reads whose planted
    adapter copies carry exactly e and e + 1 edits (e = the most non-matching columns of an alignment
    at the threshold), so window winners land at and just above the certificate bound U[a];
  * k_barcode_call at the configs[3] width: SQK-NSK007 + 96 barcode sets (97 start + 97 end slots)
    vs NanoporeRead.determine_barcode (nanopore_read.py:408-482).
"""
import ctypes
import os
import random
import subprocess
import sys

import numpy as np
import pytest

from tests import oracle_lib

SC = (3, -6, -5, -2)   # reference default (arg_parser.py:178-180)
ADPS = ['AATGTACTTCGTTCAGTTACGTATTGCT', 'GCAATACGTAACTGAACGAAGT',           # SQK-NSK007 Y_Top / Y_Bottom
        'CTTCGTTCAGTTACGTATTGCTGGCGTCTGCTT', 'CACCCAAGCAGACGCCAGCAATACGTAACT']  # 1D^2 part 2 start / end


def _rand_seq(rng, n):
    return ''.join(rng.choice('ACGT') for _ in range(n))


def _edit_exactly(rng, s, k):
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


def _reads(seed, n, mean_len, thr, copies=(1, 2, 3)):
    """Reads of ~mean_len bases with planted copies of ADPS carrying exactly e or e + 1 edits (and
    some exact ones), repeats and copies cut at the read ends."""
    rng = random.Random(seed)
    th = thr / 100.0
    reads = []
    for _ in range(n):
        r = _rand_seq(rng, max(200, int(rng.lognormvariate(0, 0.3) * mean_len)))
        for _ in range(rng.choice(copies)):
            a = rng.choice(ADPS)
            e = int(len(a) * (1 - th) / th)
            a = _edit_exactly(rng, a, rng.choice([0, e, e, e + 1, e + 1]))
            where = rng.random()
            if where < 0.1:
                r = a[rng.randint(0, 3):] + r
            elif where < 0.2:
                r = r + a[:len(a) - rng.randint(0, 3)]
            else:
                p = rng.randint(0, len(r))
                r = r[:p] + a + (a if rng.random() < 0.1 else '') + r[p:]
        reads.append(r)
    return reads


def _sorted(h):
    return h[:, np.lexsort((np.arange(h.shape[1]), h[0]))]


def _dev_scan(L, views, adps, sc, thr, profile=None, calls=1, intact=None, stream=False):
    """A FRESH scan through the device ABI (pcabi_adapters_create_scored, pcabi_scan_create,
    pcabi_middle_scan_dev): its buffers are sized on this first use (PCABI_MIDDLE_INIT_CAPS).
    profile: a float64 array of 26 that receives pcabi_scan_profile's table of the call.
    calls: scans of the same device pack with the same scan object (every call's hits must agree);
    intact: a list that receives, per call, whether the device pack is byte-identical afterwards;
    stream: on a library stream instead of the legacy one (rounds after a call's first are then
    captured into graphs on the third call and replayed from the fourth)."""
    from custom_porechop_abi_amd import _lib, engine
    vp = ctypes.c_void_p
    codes, offs, lens = views
    held = []

    def h2d(arr):
        arr = np.ascontiguousarray(arr)
        p = vp()
        _lib.check(L.pcabi_dev_malloc(ctypes.byref(p), max(arr.nbytes, 16)), 'malloc')
        held.append(p)
        _lib.check(L.pcabi_dev_h2d(p, arr.ctypes.data_as(vp), arr.nbytes), 'h2d')
        return p

    d_codes, d_off, d_len = h2d(codes), h2d(offs.astype(np.int64)), h2d(lens.astype(np.int32))
    c, o, ln = engine.encode_adapters(adps)
    tab, scan, st = vp(), vp(), vp()
    _lib.check(L.pcabi_adapters_create_scored(c.ctypes.data_as(vp), o.ctypes.data_as(vp), ln.ctypes.data_as(vp),
                                              len(adps), *sc, ctypes.byref(tab)), 'adapters')
    if stream:
        _lib.check(L.pcabi_stream_create(ctypes.byref(st)), 'stream')
    try:
        _lib.check(L.pcabi_scan_create(tab, ctypes.byref(scan)), 'scan_create')
        cap = 8 * len(lens) + 1024
        hits = np.zeros((6, cap), np.int32)
        h_len = np.ascontiguousarray(lens, np.int32)
        if profile is not None:
            assert L.pcabi_scan_profile(scan, 1, None, 0) == 26
        first = None
        for _ in range(calls):
            hits[:] = 0
            nh = L.pcabi_middle_scan_dev(scan, d_codes, d_off, d_len, h_len.ctypes.data_as(vp), len(lens), *sc,
                                         float(thr), hits.ctypes.data_as(vp), cap, st if stream else None)
            if nh < 0:
                _lib.check(int(nh), 'pcabi_middle_scan_dev')
            assert nh <= cap
            _lib.check(L.pcabi_dev_sync(), 'sync')
            if intact is not None:
                back = np.empty_like(codes)
                _lib.check(L.pcabi_dev_d2h(back.ctypes.data_as(vp), d_codes, back.nbytes), 'd2h')
                intact.append(bool(np.array_equal(back, codes)))
            got = hits[:, :nh].copy()
            if first is None:
                first = got
            else:
                assert np.array_equal(got, first), 'a second scan of the same pack differs'
        if profile is not None:
            assert L.pcabi_scan_profile(scan, 0, profile.ctypes.data_as(vp), 26) == 26
        return first
    finally:
        if scan.value:
            L.pcabi_scan_destroy(scan)
        L.pcabi_adapters_destroy(tab)
        if st.value:
            L.pcabi_stream_destroy(st)
        for p in held:
            L.pcabi_dev_free(p)


def _requeues(L):
    f = ctypes.c_int32(0)
    n = L.pcabi_middle_requeues(ctypes.byref(f))
    return int(n), int(f.value)


@pytest.fixture(scope='module')
def reads_8kb():
    from custom_porechop_abi_amd import engine
    reads = _reads(7, 160, 8000, 90.0)
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    exp = oracle_lib.middle_scan_threaded(views, ADPS, SC, 90.0)
    assert exp.shape[1] > 150
    rounds = np.bincount(exp[0]).max()
    assert rounds >= 3, 'want reads that hit in three or more rounds'
    return views, _sorted(exp)


@pytest.mark.gpu
@pytest.mark.parametrize('caps', ['256,0,0', '0,64,0', '0,0,128', '256,64,128'])
def test_overflow_grows_and_requeues_round1(gpu_lib, monkeypatch, reads_8kb, caps):
    """Round 1 of a fresh scan starts with buffers far too small (raw-hit slabs of one entry per
    block, 64 band tasks per class, 128 candidate-DP task slots): every overflow flags the round,
    the host grows that buffer and queues the round again, until it fits; the hits equal the
    oracle's."""
    views, exp = reads_8kb
    monkeypatch.setenv('PCABI_MIDDLE_SEEDS', '2')
    monkeypatch.setenv('PCABI_MIDDLE_INIT_CAPS', caps)
    n0, _ = _requeues(gpu_lib)
    got = _dev_scan(gpu_lib, views, ADPS, SC, 90.0)
    n1, flags = _requeues(gpu_lib)
    want = (1 if caps.split(',')[0] != '0' else 0) | (2 if caps.split(',')[1] != '0' else 0) | \
        (4 if caps.split(',')[2] != '0' else 0)
    assert n1 > n0, 'no round overflowed'
    assert flags & want == want, (flags, want)
    assert np.array_equal(_sorted(got), exp)


@pytest.mark.gpu
@pytest.mark.parametrize('devrounds', ['1', '0'])
@pytest.mark.parametrize('arena', ['', '0,0,0,4096'])
def test_scan_leaves_the_callers_reads_intact(gpu_lib, monkeypatch, reads_8kb, devrounds, arena):
    """The reference masks a copy of the read (nanopore_read.py:225 masked_seq, :234), so the
    caller's sequence is never touched: after pcabi_middle_scan_dev the device read pack is
    byte-identical, and scanning the same pack again with the same scan object gives the same hits
    (the oracle's) -- in the queued device rounds and in the host-driven loop
    (PCABI_MIDDLE_DEVROUNDS=0), with the default shadow arena and with one of 4 KB that has to grow
    (flag 8 in the queued rounds; the host loop grows it before the copies)."""
    views, exp = reads_8kb
    monkeypatch.setenv('PCABI_MIDDLE_SEEDS', '2')
    monkeypatch.setenv('PCABI_MIDDLE_DEVROUNDS', devrounds)
    if arena:
        monkeypatch.setenv('PCABI_MIDDLE_INIT_CAPS', arena)
    n0, _ = _requeues(gpu_lib)
    intact = []
    got = _dev_scan(gpu_lib, views, ADPS, SC, 90.0, calls=3, intact=intact)
    n1, flags = _requeues(gpu_lib)
    assert intact == [True, True, True]
    assert np.array_equal(_sorted(got), exp)
    if arena and devrounds == '1':
        assert n1 > n0 and flags & 8, 'the 4 KB arena did not overflow'


@pytest.mark.gpu
def test_host_string_scan_equals_packed_scan(gpu_lib):
    """pcabi_middle_scan_seqs (the windows as host string addresses, encoded by host threads into
    three pinned 32 MB staging slots while earlier chunks copy) returns what
    pcabi_middle_scan_host returns for the SeqPack of the same windows: ~110 MB of windows (four
    chunks, a slot refilled), odd window starts, lower-case / N / other bytes, empty windows; and
    the first reads against the oracle loop."""
    from custom_porechop_abi_amd import engine
    rng = random.Random(3)
    base = _reads(11, 120, 8000, 90.0)
    base[0] = base[0][:3000].lower() + base[0][3000:]
    base[1] = base[1][:2000] + 'NNNNRYKM' + base[1][2000:]
    seqs, total = [], 0
    while total < 110 * 10 ** 6:
        seqs.append(base[rng.randrange(len(base))])
        total += len(seqs[-1])
    st = np.array([rng.randint(0, 60) for _ in seqs], np.int64)
    ln = np.array([max(0, len(s) - a - rng.randint(0, 60)) for s, a in zip(seqs, st)], np.int64)
    ln[5] = 0
    addr, have = engine.str_buffers(seqs)
    got = engine.middle_scan_seqs(addr + st.astype(np.uint64), ln, ADPS, SC, 90.0)
    pack = engine.SeqPack.windows(seqs, st, ln)
    exp = engine.middle_scan(pack.views(np.zeros(len(seqs), np.int64), pack.lengths), ADPS, SC, 90.0)
    assert got.shape[1] > 1000
    assert np.array_equal(got, exp)
    k = 150
    ora = oracle_lib.middle_scan_seqs_threaded(addr[:k] + st[:k].astype(np.uint64), ln[:k], ADPS, SC, 90.0)
    assert np.array_equal(_sorted(got[:, got[0] < k]), _sorted(ora))


@pytest.mark.gpu
@pytest.mark.parametrize('mb,scalar', [(1, '0'), (70, '0'), (3, '1')])
def test_staging_codec_is_byte_exact(gpu_lib, monkeypatch, mb, scalar):
    """pcabi_stage_seqs_host: windows of a random byte buffer (every byte value, odd starts and
    lengths, empty windows; 70 MB = three 32 MB chunks, the last partial) carried as 2-bit codes
    + N masks and unpacked on the device == the Dna5 table applied on the host to SeqPack's
    layout, byte for byte (pads and the 16-byte tail N). scalar '1': the encoder used without AVX2."""
    import ctypes
    monkeypatch.setenv('PCABI_STAGE_SCALAR', scalar)
    from custom_porechop_abi_amd import engine
    rng = np.random.default_rng(mb)
    buf = rng.integers(0, 256, size=mb * 10 ** 6 + 100, dtype=np.uint8)
    acgt = np.frombuffer(b'ACGTacgtUuN', np.uint8)
    buf[:] = np.where(rng.random(buf.size) < 0.95, acgt[rng.integers(0, len(acgt), size=buf.size)], buf)
    starts, lens, at = [], [], 0
    while at < buf.size - 20000:
        ln = int(rng.integers(0, 20000)) if rng.random() > 0.05 else 0
        starts.append(at)
        lens.append(ln)
        at += ln + int(rng.integers(0, 7))
    starts, lens = np.array(starts, np.uint64), np.array(lens, np.int32)
    addr = np.uint64(buf.ctypes.data) + starts
    offs = np.zeros(len(lens), np.int64)
    np.cumsum(((lens.astype(np.int64) + 3) & ~3)[:-1], out=offs[1:])
    total = int(offs[-1] + ((int(lens[-1]) + 3) & ~3)) + 16
    exp = np.full(total, 4, np.uint8)
    for o, s0, ln in zip(offs.tolist(), starts.tolist(), lens.tolist()):
        exp[o:o + ln] = engine.DNA5[buf[s0:s0 + ln]]
    got = np.zeros(total, np.uint8)
    rc = engine.lib().pcabi_stage_seqs_host(0, addr.ctypes.data_as(ctypes.c_void_p), lens.ctypes.data_as(ctypes.c_void_p),
                                            len(lens), got.ctypes.data_as(ctypes.c_void_p), total)
    engine.check(rc, 'pcabi_stage_seqs_host')
    assert np.array_equal(got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize('windows', ['0', '1'])
@pytest.mark.parametrize('fault', ['0:1', '0:2', '0:4', '1:1', '1:2', '1:4', '2:7', '0:7,1:4,2:2', '0:8', '1:8',
                                   '2:15'])
def test_overflow_in_a_round_is_dropped_and_requeued(gpu_lib, monkeypatch, reads_8kb, fault, windows):
    """PCABI_MIDDLE_FAULT: the first run of round k overflows for real (its buffers shrunk to one
    entry: the seed scan's raw-hit slab, the band tasks, 64 candidate task slots, or (8) a shadow
    arena of no bytes for the round's masked copies); nothing of that
    round is kept or masked, the rounds queued behind it see no reads, and the rerun gives the same
    hits as the oracle -- in round 1 and in later rounds, with and without candidate windows."""
    from custom_porechop_abi_amd import engine
    views, exp = reads_8kb
    monkeypatch.setenv('PCABI_MIDDLE_SEEDS', '2')
    monkeypatch.setenv('PCABI_MIDDLE_WINDOWS', windows)
    monkeypatch.setenv('PCABI_MIDDLE_FAULT', fault)
    n0, f0 = _requeues(gpu_lib)
    got = engine.middle_scan(views, ADPS, SC, 90.0)
    n1, f1 = _requeues(gpu_lib)
    assert n1 - n0 >= len(fault.split(',')), 'the injected rounds did not overflow'
    assert np.array_equal(_sorted(got), exp)


@pytest.mark.gpu
@pytest.mark.parametrize('mean_len,n_reads,thr', [(8000, 120, 90.0), (20000, 60, 90.0), (8000, 100, 85.0)])
def test_candidate_windows_at_the_certificate_bound(gpu_lib, monkeypatch, mean_len, n_reads, thr):
    """PCABI_MIDDLE_WINDOWS=1 (the verified seeds' windows, the certificate, whole reads for the
    rest) vs the oracle on long reads whose copies carry exactly e or e + 1 edits, and the same scan
    with the windows off."""
    from custom_porechop_abi_amd import engine
    reads = _reads(1000 + mean_len + int(thr), n_reads, mean_len, thr)
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    exp = _sorted(oracle_lib.middle_scan_threaded(views, ADPS, SC, thr))
    assert exp.shape[1] > n_reads // 2
    monkeypatch.setenv('PCABI_MIDDLE_SEEDS', '2')
    for w in ('1', '0'):
        monkeypatch.setenv('PCABI_MIDDLE_WINDOWS', w)
        got = engine.middle_scan(views, ADPS, SC, thr)
        assert np.array_equal(_sorted(got), exp), 'windows=%s' % w


@pytest.mark.gpu
@pytest.mark.parametrize('thr', [90.0, 85.0])
def test_seed_scan_n_runs_and_short_reads(gpu_lib, monkeypatch, thr):
    """k_seed_scan (the pair byte map over packed codes) on reads with N bases, reads shorter than a
    segment and ragged ends, at 90 % (8-mers only) and 85 % (probes of 5-6 bases: the short-run
    path): the oracle's hits, and raw hits / band tasks counted (pcabi_scan_profile). (r03-r05 also
    ran the r03 bitmap scan beside it and compared the counters; that kernel is retired.)"""
    from custom_porechop_abi_amd import engine
    rng = random.Random(int(thr))
    reads = _reads(31 + int(thr), 90, 3000, thr)
    for k in range(0, len(reads), 3):                 # N runs and single Ns
        r = list(reads[k])
        for _ in range(rng.randint(1, 6)):
            p = rng.randrange(len(r))
            for q in range(p, min(len(r), p + rng.choice([1, 1, 2, 9]))):
                r[q] = 'N'
        reads[k] = ''.join(r)
    reads += [a[:n] + _rand_seq(rng, m) for a in ADPS for n, m in ((len(a), 0), (len(a), 3), (len(a) - 2, 9))]
    reads += [_rand_seq(rng, n) for n in (1, 5, 8, 31, 32, 33, 39, 40, 41)]
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    exp = _sorted(oracle_lib.middle_scan_threaded(views, ADPS, SC, thr))
    monkeypatch.setenv('PCABI_MIDDLE_SEEDS', '2')
    prof = np.zeros(26, np.float64)
    got = _dev_scan(gpu_lib, views, ADPS, SC, thr, profile=prof)
    assert np.array_equal(_sorted(got), exp), prof[7:15]
    assert prof[10] > 0


@pytest.mark.gpu
@pytest.mark.parametrize('thr', [90.0, 85.0])
def test_seed_expand_one_pass(gpu_lib, monkeypatch, thr):
    """k_seed_expand1 (a block's slabs as one flat run of hits, three per thread and pass, one walk
    to count and one to write) on reads with N runs and ragged ends: the oracle's hits; then with
    task regions far too small (every pass flags the overflow, the round grows them and reruns)."""
    from custom_porechop_abi_amd import engine
    rng = random.Random(7 + int(thr))
    reads = _reads(57 + int(thr), 120, 3000, thr)
    for k in range(0, len(reads), 4):
        r = list(reads[k])
        p = rng.randrange(len(r))
        r[p:p + 5] = 'NNNNN'
        reads[k] = ''.join(r)[:len(reads[k])]
    reads += [_rand_seq(rng, n) for n in (1, 7, 8, 33, 41)]
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    exp = _sorted(oracle_lib.middle_scan_threaded(views, ADPS, SC, thr))
    monkeypatch.setenv('PCABI_MIDDLE_SEEDS', '2')
    prof = np.zeros(26, np.float64)
    got = _dev_scan(gpu_lib, views, ADPS, SC, thr, profile=prof)
    assert np.array_equal(_sorted(got), exp)
    assert prof[11] > 0
    monkeypatch.setenv('PCABI_MIDDLE_INIT_CAPS', '0,64,0')
    n0, _ = _requeues(gpu_lib)
    got = _dev_scan(gpu_lib, views, ADPS, SC, thr)
    n1, flags = _requeues(gpu_lib)
    assert n1 > n0 and flags & 2, (n1 - n0, flags)
    assert np.array_equal(_sorted(got), exp)


@pytest.mark.gpu
@pytest.mark.parametrize('windows', ['0', '1'])
def test_round_graphs_replay(gpu_lib, monkeypatch, reads_8kb, windows):
    """Rounds after a call's first, captured into graphs (the third call of a key) and replayed (the
    fourth and fifth), on a library stream: every call equals the oracle, with and without candidate
    windows (the whole-read rounds' chunk tasks one lane each, the window rounds' on the row-split
    core, two lanes per task), and equals a fresh scan's first call (rounds queued directly)."""
    views, exp = reads_8kb
    monkeypatch.setenv('PCABI_MIDDLE_SEEDS', '2')
    monkeypatch.setenv('PCABI_MIDDLE_WINDOWS', windows)
    got = _dev_scan(gpu_lib, views, ADPS, SC, 90.0, calls=5, stream=True)
    assert np.array_equal(_sorted(got), exp)
    direct = _dev_scan(gpu_lib, views, ADPS, SC, 90.0, calls=1, stream=True)
    assert np.array_equal(got, direct)


@pytest.mark.gpu
@pytest.mark.parametrize('windows', ['0', '1'])
def test_chunk_dp_host_api(gpu_lib, monkeypatch, reads_8kb, windows):
    """The candidate DP's chunk tasks through the host API (engine.middle_scan: per-call tables,
    rounds queued directly) -- one lane per task in the whole-read rounds, two (k_align_split_chunk,
    host model: test_dp_core_cpu.py::test_row_split_chunk_core) in the candidate-window rounds --
    equal the oracle."""
    from custom_porechop_abi_amd import engine
    views, exp = reads_8kb
    monkeypatch.setenv('PCABI_MIDDLE_SEEDS', '2')
    monkeypatch.setenv('PCABI_MIDDLE_WINDOWS', windows)
    got = engine.middle_scan(views, ADPS, SC, 90.0)
    assert np.array_equal(_sorted(got), exp)


# ---- k_barcode_call at the configs[3] width ---------------------------------------------------

def _pid6(m, l):
    return float('%f' % (100.0 * m / l))


@pytest.mark.gpu
@pytest.mark.parametrize('require_two', [False, True])
def test_barcode_call_96_sets_random_scores(gpu_lib, require_two):
    """SQK-NSK007 + 96 forward barcode sets + a few reverse ones (ignored by the call) and repeated
    names (104 adapters per side, 96 slots: a repeated name's slot takes its last position),
    tie-heavy identities drawn from few (m, l2) values."""
    from custom_porechop_abi_amd import adapters as A, engine
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    from custom_porechop_abi_amd.porechop_abi import barcode_slots
    allsets = A.fresh_adapters()
    fwd = [a for a in allsets if a.name.startswith('Barcode ') and a.name.endswith('(forward)')][:96]
    rev = [a for a in allsets if a.name.startswith('Barcode ') and a.name.endswith('(reverse)')][:4]
    nsk = [a for a in allsets if a.name == 'SQK-NSK007']
    assert len(fwd) == 96
    n_read = 2000
    for seed in range(6):
        rng = random.Random(seed)
        sides = []
        for _ in range(2):
            sets = nsk + fwd + rev + rng.sample(fwd, 3)          # 104 slots, three names twice
            rng.shuffle(sets)
            ms = [rng.randint(10, 21) for _ in range(5)]
            res = np.zeros((8, len(sets) * n_read), np.int32)
            res[0] = np.where(np.array([rng.random() for _ in range(res.shape[1])]) < 0.05, -1, 3)
            res[5] = np.array([rng.choice(ms) for _ in range(res.shape[1])], np.int32)
            res[7] = 24
            for r in range(n_read):                                  # most reads: one clear best slot
                if rng.random() < 0.7:
                    k = rng.randrange(len(sets)) * n_read + r
                    res[0, k], res[5, k] = 3, 24
            sides.append((sets, res))
        ids = {}
        slots = [barcode_slots(s, 'forward', ids) for s, _ in sides]
        assert len(slots[0][0]) == 96 and len(slots[1][0]) == 96
        for (sets, _), (adp, _) in zip(sides, slots):           # repeated names -> their later table index
            last = {a.get_barcode_name(): k for k, a in enumerate(sets)
                    if a.is_barcode() and a.barcode_direction() == 'forward'}
            assert sorted(adp.tolist()) == sorted(last.values())
        names = {v: k for k, v in ids.items()}
        thr, diff = rng.choice([50.0, 75.0]), rng.choice([0.0, 5.0])
        call = engine.barcode_call(sides[0][1], sides[1][1], slots[0], slots[1], n_read, thr, diff, require_two)
        got = [names.get(int(x), 'none') for x in call]
        exp = []
        for r in range(n_read):
            read = NanoporeRead('r', 'A', '')
            for (sets, res), d in zip(sides, (read.start_barcode_scores, read.end_barcode_scores)):
                for a, s in enumerate(sets):
                    if s.is_barcode() and s.barcode_direction() == 'forward':
                        i = a * n_read + r
                        d[s.get_barcode_name()] = 0.0 if res[0, i] == -1 else _pid6(res[5, i], res[7, i])
            read.determine_barcode(thr, diff, require_two)
            exp.append(read.barcode_call)
        assert got == exp, seed
        assert sum(x != 'none' for x in exp) > 0


@pytest.mark.gpu
def test_barcode_call_96_sets_on_barcoded_reads(gpu_lib):
    """The configs[3] job: synthetic reads carrying one of 96 forward barcodes, windows of 150 bp
    aligned on the GPU against SQK-NSK007 + 96 barcode sets (97 + 97 adapters), calls on the device
    == determine_barcode over the same alignments; the first reads' alignments == the oracle's."""
    from custom_porechop_abi_amd import adapters as A, engine, synth
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    from custom_porechop_abi_amd.porechop_abi import barcode_slots
    allsets = A.fresh_adapters()
    sets = [a for a in allsets if a.name == 'SQK-NSK007'] + \
        [a for a in allsets if a.name.startswith('Barcode ') and a.name.endswith('(forward)')][:96]
    n = 3000
    reads, truth = synth.make_barcoded_reads(n, [(a.start_sequence[1], a.end_sequence[1]) for a in sets[1:]], 2000,
                                             seed=99)
    seqs = [synth.codes_to_str(r) for r in reads]
    pack = engine.SeqPack(seqs)
    sw, ew = engine.start_end_windows(pack, 150)
    sres = engine.align(sw, [a.start_sequence[1] for a in sets], SC)
    eres = engine.align(ew, [a.end_sequence[1] for a in sets], SC)
    k = 40
    for win, res, sl in ((sw, sres, lambda s: s[:150]), (ew, eres, lambda s: s[-150:])):
        adps = [a.start_sequence[1] for a in sets] if win is sw else [a.end_sequence[1] for a in sets]
        pr = np.tile(np.arange(k), len(adps))
        pa = np.repeat(np.arange(len(adps)), k)
        exp = oracle_lib.align_many([sl(s) for s in seqs[:k]], adps, (pr, pa), SC)
        got = res.reshape(8, len(adps), n)[:, :, :k].reshape(8, -1)
        assert np.array_equal(got, exp)
    ids = {}
    ss, es = barcode_slots(sets, 'forward', ids), barcode_slots(sets, 'forward', ids)
    assert len(ss[0]) == 96 and len(es[0]) == 96
    names = {v: kk for kk, v in ids.items()}
    for require_two in (False, True):
        call = engine.barcode_call(sres, eres, ss, es, n, 75.0, 5.0, require_two)
        got = [names.get(int(x), 'none') for x in call]
        exp = []
        for r in range(n):
            read = NanoporeRead('r', 'A', '')
            for res, d in ((sres, read.start_barcode_scores), (eres, read.end_barcode_scores)):
                for a, s in enumerate(sets):
                    if s.is_barcode() and s.barcode_direction() == 'forward':
                        i = a * n + r
                        d[s.get_barcode_name()] = 0.0 if res[0, i] == -1 else _pid6(res[5, i], res[7, i])
            read.determine_barcode(75.0, 5.0, require_two)
            exp.append(read.barcode_call)
        assert got == exp
        assert sum(x != 'none' for x in exp) > n // 2


@pytest.mark.gpu
@pytest.mark.parametrize('byte', ['1', '0x3f'])
def test_poisoned_scratch(gpu_lib, byte):
    """PCABI_POISON (a child process: the switch is read once per process): every fresh device
    scratch buffer and every growth starts as 0xFF bytes (every int -1) or 0x3F bytes (every int a
    huge count), and the overflow / requeue, shadow-arena, candidate-window and end-trim cases of
    tests/poisoned_middle.py still equal the oracle -- a path that reads scratch nothing wrote (r05:
    the plans' need2) no longer hides behind zeroed memory."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PCABI_POISON=byte)
    r = subprocess.run([sys.executable, '-u', os.path.join(root, 'tests', 'poisoned_middle.py')], env=env,
                       capture_output=True, text=True, timeout=400)
    print(r.stdout)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert 'all cases ok' in r.stdout

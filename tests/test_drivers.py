"""Batched phase drivers + NanoporeRead decision rules vs the reference's OWN drivers.

tests/golden/g2_decisions.json.gz holds, for the reference's test FASTQs and a seeded synthetic
set, what porechop_abi.porechop_abi (reference Python, reference SeqAn .so) decided for every
read: matching adapter sets and their discovery scores, trim amounts, recorded start/end
alignments, middle-adapter hits/trim positions and barcode scores/calls
(tools/make_golden_g2.py). Two backends run the same host logic:
  * 'oracle' (CPU, not gpu): engine.align replaced by the CPU oracle -- checks the host logic;
  * 'gpu'   : the real HIP kernels through libpcabi.so.
"""
import io

import pytest

from tests import golden_lib, oracle_lib

G2 = golden_lib.g2()
CASES = [c['case'] for c in G2['cases']]


def _records(case):
    if case['input'] == 'synthetic_reads':
        return [tuple(x) for x in G2['synthetic_reads']]
    return golden_lib.load_records(case['input'])


def _ranges(positions):
    out = []
    for p in sorted(positions):
        if out and out[-1][1] == p:
            out[-1][1] = p + 1
        else:
            out.append([p, p + 1])
    return out


def run_pipeline(case):
    from custom_porechop_abi_amd import adapters as A, porechop_abi as P
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    opts = case['opts']
    sink = io.StringIO()
    sets = A.fresh_adapters()
    reads = [NanoporeRead(n, s, q) for n, s, q in _records(case)]
    sc = opts['scoring']
    check = reads[:opts.get('check_reads', 10000)]
    matching = P.find_matching_adapter_sets(check, 0, opts['end_size'], sc, sink, opts['adapter_threshold'], 1,
                                            adapter_sets=sets)
    matching = P.fix_up_1d2_sets(matching)
    fr = P.choose_barcoding_kit(matching, 0, sink) if opts['barcodes'] else None
    set_scores = [[a.name, a.best_start_score, a.best_end_score] for a in sets if '(full sequence)' not in a.name]
    matching = P.add_full_barcode_adapter_sets(matching)
    if matching:
        P.find_adapters_at_read_ends(reads, matching, 0, opts['end_size'], opts['extra_end_trim'],
                                     opts['end_threshold'], sc, sink, opts['min_trim_size'], 1, opts['barcodes'],
                                     75.0, 5.0, opts.get('require_two', False), fr)
        P.find_adapters_in_read_middles(reads, matching, 0, opts['middle_threshold'], 10, 100, sc, sink, 1, False)
    return matching, fr, set_scores, reads


def check_case(case):
    matching, fr, set_scores, reads = run_pipeline(case)
    assert [a.name for a in matching] == case['matching']
    assert fr == case['forward_or_reverse']
    assert set_scores == case['set_scores']
    assert len(reads) == len(case['reads'])
    for r, exp in zip(reads, case['reads']):
        got = {
            'name': r.name,
            'start_trim': r.start_trim_amount, 'end_trim': r.end_trim_amount,
            'start_alns': [[a[0].name, a[1], a[2], a[3], a[4]] for a in r.start_adapter_alignments],
            'end_alns': [[a[0].name, a[1], a[2], a[3], a[4]] for a in r.end_adapter_alignments],
            'middle_pos': _ranges(r.middle_adapter_positions),
            'middle_trim': _ranges(r.middle_trim_positions),
            'middle_hit_str': r.middle_hit_str,
            'start_bc': [list(x) for x in r.start_barcode_scores.items()],
            'end_bc': [list(x) for x in r.end_barcode_scores.items()],
            'barcode_call': r.barcode_call,
        }
        assert got == exp, r.name


@pytest.mark.parametrize('case_name', CASES)
def test_drivers_match_reference_with_oracle_backend(case_name, monkeypatch):
    from custom_porechop_abi_amd import engine
    monkeypatch.setattr(engine, 'align', oracle_lib.align_windows)
    monkeypatch.setattr(engine, 'end_decisions', oracle_lib.end_decisions_windows)
    monkeypatch.setattr(engine, 'best_full_identity', oracle_lib.best_full_identity_windows)
    monkeypatch.setattr(engine, 'first_hits', oracle_lib.first_hits_windows)
    monkeypatch.setattr(engine, 'middle_scan', oracle_lib.middle_scan_windows)
    monkeypatch.setattr(engine, 'middle_scan_seqs', oracle_lib.middle_scan_seqs_windows)
    check_case([c for c in G2['cases'] if c['case'] == case_name][0])


@pytest.mark.gpu
@pytest.mark.parametrize('case_name', CASES)
def test_drivers_match_reference_on_gpu(gpu_lib, case_name):
    check_case([c for c in G2['cases'] if c['case'] == case_name][0])


def test_reference_test_expectations_one_adapter_set(monkeypatch):
    """test/test_one_adapter_set.py:51-69 (verbosity 1/2 output): 4 of 9 reads start-trimmed,
    3 of 9 end-trimmed -- on the G2 decisions and through our drivers."""
    from custom_porechop_abi_amd import engine
    monkeypatch.setattr(engine, 'align', oracle_lib.align_windows)
    monkeypatch.setattr(engine, 'end_decisions', oracle_lib.end_decisions_windows)
    monkeypatch.setattr(engine, 'best_full_identity', oracle_lib.best_full_identity_windows)
    monkeypatch.setattr(engine, 'first_hits', oracle_lib.first_hits_windows)
    monkeypatch.setattr(engine, 'middle_scan', oracle_lib.middle_scan_windows)
    monkeypatch.setattr(engine, 'middle_scan_seqs', oracle_lib.middle_scan_seqs_windows)
    case = [c for c in G2['cases'] if c['case'] == 'one_adapter_set'][0]
    _, _, _, reads = run_pipeline(case)
    assert sum(1 for r in reads if r.start_trim_amount) == 4
    assert sum(1 for r in reads if r.end_trim_amount) == 3


@pytest.mark.gpu
@pytest.mark.parametrize('case_name', ['one_adapter_set', 'barcodes', 'two_adapter_sets'])
def test_per_read_methods_on_gpu(gpu_lib, case_name):
    """The unbatched reference call pattern (one adapterAlignment per alignment through the
    legacy C ABI, porechop_abi.py:366-378 / 476-484 single-thread loops) gives the same
    decisions."""
    from custom_porechop_abi_amd import adapters as A, porechop_abi as P
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    case = [c for c in G2['cases'] if c['case'] == case_name][0]
    opts = case['opts']
    sc = opts['scoring']
    sets = A.fresh_adapters()
    reads = [NanoporeRead(n, s, q) for n, s, q in _records(case)]
    for r in reads:
        for s in sets:
            if '(full sequence)' not in s.name:
                r.align_adapter_set(s, opts['end_size'], sc)
    search = [a for a in sets if '(full sequence)' not in a.name]
    assert [[a.name, a.best_start_score, a.best_end_score] for a in search] == case['set_scores']
    matching = [a for a in search if a.best_start_or_end_score() >= opts['adapter_threshold']]
    matching = P.fix_up_1d2_sets(matching)
    fr = P.choose_barcoding_kit(matching, 0, io.StringIO()) if opts['barcodes'] else None
    matching = P.add_full_barcode_adapter_sets(matching)
    adapters, start_names, end_names = P.middle_adapter_list(matching)
    for r, exp in zip(reads, case['reads']):
        r.find_start_trim(matching, opts['end_size'], opts['extra_end_trim'], opts['end_threshold'], sc,
                          opts['min_trim_size'], opts['barcodes'], fr)
        r.find_end_trim(matching, opts['end_size'], opts['extra_end_trim'], opts['end_threshold'], sc,
                        opts['min_trim_size'], opts['barcodes'], fr)
        if opts['barcodes']:
            r.determine_barcode(75.0, 5.0, opts.get('require_two', False))
        r.find_middle_adapters(adapters, opts['middle_threshold'], 10, 100, sc, start_names, end_names)
        assert (r.start_trim_amount, r.end_trim_amount, r.barcode_call) == \
            (exp['start_trim'], exp['end_trim'], exp['barcode_call'])
        assert _ranges(r.middle_trim_positions) == exp['middle_trim']
        assert r.middle_hit_str == exp['middle_hit_str']


def _edge_reads(seed=7, n=3000):
    """Random reads with the window edge cases: empty reads, reads shorter than the window, N /
    lowercase / U bases, adapters planted at both ends."""
    import random
    from custom_porechop_abi_amd import adapters as A
    rng = random.Random(seed)
    ad = [a for a in A.fresh_adapters() if '(full sequence)' not in a.name][:8]
    out = []
    for i in range(n):
        k = rng.choice([0, 1, 3, 40, 149, 150, 151, 300, 2000])
        s = ''.join(rng.choice('ACGTACGTNacgtU') for _ in range(k))
        if k >= 150 and rng.random() < 0.5:
            a = rng.choice(ad)
            s = (a.start_sequence[1] if a.start_sequence else '') + s + (a.end_sequence[1] if a.end_sequence else '')
        out.append(s)
    return out, ad


def test_lazy_end_windows_match_pack():
    """engine.StrWindows (the window strings as addresses, pcabi_end_decisions_seqs' input) lays
    the windows out as the eager pack does, and np.asarray of it gathers the same bytes."""
    import numpy as np
    from custom_porechop_abi_amd import engine, porechop_abi as P
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    seqs, _ = _edge_reads(n=500)
    reads = [NanoporeRead('r%d' % i, s, '') for i, s in enumerate(seqs)]
    for e in (150, 40, 0, -20):
        codes, sw, ew = P.end_windows_pack(reads, e)
        lz, lsw, lew = P.end_windows_pack(reads, e, lazy=True)
        assert isinstance(lz, engine.StrWindows)
        for a, b in zip(sw + ew, lsw + lew):
            assert np.array_equal(a, b)
        assert np.array_equal(np.asarray(lz), codes)


@pytest.mark.gpu
def test_end_decisions_from_strings_on_gpu(gpu_lib):
    """pcabi_end_decisions_seqs (window strings, encoded by the library into pinned staging) ==
    pcabi_end_decisions_host (the packed Dna5 buffer) field for field, on reads with the window
    edge cases, and both == the CPU oracle on a slice."""
    import numpy as np
    from custom_porechop_abi_amd import engine, porechop_abi as P
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    seqs, ad = _edge_reads()
    reads = [NanoporeRead('r%d' % i, s, '') for i, s in enumerate(seqs)]
    starts = [a.start_sequence[1] for a in ad if a.start_sequence]
    ends = [a.end_sequence[1] for a in ad if a.end_sequence]
    sc = [3, -6, -5, -2]
    for e in (150, 40):
        lz, sw, ew = P.end_windows_pack(reads, e, lazy=True)
        codes = np.asarray(lz)
        args = (sw, ew, starts, ends, sc, e, 2, 75.0, 4)
        got = engine.end_decisions(lz, *args, bc_start=np.arange(2), bc_end=np.arange(1))
        exp = engine.end_decisions(codes, *args, bc_start=np.arange(2), bc_end=np.arange(1))
        for g, x in zip(got, exp):
            assert np.array_equal(g, x)
        k = 300
        sub = [NanoporeRead('r%d' % i, s, '') for i, s in enumerate(seqs[:k])]
        lz2, sw2, ew2 = P.end_windows_pack(sub, e, lazy=True)
        ora = oracle_lib.end_decisions_windows(lz2, sw2, ew2, starts, ends, sc, e, 2, 75.0, 4)
        gpu = engine.end_decisions(lz2, sw2, ew2, starts, ends, sc, e, 2, 75.0, 4)
        for g, x in zip(gpu[:4], ora[:4]):
            assert np.array_equal(np.asarray(g, np.int64), np.asarray(x, np.int64))


@pytest.mark.gpu
def test_middle_cut_ranges_on_device(gpu_lib):
    """pcabi_middle_cuts (the device epilogue of the middle scan) == NanoporeRead._apply_middle_hit's
    middle_trim_positions (nanopore_read.py:242-250) for random hits in discovery order: per read,
    the same ranges in the same order (CSR, the writer's cut layout)."""
    import random
    import numpy as np
    from custom_porechop_abi_amd import engine
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    rng = random.Random(12)
    n_reads, n_adp = 300, 9
    names = ['a%d' % k for k in range(n_adp)]
    start_names = set(names[:4]) | {names[7]}
    end_names = set(names[3:6]) | {names[7]}
    hits = []
    for _ in range(1500):
        r = rng.randrange(n_reads)
        a = rng.randrange(n_adp)
        s0 = rng.randrange(0, 5000)
        hits.append([r, a, s0, s0 + rng.randrange(0, 60), 20, 24])
    h = np.array(hits, np.int32).T.copy()
    bs = np.array([x in start_names for x in names], np.uint8)
    be = np.array([x in end_names for x in names], np.uint8)
    cut_off, cuts = engine.middle_cuts(h, n_reads, bs, be, 10, 100)
    assert cut_off[0] == 0 and cut_off[-1] == len(hits)
    for r in range(n_reads):
        read = NanoporeRead('r', 'A', '')
        exp = []
        for k, (rr, a, s0, e0, _, _) in enumerate(hits):
            if rr == r:
                read._apply_middle_hit(names[a], 90.0, s0, e0, 10, 100, start_names, end_names)
                exp.append((s0 - (100 if names[a] in start_names else 10), e0 + (100 if names[a] in end_names else 10)))
        got = [tuple(cuts[2 * k:2 * k + 2].tolist()) for k in range(cut_off[r], cut_off[r + 1])]
        assert got == exp, r
        pos = set()
        for a0, a1 in got:
            pos.update(range(a0, a1))
        assert pos == read.middle_trim_positions
    # no hits: every read gets an empty range list
    cut_off, cuts = engine.middle_cuts(np.zeros((6, 0), np.int32), 5, bs, be, 10, 100)
    assert cut_off.tolist() == [0] * 6 and len(cuts) == 0


@pytest.mark.gpu
@pytest.mark.parametrize('case_name', ['two_adapter_sets', 'synthetic_default'])
def test_set_search_reduced_on_device_through_rccl(gpu_lib, case_name):
    """The check phase as the sharded drivers run it on a GPU: the per-sequence maxima reduced by
    k_best_full_id straight into a device tensor, all-reduced by RCCL (a world of one rank on
    this box's GPU), then the reference's set filter: set scores and matching sets == the
    reference's (G2)."""
    import io
    import socket
    import torch
    import torch.distributed as dist
    from custom_porechop_abi_amd import adapters as A, shards
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    case = next(c for c in G2['cases'] if c['case'] == case_name)
    opts = case['opts']
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % port, rank=0, world_size=1)
    try:
        sets = A.fresh_adapters()
        if case['input'] == 'synthetic_reads':
            recs = [tuple(x) for x in G2['synthetic_reads']]
        else:
            recs = golden_lib.load_records(case['input'])
        reads = [NanoporeRead(n, sq, q) for n, sq, q in recs]
        check = reads[:opts.get('check_reads', 10000)]
        matching = shards.find_matching_adapter_sets(check, 0, opts['end_size'], opts['scoring'], io.StringIO(),
                                                     opts['adapter_threshold'], 1, adapter_sets=sets)
        got = [[a.name, a.best_start_score, a.best_end_score] for a in sets if '(full sequence)' not in a.name]
        assert got == case['set_scores']
        assert [a.name for a in matching] == [n for n in case['matching'] if '(full sequence)' not in n]
    finally:
        dist.destroy_process_group()

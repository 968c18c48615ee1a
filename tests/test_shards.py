"""Multi-process (world size 2, gloo, CPU) runs of the sharded drivers (custom_porechop_abi_amd/
shards.py) against the reference's own decisions (tests/golden/g2_decisions.json.gz).

Each rank aligns only its shard; the adapter-set search all-reduces the per-set maxima. The
alignment backend is the CPU oracle here (engine.align swapped in every rank, as in
test_drivers.py's 'oracle' backend), so this checks the sharding and the collective, not the
kernels; the GPU runs use the same module with backend "nccl".
"""
import io
import json
import os
import socket
import tempfile

import pytest

from tests import golden_lib

G2 = golden_lib.g2()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


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


def _worker(rank, world, port, case_name, out_dir):
    import torch.distributed as dist
    from custom_porechop_abi_amd import adapters as A, engine, porechop_abi as P, shards
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    from tests import oracle_lib
    engine.align = oracle_lib.align_windows            # CPU stand-ins for the HIP kernels
    engine.end_decisions = oracle_lib.end_decisions_windows
    engine.best_full_identity = oracle_lib.best_full_identity_windows
    engine.first_hits = oracle_lib.first_hits_windows
    engine.middle_scan = oracle_lib.middle_scan_windows
    engine.middle_scan_seqs = oracle_lib.middle_scan_seqs_windows
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%d' % port, rank=rank, world_size=world)
    try:
        case = next(c for c in G2['cases'] if c['case'] == case_name)
        opts = case['opts']
        sink = io.StringIO()
        sets = A.fresh_adapters()
        reads = [NanoporeRead(n, s, q) for n, s, q in _records(case)]
        sc = opts['scoring']
        check = reads[:opts.get('check_reads', 10000)]
        matching = shards.find_matching_adapter_sets(check, 0, opts['end_size'], sc, sink, opts['adapter_threshold'],
                                                     1, adapter_sets=sets)
        matching = P.fix_up_1d2_sets(matching)
        set_scores = [[a.name, a.best_start_score, a.best_end_score] for a in sets
                      if '(full sequence)' not in a.name]
        matching = P.add_full_barcode_adapter_sets(matching)
        ends = mids = (0, 0)
        if matching:
            ends = shards.find_adapters_at_read_ends(reads, matching, 0, opts['end_size'], opts['extra_end_trim'],
                                                     opts['end_threshold'], sc, sink, opts['min_trim_size'], 1,
                                                     False, 75.0, 5.0, False, None)
            shards.share_trims(reads, ends)
            mids = shards.find_adapters_in_read_middles(reads, matching, 0, opts['middle_threshold'], 10, 100, sc,
                                                        sink, 1, False)
        st, et = shards.gather_trims(reads, ends)
        out = {'rank': rank, 'matching': [a.name for a in matching], 'set_scores': set_scores,
               'ends': list(ends), 'mids': list(mids),
               'trims': {r.name: [r.start_trim_amount, r.end_trim_amount] for r in reads[ends[0]:ends[1]]},
               'middle': {r.name: _ranges(r.middle_adapter_positions) for r in reads[mids[0]:mids[1]]},
               'gathered': [st.tolist(), et.tolist()]}
        with open(os.path.join(out_dir, 'rank%d.json' % rank), 'w') as f:
            json.dump(out, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('case_name', ['two_adapter_sets', 'synthetic_default'])
def test_sharded_drivers_match_reference(case_name):
    import torch.multiprocessing as mp
    world = 2
    out_dir = tempfile.mkdtemp(prefix='pcabi_shards_')
    mp.spawn(_worker, args=(world, _free_port(), case_name, out_dir), nprocs=world, join=True)
    res = [json.load(open(os.path.join(out_dir, 'rank%d.json' % r))) for r in range(world)]
    case = next(c for c in G2['cases'] if c['case'] == case_name)
    exp_reads = {r['name']: r for r in case['reads']}
    for r in res:
        # the collective: every rank ends with the all-check-reads set maxima and the same sets
        assert r['matching'] == case['matching']
        assert r['set_scores'] == case['set_scores']
    # the shards tile the read list and each read's decisions match the reference
    assert res[0]['ends'][0] == 0 and res[0]['ends'][1] == res[1]['ends'][0]
    assert res[1]['ends'][1] == len(case['reads'])
    seen = {}
    for r in res:
        seen.update(r['trims'])
    assert len(seen) == len(case['reads'])
    for name, (s, e) in seen.items():
        assert [s, e] == [exp_reads[name]['start_trim'], exp_reads[name]['end_trim']], name
    mids = {}
    for r in res:
        mids.update(r['middle'])
    assert len(mids) == len(case['reads'])
    for name, pos in mids.items():
        assert pos == exp_reads[name]['middle_pos'], name
    # all-gathered trim amounts, original read order, identical on both ranks
    exp_st = [r['start_trim'] for r in case['reads']]
    exp_et = [r['end_trim'] for r in case['reads']]
    for r in res:
        assert r['gathered'] == [exp_st, exp_et]


def test_shard_bounds():
    from custom_porechop_abi_amd.shards import shard_bounds, shard_bounds_by_length
    for n in (0, 1, 7, 100):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, r, w) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n and all(b[k][1] == b[k + 1][0] for k in range(w - 1))
    lens = [100, 5000, 20, 20, 20, 8000, 300]
    for w in (1, 2, 3, 4):
        b = [shard_bounds_by_length(lens, r, w) for r in range(w)]
        assert b[0][0] == 0 and b[-1][1] == len(lens) and all(b[k][1] == b[k + 1][0] for k in range(w - 1))


class _OracleTrimmer(object):
    """pipeline.FileTrimmer's file loop with the batch decisions made by the batched drivers on the
    CPU oracle (TEST INFRASTRUCTURE: the GPU tests run the real FileTrimmer)."""

    def __init__(self, matching_sets, scoring_scheme_vals, end_size, end_threshold, extra_end_trim, min_trim_size,
                 middle_threshold, extra_middle_trim_good_side, extra_middle_trim_bad_side, min_split_read_size,
                 barcode_dir=None, forward_or_reverse_barcodes='forward', barcode_threshold=75.0, barcode_diff=5.0,
                 require_two_barcodes=False, untrimmed=False, discard_unassigned=False):
        from custom_porechop_abi_amd.pipeline import FileTrimmer
        self.m, self.sc, self.E, self.thr = matching_sets, scoring_scheme_vals, end_size, end_threshold
        self.extra, self.min_trim, self.mthr = extra_end_trim, min_trim_size, middle_threshold
        self.good, self.bad = extra_middle_trim_good_side, extra_middle_trim_bad_side
        self.min_split, self.discard_middle, self.times = min_split_read_size, False, {}
        self.filter_reads = bool(matching_sets)
        self.barcode_dir, self.fwd_rev = barcode_dir, forward_or_reverse_barcodes
        self.bc = (barcode_threshold, barcode_diff, require_two_barcodes)
        self.untrimmed, self.discard_unassigned = untrimmed, discard_unassigned
        self.bc_names, self.bc_ids = {}, {}
        self.trim_file = FileTrimmer.trim_file.__get__(self)
        self._tick = FileTrimmer._tick.__get__(self)
        self._write_bins = FileTrimmer._write_bins.__get__(self)

    def trim(self, batch, albacore=None):
        import numpy as np
        from custom_porechop_abi_amd import misc, porechop_abi as P
        reads = batch.nanopore_reads()
        for r in reads:                       # load_reads' Albacore barcode (porechop_abi.py:172-177)
            r.albacore_barcode_call = albacore
        sink = io.StringIO()
        if self.m:
            P.find_adapters_at_read_ends(reads, self.m, 0, self.E, self.extra, self.thr, self.sc, sink, self.min_trim, 1,
                                         self.barcode_dir is not None, self.bc[0], self.bc[1], self.bc[2], self.fwd_rev)
            P.find_adapters_in_read_middles(reads, self.m, 0, self.mthr, self.good, self.bad, self.sc, sink, 1, False)
        if self.barcode_dir is not None:
            for r in reads:
                if r.barcode_call != 'none' and r.barcode_call not in self.bc_ids:
                    self.bc_ids[r.barcode_call] = len(self.bc_ids)
                    self.bc_names[self.bc_ids[r.barcode_call]] = r.barcode_call
            self.last_calls = np.array([self.bc_ids.get(r.barcode_call, -1) for r in reads], np.int32)
        st = np.array([r.start_trim_amount for r in reads], np.int32)
        et = np.array([r.end_trim_amount for r in reads], np.int32)
        cut_off = np.zeros(len(reads) + 1, np.int64)
        flat = []
        for i, r in enumerate(reads):
            rg = misc.positions_to_ranges(sorted(r.middle_trim_positions))
            cut_off[i + 1] = cut_off[i] + len(rg)
            for a, b in rg:
                flat += [a, b]
        keep = None
        if self.filter_reads:
            keep = np.array([bool(r.start_adapter_alignments and r.end_adapter_alignments) for r in reads], np.uint8)
        return st, et, cut_off, np.array(flat, np.int64), None, keep


def _file_worker(rank, world, port, case_name, in_path, out_path, res_path, bins=None, chunk=None):
    import torch.distributed as dist
    from custom_porechop_abi_amd import engine, shards
    from tests import oracle_lib
    engine.align = oracle_lib.align_windows
    engine.end_decisions = oracle_lib.end_decisions_windows
    engine.best_full_identity = oracle_lib.best_full_identity_windows
    engine.first_hits = oracle_lib.first_hits_windows
    engine.middle_scan = oracle_lib.middle_scan_windows
    engine.middle_scan_seqs = oracle_lib.middle_scan_seqs_windows
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%d' % port, rank=rank, world_size=world)
    try:
        case = next(c for c in G2['cases'] if c['case'] == case_name)
        o = case['opts']
        counts = shards.trim_file_sharded(in_path, out_path, 'fastq', o['scoring'], o['end_size'], o['end_threshold'],
                                          o['extra_end_trim'], o['min_trim_size'], o['middle_threshold'], 10, 100, 1000,
                                          check_reads=o.get('check_reads', 10000),
                                          adapter_threshold=o['adapter_threshold'], max_reads=3 if bins else 7,
                                          trimmer_factory=_OracleTrimmer, barcode_dir=bins,
                                          require_two_barcodes=bool(o.get('require_two')), spool_chunk_bytes=chunk)
        with open(res_path % rank, 'w') as f:
            json.dump(counts, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('gz', [False, True])
@pytest.mark.parametrize('case_name', ['two_adapter_sets', 'synthetic_default'])
def test_sharded_file_pipeline_matches_reference(case_name, gz, tmp_path):
    """shards.trim_file_sharded at world size 2 (gloo): the check-read set search with one MAX
    all-reduce, record ranges split at record starts (plain input; gzip input: of the plain text
    rank 0 alone inflated), per-rank part files stitched in record order -- the written file == the reference's
    output for the same reads (G2 decisions through get_fastq, as tests/test_pipeline.py)."""
    import gzip
    import torch.multiprocessing as mp
    from tests.test_pipeline import _expected
    case = next(c for c in G2['cases'] if c['case'] == case_name)
    if case['input'] == 'synthetic_reads':
        records = [tuple(x) for x in G2['synthetic_reads']]
    else:
        records = _records(case)
    text = ''.join('@%s\n%s\n+\n%s\n' % r for r in records)
    in_path = str(tmp_path / ('in.fastq.gz' if gz else 'in.fastq'))
    if gz:
        with gzip.open(in_path, 'wt') as f:
            f.write(text)
    else:
        with open(in_path, 'w') as f:
            f.write(text)
    out_path = str(tmp_path / 'out.fastq')
    res_path = str(tmp_path / 'counts%d.json')
    mp.spawn(_file_worker, args=(2, _free_port(), case_name, in_path, out_path, res_path), nprocs=2, join=True)
    counts = [json.load(open(res_path % r)) for r in range(2)]
    assert counts[0] == counts[1] and counts[0]['reads_in'] == len(records)
    assert open(out_path).read() == _expected(case, records)
    # no part or spool file is left behind
    assert not [f for f in os.listdir(str(tmp_path)) if f.startswith('.pcabi_part') or f.startswith('.pcabi_spool')]


@pytest.mark.parametrize('fasta', [False, True])
@pytest.mark.parametrize('chunk', [1, 3000])
def test_sharded_gzip_spool_many_spans(chunk, fasta, tmp_path):
    """gzip input through the spool (shards.spool_distribute / spool_batches) in many small
    record-aligned spans, handed round-robin to the two ranks while rank 0 still inflates: both
    ranks trim spans, the stitched output == the reference's (G2), no spool file is left."""
    import gzip
    import torch.multiprocessing as mp
    from tests.test_pipeline import _expected
    case = next(c for c in G2['cases'] if c['case'] == 'synthetic_default')
    records = [tuple(x) for x in G2['synthetic_reads']]
    if fasta:
        text = ''.join('>%s\n%s\n' % (n, '\n'.join(s[k:k + 60] for k in range(0, len(s), 60))) for n, s, _ in records)
    else:
        text = ''.join('@%s\n%s\n+\n%s\n' % r for r in records)
    in_path = str(tmp_path / ('in.fasta.gz' if fasta else 'in.fastq.gz'))
    with gzip.open(in_path, 'wt') as f:
        f.write(text)
    out_path = str(tmp_path / 'out.fastq')
    res_path = str(tmp_path / 'counts%d.json')
    mp.spawn(_file_worker, args=(2, _free_port(), 'synthetic_default', in_path, out_path, res_path, None, chunk),
             nprocs=2, join=True)
    counts = [json.load(open(res_path % r)) for r in range(2)]
    assert counts[0]['reads_in'] == len(records)
    assert min(counts[0]['reads_in_per_rank']) > 0
    exp = _expected(case, [(n, s, '' if fasta else q) for n, s, q in records])
    if fasta:   # FASTA reads carry no qualities: compare the written sequences and names
        got = open(out_path).read().split('\n')[0::4]
        assert got == exp.split('\n')[0::4]
    else:
        assert open(out_path).read() == exp
    assert not [f for f in os.listdir(str(tmp_path)) if f.startswith('.pcabi_spool') or f.startswith('.pcabi_part')]


def test_sharded_gzip_spool_failure_raises_on_every_rank(tmp_path):
    """A truncated gzip input (the reference's gzip module raises EOFError): the distributor's
    error reaches both ranks, which raise instead of waiting for spans that never come, and leave
    no spool file behind in the output directory."""
    import gzip
    import torch.multiprocessing as mp
    # ~6 MB of text, cut at 90 %: the check reads (50, 'synthetic_endsize') come from the intact
    # first decode buffer, the spans run into the damage while both ranks trim
    records = [('%s_%d' % (n, k), s, q) for k in range(8) for n, s, q in G2['synthetic_reads']]
    data = gzip.compress(''.join('@%s\n%s\n+\n%s\n' % r for r in records).encode())
    in_path = str(tmp_path / 'in.fastq.gz')
    with open(in_path, 'wb') as f:
        f.write(data[:len(data) * 9 // 10])
    with pytest.raises(Exception) as ei:
        mp.spawn(_file_worker, args=(2, _free_port(), 'synthetic_endsize', in_path, str(tmp_path / 'o.fastq'),
                                     str(tmp_path / 'c%d.json'), None, 200000), nprocs=2, join=True)
    assert 'unexpected end of file' in str(ei.value) or 'distributor failed' in str(ei.value)
    # every rank's unconsumed spans, the markers and the acknowledgements are gone (shards.spool_fail_cleanup)
    left = [f for f in os.listdir(str(tmp_path)) if f.startswith('.pcabi_spool')]
    assert left == [], left


@pytest.mark.parametrize('gz', [False, True])
@pytest.mark.parametrize('case_name', ['barcodes', 'barcodes_two'])
def test_sharded_barcode_bins_match_reference(case_name, gz, tmp_path):
    """-b through shards.trim_file_sharded at world size 2 (gloo): the kit direction from the
    all-reduced set search (choose_barcoding_kit), per-rank bins with recorded byte spans,
    stitched per bin by rank 0 in record order -- every bin == the reference's (G2)."""
    import gzip
    import torch.multiprocessing as mp
    from tests.test_pipeline import _expected_bins
    case = next(c for c in G2['cases'] if c['case'] == case_name)
    records = _records(case)
    text = ''.join('@%s\n%s\n+\n%s\n' % r for r in records)
    in_path = str(tmp_path / ('in.fastq.gz' if gz else 'in.fastq'))
    with (gzip.open(in_path, 'wt') if gz else open(in_path, 'w')) as f:
        f.write(text)
    bdir = str(tmp_path / 'bins')
    res_path = str(tmp_path / 'counts%d.json')
    mp.spawn(_file_worker, args=(2, _free_port(), case_name, in_path, str(tmp_path / 'out.fastq'), res_path, bdir),
             nprocs=2, join=True)
    counts = [json.load(open(res_path % r)) for r in range(2)]
    exp = _expected_bins(case, records)
    assert counts[0]['reads_in'] == len(records) and counts[0]['bins'] == sorted(exp)
    assert sorted(os.listdir(bdir)) == sorted(k + '.fastq' for k in exp)
    for name, txt in exp.items():
        assert open(os.path.join(bdir, name + '.fastq')).read() == txt, name


ALBACORE = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'data', 'albacore')


def _albacore_worker(rank, world, port, bins, check, out_path, res_path):
    import torch.distributed as dist
    from custom_porechop_abi_amd import engine, shards
    from tests import oracle_lib
    engine.align = oracle_lib.align_windows
    engine.end_decisions = oracle_lib.end_decisions_windows
    engine.best_full_identity = oracle_lib.best_full_identity_windows
    engine.first_hits = oracle_lib.first_hits_windows
    engine.middle_scan = oracle_lib.middle_scan_windows
    engine.middle_scan_seqs = oracle_lib.middle_scan_seqs_windows
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%d' % port, rank=rank, world_size=world)
    try:
        counts = shards.trim_file_sharded(ALBACORE, out_path, 'fastq', check_reads=check, max_reads=3,
                                          trimmer_factory=_OracleTrimmer, barcode_dir=bins)
        with open(res_path % rank, 'w') as f:
            json.dump(counts, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('run', [0, 1, 2])
def test_sharded_albacore_directory_matches_reference(run, tmp_path):
    """An Albacore output directory as the input (porechop_abi.py:133-187: every *.fastq(.gz) under
    it in sorted order, the check reads spread over the files, each read tagged with its
    directory's barcode) through shards.trim_file_sharded at world size 2 (gloo), with -b (the
    device call nulled where Albacore disagrees, nanopore_read.py:479-482) and without: the bins /
    the output == what the reference's own CLI flow wrote on the reference's own test directory
    (tests/golden/g2_albacore.json.gz, tools/make_golden_albacore.py)."""
    import gzip
    import torch.multiprocessing as mp
    with gzip.open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'g2_albacore.json.gz'),
                   'rt') as f:
        exp = json.load(f)['runs'][run]
    bdir = str(tmp_path / 'bins') if exp['barcodes'] else None
    out_path = str(tmp_path / 'out.fastq')
    res_path = str(tmp_path / 'counts%d.json')
    mp.spawn(_albacore_worker, args=(2, _free_port(), bdir, exp['check_reads_arg'], out_path, res_path), nprocs=2,
             join=True)
    counts = [json.load(open(res_path % r)) for r in range(2)]
    assert counts[0]['reads_in'] == 32
    if bdir:
        assert sorted(os.listdir(bdir)) == sorted(exp['bins'])
        for name, txt in exp['bins'].items():
            assert open(os.path.join(bdir, name)).read() == txt, name
    else:
        assert open(out_path).read() == exp['output']


def test_spool_failure_reaches_a_late_rank(tmp_path):
    """rank 0 fails, acknowledges and waits wait_s for the others; rank 1 is still busy
    past wait_s. Rank 0 must leave the .error marker (and the acknowledgements) behind, so that
    rank 1, reaching spool_batches later, raises instead of polling for spans forever -- and rank 1,
    the last to acknowledge, removes every file of the job."""
    import threading
    import time
    from custom_porechop_abi_amd import shards
    spool, job, world = str(tmp_path), 'jlate', 2
    pre = shards._spool_prefix(spool, job)
    for c in (0, 1, 2):                      # spans never consumed (c % world is the owner)
        with open('%s%d_-.fq' % (pre, c), 'w') as f:
            f.write('@r\nACGT\n+\n!!!!\n')
    with open(pre + 'error', 'w') as f:      # what trim_file_sharded writes when a rank raises
        f.write('rank 0: RuntimeError: boom')
    out = {}

    def rank0():
        shards.spool_fail_cleanup(spool, job, 0, world, wait_s=0.3)
        out['r0'] = True

    def rank1():
        time.sleep(0.8)                      # past rank 0's wait
        try:
            for _ in shards.spool_batches(spool, job, 1, world, 100, stale_s=5.0):
                pass
        except RuntimeError as ex:
            out['r1_raised'] = str(ex)
        shards.spool_fail_cleanup(spool, job, 1, world, wait_s=0.3)

    ts = [threading.Thread(target=rank0, daemon=True), threading.Thread(target=rank1, daemon=True)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=20)
    assert not any(t.is_alive() for t in ts), 'a rank hung'
    assert out.get('r0') and 'input distributor failed' in out.get('r1_raised', '')
    assert not [x for x in os.listdir(spool) if x.startswith(os.path.basename(pre))], os.listdir(spool)


def test_spool_wait_is_bounded_without_a_distributor(tmp_path):
    """A distributor that died without an .error marker (its process killed) stops beating:
    spool_batches raises once its beat is older than stale_s instead of waiting forever."""
    import time
    from custom_porechop_abi_amd import shards
    spool, job = str(tmp_path), 'jdead'
    pre = shards._spool_prefix(spool, job)
    with open(pre + 'beat', 'w'):
        pass
    old = time.time() - 100
    os.utime(pre + 'beat', (old, old))
    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match='silent'):
        for _ in shards.spool_batches(spool, job, 0, 2, 100, stale_s=0.3):
            pass
    assert time.monotonic() - t0 < 10


def test_rank_device_rules(monkeypatch):
    """an explicit device needs no torch query; a node-local rank from any common
    launcher wins; a world larger than the node's GPUs without one is an error unless sharing is
    asked for (PCABI_SHARE_GPUS=1)."""
    import types
    import torch
    from custom_porechop_abi_amd import shards
    for v in ('LOCAL_RANK', 'OMPI_COMM_WORLD_LOCAL_RANK', 'MV2_COMM_WORLD_LOCAL_RANK', 'SLURM_LOCALID',
              'MPI_LOCALRANKID', 'PCABI_SHARE_GPUS'):
        monkeypatch.delenv(v, raising=False)
    assert shards.rank_device(3) == 3
    monkeypatch.setattr(torch.cuda, 'device_count', lambda: 8)
    monkeypatch.setenv('SLURM_LOCALID', '5')
    assert shards.rank_device() == 5
    monkeypatch.setenv('SLURM_LOCALID', '9')
    with pytest.raises(RuntimeError, match='one process per GPU'):
        shards.rank_device()
    monkeypatch.delenv('SLURM_LOCALID')
    fake = types.SimpleNamespace(is_available=lambda: True, is_initialized=lambda: True, get_rank=lambda: 11,
                                 get_world_size=lambda: 16)
    monkeypatch.setattr(shards, '_dist', lambda: fake)
    with pytest.raises(RuntimeError, match='PCABI_SHARE_GPUS'):
        shards.rank_device()
    monkeypatch.setenv('PCABI_SHARE_GPUS', '1')
    with pytest.warns(UserWarning):
        assert shards.rank_device() == 3
    fake.get_world_size = lambda: 8
    fake.get_rank = lambda: 6
    monkeypatch.delenv('PCABI_SHARE_GPUS')
    assert shards.rank_device() == 6

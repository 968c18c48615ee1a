"""File-to-file trimming on the GPU (custom_porechop_abi_amd/pipeline.py: native parse -> device
end trim + middle scan -> fork filter -> native writer) vs the reference's own pipeline on the
same reads: the G2 golden decisions (the reference's drivers, tools/make_golden_g2.py) applied
to NanoporeRead and written with get_fastq (checked against the reference's writer in
tests/test_io.py), for the reference's test files and the seeded synthetic set."""
import os

import pytest

from tests import golden_lib

G2 = golden_lib.g2()


def _matching(case):
    from custom_porechop_abi_amd import adapters as A, porechop_abi as P
    by_name = {a.name: a for a in A.fresh_adapters()}
    base = [by_name[n] for n in case['matching'] if '(full sequence)' not in n]
    sets = P.add_full_barcode_adapter_sets(base)
    assert [a.name for a in sets] == case['matching']
    return sets


def _expected(case, records):
    import json
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    out = []
    for (n, s, q), d in zip(records, case['reads']):
        r = NanoporeRead(n, s, q)
        assert r.name == d['name']
        r.start_trim_amount, r.end_trim_amount = int(d['start_trim']), int(d['end_trim'])
        for a, b in (json.loads(d['middle_trim']) if isinstance(d['middle_trim'], str) else d['middle_trim']):
            r.middle_trim_positions.update(range(a, b))
        alns = [d['start_alns'], d['end_alns']]
        if all(json.loads(x) if isinstance(x, str) else x for x in alns):
            out.append(r.get_fastq(1000, False))
    return ''.join(out)


@pytest.mark.gpu
@pytest.mark.parametrize('case_name', ['one_adapter_set', 'two_adapter_sets', 'barcodes', 'synthetic_default',
                                       'synthetic_linear', 'synthetic_endsize'])
def test_trim_file_matches_reference_pipeline(gpu_lib, case_name, tmp_path):
    from custom_porechop_abi_amd.pipeline import FileTrimmer
    case = [c for c in G2['cases'] if c['case'] == case_name][0]
    opts = case['opts']
    if case['input'] == 'synthetic_reads':
        records = [tuple(x) for x in G2['synthetic_reads']]
        in_path = str(tmp_path / 'in.fastq')
        with open(in_path, 'w') as f:
            for n, s, q in records:
                f.write('@%s\n%s\n+\n%s\n' % (n, s, q))
    else:
        records = golden_lib.load_records(case['input'])
        in_path = os.path.join(golden_lib.GOLDEN, 'data', case['input'] + '.gz')
        from custom_porechop_abi_amd import misc
        b = misc.load_batch(in_path)
        records = [(b.name(i), b.sequence(i), b.quals(i)) for i in range(b.n)]
    out_path = str(tmp_path / 'out.fastq')
    ft = FileTrimmer(_matching(case), opts['scoring'], opts['end_size'], opts['end_threshold'], opts['extra_end_trim'],
                     opts['min_trim_size'], opts['middle_threshold'], 10, 100, 1000)
    try:
        counts = ft.trim_file(in_path, out_path, max_reads=7)     # several batches
    finally:
        ft.close()
    assert counts['reads_in'] == len(case['reads'])
    got = open(out_path).read()
    exp = _expected(case, records)
    assert got == exp


def _fastq(path, n, seed=3):
    import random
    rng = random.Random(seed)
    with open(path, 'w') as f:
        for k in range(n):
            s = ''.join(rng.choice('ACGT') for _ in range(rng.randint(50, 300)))
            f.write('@r%d\n%s\n+\n%s\n' % (k, s, 'I' * len(s)))


def _bare_trimmer(filter_reads=True, matching=True):
    """A FileTrimmer without device state (trim() is replaced by the test): trim_file's threads
    and the native reader / writer only."""
    from custom_porechop_abi_amd.pipeline import FileTrimmer
    ft = object.__new__(FileTrimmer)
    ft.min_split, ft.discard_middle, ft.times = 1000, False, {}
    ft.filter_reads = filter_reads and matching
    return ft


@pytest.mark.parametrize('fail_at', ['trim', 'write'])
def test_trim_file_stops_on_failure_without_hanging(tmp_path, fail_at):
    """A failing trim() (device error) or write must end trim_file with that error, not a hang:
    tiny batches keep the parsed-batch queue full when the failure hits."""
    import threading
    import numpy as np
    from custom_porechop_abi_amd import misc
    in_path, out_path = str(tmp_path / 'in.fastq'), str(tmp_path / 'out.fastq')
    _fastq(in_path, 400)
    ft = _bare_trimmer()
    calls = []

    def trim(b):
        calls.append(b.n)
        if fail_at == 'trim' and len(calls) == 3:
            raise RuntimeError('injected device failure')
        z = np.zeros(b.n, np.int32)
        return z, z, np.zeros(b.n + 1, np.int64), np.zeros(0, np.int64), None, np.ones(b.n, np.uint8)
    ft.trim = trim
    if fail_at == 'write':
        real = misc.write_reads

        def bad_write(*a, **k):
            raise OSError('injected write failure')
        misc.write_reads = bad_write
    res = {}

    def run():
        try:
            ft.trim_file(in_path, out_path, max_reads=5)
        except BaseException as ex:
            res['ex'] = ex
    th = threading.Thread(target=run, daemon=True)
    th.start()
    th.join(30)
    if fail_at == 'write':
        misc.write_reads = real
    assert not th.is_alive(), 'trim_file hung after a failure'
    assert 'injected' in str(res.get('ex')), res
    if fail_at == 'write':
        assert len(calls) < 80, 'the run did not stop early after the write failure'


@pytest.mark.gpu
def test_trim_file_without_matching_sets_writes_reads_unchanged(gpu_lib, tmp_path):
    """No adapter set matched: the reference writes every read unchanged (porechop_abi.py:93-125
    applies filter_reads_by_adapter only inside `if matching_sets:`)."""
    from custom_porechop_abi_amd.pipeline import FileTrimmer
    in_path, out_path = str(tmp_path / 'in.fastq'), str(tmp_path / 'out.fastq')
    _fastq(in_path, 30)
    ft = FileTrimmer([])
    try:
        counts = ft.trim_file(in_path, out_path, max_reads=7)
    finally:
        ft.close()
    assert counts == {'reads_in': 30, 'reads_kept': 30}
    assert open(out_path).read() == open(in_path).read()


@pytest.mark.gpu
@pytest.mark.parametrize('gz', [False, True])
def test_sharded_file_pipeline_on_gpu(gpu_lib, tmp_path, gz):
    """shards.trim_file_sharded with the real FileTrimmer on this box's GPU, the set search
    all-reduced by RCCL (a world of one rank): the written file == the reference's output (G2)."""
    import gzip
    import socket
    import torch.distributed as dist
    from custom_porechop_abi_amd import shards
    case = [c for c in G2['cases'] if c['case'] == 'synthetic_default'][0]
    o = case['opts']
    records = [tuple(x) for x in G2['synthetic_reads']]
    text = ''.join('@%s\n%s\n+\n%s\n' % r for r in records)
    in_path = str(tmp_path / ('in.fastq.gz' if gz else 'in.fastq'))
    with (gzip.open(in_path, 'wt') if gz else open(in_path, 'w')) as f:
        f.write(text)
    out_path = str(tmp_path / 'out.fastq')
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % port, rank=0, world_size=1)
    try:
        counts = shards.trim_file_sharded(in_path, out_path, 'fastq', o['scoring'], o['end_size'], o['end_threshold'],
                                          o['extra_end_trim'], o['min_trim_size'], o['middle_threshold'], 10, 100, 1000,
                                          check_reads=o.get('check_reads', 10000),
                                          adapter_threshold=o['adapter_threshold'], max_reads=7, device=0)
    finally:
        dist.destroy_process_group()
    assert counts['reads_in'] == len(records)
    assert open(out_path).read() == _expected(case, records)


def _expected_bins(case, records, discard_unassigned=False, untrimmed=False, fasta=False):
    """The reference's barcode bins (porechop_abi.py:581-610) from its own decisions (G2): the
    reads with start and end alignments (the fork's filter), each into <barcode_call>.<fmt>."""
    import json
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    bins = {}
    for (n, s, q), d in zip(records, case['reads']):
        r = NanoporeRead(n, s, q)
        r.start_trim_amount, r.end_trim_amount = int(d['start_trim']), int(d['end_trim'])
        for a, b in (json.loads(d['middle_trim']) if isinstance(d['middle_trim'], str) else d['middle_trim']):
            r.middle_trim_positions.update(range(a, b))
        alns = [d['start_alns'], d['end_alns']]
        if not all(json.loads(x) if isinstance(x, str) else x for x in alns):
            continue
        call = d['barcode_call']
        if discard_unassigned and call == 'none':
            continue
        txt = r.get_fasta(1000, False, untrimmed) if fasta else r.get_fastq(1000, False, untrimmed)
        if txt:
            bins[call] = bins.get(call, '') + txt
    return bins


def _records(case, tmp_path):
    from custom_porechop_abi_amd import misc
    in_path = os.path.join(golden_lib.GOLDEN, 'data', case['input'] + '.gz')
    b = misc.load_batch(in_path)
    return in_path, [(b.name(i), b.sequence(i), b.quals(i)) for i in range(b.n)]


@pytest.mark.gpu
@pytest.mark.parametrize('case_name,flags', [('barcodes', {}), ('barcodes_two', {}),
                                             ('barcodes', {'discard_unassigned': True, 'untrimmed': True}),
                                             ('barcodes', {'gz': True})])
def test_trim_file_barcode_bins_match_reference(gpu_lib, case_name, flags, tmp_path):
    """-b: FileTrimmer's barcode bins (device barcode call + per-bin native writes) == the
    reference's output_reads bins built from its own decisions and calls (G2)."""
    import gzip
    from custom_porechop_abi_amd.pipeline import FileTrimmer
    case = [c for c in G2['cases'] if c['case'] == case_name][0]
    opts = case['opts']
    in_path, records = _records(case, tmp_path)
    bdir = str(tmp_path / 'bins')
    fmt = 'fastq.gz' if flags.get('gz') else 'fastq'
    ft = FileTrimmer(_matching(case), opts['scoring'], opts['end_size'], opts['end_threshold'], opts['extra_end_trim'],
                     opts['min_trim_size'], opts['middle_threshold'], 10, 100, 1000, barcode_dir=bdir,
                     forward_or_reverse_barcodes=case['forward_or_reverse'],
                     require_two_barcodes=bool(opts.get('require_two')),
                     discard_unassigned=flags.get('discard_unassigned', False), untrimmed=flags.get('untrimmed', False))
    try:
        counts = ft.trim_file(in_path, str(tmp_path / 'unused.fastq'), fmt, max_reads=3)   # several batches
    finally:
        ft.close()
    exp = _expected_bins(case, records, flags.get('discard_unassigned', False), flags.get('untrimmed', False))
    assert exp and sorted(counts['bins']) == sorted(exp)
    assert sorted(os.listdir(bdir)) == sorted(k + '.' + fmt for k in exp)
    for name, txt in exp.items():
        path = os.path.join(bdir, name + '.' + fmt)
        got = gzip.open(path, 'rt').read() if fmt.endswith('.gz') else open(path).read()
        assert got == txt, name


@pytest.mark.parametrize('flags', [{}, {'discard_unassigned': True, 'untrimmed': True}, {'gz': True}])
def test_output_reads_barcode_bins_and_file(flags, tmp_path):
    """porechop_abi.output_reads (porechop_abi.py:535-668) on NanoporeRead objects carrying the
    reference's decisions (G2): the bins, and the single-file output (where --untrimmed does
    not apply, as in the reference)."""
    import gzip
    import io
    import json
    from custom_porechop_abi_amd import porechop_abi as P
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    case = [c for c in G2['cases'] if c['case'] == 'barcodes'][0]
    _, records = _records(case, tmp_path)
    reads = []
    for (n, s, q), d in zip(records, case['reads']):
        r = NanoporeRead(n, s, q)
        r.start_trim_amount, r.end_trim_amount = int(d['start_trim']), int(d['end_trim'])
        for a, b in (json.loads(d['middle_trim']) if isinstance(d['middle_trim'], str) else d['middle_trim']):
            r.middle_trim_positions.update(range(a, b))
        alns = [d['start_alns'], d['end_alns']]
        if all(json.loads(x) if isinstance(x, str) else x for x in alns):
            r.barcode_call = d['barcode_call']
            reads.append(r)
    gz = flags.get('gz', False)
    fmt = 'fastq.gz' if gz else 'fastq'
    bdir = str(tmp_path / 'bins')
    log = io.StringIO()
    P.output_reads(reads, fmt, None, 'FASTQ', 1, False, 1000, log, bdir, 'in.fastq',
                   flags.get('untrimmed', False), 1, flags.get('discard_unassigned', False))
    exp = _expected_bins(case, records, flags.get('discard_unassigned', False), flags.get('untrimmed', False))
    assert sorted(os.listdir(bdir)) == sorted(k + '.' + fmt for k in exp)
    for name, txt in exp.items():
        path = os.path.join(bdir, name + '.' + fmt)
        assert (gzip.open(path, 'rt').read() if gz else open(path).read()) == txt
    assert 'Barcode' in log.getvalue() and 'barcode-specific files' in log.getvalue()
    out = str(tmp_path / ('all.' + fmt))
    P.output_reads(reads, 'auto', out, 'FASTQ', 0, False, 1000, io.StringIO(), None, 'in.fastq',
                   flags.get('untrimmed', False), 1, False)
    got = gzip.open(out, 'rt').read() if gz else open(out).read()
    assert got == ''.join(r.get_fastq(1000, False) for r in reads)


@pytest.mark.gpu
@pytest.mark.parametrize('run', [0, 1, 2])
def test_albacore_directory_on_gpu(gpu_lib, tmp_path, run):
    """An Albacore output directory (the reference's own test/test_albacore_directory: barcode01..03
    and unclassified) through shards.trim_file_sharded with the real FileTrimmer on this GPU and
    the set search through RCCL: the check reads spread over the files, -b calls nulled where the
    directory's barcode disagrees (nanopore_read.py:479-482) -- bins / output == the reference's own
    CLI flow on the same directory (tests/golden/g2_albacore.json.gz)."""
    import gzip
    import json
    import socket
    import torch.distributed as dist
    from custom_porechop_abi_amd import shards
    with gzip.open(os.path.join(golden_lib.GOLDEN, 'g2_albacore.json.gz'), 'rt') as f:
        exp = json.load(f)['runs'][run]
    in_dir = os.path.join(golden_lib.GOLDEN, 'data', 'albacore')
    bdir = str(tmp_path / 'bins') if exp['barcodes'] else None
    out_path = str(tmp_path / 'out.fastq')
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % port, rank=0, world_size=1)
    try:
        counts = shards.trim_file_sharded(in_dir, out_path, 'fastq', check_reads=exp['check_reads_arg'], max_reads=5,
                                          device=0, barcode_dir=bdir)
    finally:
        dist.destroy_process_group()
    assert counts['reads_in'] == 32

    def same(got, want, what):
        if got == want:
            return
        g, w = got.split('\n'), want.split('\n')
        k = next((i for i, (x, y) in enumerate(zip(g, w)) if x != y), min(len(g), len(w)))
        ctx = lambda lines: [x[:80] + ('...%d' % len(x) if len(x) > 80 else '') for x in lines[max(0, k - 2):k + 2]]
        raise AssertionError('%s: %d vs %d lines, first difference at line %d: got %s want %s'
                             % (what, len(g), len(w), k, ctx(g), ctx(w)))
    if bdir:
        assert sorted(os.listdir(bdir)) == sorted(exp['bins'])
        for name, txt in exp['bins'].items():
            same(open(os.path.join(bdir, name)).read(), txt, name)
    else:
        same(open(out_path).read(), exp['output'], 'output')

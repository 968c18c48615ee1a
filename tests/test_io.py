"""Sequence-file I/O (csrc/pcabi_io.cpp through custom_porechop_abi_amd/misc.py) vs the
reference's own code on the same files (tests/golden/g3_io.json.gz, tools/make_golden_g3.py):
  * misc.load_fasta_or_fastq == porechop_abi.misc.load_fasta_or_fastq (misc.py:108-165), on the
    reference's test files and on edge cases (CRLF / lone CR endings, blank and whitespace lines,
    an empty FASTA header whose sequence carries over, lower case, RNA, IUPAC, short qualities,
    tabs / spaces in headers, gzip);
  * the native batch == NanoporeRead's normalised fields (nanopore_read.py:31-44), and its Dna5
    codes == engine.SeqPack's layout;
  * the native writer and the NanoporeRead mirror == the reference's get_fasta / get_fastq with
    start / end trims (Python slice semantics, over-long trims), middle splits, min split size,
    discard_middle and untrimmed output.
No GPU needed."""
import gzip
import json
import os

import numpy as np
import pytest

from tests import golden_lib

G3 = json.load(gzip.open(os.path.join(golden_lib.GOLDEN, 'g3_io.json.gz'), 'rt'))
GOLDEN_IO = os.path.join(golden_lib.GOLDEN, "io")
CASES = G3['cases']


def _path(case):
    return os.path.join(golden_lib.GOLDEN, case['file'])


@pytest.mark.parametrize('case', CASES, ids=[c['file'] for c in CASES])
def test_load_fasta_or_fastq_matches_reference(case):
    from custom_porechop_abi_amd import misc
    recs, kind = misc.load_fasta_or_fastq(_path(case))
    assert kind == case['type']
    assert [list(x) for x in recs] == case['records']


@pytest.mark.parametrize('case', CASES, ids=[c['file'] for c in CASES])
def test_native_batch_matches_nanopore_read(case):
    from custom_porechop_abi_amd import engine, misc
    b = misc.load_batch(_path(case))
    assert b.n == len(case['reads'])
    for i, (name, seq, quals, rna) in enumerate(case['reads']):
        assert (b.name(i), b.sequence(i), b.quals(i), bool(b.rna[i])) == (name, seq, quals, rna)
    pack = engine.SeqPack([r[1] for r in case['reads']])
    assert np.array_equal(b.code_off, pack.offsets) and np.array_equal(b.lengths, pack.lengths)
    assert np.array_equal(b.codes, pack.codes)
    reads = b.nanopore_reads()
    assert [(r.name, r.seq, r.quals, r.rna) for r in reads] == [tuple(x) for x in case['reads']]


@pytest.mark.parametrize('case', CASES, ids=[c['file'] for c in CASES])
def test_streaming_batches_concatenate(case):
    from custom_porechop_abi_amd import misc
    got = []
    for b in misc.read_batches(_path(case), max_reads=3, max_bases=500):
        assert 0 < b.n <= 3
        got += [[b.name(i), b.sequence(i), b.quals(i), bool(b.rna[i])] for i in range(b.n)]
    assert got == case['reads']


def _apply(reads, o):
    from custom_porechop_abi_amd import misc
    for r, (st, et), cut in zip(reads, o['trims'], o['cuts']):
        r.start_trim_amount, r.end_trim_amount = st, et
        r.middle_trim_positions = set(cut)
    return [misc.positions_to_ranges(c) for c in o['cuts']]


@pytest.mark.parametrize('case', CASES, ids=[c['file'] for c in CASES])
def test_writers_match_reference_output(case, tmp_path):
    from custom_porechop_abi_amd import misc
    b = misc.load_batch(_path(case))
    reads = b.nanopore_reads()
    for k, o in enumerate(case['outputs']):
        cuts = _apply(reads, o)
        for fmt in ('fasta', 'fastq'):
            exp = o[fmt]
            if exp is None:
                continue
            # mirror (per-read Python interface)
            got = ''.join(getattr(r, 'get_' + fmt)(o['min_split'], o['discard_middle'], o['untrimmed'])
                          for r in reads)
            assert got == exp, (fmt, k)
            # native batch writer, plain and gzip
            for gz in (False, True):
                out = str(tmp_path / ('o%d.%s%s' % (k, fmt, '.gz' if gz else '')))
                misc.write_reads(b, out, fmt + ('.gz' if gz else ''), [t[0] for t in o['trims']],
                                 [t[1] for t in o['trims']], cuts, o['min_split'], o['discard_middle'],
                                 untrimmed=o['untrimmed'])
                data = (gzip.open(out, 'rb') if gz else open(out, 'rb')).read().decode()
                assert data == exp, (fmt, k, gz)


def test_parse_errors(tmp_path):
    from custom_porechop_abi_amd import misc
    bad = tmp_path / 'x.txt'
    bad.write_text('hello\n')
    with pytest.raises(ValueError):
        misc.load_batch(str(bad))
    trunc = tmp_path / 't.fastq'
    trunc.write_text('@r1\nACGT\n+\nIIII\n@r2\nACGT\n')
    with pytest.raises(ValueError):
        misc.load_batch(str(trunc))
    blank = tmp_path / 'b.fastq'
    blank.write_text('@r1\nACGT\n+\nIIII\n\n')     # the reference dies on the trailing blank line
    with pytest.raises(ValueError):
        misc.load_batch(str(blank))
    with pytest.raises(SystemExit):
        misc.load_fasta_or_fastq(str(bad))
    bz = tmp_path / 'z.fastq'
    bz.write_bytes(b'BZh91AY&SY')
    with pytest.raises(SystemExit):
        misc.load_fasta_or_fastq(str(bz))


def test_large_gzip_streaming_and_threads(tmp_path, monkeypatch):
    """Batches that outgrow the 4 MB decode buffer (pinned refills), plain (memory-mapped) and
    gzip input, one and several parse threads: all equal the reference's rules restated."""
    import random
    from custom_porechop_abi_amd import misc
    rng = random.Random(3)
    recs = []
    for k in range(3000):
        n = rng.randint(0, 6000)
        s = ''.join(rng.choice('ACGTacgtNU') for _ in range(n))
        q = ''.join(rng.choice('!#5?I') for _ in range(max(0, n - rng.randint(0, 3))))
        recs.append(('r%d x=%d' % (k, k), s, q))
    text = ''.join('@%s\n%s\n+\n%s\n' % r for r in recs)
    plain = tmp_path / 'big.fastq'
    plain.write_text(text.replace('\n', '\r\n') if False else text)
    gz = tmp_path / 'big.fastq.gz'
    with gzip.open(gz, 'wt') as f:
        f.write(text)

    def expect():
        out = []
        for name, s, q in recs:
            u = s.upper()
            rna = u.count('U') > u.count('T')
            u = u.replace('U', 'T') if rna else u
            out.append([name, u, q + '+' * (len(s) - len(q)), rna])
        return out

    exp = expect()
    for threads in ('1', '7'):
        monkeypatch.setenv('PCABI_IO_THREADS', threads)
        for path in (str(plain), str(gz)):
            got = []
            for b in misc.read_batches(path, max_reads=700, max_bases=2_000_000):
                got += [[b.name(i), b.sequence(i), b.quals(i), bool(b.rna[i])] for i in range(b.n)]
            assert got == exp, (threads, path)
            b = misc.load_batch(path)
            assert b.n == len(exp) and b.sequence(len(exp) - 1) == exp[-1][1]


def _batches_text(path, byte_range=None, max_reads=3):
    from custom_porechop_abi_amd import misc
    out = []
    for b in misc.read_batches(path, max_reads=max_reads, byte_range=byte_range):
        out += [(b.name(i), b.sequence(i), b.quals(i), int(b.rna[i])) for i in range(b.n)]
    return out


def test_byte_range_shards_cover_every_record_once(tmp_path):
    """Reads split into byte ranges at record starts (misc.record_boundaries /
    pcabi_fastx_record_start, the sharded file pipeline's split): for every cut position of the
    plain fixtures (CRLF / lone-CR endings, blank and whitespace lines, empty FASTA headers whose
    sequence runs on, qualities starting with '@'), the ranges' records concatenated == the
    whole file's records."""
    import random
    from custom_porechop_abi_amd import _lib, misc
    L = misc._declare(_lib.lib())
    import ctypes
    files = [os.path.join(GOLDEN_IO, f) for f in sorted(os.listdir(GOLDEN_IO)) if not f.endswith('.gz')]
    # FASTQ whose qualities start with '@' and FASTA with empty headers in the middle
    rng = random.Random(8)
    q = str(tmp_path / 'at_quals.fastq')
    with open(q, 'w') as f:
        for k in range(40):
            s = ''.join(rng.choice('ACGT') for _ in range(rng.randint(0, 30)))
            f.write('@r%d x\n%s\n+\n%s\n' % (k, s, '@' * len(s) if k % 2 else ''.join(rng.choice('@+!#I') for _ in s)))
    a = str(tmp_path / 'empty_headers.fasta')
    with open(a, 'w') as f:
        for k in range(30):
            f.write('>%s\n%s\n\n%s\n' % ('' if k % 4 == 1 else 'r%d' % k, 'ACGT' * (k % 5), 'GG' * (k % 3)))
    files += [q, a]
    for path in files:
        whole = _batches_text(path, max_reads=1 << 20)
        size = os.path.getsize(path)
        h = ctypes.c_void_p()
        assert L.pcabi_fastx_open(os.fsencode(path), 0, ctypes.byref(h)) == 0
        try:
            starts = sorted({int(L.pcabi_fastx_record_start(h, b)) for b in range(size + 1)})
        finally:
            L.pcabi_fastx_close(h)
        assert starts[-1] == size
        for cut in starts:
            got = _batches_text(path, (0, cut)) + _batches_text(path, (cut, size))
            assert got == whole, (path, cut)
        for parts in (2, 3, 5):
            b = misc.record_boundaries(path, parts)
            got = []
            for k in range(parts):
                got += _batches_text(path, (b[k], b[k + 1]))
            assert got == whole, (path, parts)
    assert misc.record_boundaries(os.path.join(GOLDEN_IO, 'plain_mixed.fastq.gz'), 2) is None


def test_text_chunks_reparse_to_the_same_records(tmp_path):
    """misc.text_chunks (pcabi_fastx_next_text, the sharded pipeline's distributor): for every
    fixture, plain and gzip, and chunk sizes from one byte up, each span written to its own file and
    parsed afresh gives, concatenated, exactly the whole file's records (CRLF / lone-CR endings,
    blank and whitespace lines, empty FASTA headers whose sequence runs on, '@'-leading qualities)."""
    import random
    from custom_porechop_abi_amd import misc
    files = [os.path.join(GOLDEN_IO, f) for f in sorted(os.listdir(GOLDEN_IO))]
    rng = random.Random(9)
    q = str(tmp_path / 'at_quals.fastq.gz')
    with gzip.open(q, 'wt') as f:
        for k in range(60):
            s = ''.join(rng.choice('ACGT') for _ in range(rng.randint(0, 40)))
            f.write('@r%d x\n%s\n+\n%s\n' % (k, s, '@' * len(s) if k % 2 else ''.join(rng.choice('@+!#I') for _ in s)))
    a = str(tmp_path / 'empty_headers.fasta.gz')
    with gzip.open(a, 'wt') as f:
        for k in range(40):
            f.write('>%s\n%s\n\n%s\n' % ('' if k % 4 == 1 else 'r%d' % k, 'ACGT' * (k % 5), 'GG' * (k % 3)))
    files += [q, a]
    for path in files:
        whole = _batches_text(path, max_reads=1 << 20)
        for size in (1, 7, 64, 500, 1 << 20):
            got, n_chunks = [], 0
            for k, mv in enumerate(misc.text_chunks(path, size)):
                part = str(tmp_path / ('chunk%d' % k))
                with open(part, 'wb') as f:
                    f.write(mv)
                got += _batches_text(part, max_reads=1 << 20)
                n_chunks += 1
            assert got == whole, (path, size)
            if size == 1:
                assert n_chunks > 1 or len(whole) <= 1, path

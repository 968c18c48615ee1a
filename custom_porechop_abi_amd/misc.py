"""Sequence-file I/O on both sides of the alignment engine (mirror of porechop_abi/misc.py:60-168
and the read loading / output of porechop_abi/porechop_abi.py:133-187, 535-668).

The parsing and writing run in libpcabi's native host unit (csrc/pcabi_io.cpp: zlib, the
reference's parse rules, NanoporeRead's normalisation); this module is the Python surface:
  * load_fasta_or_fastq(filename) -> (records, 'FASTA' | 'FASTQ'), the reference's tuples
    (FASTA: (short_name, seq, full_name); FASTQ: (short_name, seq, spacer, quals, full_name));
    the sequence text is the file's own (the reference normalises it later, in NanoporeRead);
  * load_reads(path, verbosity, print_dest, check_read_count) -> (reads, check_reads, read_type)
    with NanoporeRead objects, for a file or an Albacore-style directory of FASTQs;
  * ReadBatch / read_batches(path): the batched path -- names, normalised sequences, qualities
    and the Dna5 codes already in the engine's packed layout (engine.SeqPack's), no per-read
    Python objects;
  * write_reads(batch, path, ...): the reference's trimmed FASTA / FASTQ output for a batch.
"""
import ctypes
import os
import sys

import numpy as np

from ._lib import check, lib

FASTA, FASTQ = 0, 1


class _View(ctypes.Structure):
    _fields_ = [('n', ctypes.c_int64), ('type', ctypes.c_int32), ('names', ctypes.c_void_p),
                ('name_off', ctypes.c_void_p), ('seq', ctypes.c_void_p), ('seq_off', ctypes.c_void_p),
                ('qual', ctypes.c_void_p), ('qual_off', ctypes.c_void_p), ('rna', ctypes.c_void_p),
                ('spacer', ctypes.c_void_p), ('spacer_off', ctypes.c_void_p), ('codes', ctypes.c_void_p), ('codes_len', ctypes.c_int64), ('code_off', ctypes.c_void_p),
                ('len', ctypes.c_void_p)]


def _declare(L):
    if getattr(L, '_io_declared', False):
        return L
    P, i64, c_int = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    sig = {
        'pcabi_fastx_open': ([ctypes.c_char_p, c_int, ctypes.POINTER(P)], c_int),
        'pcabi_fastx_type': ([P], c_int),
        'pcabi_fastx_next': ([P, i64, i64, ctypes.POINTER(P)], i64),
        'pcabi_fastx_close': ([P], None),
        'pcabi_fastx_load': ([ctypes.c_char_p, c_int, ctypes.POINTER(P)], c_int),
        'pcabi_reads_count': ([P], i64),
        'pcabi_reads_type': ([P], c_int),
        'pcabi_reads_views': ([P, ctypes.POINTER(_View)], c_int),
        'pcabi_reads_free': ([P], None),
        'pcabi_reads_write': ([P, ctypes.c_char_p, c_int, c_int, c_int, P, P, P, P, c_int, c_int, c_int, P], c_int),
        'pcabi_fastx_record_start': ([P, i64], i64),
        'pcabi_fastx_set_range': ([P, i64, i64], c_int),
        'pcabi_fastx_remaining': ([P], i64),
        'pcabi_fastx_next_text': ([P, i64, ctypes.POINTER(P), ctypes.POINTER(i64)], c_int),
    }
    for name, (a, r) in sig.items():
        f = getattr(L, name)
        f.argtypes, f.restype = a, r
    L._io_declared = True
    return L


class _Owner(object):
    """Owns a native batch; numpy views into its buffers keep it alive (zero-copy)."""

    def __init__(self, handle):
        self.h = handle

    def __del__(self):
        h, self.h = self.h, None
        if h:
            try:
                _declare(lib()).pcabi_reads_free(h)
            except Exception:
                pass


def _view(owner, ptr, dtype, n):
    """numpy view of n items at ptr inside owner's batch (no copy)."""
    dtype = np.dtype(dtype)
    if n == 0 or not ptr:
        return np.zeros(0, dtype)
    raw = (ctypes.c_uint8 * (n * dtype.itemsize)).from_address(ptr)
    raw._owner = owner                         # the ctypes buffer keeps the batch alive
    return np.frombuffer(raw, dtype=dtype, count=n)


class ReadBatch(object):
    """One batch of parsed reads, as zero-copy numpy views of the native buffers.

    names / seq / qual: uint8 buffers with int64 offsets [n + 1]; rna: uint8 [n];
    codes: Dna5 uint8 buffer, code_off int64 [n] (4-aligned), lengths int32 [n] -- the layout
    engine.SeqPack builds, so (codes, code_off + start, length) are engine windows directly.
    The native batch lives as long as this object or any of its arrays (write_reads uses it)."""

    def __init__(self, handle):
        L = _declare(lib())
        v = _View()
        self._owner = _Owner(handle)
        check(L.pcabi_reads_views(handle, ctypes.byref(v)), 'pcabi_reads_views')
        n = int(v.n)
        o = self._owner
        self.type = int(v.type)
        self.n = n
        self.name_off = _view(o, v.name_off, np.int64, n + 1)
        self.seq_off = _view(o, v.seq_off, np.int64, n + 1)
        self.qual_off = _view(o, v.qual_off, np.int64, n + 1)
        self.spacer_off = _view(o, v.spacer_off, np.int64, n + 1)
        self.names = _view(o, v.names, np.uint8, int(self.name_off[-1]) if n else 0)
        self.seq = _view(o, v.seq, np.uint8, int(self.seq_off[-1]) if n else 0)
        self.qual = _view(o, v.qual, np.uint8, int(self.qual_off[-1]) if n else 0)
        self.spacer = _view(o, v.spacer, np.uint8, int(self.spacer_off[-1]) if n else 0)
        self.rna = _view(o, v.rna, np.uint8, n)
        self.codes = _view(o, v.codes, np.uint8, int(v.codes_len))
        self.code_off = _view(o, v.code_off, np.int64, n)
        self.lengths = _view(o, v.len, np.int32, n)

    @property
    def _h(self):
        return self._owner.h

    def __len__(self):
        return self.n

    def _text(self, buf, off, i):
        return buf[off[i]:off[i + 1]].tobytes().decode()

    def name(self, i):
        return self._text(self.names, self.name_off, i)

    def sequence(self, i):
        return self._text(self.seq, self.seq_off, i)

    def quals(self, i):
        return self._text(self.qual, self.qual_off, i)

    def spacer_line(self, i):
        return self._text(self.spacer, self.spacer_off, i)

    def views(self, starts=None, lengths=None):
        """Engine windows (codes, offsets, lengths) of [start, start + length) of every read."""
        st = np.zeros(self.n, np.int64) if starts is None else np.asarray(starts, np.int64)
        ln = self.lengths if lengths is None else np.asarray(lengths, np.int32)
        return self.codes, self.code_off + st, ln

    def nanopore_reads(self):
        """The reference's NanoporeRead objects (name = full header; seq / quals already
        normalised, so the constructor leaves them unchanged except for the rna flag)."""
        from .nanopore_read import NanoporeRead
        out = []
        for i in range(self.n):
            r = NanoporeRead(self.name(i), self.sequence(i), self.quals(i))
            r.rna = bool(self.rna[i])
            out.append(r)
        return out


def _open_error(path):
    msg = lib().pcabi_last_error()
    return msg.decode() if msg else path


def input_files(path):
    """The sequence files of an input, as load_reads sees it (porechop_abi.py:133-187): a file is
    itself (albacore barcode None); a directory is an Albacore output directory -- every *.fastq /
    *.fastq.gz under it, sorted by path, each with the barcode its path names
    (get_albacore_barcode_from_path). Exits like the reference when nothing is found."""
    if os.path.isfile(path):
        return [(path, None)]
    if os.path.isdir(path):
        fastqs = sorted([os.path.join(d, f) for d, _, fs in os.walk(path) for f in fs
                         if f.lower().endswith('.fastq') or f.lower().endswith('.fastq.gz')])
        if not fastqs:
            sys.exit('Error: could not find fastq files in ' + path)
        return [(f, get_albacore_barcode_from_path(f)) for f in fastqs]
    sys.exit('Error: could not find ' + path)


def load_check_reads(path, check_read_count):
    """The check reads of load_reads (porechop_abi.py:133-187) as NanoporeRead objects: a file's
    first check_read_count records; for an Albacore directory the first
    round(check_read_count / files) records of every file, in file order."""
    files = input_files(path)
    per_file = check_read_count if os.path.isfile(path) else int(round(check_read_count / len(files)))
    out = []
    for f, _ in files:
        if per_file <= 0:
            break
        for b in read_batches(f, max_reads=per_file, max_bases=1 << 62):
            out += b.nanopore_reads()
            break
    return out


def record_boundaries(path, parts):
    """Byte offsets [parts + 1] splitting a plain FASTA / FASTQ file into `parts` contiguous record
    ranges of about equal size (so about equal bases): each cut is moved forward to the next record
    start (pcabi_fastx_record_start). None for a gzip file (it cannot be entered mid-stream) and for
    a directory (its files are streamed in order)."""
    if os.path.isdir(path):
        return None
    L = _declare(lib())
    h = ctypes.c_void_p()
    rc = L.pcabi_fastx_open(os.fsencode(path), 0, ctypes.byref(h))
    if rc != 0:
        raise ValueError(_open_error(path))
    try:
        if get_compression_type(path) != 'plain':
            return None
        size = os.path.getsize(path)
        cuts = [0]
        for k in range(1, parts):
            b = L.pcabi_fastx_record_start(h, size * k // parts)
            if b < 0:
                return None
            cuts.append(max(int(b), cuts[-1]))
        cuts.append(size)
        return cuts
    finally:
        L.pcabi_fastx_close(h)


def ramp_sizes(max_reads, remaining_reads=None, done=0):
    """The next batch's read count for a pipeline's ramp (misc.read_batches ramp=True): batches
    grow from max_reads / 8 by doubling (the later stages start after a small first parse) and,
    once fewer than 1.5 x max_reads reads remain (remaining_reads, estimated from the bytes left),
    take half of what remains, down to max_reads / 8 (the last write is a small one, overlapped by
    the trims before it). done: batches already read."""
    lo = max(1, max_reads // 8)
    want = min(max_reads, lo << done)
    if remaining_reads is not None and remaining_reads < 1.5 * max_reads:
        want = min(want, remaining_reads if remaining_reads <= 2 * lo else (remaining_reads + 1) // 2)
    return max(1, int(want))


def read_batches(path, max_reads=100000, max_bases=1 << 30, raw=False, byte_range=None, first_reads=None,
                 ramp=False):
    """Stream a FASTA / FASTQ(.gz) file as ReadBatch objects (pcabi_fastx_next); byte_range =
    (begin, end) record starts of a plain file (record_boundaries) reads only that range;
    first_reads: the first batch's size, if other than max_reads (a pipeline starts its later
    stages sooner on a small first batch); ramp: batch sizes from ramp_sizes (a plain file's last
    batches shrink too, from the bytes left and the bytes per read so far). Batching never changes
    what is read or written, only when."""
    L = _declare(lib())
    h = ctypes.c_void_p()
    rc = L.pcabi_fastx_open(os.fsencode(path), int(raw), ctypes.byref(h))
    if rc != 0:
        raise ValueError(_open_error(path))
    if byte_range is not None and L.pcabi_fastx_set_range(h, int(byte_range[0]), int(byte_range[1])) != 0:
        L.pcabi_fastx_close(h)
        raise ValueError(_open_error(path))
    try:
        want = int(first_reads) if first_reads else (ramp_sizes(int(max_reads)) if ramp else int(max_reads))
        left0 = L.pcabi_fastx_remaining(h)
        n_done, b_done, k = 0, 0, 0
        while True:
            b = ctypes.c_void_p()
            n = L.pcabi_fastx_next(h, want, int(max_bases), ctypes.byref(b))
            if n < 0:
                raise ValueError(_open_error(path))
            if n == 0:
                L.pcabi_reads_free(b)
                return
            k += 1
            want = int(max_reads)
            if ramp:
                left = L.pcabi_fastx_remaining(h)
                n_done += n
                est = None
                if left >= 0 and left0 > 0:
                    b_done = left0 - left
                    est = int(left * n_done / max(1, b_done))
                want = ramp_sizes(int(max_reads), est, k)
            yield ReadBatch(b)
    finally:
        L.pcabi_fastx_close(h)


def text_chunks(path, chunk_bytes):
    """Stream a FASTA / FASTQ(.gz) file as spans of its decoded text holding whole records, cut
    where a fresh reader parses the same records (pcabi_fastx_next_text): yields memoryviews of at
    least chunk_bytes (the last may be shorter), each valid until the next one is requested."""
    L = _declare(lib())
    h = ctypes.c_void_p()
    rc = L.pcabi_fastx_open(os.fsencode(path), 0, ctypes.byref(h))
    if rc != 0:
        raise ValueError(_open_error(path))
    try:
        while True:
            p, n = ctypes.c_void_p(), ctypes.c_int64()
            rc = L.pcabi_fastx_next_text(h, int(chunk_bytes), ctypes.byref(p), ctypes.byref(n))
            if rc < 0:
                raise ValueError(_open_error(path))
            if rc == 0:
                return
            yield memoryview((ctypes.c_char * int(n.value)).from_address(p.value)).cast('B')
    finally:
        L.pcabi_fastx_close(h)


def load_batch(path, raw=False):
    """The whole file as one ReadBatch (pcabi_fastx_load); raw keeps the file's own text."""
    L = _declare(lib())
    b = ctypes.c_void_p()
    rc = L.pcabi_fastx_load(os.fsencode(path), int(raw), ctypes.byref(b))
    if rc != 0:
        raise ValueError(_open_error(path))
    return ReadBatch(b)


# ---- the reference's Python surface (porechop_abi/misc.py) -----------------------------------
def get_compression_type(filename):
    """misc.py:60-81: 'gz' / 'plain' by magic bytes; bzip2 / zip exit with the reference's text."""
    with open(filename, 'rb') as f:
        start = f.read(4)
    if start.startswith(b'\x1f\x8b\x08'):
        return 'gz'
    if start.startswith(b'\x42\x5a\x68'):
        sys.exit('Error: cannot use bzip2 format - use gzip instead')
    if start.startswith(b'\x50\x4b\x03\x04'):
        sys.exit('Error: cannot use zip format - use gzip instead')
    return 'plain'


def load_fasta_or_fastq(filename):
    """misc.py:108-120 through the native reader in raw mode (the file's own text; the reference
    normalises it later, in NanoporeRead)."""
    if not os.path.isfile(filename):
        sys.exit('Error: could not find ' + filename)
    get_compression_type(filename)
    try:
        b = load_batch(filename, raw=True)
    except ValueError:
        sys.exit('\nError: ' + filename + ' could not be parsed - is it formatted correctly?')
    if b.type == FASTA:
        recs = []
        for i in range(b.n):
            full = b.name(i)
            recs.append((full.split()[0], b.sequence(i), full))
        return recs, 'FASTA'
    recs = []
    for i in range(b.n):
        full = b.name(i)
        recs.append((full.split()[0], b.sequence(i), b.spacer_line(i), b.quals(i), full))
    return recs, 'FASTQ'


# Terminal formatting of the verbose output (misc.py:270-316): the same escape codes.
END_FORMATTING = '\033[0m'
BOLD = '\033[1m'
UNDERLINE = '\033[4m'
RED = '\033[31m'
YELLOW = '\033[93m'


def red(text):
    return RED + text + END_FORMATTING


def yellow(text):
    return YELLOW + text + END_FORMATTING


def add_line_breaks_to_sequence(sequence, line_length):
    """misc.py:327-338."""
    if not sequence:
        return '\n'
    return ''.join(sequence[p:p + line_length] + '\n' for p in range(0, len(sequence), line_length))


def load_reads(input_file_or_directory, verbosity, print_dest, check_read_count):
    """porechop_abi.py:133-187: NanoporeRead objects from a file, or from every *.fastq(.gz)
    under an Albacore-style directory (check reads spread over the files, barcode from the path)."""
    if os.path.isfile(input_file_or_directory):
        if verbosity > 0:
            print('\nLoading reads', flush=True, file=print_dest)
            print(input_file_or_directory, flush=True, file=print_dest)
        get_compression_type(input_file_or_directory)
        try:
            b = load_batch(input_file_or_directory)
        except ValueError:
            sys.exit('\nError: ' + input_file_or_directory + ' could not be parsed - is it formatted correctly?')
        reads = b.nanopore_reads()
        read_type = 'FASTA' if b.type == FASTA else 'FASTQ'
        check_reads = reads[:check_read_count]
    elif os.path.isdir(input_file_or_directory):
        fastqs = sorted([os.path.join(d, f) for d, _, fs in os.walk(input_file_or_directory) for f in fs
                         if f.lower().endswith('.fastq') or f.lower().endswith('.fastq.gz')])
        if not fastqs:
            sys.exit('Error: could not find fastq files in ' + input_file_or_directory)
        reads, check_reads, read_type = [], [], 'FASTQ'
        per_file = int(round(check_read_count / len(fastqs)))
        for fq in fastqs:
            if verbosity > 0:
                print(fq, flush=True, file=print_dest)
            file_reads = load_batch(fq).nanopore_reads()
            bc = get_albacore_barcode_from_path(fq)
            for r in file_reads:
                r.albacore_barcode_call = bc
            reads += file_reads
            check_reads += file_reads[:per_file]
    else:
        sys.exit('Error: could not find ' + input_file_or_directory)
    if verbosity > 0:
        print('{:,}'.format(len(reads)) + ' reads loaded\n\n', flush=True, file=print_dest)
    return reads, check_reads, read_type


def get_albacore_barcode_from_path(albacore_path):
    """porechop_abi.py:190-197: the last /barcodeNN/ directory of the path."""
    import re
    if '/unclassified/' in albacore_path:
        return 'none'
    matches = re.findall('/barcode(\\d\\d)/', albacore_path)
    return 'BC' + matches[-1] if matches else None


def write_reads(batch, path, out_format='fastq', start_trim=None, end_trim=None, middle_cuts=None,
                min_split_read_size=1000, discard_middle=False, untrimmed=False, select=None, append=False,
                cut_arrays=None):
    """NanoporeRead.get_fasta / get_fastq for every read of a ReadBatch, natively
    (pcabi_reads_write). Returns how many reads produced output (a non-empty read string). out_format: 'fasta' | 'fastq' | 'fasta.gz' | 'fastq.gz'.
    middle_cuts: per read a list of (begin, end) ranges of the trimmed sequence (the reference's
    middle_trim_positions as ranges), or None; cut_arrays: the same as (cut_off int64 [n + 1],
    cuts int64 [2 * n_cuts]) arrays."""
    L = _declare(lib())
    gz = out_format.endswith('.gz')
    fasta = out_format.startswith('fasta')
    n = batch.n
    st = None if start_trim is None else np.ascontiguousarray(start_trim, np.int32)
    et = None if end_trim is None else np.ascontiguousarray(end_trim, np.int32)
    co = cu = None
    if cut_arrays is not None:
        co = np.ascontiguousarray(cut_arrays[0], np.int64)
        cu = np.ascontiguousarray(cut_arrays[1], np.int64)
        if cu.size == 0:
            cu = np.zeros(2, np.int64)
    elif middle_cuts is not None:
        co = np.zeros(n + 1, np.int64)
        flat = []
        for i, rg in enumerate(middle_cuts):
            rg = [(int(a), int(b)) for a, b in (rg or []) if b > a]
            co[i + 1] = co[i] + len(rg)
            for a, b in rg:
                flat += [a, b]
        cu = np.array(flat if flat else [0, 0], np.int64)
    sel = None if select is None else np.ascontiguousarray(select, np.uint8)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p) if a is not None else None
    rc = L.pcabi_reads_write(batch._h, os.fsencode(path), int(append), int(gz), int(fasta), p(st), p(et), p(co), p(cu),
                             int(min_split_read_size), int(discard_middle), int(untrimmed), p(sel))
    if rc < 0:
        check(rc, 'pcabi_reads_write')
    return int(rc)


def positions_to_ranges(positions):
    """A set of positions (NanoporeRead.middle_trim_positions) -> sorted disjoint [a, b) ranges."""
    out = []
    for x in sorted(positions):
        if out and out[-1][1] == x:
            out[-1][1] = x + 1
        else:
            out.append([x, x + 1])
    return [tuple(r) for r in out]

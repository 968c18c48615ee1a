"""Batched host interface to the MI355X adapter-alignment engine (libpcabi.so).

Sequences travel as Dna5 codes (A=0 C=1 G=2 T/U=3 other=4; the table of
S/basic/alphabet_residue_tabs.h:113-140 in the reference's vendored SeqAn) packed in one
byte buffer. A *window* is an (offset, length) view into that buffer (any offset); the buffer
carries 16 bytes of padding past its last sequence, as libpcabi requires (include/pcabi.h).

The reference encodes each Python str with UTF-8 before handing it to SeqAn
(porechop_abi/cpp_function_wrappers.py:52), so a non-ASCII character becomes several N codes;
``encode_seq`` reproduces that byte-for-byte.
"""
import ctypes
import itertools

import numpy as np

from ._lib import NFIELDS, check, lib

DNA5 = np.full(256, 4, dtype=np.uint8)
for _c, _v in (('A', 0), ('C', 1), ('G', 2), ('T', 3), ('U', 3)):
    DNA5[ord(_c)] = _v
    DNA5[ord(_c.lower())] = _v

PAD = 16


_AS_UTF8 = None


try:
    from . import _pystr   # the drivers' host helpers (csrc/pystr.c, built by __graft_entry__.build)
except ImportError:        # not built: the same results through Python-level passes
    _pystr = None


def str_buffers(seqs):
    """(character addresses uint64[n], lengths int64[n]) of a list of ASCII strs in one native
    pass (_pystr.ascii_buffers), or None when an item is not an ASCII str. The addresses are
    valid while the strs live."""
    n = len(seqs)
    if n == 0:
        return None
    if _pystr is None:
        try:
            if not all(map(str.isascii, seqs)):
                return None
        except TypeError:
            return None
        return (np.fromiter(map(_as_utf8(), seqs), np.uint64, n), np.fromiter(map(len, seqs), np.int64, n))
    addr = np.empty(n, np.uint64)
    lens = np.empty(n, np.int64)
    return (addr, lens) if _pystr.ascii_buffers(seqs, addr, lens) else None


def _as_utf8():
    global _AS_UTF8
    if _AS_UTF8 is None:
        f = ctypes.pythonapi.PyUnicode_AsUTF8
        f.restype, f.argtypes = ctypes.c_void_p, [ctypes.py_object]
        _AS_UTF8 = f
    return _AS_UTF8


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def encode_seq(seq):
    """str -> Dna5 codes (uint8 array), byte-exact with the reference's UTF-8 marshalling."""
    return DNA5[np.frombuffer(seq.encode('utf-8'), dtype=np.uint8)]


class SeqPack(object):
    """Sequences packed back to back (4-aligned starts, 16 bytes tail padding)."""

    def __init__(self, seqs):
        raw = self._pack_ascii(seqs)
        if raw is None:
            parts = []
            offs = np.zeros(len(seqs), dtype=np.int64)
            lens = np.zeros(len(seqs), dtype=np.int32)
            pos = 0
            for k, s in enumerate(seqs):
                b = s.encode('utf-8') if isinstance(s, str) else bytes(s)
                n = len(b)
                offs[k] = pos
                lens[k] = n
                pad = (-n) & 3
                parts.append(b)
                if pad:
                    parts.append(b'N' * pad)
                pos += n + pad
            parts.append(b'N' * PAD)
            raw = b''.join(parts)
        else:
            raw, offs, lens = raw
        self.codes = np.empty(len(raw), dtype=np.uint8)
        # the S/basic/alphabet_residue_tabs.h table, in C (threads for large batches)
        lib().pcabi_encode_dna5(raw, self.codes.ctypes.data_as(ctypes.c_void_p), len(raw))
        self.offsets = offs
        self.lengths = lens

    @staticmethod
    def _pack_ascii(seqs):
        """The same layout for a list of ASCII str (reads always are): one join and one encode
        instead of one encode per sequence (8 kb reads: ~4x faster). None for anything else."""
        if not seqs or not all(type(x) is str for x in seqs):
            return None
        if sum(map(len, seqs)) > 2000 * len(seqs):         # long reads: the copies dominate, no gain
            return None
        lens = np.fromiter(map(len, seqs), dtype=np.int64, count=len(seqs))
        pads = (-lens) & 3
        fill = ('', 'N', 'NN', 'NNN')
        joined = ''.join(itertools.chain(itertools.chain.from_iterable(zip(seqs, map(fill.__getitem__, pads.tolist()))),
                                         ('N' * PAD,)))
        if not joined.isascii():                       # multi-byte UTF-8: byte lengths differ
            return None
        offs = np.zeros(len(seqs), dtype=np.int64)
        np.cumsum((lens + pads)[:-1], out=offs[1:])
        return joined.encode('ascii'), offs, lens.astype(np.int32)

    @classmethod
    def windows(cls, seqs, starts, lengths, index=None, bufs=None, lazy=False):
        """The pack of [seqs[k][a:a + l] for k, a, l in zip(index, starts, lengths)] (index
        defaults to every sequence once; same layout as SeqPack of those slices) without making
        them: for ASCII str the codes are gathered from the strs' own buffers by
        pcabi_encode_dna5_gather (one byte per base, so character positions are byte positions).
        `starts` / `lengths` must lie inside each sequence. bufs: str_buffers(seqs) when the caller
        has it already. lazy: for ASCII str, a StrWindows (the same layout, not yet gathered) instead."""
        starts = np.asarray(starts, np.int64)
        lengths = np.asarray(lengths, np.int64)
        idx = np.arange(len(seqs)) if index is None else np.asarray(index, np.int64)
        n = len(idx)
        # CPython keeps an ASCII str's bytes inside the object: PyUnicode_AsUTF8 is their address
        # (no copy), valid while `seqs` holds the strs -- i.e. for this call
        if bufs is None and n > 0:
            bufs = str_buffers(seqs)
        if n == 0 or bufs is None:                     # bytes / arrays / non-ASCII: the slicing path
            return cls([seqs[k][a:a + l] for k, a, l in zip(idx.tolist(), starts.tolist(), lengths.tolist())])
        have = bufs[1][idx]
        if len(starts) != n or len(lengths) != n or (starts < 0).any() or (lengths < 0).any() or \
                (starts + lengths > have).any():
            raise ValueError('SeqPack.windows: a window lies outside its sequence')
        addr = bufs[0][idx] + starts.astype(np.uint64)
        offs = np.zeros(n, np.int64)
        np.cumsum((lengths + ((-lengths) & 3))[:-1], out=offs[1:])
        total = int(offs[-1] + lengths[-1] + ((-lengths[-1]) & 3)) + PAD
        if lazy:
            return StrWindows(seqs, addr, lengths, offs, total)
        self = cls.__new__(cls)
        self.codes = np.empty(total, np.uint8)
        lib().pcabi_encode_dna5_gather(_ptr(addr), _ptr(lengths), _ptr(offs), n, _ptr(self.codes), total)
        self.offsets = offs
        self.lengths = lengths.astype(np.int32)
        return self

    def __len__(self):
        return len(self.lengths)

    def views(self, starts, lengths, index=None):
        """Window views [start, start+len) of packed sequences (start relative to each sequence):
        (codes, offsets, lengths). No copy -- the kernels accept any offset."""
        idx = np.arange(len(self.lengths)) if index is None else np.asarray(index)
        starts = np.asarray(starts, dtype=np.int64)
        lengths = np.asarray(lengths, dtype=np.int32)
        return self.codes, self.offsets[idx] + starts, lengths


class StrWindows(object):
    """A window pack not made yet: the windows as addresses into ASCII strs (str_buffers) and
    lengths, at SeqPack.windows' offsets. engine.end_decisions hands the addresses to the library,
    which gathers and encodes them into pinned staging buffers itself (pcabi_end_decisions_seqs);
    np.asarray(w) makes the Dna5 pack for anything that needs the bytes. `codes` is the object
    itself, so it stands where a SeqPack's codes buffer goes; it keeps `seqs` (the strs) alive."""

    def __init__(self, seqs, addr, lengths, offsets, total):
        self.seqs = seqs
        self.addr = np.ascontiguousarray(addr, np.uint64)
        self._lens64 = np.ascontiguousarray(lengths, np.int64)
        self.lengths = self._lens64.astype(np.int32)
        self.offsets = np.ascontiguousarray(offsets, np.int64)
        self.size = int(total)
        self.codes = self

    def __len__(self):
        return self.size

    def __array__(self, dtype=None, copy=None):
        codes = np.empty(self.size, np.uint8)
        lib().pcabi_encode_dna5_gather(_ptr(self.addr), _ptr(self._lens64), _ptr(self.offsets), len(self.lengths),
                                       _ptr(codes), self.size)
        return codes if dtype is None else codes.astype(dtype, copy=False)


def start_end_windows(pack, end_size):
    """(start windows, end windows) exactly as seq[:end_size] and seq[-end_size:]
    (porechop_abi/nanopore_read.py:164,169,181,203), as packed views."""
    n = pack.lengths.astype(np.int64)
    e = int(end_size)
    s_len = np.minimum(n, e) if e >= 0 else np.maximum(n + e, 0)
    if e > 0:
        e_start = np.maximum(n - e, 0)
    elif e == 0:
        e_start = np.zeros_like(n)          # seq[-0:] is the whole sequence
    else:
        e_start = np.minimum(-e, n)
    e_len = n - e_start
    sw = pack.views(np.zeros_like(n), s_len.astype(np.int32))
    ew = pack.views(e_start, e_len.astype(np.int32))
    return sw, ew


def encode_adapters(adapter_seqs):
    b = [encode_seq(s) for s in adapter_seqs]
    lens = np.array([len(x) for x in b], dtype=np.int32)
    offs = np.zeros(len(b), dtype=np.int32)
    if len(b) > 1:
        offs[1:] = np.cumsum(lens)[:-1]
    codes = np.concatenate(b + [np.zeros(PAD, np.uint8)]).astype(np.uint8)
    return codes, offs, lens


def align(windows, adapter_seqs, scoring_scheme_vals, pairs=None, device=0):
    """Align windows against adapters on the GPU.

    windows: (codes uint8, offsets int64, lengths int32) as from SeqPack.views.
    pairs=None -> cross product, result column a*n_win + w; else (win_idx, adp_idx) arrays.
    Returns int32 array (8, n_results): rs, re, as, ae, score, m, l1, l2 (pcabi.h field order).
    """
    codes, offs, lens = windows
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    lens = np.ascontiguousarray(lens, dtype=np.int32)
    acodes, aoffs, alens = encode_adapters(adapter_seqs)
    n_win = len(lens)
    n_adp = len(alens)
    if pairs is None:
        tw = ta = None
        n_task = 0
        n_res = n_win * n_adp
    else:
        tw = np.ascontiguousarray(pairs[0], dtype=np.int32)
        ta = np.ascontiguousarray(pairs[1], dtype=np.int32)
        n_task = len(tw)
        n_res = n_task
    out = np.zeros((NFIELDS, n_res), dtype=np.int32)
    if n_res == 0:
        return out
    m, mm, go, ge = (int(x) for x in scoring_scheme_vals[:4])
    rc = lib().pcabi_align_host(device, _ptr(codes), codes.size, _ptr(offs), _ptr(lens), n_win,
                                _ptr(acodes), _ptr(aoffs), _ptr(alens), n_adp,
                                _ptr(tw), _ptr(ta), n_task, m, mm, go, ge, _ptr(out))
    check(rc, 'pcabi_align_host')
    return out


def first_hits(windows, adapter_seqs, scoring_scheme_vals, threshold, device=0):
    """Middle-scan round 1 on the GPU (pcabi_first_hits_host): for every window, the first adapter
    in list order whose full-adapter identity is not below `threshold`.
    Returns int32 (5, n_win): adapter index (-1 = none), rs, re (inclusive), m, l2."""
    codes, offs, lens = windows
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    lens = np.ascontiguousarray(lens, dtype=np.int32)
    acodes, aoffs, alens = encode_adapters(adapter_seqs)
    n_win = len(lens)
    out = np.zeros((5, n_win), dtype=np.int32)
    if n_win == 0:
        return out
    m, mm, go, ge = (int(x) for x in scoring_scheme_vals[:4])
    rc = lib().pcabi_first_hits_host(device, _ptr(codes), codes.size, _ptr(offs), _ptr(lens), n_win,
                                     _ptr(acodes), _ptr(aoffs), _ptr(alens), len(alens), m, mm, go, ge,
                                     float(threshold), _ptr(out))
    check(rc, 'pcabi_first_hits_host')
    return out


def middle_scan(windows, adapter_seqs, scoring_scheme_vals, threshold, device=0):
    """The reference's masked re-alignment loop (nanopore_read.py:219-252) for a batch of reads,
    in rounds on the GPU (pcabi_middle_scan_host). Returns int32 (6, n_hits): read, adapter,
    read_start, read_end (exclusive), m, l2, in discovery order (per read: the reference's order)."""
    codes, offs, lens = windows
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    lens = np.ascontiguousarray(lens, dtype=np.int32)
    acodes, aoffs, alens = encode_adapters(adapter_seqs)
    n_win = len(lens)
    if n_win == 0 or not len(alens):
        return np.zeros((6, 0), np.int32)
    m, mm, go, ge = (int(x) for x in scoring_scheme_vals[:4])
    cap = max(1024, n_win // 4)
    while True:
        out = np.zeros((6, cap), dtype=np.int32)
        n = lib().pcabi_middle_scan_host(device, _ptr(codes), codes.size, _ptr(offs), _ptr(lens), n_win,
                                         _ptr(acodes), _ptr(aoffs), _ptr(alens), len(alens), m, mm, go, ge,
                                         float(threshold), _ptr(out), cap)
        if n < 0:
            check(int(n), 'pcabi_middle_scan_host')
        if n <= cap:
            return out[:, :n]
        cap = int(n)


def middle_scan_seqs(addr, lens, adapter_seqs, scoring_scheme_vals, threshold, device=0):
    """middle_scan over windows given as host string addresses (pcabi_middle_scan_seqs): addr
    uint64[n] the address of each window's first character (an ASCII str's own bytes, see
    str_buffers), lens its length; the library encodes them into pinned staging buffers while the
    earlier chunks copy to the device -- no Dna5 pack in pageable memory. Same result as
    middle_scan over the packed windows."""
    addr = np.ascontiguousarray(addr, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.int32)
    acodes, aoffs, alens = encode_adapters(adapter_seqs)
    n_win = len(lens)
    if n_win == 0 or not len(alens):
        return np.zeros((6, 0), np.int32)
    m, mm, go, ge = (int(x) for x in scoring_scheme_vals[:4])
    cap = max(1024, n_win // 4)
    while True:
        out = np.zeros((6, cap), dtype=np.int32)
        n = lib().pcabi_middle_scan_seqs(device, _ptr(addr), _ptr(lens), n_win, _ptr(acodes), _ptr(aoffs),
                                         _ptr(alens), len(alens), m, mm, go, ge, float(threshold), _ptr(out), cap)
        if n < 0:
            check(int(n), 'pcabi_middle_scan_seqs')
        if n <= cap:
            return out[:, :n]
        cap = int(n)


def best_full_identity(windows, adapter_seqs, scoring_scheme_vals, best=None, device=0, best_device_ptr=None):
    """Adapter-set search reduction on the GPU (pcabi_best_full_identity_host,
    porechop_abi/nanopore_read.py:158-173): best[a] = max(best[a], max over windows of the full
    identity of (window, adapter a)), the (adapter, window) results never leaving the device.
    best: float64[n_adp] start values (zeros if None), returned updated. best_device_ptr: an int
    device address of float64[n_adp] on `device` to update in place instead (e.g. the tensor an
    RCCL all-reduce reduces next); then None is returned."""
    codes, offs, lens = windows
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    lens = np.ascontiguousarray(lens, dtype=np.int32)
    acodes, aoffs, alens = encode_adapters(adapter_seqs)
    m, mm, go, ge = (int(x) for x in scoring_scheme_vals[:4])
    if best_device_ptr is not None:
        rc = lib().pcabi_best_full_identity_host(device, _ptr(codes), codes.size, _ptr(offs), _ptr(lens), len(lens),
                                                 _ptr(acodes), _ptr(aoffs), _ptr(alens), len(alens), m, mm, go, ge,
                                                 ctypes.c_void_p(int(best_device_ptr)), 1)
        check(rc, 'pcabi_best_full_identity_host')
        return None
    out = np.zeros(len(alens), np.float64) if best is None else np.array(best, dtype=np.float64)
    rc = lib().pcabi_best_full_identity_host(device, _ptr(codes), codes.size, _ptr(offs), _ptr(lens), len(lens),
                                             _ptr(acodes), _ptr(aoffs), _ptr(alens), len(alens), m, mm, go, ge,
                                             _ptr(out), 0)
    check(rc, 'pcabi_best_full_identity_host')
    return out


_END_LIST_RATIO = [4.0]


def end_decisions(codes, start_windows, end_windows, start_seqs, end_seqs, scoring_scheme_vals, end_size, extra_trim,
                  end_threshold, min_trim_size, bc_start=None, bc_end=None, device=0):
    """find_start_trim / find_end_trim for a batch of reads on the GPU (pcabi_end_decisions_host,
    porechop_abi/nanopore_read.py:175-217): only the decisions come back, never the result matrix.

    codes: one Dna5 buffer holding both window sets, or the StrWindows they are views of (start
    windows, then end windows: pcabi_end_decisions_seqs); start_windows / end_windows: (offsets
    int64, lengths int32). Returns (start_trim int32[n], end_trim int32[n], start_list, end_list,
    bc_full): each list is int32 (7, k) -- read, adapter, rs, re (inclusive), m, l1, l2 -- of the
    alignments the reference records, read-major in adapter order; bc_full is float64
    (len(bc_start) + len(bc_end), n) full identities of the listed adapters (None without them)."""
    s_off = np.ascontiguousarray(start_windows[0], dtype=np.int64)
    s_len = np.ascontiguousarray(start_windows[1], dtype=np.int32)
    e_off = np.ascontiguousarray(end_windows[0], dtype=np.int64)
    e_len = np.ascontiguousarray(end_windows[1], dtype=np.int32)
    n = len(s_len)
    # window strings (StrWindows: start windows then end windows, the views its own) go to the
    # library as addresses; anything else as a Dna5 buffer
    strs = isinstance(codes, StrWindows) and len(codes.lengths) == 2 * n and \
        np.array_equal(codes.offsets, np.concatenate([s_off, e_off])) and \
        np.array_equal(codes.lengths, np.concatenate([s_len, e_len]))
    if not strs:
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
    sa, so, sl = encode_adapters(start_seqs)
    ea, eo, el = encode_adapters(end_seqs)
    bs = np.ascontiguousarray(bc_start if bc_start is not None else [], dtype=np.int32)
    be = np.ascontiguousarray(bc_end if bc_end is not None else [], dtype=np.int32)
    st = np.zeros(n, np.int32)
    et = np.zeros(n, np.int32)
    nb = len(bs) + len(be)
    bc_full = np.zeros((nb, n), np.float64) if nb else None
    # list capacity from the most alignments per read seen so far (a call whose lists overflow runs
    # again -- the whole decision, ~half the driver's library time, r05); the lists are np.empty:
    # only the columns written are ever touched, so headroom costs address space, not time
    cap = int(n * _END_LIST_RATIO[0] * 1.25) + 1024
    m, mm, go, ge = (int(x) for x in scoring_scheme_vals[:4])
    while True:
        sh = np.empty((7, cap), np.int32)
        eh = np.empty((7, cap), np.int32)
        cnt = np.zeros(2, np.int64)
        if strs:
            rc = lib().pcabi_end_decisions_seqs(device, _ptr(codes.addr), _ptr(codes.lengths), n, _ptr(sa), _ptr(so),
                                                _ptr(sl), len(sl), _ptr(ea), _ptr(eo), _ptr(el), len(el), m, mm, go, ge,
                                                int(end_size), int(extra_trim), float(end_threshold),
                                                int(min_trim_size), _ptr(st), _ptr(et), _ptr(sh), _ptr(eh), cap,
                                                _ptr(cnt), _ptr(bs), len(bs), _ptr(be), len(be), _ptr(bc_full))
            check(rc, 'pcabi_end_decisions_seqs')
        else:
            rc = lib().pcabi_end_decisions_host(device, _ptr(codes), codes.size, _ptr(s_off), _ptr(s_len),
                                                _ptr(e_off), _ptr(e_len), n, _ptr(sa), _ptr(so), _ptr(sl), len(sl),
                                                _ptr(ea), _ptr(eo), _ptr(el), len(el), m, mm, go, ge, int(end_size),
                                                int(extra_trim), float(end_threshold), int(min_trim_size), _ptr(st),
                                                _ptr(et), _ptr(sh), _ptr(eh), cap, _ptr(cnt), _ptr(bs), len(bs),
                                                _ptr(be), len(be), _ptr(bc_full))
            check(rc, 'pcabi_end_decisions_host')
        if n:
            _END_LIST_RATIO[0] = max(_END_LIST_RATIO[0], float(cnt.max()) / n)
        if cnt.max() <= cap:
            return st, et, sh[:, :cnt[0]], eh[:, :cnt[1]], bc_full
        cap = int(cnt.max())


def middle_cuts(hits, n_reads, bad_start, bad_end, good_side, bad_side, device=0):
    """Middle trim ranges of a scan's hits on the GPU (pcabi_middle_cuts_host,
    porechop_abi/nanopore_read.py:233-250): hits int32 (>= 4, n_hits) rows read, adapter,
    read_start, read_end (exclusive); bad_start / bad_end: per adapter, its name is a start / end
    sequence name. Returns (cut_off int64[n_reads + 1], cuts int64[2 * n_hits]) grouped per read
    in discovery order -- pcabi_reads_write's cut layout."""
    hits = np.ascontiguousarray(hits, dtype=np.int32)
    n_hits = hits.shape[1] if hits.ndim == 2 else 0
    bs = np.ascontiguousarray(bad_start, dtype=np.uint8)
    be = np.ascontiguousarray(bad_end, dtype=np.uint8)
    cut_off = np.zeros(n_reads + 1, np.int64)
    cuts = np.zeros(2 * n_hits, np.int64)
    rc = lib().pcabi_middle_cuts_host(device, _ptr(hits), n_hits, n_hits, n_reads, _ptr(bs), _ptr(be), len(bs),
                                      int(good_side), int(bad_side), _ptr(cut_off), _ptr(cuts))
    check(rc, 'pcabi_middle_cuts_host')
    return cut_off, cuts


_PID6_TAB = []


def pid6(m, l):
    """float('%f' % (100*m/l)) elementwise (NaN where l == 0), the reference's identity text
    round trip (porechop_abi/src/alignment.cpp:118-119, porechop_abi/nanopore_read.py:497-498).
    Pairs with 0 <= m, l < 256 (every end-window alignment) come from a table the library filled
    once (pcabi_pid6_host over all 65,536 pairs): the drivers convert ~10^6 pairs per batch."""
    m = np.ascontiguousarray(m, dtype=np.int32)
    l = np.ascontiguousarray(l, dtype=np.int32)
    if m.size > 4096 and m.shape == l.shape:
        small = ((m | l) & ~255) == 0
        if small.all():
            if not _PID6_TAB:
                mm, ll = np.divmod(np.arange(65536, dtype=np.int32), 256)
                tab = np.empty(65536, dtype=np.float64)
                lib().pcabi_pid6_host(_ptr(np.ascontiguousarray(mm)), _ptr(np.ascontiguousarray(ll)), 65536, _ptr(tab))
                _PID6_TAB.append(tab)
            return _PID6_TAB[0][(m << 8) | l]
    out = np.empty(m.shape, dtype=np.float64)
    lib().pcabi_pid6_host(_ptr(m), _ptr(l), m.size, _ptr(out))
    return out


def identities(res):
    """(full_adapter_identity, aligned_region_identity, read_start, read_end_exclusive) arrays,
    the tuple align_adapter returns (porechop_abi/nanopore_read.py:485-500)."""
    rs = res[0]
    failed = rs == -1
    full = pid6(res[5], res[7])
    part = pid6(res[5], res[6])
    full[failed] = 0.0
    part[failed] = 0.0
    read_end = np.where(failed, 0, res[1] + 1).astype(np.int64)
    return full, part, rs.astype(np.int64), read_end


def barcode_call(start_res, end_res, start_slots, end_slots, n_read, barcode_threshold, barcode_diff,
                 require_two, device=0, with_scores=False):
    """determine_barcode for a batch of reads on the GPU (pcabi_barcode_call_host,
    porechop_abi/nanopore_read.py:408-482).

    start_res / end_res: int32 (8, n_adp * n_read) cross-product results (column a*n_read + r).
    *_slots: (slot_adp, slot_name) int32 arrays, the side's barcode dict in insertion order
    (porechop_abi.barcode_slots). Returns call int32[n_read] (barcode id, -1 = 'none') and, with
    with_scores, float64 (n_read, 4)."""
    def side(res, slots):
        res = np.ascontiguousarray(res, dtype=np.int32).reshape(NFIELDS, -1)
        adp = np.ascontiguousarray(slots[0], dtype=np.int32)
        name = np.ascontiguousarray(slots[1], dtype=np.int32)
        n_adp = res.shape[1] // n_read if n_read else 0
        return res, adp, name, n_adp

    sr, sa, sn, n_sa = side(start_res, start_slots)
    er, ea, en, n_ea = side(end_res, end_slots)
    call = np.full(n_read, -1, dtype=np.int32)
    scores = np.zeros((n_read, 4), dtype=np.float64) if with_scores else None
    if n_read:
        rc = lib().pcabi_barcode_call_host(device, _ptr(sr), n_sa, _ptr(sa), _ptr(sn), len(sa), _ptr(er), n_ea,
                                           _ptr(ea), _ptr(en), len(ea), n_read, float(barcode_threshold),
                                           float(barcode_diff), int(bool(require_two)), _ptr(call),
                                           _ptr(scores) if with_scores else None)
        check(rc, 'pcabi_barcode_call_host')
    return (call, scores) if with_scores else call

"""ctypes access to the CPU oracle (oracle/pcabi_oracle.c). TEST INFRASTRUCTURE ONLY."""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, 'oracle', 'liboracle.so')


class Result(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int) for k in ('rs', 're', 'as_', 'ae', 'score', 'm', 'l1', 'l2')]


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(ROOT, 'oracle', 'pcabi_oracle.c')
    if not os.path.isfile(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.check_call(['make', '-s', '-C', os.path.join(ROOT, 'oracle')])
    L = ctypes.CDLL(SO)
    L.pcabi_oracle_align.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int] + \
        [ctypes.c_int] * 4 + [ctypes.POINTER(Result)]
    L.pcabi_oracle_adapter_alignment.argtypes = [ctypes.c_char_p, ctypes.c_char_p] + [ctypes.c_int] * 4
    L.pcabi_oracle_adapter_alignment.restype = ctypes.c_void_p
    L.pcabi_oracle_free.argtypes = [ctypes.c_void_p]
    L.pcabi_oracle_align_batch.argtypes = [ctypes.c_void_p] * 7 + [ctypes.c_longlong] + \
        [ctypes.c_int] * 4 + [ctypes.c_void_p]
    _lib = L
    return L


def align(read, adapter, scoring):
    """8 ints (rs, re, as, ae, score, m, l1, l2) for one pair; read/adapter are str."""
    L = load()
    r = Result()
    rb, ab = read.encode('utf-8'), adapter.encode('utf-8')
    L.pcabi_oracle_align(rb, len(rb), ab, len(ab), *scoring[:4], ctypes.byref(r))
    return [r.rs, r.re, r.as_, r.ae, r.score, r.m, r.l1, r.l2]


def result_string(read, adapter, scoring):
    L = load()
    p = L.pcabi_oracle_adapter_alignment(read.encode('utf-8'), adapter.encode('utf-8'), *scoring[:4])
    s = ctypes.cast(p, ctypes.c_char_p).value.decode()
    L.pcabi_oracle_free(p)
    return s


def align_many(reads, adapters, pairs, scoring):
    """(8, n_pairs) int32 for explicit (read_idx, adapter_idx) pairs."""
    L = load()
    rb = [r.encode('utf-8') for r in reads]
    ab = [a.encode('utf-8') for a in adapters]
    rbuf = b''.join(rb) + b'\0'
    abuf = b''.join(ab) + b'\0'
    roff = np.zeros(len(rb), np.int64)
    roff[1:] = np.cumsum([len(x) for x in rb])[:-1] if len(rb) > 1 else []
    rlen = np.array([len(x) for x in rb], np.int32)
    aoff = np.zeros(len(ab), np.int32)
    aoff[1:] = np.cumsum([len(x) for x in ab])[:-1] if len(ab) > 1 else []
    alen = np.array([len(x) for x in ab], np.int32)
    pr = np.asarray(pairs[0], np.int64)
    pa = np.ascontiguousarray(pairs[1], np.int32)
    off_p = np.ascontiguousarray(roff[pr])
    len_p = np.ascontiguousarray(rlen[pr])
    out = np.zeros((len(pr), 8), np.int32)
    rbufa = np.frombuffer(rbuf, np.uint8)
    abufa = np.frombuffer(abuf, np.uint8)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    L.pcabi_oracle_align_batch(vp(rbufa), vp(off_p), vp(len_p), vp(abufa), vp(aoff), vp(alen), vp(pa),
                               len(pr), *scoring[:4], vp(out))
    return out.T.copy()


_LETTERS = np.frombuffer(b'ACGTNNNN', dtype=np.uint8)


def align_windows(windows, adapter_seqs, scoring, pairs=None, device=0):
    """Drop-in for custom_porechop_abi_amd.engine.align computed by the oracle (CPU).
    Used by tests to exercise the batched host logic without a GPU."""
    codes, offs, lens = windows
    reads = [_LETTERS[codes[o:o + l]].tobytes().decode() for o, l in zip(offs.tolist(), lens.tolist())]
    n_win, n_adp = len(reads), len(adapter_seqs)
    if pairs is None:
        pr = np.tile(np.arange(n_win), n_adp)
        pa = np.repeat(np.arange(n_adp), n_win)
    else:
        pr, pa = np.asarray(pairs[0]), np.asarray(pairs[1])
    if len(pr) == 0:
        return np.zeros((8, 0), np.int32)
    return align_many(reads, list(adapter_seqs), (pr, pa), scoring)


def first_hits_windows(windows, adapter_seqs, scoring, threshold, device=0):
    """Drop-in for custom_porechop_abi_amd.engine.first_hits computed by the oracle (CPU): the
    first adapter (list order) whose full identity is not below threshold, per window."""
    from custom_porechop_abi_amd.engine import pid6
    n_win = len(windows[2])
    out = np.zeros((5, n_win), np.int32)
    out[0] = -1
    out[1] = -1
    if n_win == 0 or not adapter_seqs:
        return out
    res = align_windows(windows, adapter_seqs, scoring)
    n_adp = len(adapter_seqs)
    full = np.where(res[0] == -1, 0.0, pid6(res[5], res[7])).reshape(n_adp, n_win)
    strong = ~(full < threshold)
    for w in range(n_win):
        hit = np.nonzero(strong[:, w])[0]
        if len(hit):
            i = int(hit[0]) * n_win + w
            out[:, w] = [int(hit[0]), res[0, i], res[1, i], res[5, i], res[7, i]]
    return out


def middle_scan_windows(windows, adapter_seqs, scoring, threshold, device=0):
    """Drop-in for custom_porechop_abi_amd.engine.middle_scan computed by the oracle (CPU): the
    reference's loop (porechop_abi/nanopore_read.py:236-246) restated per read -- for each adapter
    in order, re-align while the full identity is not below the threshold, masking each hit."""
    from custom_porechop_abi_amd.engine import pid6
    codes, offs, lens = windows
    out = []
    for w, (o, l) in enumerate(zip(offs.tolist(), lens.tolist())):
        masked = _LETTERS[codes[o:o + l]].tobytes().decode()
        for a, adp in enumerate(adapter_seqs):
            while True:
                r = align(masked, adp, scoring)
                full = 0.0 if r[0] == -1 else float(pid6(np.array([r[5]]), np.array([r[7]]))[0])
                if full < threshold:
                    break
                rs, rend = (r[0], r[1] + 1) if r[0] != -1 else (-1, 0)
                masked = masked[:rs] + '-' * (rend - rs) + masked[rend:]
                out.append([w, a, rs, rend, r[5], r[7]])
    return np.array(out, np.int32).reshape(-1, 6).T.copy()


def middle_scan_threaded(windows, adapter_seqs, scoring, threshold, threads=None):
    """middle_scan_windows in C (pcabi_oracle_middle_scan), the reads spread over threads: the
    checker for bench-sized middle scans (thousands of reads x the 98-adapter list)."""
    L = load()
    L.pcabi_oracle_middle_scan.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int] + \
        [ctypes.c_int] * 4 + [ctypes.c_double, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong]
    L.pcabi_oracle_middle_scan.restype = ctypes.c_longlong
    codes, offs, lens = windows
    text = _LETTERS[np.asarray(codes)]                     # '-'-free: masked bases are N, as '-' is
    roff = np.ascontiguousarray(offs, np.int64)
    rlen = np.ascontiguousarray(lens, np.int32)
    ab = [a.encode() for a in adapter_seqs]
    abuf = np.frombuffer(b''.join(ab) + b'\0', np.uint8)
    alen = np.array([len(x) for x in ab], np.int32)
    aoff = np.zeros(len(ab), np.int32)
    if len(ab) > 1:
        aoff[1:] = np.cumsum(alen)[:-1]
    threads = threads or min(16, os.cpu_count() or 1)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    cap = 1 << 16
    while True:
        out = np.zeros((6, cap), np.int32)
        nh = L.pcabi_oracle_middle_scan(vp(text), vp(roff), vp(rlen), len(rlen), vp(abuf), vp(aoff), vp(alen), len(ab),
                                        *scoring[:4], float(threshold), threads, vp(out), cap)
        if nh <= cap:
            return out[:, :nh].copy()
        cap = int(nh)


def seqs_windows(addr, lens):
    """The windows engine.middle_scan_seqs takes (host character addresses, lengths) as the packed
    (codes, offsets, lengths) the windowed checkers take: the bytes read back with ctypes, encoded
    with the Dna5 table, 4-aligned offsets as SeqPack lays them out."""
    from custom_porechop_abi_amd.engine import DNA5, PAD
    lens = np.asarray(lens, np.int64)
    offs = np.zeros(len(lens), np.int64)
    if len(lens) > 1:
        offs[1:] = np.cumsum((lens + 3) & ~3)[:-1]
    total = int(offs[-1] + ((lens[-1] + 3) & ~3)) + PAD if len(lens) else PAD
    codes = np.full(total, 4, np.uint8)
    for a, o, l in zip(np.asarray(addr, np.uint64).tolist(), offs.tolist(), lens.tolist()):
        if l:
            codes[o:o + l] = DNA5[np.frombuffer(ctypes.string_at(a, l), np.uint8)]
    return codes, offs, lens.astype(np.int32)


def middle_scan_seqs_windows(addr, lens, adapter_seqs, scoring, threshold, device=0):
    """Drop-in for custom_porechop_abi_amd.engine.middle_scan_seqs computed by the oracle (CPU)."""
    return middle_scan_windows(seqs_windows(addr, lens), adapter_seqs, scoring, threshold)


def middle_scan_seqs_threaded(addr, lens, adapter_seqs, scoring, threshold, device=0):
    """middle_scan_seqs_windows on the C loop (middle_scan_threaded)."""
    return middle_scan_threaded(seqs_windows(addr, lens), adapter_seqs, scoring, threshold)


def best_full_identity_windows(windows, adapter_seqs, scoring, best=None, device=0, best_device_ptr=None):
    """Drop-in for custom_porechop_abi_amd.engine.best_full_identity computed by the oracle (CPU)."""
    from custom_porechop_abi_amd.engine import pid6
    assert best_device_ptr is None, 'the CPU stand-in has no device buffer'
    n_win, n_adp = len(windows[2]), len(adapter_seqs)
    out = np.zeros(n_adp, np.float64) if best is None else np.array(best, dtype=np.float64)
    if n_win == 0 or n_adp == 0:
        return out
    res = align_windows(windows, adapter_seqs, scoring)
    full = np.where(res[0] == -1, 0.0, pid6(res[5], res[7])).reshape(n_adp, n_win)
    return np.maximum(out, full.max(axis=1))


def end_decisions_windows(codes, start_windows, end_windows, start_seqs, end_seqs, scoring, end_size, extra_trim,
                          end_threshold, min_trim_size, bc_start=None, bc_end=None, device=0):
    """Drop-in for custom_porechop_abi_amd.engine.end_decisions computed by the oracle (CPU): the
    alignments of both sides, find_start_trim / find_end_trim's rules (nanopore_read.py:175-217)
    restated over them, the recorded alignments as (read, adapter, rs, re, m, l1, l2) lists in the
    reference's order, and the listed adapters' full identities."""
    from custom_porechop_abi_amd.engine import pid6
    codes = np.asarray(codes, np.uint8)             # an engine.StrWindows is gathered here
    n = len(start_windows[1])
    trims, lists, fulls = [], [], []
    for side, (win, seqs, sel) in enumerate(((start_windows, start_seqs, bc_start), (end_windows, end_seqs, bc_end))):
        na = len(seqs)
        if na == 0 or n == 0:
            trims.append(np.zeros(n, np.int32))
            lists.append(np.zeros((7, 0), np.int32))
            continue
        res = align_windows((codes, win[0], win[1]), list(seqs), scoring).reshape(8, na, n)
        rs = res[0]
        failed = rs == -1
        re1 = np.where(failed, 0, res[1] + 1)
        part = np.where(failed, 0.0, pid6(res[5].ravel(), res[6].ravel()).reshape(na, n))
        full = np.where(failed, 0.0, pid6(res[5].ravel(), res[7].ravel()).reshape(na, n))
        edge = (re1 != end_size) if side == 0 else (rs != 0)
        ok = (part > end_threshold) & edge & (re1 - rs >= min_trim_size)
        amount = np.where(ok, (re1 + extra_trim) if side == 0 else (end_size - rs) + extra_trim, 0)
        trims.append(np.maximum(amount.max(axis=0), 0).astype(np.int32))
        r, a = np.nonzero(ok.T)                    # read-major, adapter order within a read
        lists.append(np.stack([r, a, rs[a, r], res[1][a, r], res[5][a, r], res[6][a, r], res[7][a, r]]).astype(np.int32))
        if sel is not None and len(sel):
            fulls.append(full[np.asarray(sel)])
    bc_full = np.concatenate(fulls, axis=0) if fulls else None
    return trims[0], trims[1], lists[0], lists[1], bc_full

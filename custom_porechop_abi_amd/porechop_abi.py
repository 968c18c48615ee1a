"""Batched phase drivers (mirror of the hot-path drivers in porechop_abi/porechop_abi.py).

The reference fans every read (or read x adapter-set pair) out over a ThreadPool that calls
the per-pair C++ aligner once per alignment (porechop_abi.py:200-245, 359-438, 457-522). Here
each phase packs its windows once, runs ALL alignments of the phase as one GPU batch
(engine.align -> libpcabi k_align), and then applies the reference's per-read decision rules
(NanoporeRead._apply_* -- the same code the per-read methods use) in the reference's order.
Signatures are unchanged; `threads` is accepted and ignored (the GPU is the parallelism).

Middle-adapter scan (porechop_abi.py:457-522 / nanopore_read.py:219-252): the reference masks
every strong hit with '-' and re-aligns the SAME adapter, and the mask carries over to the
following adapters. The batched scan reproduces that order exactly in rounds: round 1 aligns
every read against every adapter on the unmasked read; for each read the first adapter (in
list order) with a hit is final for all adapters before it; the hit is masked and the read
re-enters the next round from that adapter on. Rounds repeat until no read has a hit.
"""
import contextlib
import gc
import sys
import threading

import numpy as np

from . import adapters as _adapters
from .adapters import make_full_native_barcode_adapter, make_new_full_rapid_barcode_adapter, \
    make_old_full_rapid_barcode_adapter
from . import engine
from .engine import SeqPack
from .misc import red

END_FORMATTING = '\033[0m'
BOLD = '\033[1m'
UNDERLINE = '\033[4m'


def int_to_str(num, max_num=0):
    s = 'n/a' if num is None else '{:,}'.format(num)
    return s.rjust(len('{:,}'.format(int(max_num))))


def bold_underline(text):
    return BOLD + UNDERLINE + text + END_FORMATTING


def output_progress_line(completed, total, print_dest, end_newline=False, step=10):
    if step > 1 and completed % step != 0 and completed != total:
        return
    pct = 100.0 * completed / total if total > 0 else 0.0
    line = '\r%s / %s (%.1f%%)' % (int_to_str(completed), int_to_str(total), pct)
    print(line, end='\n' if end_newline else '', flush=True, file=print_dest)


def _replay_progress(read_count, print_dest, plus_one=False):
    """The progress lines the reference's per-read loop prints after each read (every 10th and the
    last, output_progress_line's step), emitted after the batch. plus_one: the middle phase's
    thread-pool loop reports finished_count + 1 (porechop_abi.py:513-515)."""
    for k in range(1, read_count + 1):
        output_progress_line(k + 1 if plus_one else k, read_count, print_dest)


def _unique(seqs):
    """Deduplicate adapter sequences: (unique list, index of each input in it)."""
    pos, uniq, idx = {}, [], []
    for s in seqs:
        if s not in pos:
            pos[s] = len(uniq)
            uniq.append(s)
        idx.append(pos[s])
    return uniq, np.array(idx, dtype=np.int64)


# ---------------------------------------------------------------------------------------------
def find_matching_adapter_sets(check_reads, verbosity, end_size, scoring_scheme_vals, print_dest,
                               adapter_threshold, threads, adapter_sets=None):
    """Adapter-set discovery over the check reads (porechop_abi.py:200-245): every non-"full
    sequence" set's start/end sequence against every check read's start/end window; keeps the
    sets whose best start-or-end full-adapter identity reaches adapter_threshold."""
    if adapter_sets is None:
        adapter_sets = _adapters.ADAPTERS
    read_count = len(check_reads)
    if verbosity > 0:
        print(bold_underline('Looking for known adapter sets'), flush=True, file=print_dest)
        output_progress_line(0, read_count, print_dest)
    search = [a for a in adapter_sets if '(full sequence)' not in a.name]
    if check_reads:
        maxima = set_search_maxima(check_reads, end_size, scoring_scheme_vals, search)
        apply_set_maxima(search, maxima)
    if verbosity > 0:
        _replay_progress(read_count, print_dest)
        output_progress_line(read_count, read_count, print_dest, end_newline=True)
    return [a for a in search if a.best_start_or_end_score() >= adapter_threshold]


def set_search_maxima(check_reads, end_size, scoring_scheme_vals, search, out_device_ptr=None, device=0):
    """The check phase's reduction (nanopore_read.py:158-173 over every check read): per distinct
    start sequence, then per distinct end sequence of the searched sets, the best full-adapter
    identity over the reads' windows -- reduced on GPU `device` (engine.best_full_identity), the
    (adapter, window) results never leaving it. Returns the float64 maxima (start sequences
    first), or, with out_device_ptr (an int device address of as many float64 ON `device`),
    writes them there and returns None (the buffer the sharded drivers all-reduce)."""
    starts_u, _ = _unique([a.start_sequence[1] for a in search if a.start_sequence])
    ends_u, _ = _unique([a.end_sequence[1] for a in search if a.end_sequence])
    codes, (s_off, s_len), (e_off, e_len) = end_windows_pack(check_reads, end_size)
    sw, ew = (codes, s_off, s_len), (codes, e_off, e_len)
    if out_device_ptr is not None:
        if starts_u and len(check_reads):
            engine.best_full_identity(sw, starts_u, scoring_scheme_vals, device=device, best_device_ptr=out_device_ptr)
        if ends_u and len(check_reads):
            engine.best_full_identity(ew, ends_u, scoring_scheme_vals, device=device,
                                      best_device_ptr=out_device_ptr + 8 * len(starts_u))
        return None
    out = np.zeros(len(starts_u) + len(ends_u), np.float64)
    if len(check_reads):
        if starts_u:
            out[:len(starts_u)] = engine.best_full_identity(sw, starts_u, scoring_scheme_vals, device=device)
        if ends_u:
            out[len(starts_u):] = engine.best_full_identity(ew, ends_u, scoring_scheme_vals, device=device)
    return out


def apply_set_maxima(search, maxima):
    """best_start_score / best_end_score of every searched set = max(itself, its sequence's maximum)."""
    starts = [a for a in search if a.start_sequence]
    ends = [a for a in search if a.end_sequence]
    starts_u, s_idx = _unique([a.start_sequence[1] for a in starts])
    _, e_idx = _unique([a.end_sequence[1] for a in ends])
    maxima = np.asarray(maxima, dtype=np.float64)
    for a, k in zip(starts, s_idx.tolist()):
        a.best_start_score = max(a.best_start_score, float(maxima[k]))
    for a, k in zip(ends, e_idx.tolist()):
        a.best_end_score = max(a.best_end_score, float(maxima[len(starts_u) + k]))


def fix_up_1d2_sets(matching_sets):
    """porechop_abi.py:283-304. Note the reference compares against 'SQK-MAP006 Short' while
    the database names the set 'SQK-MAP006 short', so this never fires there; kept verbatim."""
    names = [x.name for x in matching_sets]
    if '1D^2 part 1' in names and '1D^2 part 2' in names and 'SQK-MAP006 Short' in names:
        score = {x.name: x.best_start_or_end_score() for x in matching_sets}
        if score['1D^2 part 1'] >= score['SQK-MAP006 Short'] and \
                score['1D^2 part 2'] >= score['SQK-MAP006 Short']:
            matching_sets = [x for x in matching_sets if x.name != 'SQK-MAP006 Short']
    return matching_sets


def choose_barcoding_kit(adapter_sets, verbosity, print_dest):
    """porechop_abi.py:248-280: pick forward or reverse barcodes from the discovery scores
    (best start-or-end first, then start+end sums). Exits like the reference when undecidable."""
    fwd_or = rev_or = fwd_and = rev_and = 0
    for s in adapter_sets:
        low = s.name.lower()
        if 'barcode' not in low:
            continue
        if '(forward)' in low:
            fwd_or += s.best_start_or_end_score()
            fwd_and += s.best_start_score + s.best_end_score
        elif '(reverse)' in low:
            rev_or += s.best_start_or_end_score()
            rev_and += s.best_start_score + s.best_end_score
    if fwd_or == 0 and rev_or == 0:
        sys.exit('Error: no barcodes were found, so Porechop cannot perform barcode demultiplexing')
    if fwd_or != rev_or:
        orientation = 'forward' if fwd_or > rev_or else 'reverse'
    elif fwd_and != rev_and:
        orientation = 'forward' if fwd_and > rev_and else 'reverse'
    else:
        sys.exit('Error: Porechop could not determine barcode orientation')
    if verbosity > 0:
        print('\nBarcodes determined to be in ' + orientation + ' orientation', file=print_dest)
    return orientation


def add_full_barcode_adapter_sets(matching_sets):
    """porechop_abi.py:324-348: add full native / rapid barcode adapters for found barcodes."""
    names = [x.name for x in matching_sets]
    for i in range(1, 97):
        if 'SQK-NSK007' in names and 'Barcode %d (reverse)' % i in names:
            matching_sets.append(make_full_native_barcode_adapter(i))
        if 'Rapid' in names and 'Barcode %d (forward)' % i in names:
            if 'RBK004_upstream' in names:
                matching_sets.append(make_new_full_rapid_barcode_adapter(i))
            elif 'SQK-NSK007' in names:
                matching_sets.append(make_old_full_rapid_barcode_adapter(i))
    return matching_sets


# ---------------------------------------------------------------------------------------------
def find_adapters_at_read_ends(reads, matching_sets, verbosity, end_size, extra_trim_size,
                               end_threshold, scoring_scheme_vals, print_dest, min_trim_size,
                               threads, check_barcodes, barcode_threshold, barcode_diff,
                               require_two_barcodes, forward_or_reverse_barcodes):
    """End trimming (porechop_abi.py:359-438): start window x start sequences and end window x
    end sequences of the matching sets for every read, then the per-read decisions of
    find_start_trim / find_end_trim / determine_barcode."""
    if verbosity > 0:
        print(bold_underline('Trimming adapters from read ends'), file=print_dest)
        name_len = max(max(len(x.start_sequence[0]) if x.start_sequence else 0 for x in matching_sets),
                       max(len(x.end_sequence[0]) if x.end_sequence else 0 for x in matching_sets))
        for s in matching_sets:
            for seq in (s.start_sequence, s.end_sequence):
                if seq:
                    print('  ' + seq[0].rjust(name_len) + ': ' + red(seq[1]), file=print_dest)
        print('', file=print_dest)
    read_count = len(reads)
    if verbosity == 1:
        output_progress_line(0, read_count, print_dest)
    if reads:
        starts = [a for a in matching_sets if a.start_sequence]
        ends = [a for a in matching_sets if a.end_sequence]
        _end_decisions(reads, starts, ends, end_size, extra_trim_size, end_threshold, scoring_scheme_vals,
                       min_trim_size, check_barcodes, forward_or_reverse_barcodes)
        if check_barcodes:
            for r in reads:
                r.determine_barcode(barcode_threshold, barcode_diff, require_two_barcodes)
    # per read, in read order, what the reference's loop prints after each read (:395-402, 426-432)
    if verbosity == 1:
        _replay_progress(read_count, print_dest)
    elif verbosity == 2:
        for r in reads:
            print(r.formatted_start_and_end_seq(end_size, extra_trim_size, check_barcodes), file=print_dest)
    elif verbosity > 2:
        for r in reads:
            print(r.full_start_end_output(end_size, extra_trim_size, check_barcodes), file=print_dest)
    if verbosity == 1:
        output_progress_line(read_count, read_count, print_dest, end_newline=True)
    if verbosity > 0:
        print('', file=print_dest)


def end_windows_pack(reads, end_size, lazy=False):
    """The reads' start and end windows, seq[:end_size] and seq[-end_size:] as the reference slices
    them (nanopore_read.py:181, 203), packed into one Dna5 buffer: (codes, start views, end views)
    -- only the 2 x end_size bases per read travel, not the whole reads. lazy: `codes` may be an
    engine.StrWindows (the windows as addresses into the reads' strs; the library encodes them)."""
    n = len(reads)
    seqs = _attrs(reads, 'seq')
    bufs = engine.str_buffers(seqs)
    ln = bufs[1] if bufs is not None else np.fromiter(map(len, seqs), np.int64, n)
    e = int(end_size)
    s_len = np.clip(ln + e if e < 0 else np.minimum(ln, e), 0, None)      # seq[:e]
    e_start = np.zeros(n, np.int64) if e == 0 else (np.maximum(ln - e, 0) if e > 0 else np.minimum(-e, ln))
    pack = SeqPack.windows(seqs, np.concatenate([np.zeros(n, np.int64), e_start]),
                           np.concatenate([s_len, ln - e_start]), index=np.tile(np.arange(n), 2),
                           bufs=bufs, lazy=lazy)   # seq[-e:]
    return pack.codes, (pack.offsets[:n], pack.lengths[:n]), (pack.offsets[n:], pack.lengths[n:])


_gc_lock = threading.Lock()
_gc_state = {'depth': 0, 'froze': False}


@contextlib.contextmanager
def _gc_paused():
    """While a driver makes its ~10^5 result tuples / lists, every object alive at the start (the
    batch's NanoporeRead objects among them) sits in the collector's permanent generation
    (gc.freeze), so the collections the new objects trigger do not walk the whole batch (a full
    pass over 100k reads cost a third of the end-trim driver's host time). The collector stays on:
    other threads' cyclic garbage is still collected. Freezing is process-wide, so it is done only
    when nothing is frozen yet (an application that froze its own objects, e.g. before a fork, keeps
    them frozen: the drivers then run without the shortcut), and nested or concurrent drivers share
    one freeze, undone by the last one out."""
    with _gc_lock:
        if _gc_state['depth'] == 0:
            _gc_state['froze'] = gc.get_freeze_count() == 0
            if _gc_state['froze']:
                gc.freeze()
        _gc_state['depth'] += 1
    try:
        yield
    finally:
        with _gc_lock:
            _gc_state['depth'] -= 1
            if _gc_state['depth'] == 0 and _gc_state['froze']:
                gc.unfreeze()
                _gc_state['froze'] = False


def _attrs(objs, name):
    """[getattr(o, name) for o in objs], in one native pass when the host helpers are built."""
    if engine._pystr is not None:
        return engine._pystr.attr_list(objs, name)
    return [getattr(o, name) for o in objs]


def _end_decisions(*args):
    with _gc_paused():
        _end_decisions_batch(*args)


def _end_decisions_batch(reads, starts, ends, end_size, extra, thr, scoring_scheme_vals, min_trim, check_barcodes,
                         fwd_rev):
    """The decisions of find_start_trim / find_end_trim (nanopore_read.py:175-217) for every read at
    once, on the device (engine.end_decisions: k_end_trim, then only the recorded alignments and --
    with -b -- the barcode identities come back): trim amounts, the start / end alignment lists in
    the reference's order (read, then set order) and the barcode dicts. Distinct sequences are
    aligned once; a list entry is made for every set holding the sequence."""
    codes, sw, ew = end_windows_pack(reads, end_size, lazy=True)
    s_u, s_idx = _unique([a.start_sequence[1] for a in starts])
    e_u, e_idx = _unique([a.end_sequence[1] for a in ends])
    bc = [[k for k, a in enumerate(sets) if check_barcodes and a.is_barcode() and a.barcode_direction() == fwd_rev]
          for sets in (starts, ends)]
    st, et, s_list, e_list, bc_full = engine.end_decisions(
        codes, sw, ew, s_u, e_u, scoring_scheme_vals, end_size, extra, thr, min_trim,
        bc_start=s_idx[bc[0]] if bc[0] else None, bc_end=e_idx[bc[1]] if bc[1] else None)
    if engine._pystr is not None:                 # one native pass: the same max-updates
        engine._pystr.raise_trims(reads, np.ascontiguousarray(st, np.int32), np.ascontiguousarray(et, np.int32))
    else:
        for r, a, b in zip(reads, st.tolist(), et.tolist()):
            if a > r.start_trim_amount:
                r.start_trim_amount = a
            if b > r.end_trim_amount:
                r.end_trim_amount = b
    for sets, idx, lst, attr in ((starts, s_idx, s_list, 'start_adapter_alignments'),
                                 (ends, e_idx, e_list, 'end_adapter_alignments')):
        if not sets or not lst.shape[1]:
            continue
        # distinct sequence -> the sets holding it (set order), as index arrays: `mem` lists the
        # sets grouped by distinct sequence, `first` / `cnt` each sequence's slice of it
        idx = np.asarray(idx, np.int64)
        cnt = np.bincount(idx, minlength=int(idx.max()) + 1)
        mem = np.argsort(idx, kind='stable')
        first = np.cumsum(cnt) - cnt
        read, u, rs, re_, m, l1, l2 = lst
        failed = rs == -1
        full = np.where(failed, 0.0, engine.pid6(m, l2))
        part = np.where(failed, 0.0, engine.pid6(m, l1))
        re_x = np.where(failed, 0, re_ + 1)
        if int(cnt.max()) == 1:
            # every distinct sequence in one set (the usual table): a row per alignment, and the
            # device's read-major lists are in set order within a read whenever the distinct
            # sequences are numbered in set order -- then nothing is expanded or sorted (r05)
            set_k = mem[u]
            key = read.astype(np.int64) * max(1, len(sets)) + set_k
            if key.size < 2 or bool(np.all(key[1:] > key[:-1])):
                order = None
            else:
                order = np.argsort(key, kind='stable')
            rd = read if order is None else read[order]
            if order is not None:
                set_k, full, part, rs, re_x = (x[order] for x in (set_k, full, part, rs, re_x))
        else:
            rep = cnt[u]
            within = np.arange(int(rep.sum())) - np.repeat(np.cumsum(rep) - rep, rep)
            set_k = mem[np.repeat(first[u], rep) + within]
            read = np.repeat(read, rep)
            # read-major, set order within a read: one stable sort of a combined key (the rows come
            # read-major already, so the sort's runs are long: ~6x faster than lexsort on 500 k rows)
            order = np.argsort(read.astype(np.int64) * max(1, len(sets)) + set_k, kind='stable')
            full, part, rs, re_x = (np.repeat(x, rep)[order] for x in (full, part, rs, re_x))
            rd = read[order]
            set_k = set_k[order]
        if engine._pystr is not None:             # the tuples made and appended in one native pass
            engine._pystr.append_rows(reads, attr, sets, rd.astype(np.int64), set_k.astype(np.int64),
                                      full.astype(np.float64), part.astype(np.float64), rs.astype(np.int64),
                                      re_x.astype(np.int64))
            continue
        # the tuples in one pass, then one extend per read (not one append per alignment)
        rows = list(zip(map(sets.__getitem__, set_k.tolist()), full.tolist(), part.tolist(), rs.tolist(),
                        re_x.tolist()))
        cut = np.flatnonzero(np.diff(rd)) + 1
        lo = np.concatenate([[0], cut]).tolist()
        hi = np.concatenate([cut, [len(rd)]]).tolist()
        for i, a, b in zip(rd[lo].tolist() if len(rd) else [], lo, hi):
            getattr(reads[i], attr).extend(rows[a:b])
    if bc_full is not None:
        j0 = 0
        for side, sets in ((0, starts), (1, ends)):
            names = [sets[k].get_barcode_name() for k in bc[side]]
            block = bc_full[j0:j0 + len(names)]
            j0 += len(names)
            if not names:
                continue
            for i, r in enumerate(reads):
                d = r.start_barcode_scores if side == 0 else r.end_barcode_scores
                for name, v in zip(names, block[:, i].tolist()):
                    d[name] = v


def barcode_slots(sets, forward_or_reverse, name_ids):
    """The barcode dict find_start_trim / find_end_trim build for every read
    (nanopore_read.py:193-195, 215-217) as slots for pcabi_barcode_call: in insertion order, the
    table index (among `sets`, the side's adapter table) of the adapter whose identity is the
    entry's final value -- a dict keeps a name's first position and its last value -- and the
    name's id in `name_ids` (extended in place, shared by both sides)."""
    pos, adp, name = {}, [], []
    for k, a in enumerate(sets):
        if not (a.is_barcode() and a.barcode_direction() == forward_or_reverse):
            continue
        nm = a.get_barcode_name()
        if nm not in name_ids:
            name_ids[nm] = len(name_ids)
        if nm in pos:
            adp[pos[nm]] = k
        else:
            pos[nm] = len(adp)
            adp.append(k)
            name.append(name_ids[nm])
    return np.array(adp, np.int32), np.array(name, np.int32)


# ---------------------------------------------------------------------------------------------
def middle_adapter_list(matching_sets):
    """porechop_abi.py:465-479: start sequences, plus end sequences that differ from their
    set's start sequence; and the start / end sequence-name sets."""
    adapters = []
    for s in matching_sets:
        if s.start_sequence:
            adapters.append(s.start_sequence)
        if s.end_sequence and (not s.start_sequence or s.end_sequence[1] != s.start_sequence[1]):
            adapters.append(s.end_sequence)
    start_names = {s.start_sequence[0] for s in matching_sets if s.start_sequence}
    end_names = {s.end_sequence[0] for s in matching_sets if s.end_sequence}
    return adapters, start_names, end_names


def trimmed_bounds(reads, seq_lens=None):
    """(start, length) of get_seq_with_start_end_adapters_trimmed() inside each read's seq, with
    Python's slice rules for seq[s:len(seq) - e] (a negative stop counts from the end, both ends
    clipped) -- the trimmed reads as views of the untrimmed ones, no copy. `seq_lens`: the reads'
    seq lengths when the caller has them already."""
    n = np.fromiter(map(len, _attrs(reads, 'seq')), np.int64, len(reads)) if seq_lens is None else \
        np.asarray(seq_lens, np.int64)
    if engine._pystr is not None:                 # one native pass per field, straight into int64
        s, e = np.empty(len(reads), np.int64), np.empty(len(reads), np.int64)
        engine._pystr.int_attrs(reads, 'start_trim_amount', s)
        engine._pystr.int_attrs(reads, 'end_trim_amount', e)
    else:
        s = np.array(_attrs(reads, 'start_trim_amount'), np.int64).reshape(-1)
        e = np.array(_attrs(reads, 'end_trim_amount'), np.int64).reshape(-1)
    a = np.minimum(s, n)
    b = n - e
    b = np.clip(np.where(b < 0, b + n, b), 0, n)
    return a, np.maximum(b - a, 0)


def scan_middles(seqs, adapter_seqs, middle_threshold, scoring_scheme_vals, device=0, bounds=None):
    """Exact batched equivalent of the reference's masked re-alignment loop
    (porechop_abi/nanopore_read.py:219-252), run on the GPU in rounds (engine.middle_scan,
    pcabi_middle_scan_host): round 1 keeps each read's first adapter over the threshold, later
    rounds re-align only the reads that just hit -- masked with '-' (Dna5 N) -- from that adapter
    onwards. `bounds` = (start, length) arrays scans those windows of `seqs` (in the sequences,
    as trimmed_bounds gives them) instead of the whole sequences; positions are relative to the
    window start.

    Returns, per read, the ordered list of hits (adapter_index, full_identity, read_start,
    read_end) that nanopore_read.find_middle_adapters would record."""
    hits = [[] for _ in range(len(seqs))]
    for r, lst in _middle_hits_by_read(seqs, adapter_seqs, middle_threshold, scoring_scheme_vals, device, bounds):
        hits[r] = lst
    return hits


def _middle_hits_by_read(seqs, adapter_seqs, middle_threshold, scoring_scheme_vals, device=0, bounds=None,
                         bufs=None):
    """scan_middles' hits as (read index, ordered hit list) for the reads that have any, in read
    order: the drivers then touch only those reads (a few percent of a batch), not every read.
    bufs: engine.str_buffers(seqs) when the caller has it."""
    n = len(seqs)
    if n == 0 or not adapter_seqs:
        return []
    if bufs is None:
        bufs = engine.str_buffers(seqs)
    if bufs is not None:
        # ASCII strs: the windows go to the library as addresses into the strs' own bytes, encoded
        # there into pinned staging buffers while earlier chunks copy (no pack in pageable memory)
        starts, lengths = (np.zeros(n, np.int64), bufs[1]) if bounds is None else \
            (np.asarray(bounds[0], np.int64), np.asarray(bounds[1], np.int64))
        if len(starts) != n or len(lengths) != n or (starts < 0).any() or (lengths < 0).any() or \
                (starts + lengths > bufs[1]).any():
            raise ValueError('middle scan: a window lies outside its sequence')
        h = engine.middle_scan_seqs(bufs[0] + starts.astype(np.uint64), lengths, adapter_seqs, scoring_scheme_vals,
                                    middle_threshold, device=device)
    else:
        pack = SeqPack(seqs) if bounds is None else SeqPack.windows(seqs, *bounds, bufs=bufs)
        views = pack.views(np.zeros(n, np.int64), pack.lengths)
        h = engine.middle_scan(views, adapter_seqs, scoring_scheme_vals, middle_threshold, device=device)
    if not h.shape[1]:
        return []
    full = engine.pid6(h[4], h[5])
    full[h[2] == -1] = 0.0
    # a read's hits keep their discovery order (rounds come back round-major): stable sort by read
    order = np.argsort(h[0], kind='stable')
    rd = h[0][order]
    rows = list(zip(h[1][order].tolist(), full[order].tolist(), h[2][order].tolist(), h[3][order].tolist()))
    cut = (np.flatnonzero(np.diff(rd)) + 1).tolist()
    lo, hi = [0] + cut, cut + [len(rows)]
    return [(r, rows[a:b]) for r, a, b in zip(rd[lo].tolist(), lo, hi)]


def find_adapters_in_read_middles(reads, matching_sets, verbosity, middle_threshold,
                                  extra_trim_good_side, extra_trim_bad_side, scoring_scheme_vals,
                                  print_dest, threads, discard_middle):
    """Middle-adapter split scan (porechop_abi.py:457-522)."""
    if verbosity > 0:
        verb = 'Discarding' if discard_middle else 'Splitting'
        print(bold_underline(verb + ' reads containing middle adapters'), file=print_dest)
    adapters, start_names, end_names = middle_adapter_list(matching_sets)
    read_count = len(reads)
    if verbosity == 1:
        output_progress_line(0, read_count, print_dest)
    # the trimmed reads packed straight from the untrimmed strs (SeqPack.windows), no slices
    with _gc_paused():
        seqs = _attrs(reads, 'seq')
        bufs = engine.str_buffers(seqs)
        by_read = _middle_hits_by_read(seqs, [a[1] for a in adapters], middle_threshold, scoring_scheme_vals,
                                       bounds=trimmed_bounds(reads, None if bufs is None else bufs[1]), bufs=bufs)
    # only reads with hits change; at verbosity > 1 every read is visited in order, since a read
    # with positions from an earlier call prints too (the reference's per-read loop, porechop_abi.py:487-495)
    visit = [(i, h.get(i, ())) for h in (dict(by_read),) for i in range(read_count)] if verbosity > 1 else by_read
    for i, hits in visit:
        r = reads[i]
        for a, full, s0, e0 in hits:
            r._apply_middle_hit(adapters[a][0], full, s0, e0, extra_trim_good_side, extra_trim_bad_side,
                                start_names, end_names)
        if r.middle_adapter_positions and verbosity > 1:
            print(r.middle_adapter_results(verbosity), file=print_dest, flush=True)
    if verbosity == 1:
        # the single-thread loop reports each read, the thread pool's loop one ahead (:492-493, 513-515)
        _replay_progress(read_count, print_dest, plus_one=threads != 1)
        output_progress_line(read_count, read_count, print_dest, end_newline=True)
        print('', flush=True, file=print_dest)


def filter_reads_by_adapter(reads, print_dest=sys.stdout):
    """The fork's filter (porechop_abi.py:36-39): keep reads with start AND end alignments."""
    kept = [r for r in reads if r.adapters_found()]
    print('Filtered reads: %d' % len(kept), file=print_dest)
    return kept


# ---------------------------------------------------------------------------------------------
def _print_table(table, print_dest, alignments='', col_separation=2, indent=2):
    """Plain-text table (the reference's misc.print_table without colours or wrapping): display
    only."""
    n = len(table[0])
    alignments = (alignments + 'L' * n)[:n]
    widths = [max(len(str(r[c])) for r in table) for c in range(n)]
    for r in table:
        cells = [str(x).ljust(w) if a == 'L' else str(x).rjust(w) for x, w, a in zip(r, widths, alignments)]
        print(' ' * indent + (' ' * col_separation).join(cells).rstrip(), file=print_dest)


def output_reads(reads, out_format, output, read_type, verbosity, discard_middle, min_split_size, print_dest,
                 barcode_dir, input_filename, untrimmed, threads, discard_unassigned):
    """porechop_abi.py:535-668 for a list of NanoporeRead: barcode bins (-b), stdout, or a file;
    the output format from `out_format` / the output name / the input read type as the reference
    ('auto'). Gzipped outputs are compressed here (gzip module) rather than by a gzip / pigz
    subprocess: the decompressed contents are the reference's byte for byte. As in the
    reference, `untrimmed` only applies to barcode bins. For files of millions of reads the
    native path is pipeline.FileTrimmer (barcode_dir included)."""
    import gzip
    import os
    from collections import defaultdict
    if verbosity > 0:
        trimmed_or_untrimmed = 'untrimmed' if untrimmed else 'trimmed'
        if barcode_dir is not None:
            verb, destination = 'Saving ', 'barcode-specific files'
        elif output is None:
            verb, destination = 'Outputting ', 'stdout'
        else:
            verb, destination = 'Saving ', 'file'
        print(bold_underline(verb + trimmed_or_untrimmed + ' reads to ' + destination), flush=True, file=print_dest)
    if out_format == 'auto':
        if output is None:
            out_format = read_type.lower()
            if barcode_dir is not None and input_filename.lower().endswith('.gz'):
                out_format += '.gz'
        elif '.fasta.gz' in output.lower():
            out_format = 'fasta.gz'
        elif '.fastq.gz' in output.lower():
            out_format = 'fastq.gz'
        elif '.fasta' in output.lower():
            out_format = 'fasta'
        elif '.fastq' in output.lower():
            out_format = 'fastq'
        else:
            out_format = read_type.lower()
    gzipped_out = False
    if out_format.endswith('.gz') and (barcode_dir is not None or output is not None):
        gzipped_out = True
        out_format = out_format[:-3]

    def read_string(read, with_untrimmed):
        if out_format == 'fasta':
            return read.get_fasta(min_split_size, discard_middle, untrimmed) if with_untrimmed \
                else read.get_fasta(min_split_size, discard_middle)
        return read.get_fastq(min_split_size, discard_middle, untrimmed) if with_untrimmed \
            else read.get_fastq(min_split_size, discard_middle)

    if barcode_dir is not None:
        os.makedirs(barcode_dir, exist_ok=True)
        parts = defaultdict(list)
        read_counts, base_counts = defaultdict(int), defaultdict(int)
        for read in reads:
            name = read.barcode_call
            if discard_unassigned and name == 'none':
                continue
            s = read_string(read, True)
            if not s:
                continue
            parts[name].append(s)
            read_counts[name] += 1
            base_counts[name] += len(read.seq) if untrimmed else read.seq_length_with_start_end_adapters_trimmed()
        table = [['Barcode', 'Reads', 'Bases', 'File']]
        for name in sorted(parts):
            path = os.path.join(barcode_dir, name + '.' + out_format)
            data = ''.join(parts[name]).encode()
            if gzipped_out:
                if os.path.isfile(path):
                    os.remove(path)
                path += '.gz'
                with gzip.open(path, 'wb') as f:
                    f.write(data)
            else:
                with open(path, 'wb') as f:
                    f.write(data)
            table.append([name, int_to_str(read_counts[name]), int_to_str(base_counts[name]), path])
        if verbosity > 0:
            print('', file=print_dest)
            _print_table(table, print_dest, alignments='LRRL')
    elif output is None:
        for read in reads:
            print(read_string(read, False), end='')
        if verbosity > 0:
            print('Done', flush=True, file=print_dest)
    else:
        data = ''.join(read_string(read, False) for read in reads).encode()
        if gzipped_out:
            with gzip.open(output, 'wb') as f:
                f.write(data)
        else:
            with open(output, 'wb') as f:
                f.write(data)
        if verbosity > 0:
            print('\nSaved result to ' + os.path.abspath(output), file=print_dest)
    if verbosity > 0:
        print('', flush=True, file=print_dest)

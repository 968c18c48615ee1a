"""File-to-file trimming on one GPU: the CLI's hot path without per-read Python objects
(porechop_abi/porechop_abi.py:41-131 after adapter-set discovery).

    ReadBatch (native parse, misc.read_batches)
      -> H2D of the packed Dna5 codes, start / end window views        (engine layout, no repack)
      -> k_tile_windows / k_align cross products / k_end_trim           (find_adapters_at_read_ends)
      -> trims D2H (8 B / read)
      -> pcabi_middle_scan_dev over the trimmed reads                   (find_adapters_in_read_middles)
      -> middle cut ranges (NanoporeRead._apply_middle_hit: pcabi_middle_cuts on the device)
      -> the fork's start-and-end filter (porechop_abi.py:36-39)
      -> native trimmed FASTA / FASTQ writer                             (output_reads, get_fastq)

Decisions are the reference's (same kernels and epilogues the parity tests cover); barcode
demultiplexing and verbose output stay with the per-read drivers (porechop_abi.py here).
"""
import ctypes
import os
import queue
import threading
import time

import numpy as np

from . import misc
from ._lib import check, cross_regions, lib
from .engine import encode_adapters, middle_cuts
from .porechop_abi import middle_adapter_list

VP = ctypes.c_void_p


class FileTrimmer(object):
    """Device state for trimming batches against one list of matching adapter sets.

    Options follow the reference's arguments (arg_parser.py defaults): end_size 150,
    end_threshold 75, extra_end_trim 2, min_trim_size 4, middle_threshold 90, extra middle trim
    10 (good side) / 100 (bad side), min_split_read_size 1000, no_split False, discard_middle
    False, adapter filter on (the fork's)."""

    barcode_dir = None                    # -b off (set by __init__)

    def __init__(self, matching_sets, scoring_scheme_vals=(3, -6, -5, -2), end_size=150, end_threshold=75.0,
                 extra_end_trim=2, min_trim_size=4, middle_threshold=90.0, extra_middle_trim_good_side=10,
                 extra_middle_trim_bad_side=100, min_split_read_size=1000, no_split=False, discard_middle=False,
                 filter_reads=True, device=0, barcode_dir=None, forward_or_reverse_barcodes='forward',
                 barcode_threshold=75.0, barcode_diff=5.0, require_two_barcodes=False, untrimmed=False,
                 discard_unassigned=False):
        self.L = L = lib()
        self.device = int(device)
        check(L.pcabi_dev_set(device), 'pcabi_dev_set')
        self.sc = tuple(int(x) for x in scoring_scheme_vals[:4])
        self.E, self.thr, self.extra, self.min_trim = int(end_size), float(end_threshold), int(extra_end_trim), \
            int(min_trim_size)
        self.mthr, self.good, self.bad = float(middle_threshold), int(extra_middle_trim_good_side), \
            int(extra_middle_trim_bad_side)
        self.min_split, self.no_split, self.discard_middle = int(min_split_read_size), bool(no_split), \
            bool(discard_middle)
        # the reference filters only when some adapter set matched (porechop_abi.py:93-122); with
        # none, every read is written unchanged
        self.filter_reads = bool(filter_reads) and bool(matching_sets)
        self.start_adps = [a.start_sequence[1] for a in matching_sets if a.start_sequence]
        self.end_adps = [a.end_sequence[1] for a in matching_sets if a.end_sequence]
        mids, start_names, end_names = middle_adapter_list(matching_sets)
        self.mid_adps = [x[1] for x in mids]
        self.bad_start = np.array([x[0] in start_names for x in mids], bool)
        self.bad_end = np.array([x[0] in end_names for x in mids], bool)
        self.tabs = [self._table(x) for x in (self.start_adps, self.end_adps, self.mid_adps)]
        self.scan = VP()
        if self.mid_adps:
            check(L.pcabi_scan_create(self.tabs[2], ctypes.byref(self.scan)), 'pcabi_scan_create')
        self.stream = VP()
        check(L.pcabi_stream_create(ctypes.byref(self.stream)), 'pcabi_stream_create')
        self.dev = {}
        self.times = {}
        # -b: barcode bins (porechop_abi.py:80-104, 581-638). The dicts find_start_trim /
        # find_end_trim fill become slot tables (porechop_abi.barcode_slots), the call runs on the
        # device after the end trim (pcabi_barcode_call_dev), and the writer sends every read to
        # <barcode_dir>/<call>.<format>; --untrimmed and --discard_unassigned as the reference
        # (the former only applies to bins there too).
        self.barcode_dir = barcode_dir
        if barcode_dir is not None:
            from .porechop_abi import barcode_slots
            ids = {}
            start_sets = [a for a in matching_sets if a.start_sequence]
            end_sets = [a for a in matching_sets if a.end_sequence]
            self.bc_slots = (barcode_slots(start_sets, forward_or_reverse_barcodes, ids),
                             barcode_slots(end_sets, forward_or_reverse_barcodes, ids))
            self.bc_names = {v: k for k, v in ids.items()}
            self.bc_thr, self.bc_diff, self.bc_two = float(barcode_threshold), float(barcode_diff), \
                bool(require_two_barcodes)
            self.untrimmed, self.discard_unassigned = bool(untrimmed), bool(discard_unassigned)

    def _table(self, seqs):
        if not seqs:
            return None
        c, o, l = encode_adapters(seqs)
        t = VP()
        check(self.L.pcabi_adapters_create_scored(c.ctypes.data_as(VP), o.ctypes.data_as(VP), l.ctypes.data_as(VP),
                                                  len(seqs), *self.sc, ctypes.byref(t)), 'pcabi_adapters_create')
        return t

    def _buf(self, key, nbytes):
        nbytes = max(int(nbytes), 16)
        if key not in self.dev or self.dev[key][1] < nbytes:
            if key in self.dev:
                # grown with headroom: batches of varying size do not reallocate (a free waits for
                # the device) every time one is a little larger than the last
                nbytes = max(nbytes, self.dev[key][1] + self.dev[key][1] // 4)
                self.L.pcabi_dev_free(self.dev[key][0])
            p = VP()
            check(self.L.pcabi_dev_malloc(ctypes.byref(p), nbytes), 'pcabi_dev_malloc')
            self.dev[key] = (p, nbytes)
        return self.dev[key][0]

    def _h2d(self, key, arr):
        arr = np.ascontiguousarray(arr)
        p = self._buf(key, arr.nbytes)
        if arr.nbytes:
            check(self.L.pcabi_dev_copy_async(p, arr.ctypes.data_as(VP), arr.nbytes, 0, self.stream), 'h2d')
        return p

    def _tick(self, key, t):
        now = time.perf_counter()
        self.times[key] = self.times.get(key, 0.0) + now - t
        return now

    def trim(self, batch, albacore=None):
        """Decisions for one ReadBatch: (start_trim, end_trim, cut_off, cuts, hits, keep).
        albacore: the barcode of the Albacore directory the batch came from (misc.input_files), or
        None; with -b a device call that disagrees with it becomes 'none' (nanopore_read.py:479-482)."""
        L, sc, nb = self.L, self.sc, batch.n
        t = time.perf_counter()
        lens = batch.lengths.astype(np.int64)
        E = self.E
        s_len = (np.minimum(lens, E) if E >= 0 else np.maximum(lens + E, 0)).astype(np.int32)
        if E > 0:
            e_start = np.maximum(lens - E, 0)
        elif E == 0:
            e_start = np.zeros_like(lens)
        else:
            e_start = np.minimum(-E, lens)
        e_len = (lens - e_start).astype(np.int32)
        d_codes = self._h2d('codes', batch.codes)
        trims = np.zeros((2, nb), np.int32)
        res = [None, None]
        regions = []
        n_ad = (len(self.start_adps), len(self.end_adps))
        for side, (w_off, w_len) in enumerate(((batch.code_off, s_len), (batch.code_off + e_start, e_len))):
            res[side] = self._buf('res%d' % side, 4 * 8 * max(1, n_ad[side]) * nb)
            if not n_ad[side] or nb == 0:
                continue
            toff = np.zeros((nb + 255) // 256 + 1, np.int64)
            nd = L.pcabi_tile_layout(w_len.ctypes.data_as(VP), nb, toff.ctypes.data_as(VP))
            d_off, d_len = self._h2d('off%d' % side, w_off), self._h2d('len%d' % side, w_len)
            d_toff = self._h2d('toff%d' % side, toff)
            d_tiles = self._buf('tiles%d' % side, 4 * nd)
            check(L.pcabi_tile_windows_dev(d_codes, d_off, d_len, nb, d_toff, int(np.diff(toff).max() // 256), d_tiles,
                                           self.stream), 'tile')
            regions.append((d_tiles, d_toff, d_len, nb, int(w_len.max()), self.tabs[side], res[side], n_ad[side] * nb))
        if regions:
            # both read ends in one call: their register buckets in grouped launches (r06)
            arr = cross_regions(regions)
            check(L.pcabi_align_cross_multi_dev(arr, len(regions), *sc, self.stream, None, None), 'align')
        if nb:
            d_st, d_et = self._buf('st', 4 * nb), self._buf('et', 4 * nb)
            check(L.pcabi_end_trim_dev(res[0], n_ad[0] * nb, n_ad[0], res[1], n_ad[1] * nb, n_ad[1], nb, E, self.extra,
                                       self.thr, self.min_trim, d_st, d_et, None, None, self.stream), 'end_trim')
            check(L.pcabi_dev_copy_async(trims[0].ctypes.data_as(VP), d_st, 4 * nb, 1, self.stream), 'd2h')
            check(L.pcabi_dev_copy_async(trims[1].ctypes.data_as(VP), d_et, 4 * nb, 1, self.stream), 'd2h')
            if self.barcode_dir is not None:
                calls = np.full(nb, -1, np.int32)
                (sa, sn), (ea, en) = self.bc_slots
                d_call = self._buf('bcall', 4 * nb)
                slots = [self._h2d('bc%d' % i, x) for i, x in enumerate((sa, sn, ea, en))]
                check(L.pcabi_barcode_call_dev(res[0], n_ad[0] * nb, slots[0], slots[1], len(sa), res[1],
                                               n_ad[1] * nb, slots[2], slots[3], len(ea), nb, self.bc_thr,
                                               self.bc_diff, int(self.bc_two), d_call, None, self.stream),
                      'barcode_call')
                check(L.pcabi_dev_copy_async(calls.ctypes.data_as(VP), d_call, 4 * nb, 1, self.stream), 'd2h')
                self.last_calls = calls
            check(L.pcabi_stream_sync(self.stream), 'sync')
            if self.barcode_dir is not None and albacore is not None:
                self.last_calls = self.albacore_filter(self.last_calls, albacore)
        elif self.barcode_dir is not None:
            self.last_calls = np.full(nb, -1, np.int32)
        t = self._tick('end_trim', t)
        cut_off = np.zeros(nb + 1, np.int64)
        cuts = np.zeros(0, np.int64)
        hits = np.zeros((6, 0), np.int32)
        if self.mid_adps and not self.no_split and nb:
            # get_seq_with_start_end_adapters_trimmed (nanopore_read.py:66-71): the Python slice
            # seq[st:len - et] of the reference, as a window of the packed read
            st, et = trims[0].astype(np.int64), trims[1].astype(np.int64)
            trimmed = (st > 0) | (et > 0)
            end = lens - et
            end = np.where(end < 0, np.maximum(lens + end, 0), end)
            a = np.minimum(st, lens)
            t_len = np.where(trimmed, np.maximum(end - a, 0), lens).astype(np.int32)
            t_off = batch.code_off + np.where(trimmed, a, 0)
            d_toff, d_tlen = self._h2d('toffm', t_off), self._h2d('tlenm', t_len)
            cap = max(4096, nb)
            while True:
                hits = np.zeros((6, cap), np.int32)
                nh = L.pcabi_middle_scan_dev(self.scan, d_codes, d_toff, d_tlen, t_len.ctypes.data_as(VP), nb, *sc,
                                             self.mthr, hits.ctypes.data_as(VP), cap, self.stream)
                if nh < 0:
                    check(int(nh), 'pcabi_middle_scan_dev')
                if nh <= cap:
                    break
                cap = int(nh)                 # the scan leaves the codes intact: rerun, larger

            hits = hits[:, :int(nh)]
            # NanoporeRead._apply_middle_hit's trim ranges (nanopore_read.py:242-250) on the device,
            # grouped per read in the writer's cut layout
            cut_off, cuts = middle_cuts(hits, nb, self.bad_start, self.bad_end, self.good, self.bad, self.device)
        t = self._tick('middle', t)
        keep = None
        if self.filter_reads:
            # the fork's filter: start AND end alignments (a recorded alignment always trims >= 1)
            keep = ((trims[0] > 0) & (trims[1] > 0)).astype(np.uint8)
        return trims[0], trims[1], cut_off, cuts, hits, keep

    def albacore_filter(self, calls, albacore):
        """determine_barcode's Albacore cross-check (nanopore_read.py:479-482): a read binned by
        Albacore keeps Porechop's call only when both agree, else it is 'none' (-1); reads of the
        'unclassified' directory (albacore 'none') all become 'none'."""
        ids = {v: k for k, v in self.bc_names.items()}
        want = ids.get(albacore, -2)
        return np.where(calls == want, calls, -1).astype(np.int32)

    def trim_file(self, in_path, out_path, out_format='fastq', max_reads=200000, byte_range=None, batch_filter=None,
                  segments=None, source=None):
        """Trim a FASTA / FASTQ(.gz) file -- or an Albacore output directory, its *.fastq(.gz) files
        in sorted order as load_reads reads them (porechop_abi.py:133-187), each batch carrying
        its file's barcode for the -b cross-check -- batch by batch into out_path. Returns read
        counts.

        Shards (shards.trim_file_sharded): byte_range = (begin, end) record starts of a plain file
        reads only that range; batch_filter(k) False skips batch k (parsed, not trimmed or
        written); segments, a list, receives (k, begin, end) byte spans of out_path per written batch;
        source, an iterable of (key, ReadBatch, albacore barcode), replaces reading in_path (the
        spooled chunks of shards.spool_batches; key is what segments record).

        Three stages overlap across batches: a reader thread parses the next batch, this thread
        runs the device work, a writer thread writes the previous batch (in file order). The
        library's parse, alignment and write calls release the GIL. times: 'parse' / 'write_wait'
        are this thread's waits, 'read' / 'write' the reader's / writer's own busy time (overlapped)."""
        counts = {'reads_in': 0, 'reads_kept': 0}
        # PCABI_PIPE_TRACE=1: (stage, batch, begin, end) per stage and batch in self.trace (the
        # pipeline's timeline: which stage holds the others up)
        trace = self.trace = [] if os.environ.get('PCABI_PIPE_TRACE') == '1' else None
        bins = {}                             # barcode name -> (path, reads selected for it)
        if self.barcode_dir is not None:
            os.makedirs(self.barcode_dir, exist_ok=True)
            counts['bins'] = bins
        # batches parsed ahead / trimmed and waiting for the writer (PCABI_PIPE_DEPTH, default 2)
        depth = max(1, int(os.environ.get('PCABI_PIPE_DEPTH', '2')))
        pq = queue.Queue(maxsize=depth)
        wq = queue.Queue(maxsize=depth)
        errors = []
        stop = threading.Event()          # set when this thread leaves: the reader stops putting

        def put_parsed(item):
            while not stop.is_set():
                try:
                    pq.put(item, timeout=0.05)
                    return True
                except queue.Full:
                    pass
            return False

        def batches():
            files = misc.input_files(in_path)
            if len(files) > 1 or files[0][1] is not None:
                if byte_range is not None:
                    raise ValueError('byte ranges apply to a single plain file, not to a directory')
            for f, alb in files:
                # batch sizes ramp up at the start and down at the end (misc.ramp_sizes): the first
                # parse and the last write are small, so they overlap the other stages
                for b in misc.read_batches(f, max_reads=max_reads, byte_range=byte_range, ramp=True):
                    yield b, alb

        def produce():
            try:
                items = iter(source if source is not None else
                             ((k, b, alb) for k, (b, alb) in enumerate(batches())))
                while True:
                    t0 = time.perf_counter()
                    item = next(items, None)
                    # the reader's own busy time (parse; overlapped like 'write')
                    t1 = time.perf_counter()
                    self.times['read'] = self.times.get('read', 0.0) + t1 - t0
                    if trace is not None:
                        trace.append(('read', item[0] if item is not None else -1, t0, t1))
                    if item is None:
                        break
                    k, b, alb = item
                    if batch_filter is not None and not batch_filter(k):
                        continue
                    if not put_parsed((k, b, alb)):
                        return
                put_parsed(None)
            except BaseException as ex:   # handed to the consumer
                put_parsed(ex)

        def consume_writes():
            first = True
            while True:
                item = wq.get()
                if item is None:
                    break
                if errors:
                    continue                 # drain after a failure
                k, b, st, et, co, cu, keep, calls = item
                t0 = time.perf_counter()
                try:
                    if calls is not None:
                        self._write_bins(b, out_format, st, et, co, cu, keep, calls, bins, k, segments)
                    else:
                        at = os.path.getsize(out_path) if (segments is not None and not first) else 0
                        misc.write_reads(b, out_path, out_format, st, et, None, self.min_split, self.discard_middle,
                                         select=keep, append=not first, cut_arrays=(co, cu))
                        if segments is not None:
                            segments.append((k, at, os.path.getsize(out_path)))
                except BaseException as ex:
                    errors.append(ex)
                first = False
                counts['reads_in'] += b.n
                counts['reads_kept'] += int(keep.sum()) if keep is not None else b.n
                t1 = time.perf_counter()
                self.times['write'] = self.times.get('write', 0.0) + t1 - t0
                if trace is not None:
                    trace.append(('write', k, t0, t1))
            if first and not errors and self.barcode_dir is None:   # empty input: still create the output
                open(out_path, 'wb').close()

        reader = threading.Thread(target=produce, daemon=True)
        writer = threading.Thread(target=consume_writes, daemon=True)
        reader.start()
        writer.start()
        t = time.perf_counter()
        try:
            while not errors:                # a failed write stops the run at the next batch
                b = pq.get()
                t = self._tick('parse', t)   # waiting for a parsed batch
                if b is None:
                    break
                if isinstance(b, BaseException):
                    raise b
                k, b, alb = b
                t0 = t
                st, et, co, cu, _, keep = self.trim(b) if alb is None else self.trim(b, albacore=alb)
                calls = self.last_calls if self.barcode_dir is not None else None
                t1 = time.perf_counter()
                wq.put((k, b, st, et, co, cu, keep, calls))   # the writer drains even after a failure
                del b
                t = time.perf_counter()
                self.times['put_wait'] = self.times.get('put_wait', 0.0) + t - t1
                if trace is not None:
                    trace.append(('trim', k, t0, t1))
                    trace.append(('put', k, t1, t))
        finally:
            # on every exit (errors included) the reader's pending put times out on `stop`, so
            # joining it cannot block on a full queue
            stop.set()
            wq.put(None)
            writer.join()
            reader.join()
        self._tick('write_wait', t)
        if errors:
            raise errors[0]
        return counts

    def _write_bins(self, b, out_format, st, et, co, cu, keep, calls, bins, k=0, segments=None):
        """One batch into the barcode bins (porechop_abi.py:581-610): the reads of each call, in
        read order, appended to <barcode_dir>/<name>.<format> (created, not appended, the first
        time the run writes it, as the reference opens each bin with 'wt'). segments (sharded
        runs) receives (k, name, begin, end) byte spans per bin write. As in the reference
        (porechop_abi.py:598-604) a bin exists only once some read of it produced output, and it
        counts only those reads: a write that emitted nothing leaves no file and no span."""
        sel = np.ones(b.n, bool) if keep is None else keep.astype(bool)
        if self.discard_unassigned:
            sel &= calls >= 0
        for cid in np.unique(calls[sel]).tolist():
            name = self.bc_names.get(cid, 'none') if cid >= 0 else 'none'
            mask = (sel & (calls == cid)).astype(np.uint8)
            path = os.path.join(self.barcode_dir, name + '.' + out_format)
            fresh = name not in bins
            at = 0 if fresh else os.path.getsize(path)
            emitted = misc.write_reads(b, path, out_format, st, et, None, self.min_split, self.discard_middle,
                                       untrimmed=self.untrimmed, select=mask, append=not fresh, cut_arrays=(co, cu))
            if emitted == 0:
                if fresh and os.path.exists(path):
                    os.remove(path)             # the reference never opens an empty bin
                continue
            bins[name] = (path, (0 if fresh else bins[name][1]) + emitted)
            if segments is not None:
                segments.append((k, name, at, os.path.getsize(path)))

    def close(self):
        L = self.L
        for p, _ in self.dev.values():
            L.pcabi_dev_free(p)
        self.dev = {}
        if self.scan:
            L.pcabi_scan_destroy(self.scan)
            self.scan = VP()
        for t in self.tabs:
            if t:
                L.pcabi_adapters_destroy(t)
        self.tabs = []
        if self.stream:
            L.pcabi_stream_destroy(self.stream)
            self.stream = VP()

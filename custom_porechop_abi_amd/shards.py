"""Multi-GPU drivers: one process per GPU, each owning a contiguous shard of the reads
(SURVEY.md §8(e)).

Every (read, adapter) alignment is independent, so the trimming phases need no exchange at all:
a rank runs the batched drivers of porechop_abi.py on its own reads. The one real exchange is
the adapter-set search (porechop_abi/porechop_abi.py:200-245): a set is kept when its best
full-adapter identity over ALL check reads reaches the threshold, so the per-sequence maxima
(one float64 per distinct start / end sequence, exact and order-free) are all-reduced with MAX
before the same filter runs on every rank. With backend "nccl" (RCCL over xGMI on MI355X) the
GPU reduction writes them straight into the device buffer the collective reduces; with "gloo"
they go through the host (the CPU tests).

Shards are contiguous read ranges, balanced by read count (end windows: equal work per read) or
by total bases (middle scan: work grows with read length). gather_trims() brings the per-read
trim amounts back to every rank in the original read order; share_trims() writes them into the
reads so the middle scan (which works on the end-trimmed sequence) can use its own shards.
"""
import numpy as np

from . import porechop_abi as P
from . import adapters as _adapters


def _dist():
    import torch.distributed as dist
    return dist


def shard_bounds(n, rank, world):
    """[lo, hi) of an equal-count contiguous split of n items."""
    lo = n * rank // world
    hi = n * (rank + 1) // world
    return lo, hi


def shard_bounds_by_length(lengths, rank, world):
    """[lo, hi) of a contiguous split balanced by the running sum of lengths (middle scan)."""
    lengths = np.asarray(lengths, dtype=np.int64)
    n = len(lengths)
    if n == 0:
        return 0, 0
    cum = np.concatenate([[0], np.cumsum(lengths)])
    total = cum[-1]
    cut = lambda r: int(np.searchsorted(cum, total * r / world, side='left')) if 0 < r < world else (0 if r == 0 else n)
    return min(cut(rank), n), min(cut(rank + 1), n)


def _device_tensor(values, group):
    import torch
    dist = _dist()
    t = torch.tensor(values, dtype=torch.float64)
    if dist.get_backend(group) == 'nccl':
        t = t.cuda()
    return t


def rank_device(device=None):
    """The GPU of this rank: `device` if given, else the node-local rank a launcher publishes
    (LOCAL_RANK from torch.distributed.run, or Open MPI's / MVAPICH's / Slurm's / Intel MPI's; one
    past the node's GPU count is an error, not a shared card), else the global rank when the world
    fits the node's GPUs; a larger world without a local rank is an error unless PCABI_SHARE_GPUS=1
    (rank mod GPUs). 0 outside torch.distributed."""
    import os
    import warnings
    if device is not None:
        return int(device)
    import torch
    n = torch.cuda.device_count()   # counting does not initialise the GPU
    # the node-local rank as torchrun, Open MPI, MVAPICH, Slurm or Intel MPI publish it
    for var in ('LOCAL_RANK', 'OMPI_COMM_WORLD_LOCAL_RANK', 'MV2_COMM_WORLD_LOCAL_RANK', 'SLURM_LOCALID',
                'MPI_LOCALRANKID'):
        if var in os.environ:
            dev = int(os.environ[var])
            if n > 0 and dev >= n:
                raise RuntimeError('%s %d but this node has %d GPU(s): one process per GPU' % (var, dev, n))
            return dev
    dist = _dist()
    if not (dist.is_available() and dist.is_initialized()):
        return 0
    rank, world = dist.get_rank(), dist.get_world_size()
    if n > 0 and world > n:
        # no node-local rank: one node oversubscribed, or a launcher that publishes none. Sharing
        # cards (rank mod GPUs) is opt-in (PCABI_SHARE_GPUS=1), not a silent fallback.
        if os.environ.get('PCABI_SHARE_GPUS') != '1':
            raise RuntimeError('the world (%d ranks) exceeds this node\'s %d GPU(s) and no node-local rank is set '
                               '(LOCAL_RANK, OMPI_COMM_WORLD_LOCAL_RANK, SLURM_LOCALID, ...): one process per GPU; '
                               'PCABI_SHARE_GPUS=1 lets rank r take GPU r mod %d' % (world, n, n))
        warnings.warn('PCABI_SHARE_GPUS=1: rank %d takes GPU %d of %d' % (rank, rank % n, n))
    return rank % n if n > 0 else rank


def find_matching_adapter_sets(check_reads, verbosity, end_size, scoring_scheme_vals, print_dest,
                               adapter_threshold, threads, adapter_sets=None, group=None, device=None):
    """Sharded porechop_abi.find_matching_adapter_sets: check_reads is the FULL check list (same
    on every rank); each rank reduces its shard's windows on its GPU (rank_device(device)) into
    the per-sequence maxima (porechop_abi.set_search_maxima: the (adapter, window) results never
    leave the device), and those maxima are all-reduced with MAX. With "nccl" (RCCL) the kernel
    writes them straight into the device buffer the collective reduces -- allocated on the same
    GPU the kernel runs on (include/pcabi.h: `best` lives on `device`); with "gloo" they go
    through the host."""
    dist = _dist()
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    dev = rank_device(device)
    if adapter_sets is None:
        adapter_sets = _adapters.ADAPTERS
    if not dist.is_initialized():
        return P.find_matching_adapter_sets(check_reads, verbosity, end_size, scoring_scheme_vals, print_dest,
                                            adapter_threshold, threads, adapter_sets=adapter_sets)
    lo, hi = shard_bounds(len(check_reads), rank, world)
    search = [a for a in adapter_sets if '(full sequence)' not in a.name]
    n_u = len(set(a.start_sequence[1] for a in search if a.start_sequence)) + \
        len(set(a.end_sequence[1] for a in search if a.end_sequence))
    import torch
    if dist.get_backend(group) == 'nccl':
        # RCCL reduces on the current device: make it the rank's, and put the buffer there
        torch.cuda.set_device(dev)
        t = torch.zeros(max(n_u, 1), dtype=torch.float64, device=torch.device('cuda', dev))
        if t.device.index != dev:
            raise RuntimeError('set-search buffer on cuda:%s, kernels on device %d' % (t.device.index, dev))
        torch.cuda.synchronize(dev)
        P.set_search_maxima(check_reads[lo:hi], end_size, scoring_scheme_vals, search, out_device_ptr=t.data_ptr(),
                            device=dev)
    else:
        t = torch.zeros(max(n_u, 1), dtype=torch.float64)
        t[:n_u] = torch.from_numpy(P.set_search_maxima(check_reads[lo:hi], end_size, scoring_scheme_vals, search,
                                                       device=dev))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    P.apply_set_maxima(search, t.cpu().numpy()[:n_u])
    return [a for a in search if a.best_start_or_end_score() >= adapter_threshold]


def local_reads(reads, group=None, by_length=False):
    """This rank's contiguous shard of `reads` and its [lo, hi) bounds."""
    dist = _dist()
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if by_length:
        lo, hi = shard_bounds_by_length([len(r.seq) for r in reads], rank, world)
    else:
        lo, hi = shard_bounds(len(reads), rank, world)
    return reads[lo:hi], (lo, hi)


def find_adapters_at_read_ends(reads, matching_sets, *args, group=None, **kwargs):
    """Sharded end trimming: each rank trims its own shard of `reads` (no collective).
    Returns (lo, hi) of the shard this rank processed."""
    mine, bounds = local_reads(reads, group)
    P.find_adapters_at_read_ends(mine, matching_sets, *args, **kwargs)
    return bounds


def find_adapters_in_read_middles(reads, matching_sets, *args, group=None, **kwargs):
    """Sharded middle-adapter scan, shards balanced by bases (no collective). The scan reads each
    read's end-trim amounts (NanoporeRead.get_seq_with_start_end_adapters_trimmed), so they must
    be set on every read first: share_trims() after the sharded end trimming.
    Returns (lo, hi) of the shard this rank processed."""
    mine, bounds = local_reads(reads, group, by_length=True)
    P.find_adapters_in_read_middles(mine, matching_sets, *args, **kwargs)
    return bounds


def share_trims(reads, bounds, group=None):
    """Write every rank's end-trim amounts into all of `reads` (one all-gather, 16 B per read)."""
    st, et = gather_trims(reads, bounds, group)
    for r, s, e in zip(reads, st.tolist(), et.tolist()):
        r.start_trim_amount, r.end_trim_amount = s, e


def gather_trims(reads, bounds, group=None):
    """All-gather the (start_trim, end_trim) amounts of every rank's shard into arrays over the
    full read list (original order). `bounds` = the (lo, hi) this rank processed."""
    dist = _dist()
    lo, hi = bounds
    mine = np.array([[r.start_trim_amount, r.end_trim_amount] for r in reads[lo:hi]], np.float64).reshape(-1, 2)
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return mine[:, 0].astype(np.int64), mine[:, 1].astype(np.int64)
    world = dist.get_world_size(group)
    sizes = _device_tensor([float(hi - lo)], group)
    all_sizes = [sizes.clone() for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    counts = [int(s.item()) for s in all_sizes]
    width = max(counts) if counts else 0
    buf = np.zeros((width, 2), np.float64)
    buf[:len(mine)] = mine
    t = _device_tensor(buf.tolist() if width else [[0.0, 0.0]], group)
    parts = [t.clone() for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    rows = np.concatenate([p.cpu().numpy()[:c] for p, c in zip(parts, counts)], axis=0)
    return rows[:, 0].astype(np.int64), rows[:, 1].astype(np.int64)


# ---- spooled input: gzip files and Albacore directories ----------------------------------------
# A gzip stream cannot be entered mid-way, so one reader (rank 0's distributor thread) inflates it
# once, cut into spans of whole records (misc.text_chunks), and writes span c to a spool file that
# rank c % world parses and trims as soon as it is there. Every rank, rank 0's own trimming
# included, consumes its spans in order; at most SPOOL_DEPTH spans per rank wait on disk (the
# distributor blocks until the rank has deleted one), so no full-size scratch copy is made and
# nobody waits for the whole inflate. A failure of the distributor leaves an .error marker that
# makes every consumer raise instead of waiting. The spool directory must be visible to every rank
# (the output directory by default; /dev/shm only when all ranks share a node).
SPOOL_CHUNK_BYTES = 128 << 20
SPOOL_DEPTH = 2


def _spool_prefix(spool, job):
    import os
    return os.path.join(spool, '.pcabi_spool_%s_' % job)


def spool_distribute(in_path, spool, job, world, chunk_bytes=None, depth=SPOOL_DEPTH, stop=None):
    """Rank 0's distributor (run in a thread): every input file in load_reads' order
    (misc.input_files), cut into record-aligned spans of ~chunk_bytes, span c written to
    <spool>/.pcabi_spool_<job>_<c>_<albacore>.fq for rank c % world; then an .end marker holding
    the span count, or an .error marker holding the failure."""
    import os
    import time
    from . import misc
    pre = _spool_prefix(spool, job)
    chunk_bytes = int(chunk_bytes or SPOOL_CHUNK_BYTES)
    pending = [[] for _ in range(world)]
    c = 0

    def beat():                               # liveness for the consumers' bounded wait
        with open(pre + 'beat', 'w'):
            pass

    try:
        beat()
        for f, alb in misc.input_files(in_path):
            for mv in misc.text_chunks(f, chunk_bytes):
                r = c % world
                t_beat = time.monotonic()
                while True:
                    pending[r] = [x for x in pending[r] if os.path.exists(x)]
                    if len(pending[r]) < depth:
                        break
                    if (stop is not None and stop.is_set()) or os.path.exists(pre + 'error'):
                        return                 # this rank or another one gave up
                    if time.monotonic() - t_beat > 1.0:
                        beat()
                        t_beat = time.monotonic()
                    time.sleep(0.005)
                path = '%s%d_%s.fq' % (pre, c, alb if alb is not None else '-')
                with open(path + '.tmp', 'wb') as fo:
                    fo.write(mv)
                os.replace(path + '.tmp', path)
                pending[r].append(path)
                beat()
                c += 1
        with open(pre + 'end.tmp', 'w') as fo:
            fo.write(str(c))
        os.replace(pre + 'end.tmp', pre + 'end')
    except BaseException as ex:   # every consumer raises it instead of waiting
        with open(pre + 'error', 'w') as fo:
            fo.write('%s: %s' % (type(ex).__name__, ex))


def spool_fail_cleanup(spool, job, rank, world, wait_s=30.0, poll=0.01):
    """A failed rank's share of the spool cleanup (the job raised on this rank): its own spans that
    were never consumed go (span c belongs to rank c % world), then an acknowledgement marker. Rank
    0 -- which has joined the distributor, so nothing new appears -- removes every file of the job
    once every rank has acknowledged; the other ranks wait (bounded) until it has, so a launcher that
    kills the rest of a job when one process fails (torch.multiprocessing.spawn) cannot cut rank 0's
    cleanup short. If some rank has not acknowledged within wait_s (it is still trimming a span and
    has not seen the failure yet), rank 0 removes the spans but leaves the .error / .end markers and
    the acknowledgements, plus a .left marker: the late rank still finds the error and raises
    instead of polling for spans forever, and the last rank to acknowledge removes what is left."""
    import os
    import time
    pre = _spool_prefix(spool, job)
    d, base = os.path.split(pre)

    def rm(name):
        try:
            os.remove(os.path.join(d, name))
        except FileNotFoundError:
            pass

    for f in os.listdir(d):
        head = f[len(base):].split('_', 1)[0] if f.startswith(base) else ''
        if head.isdigit() and int(head) % world == rank:
            rm(f)                                 # a span (or its .tmp) of this rank
    with open(pre + 'ack%d' % rank, 'w'):
        pass

    def all_acked(names):
        return all(base + 'ack%d' % r in names for r in range(world))

    def rm_all():
        for f in os.listdir(d):
            if f.startswith(base):
                rm(f)

    t_end = time.monotonic() + wait_s
    while time.monotonic() < t_end:
        names = set(os.listdir(d))
        if rank == 0 and all_acked(names):
            rm_all()
            return
        if rank != 0:
            if base + 'ack%d' % rank not in names:
                return                            # rank 0 has cleaned up
            if base + 'left' in names and all_acked(names):
                rm_all()                          # rank 0 left first: the last rank cleans up
                return
        time.sleep(poll)
    if rank == 0:
        # a rank has not seen the failure yet: everything but the markers it needs to raise
        keep = {base + x for x in ('error', 'end', 'left')} | {base + 'ack%d' % r for r in range(world)}
        for f in os.listdir(d):
            if f.startswith(base) and f not in keep:
                rm(f)
        with open(pre + 'left', 'w'):
            pass
        if all_acked(set(os.listdir(d))):         # it acknowledged meanwhile
            rm_all()


def spool_batches(spool, job, rank, world, max_reads, poll=0.005, stale_s=600.0):
    """This rank's spans from the distributor, parsed: yields ((c, j), ReadBatch, albacore) for
    batch j of span c = rank, rank + world, ... in order, deleting each span file once parsed.
    The wait for a span is bounded: the distributor touches a .beat marker while it runs (each span
    written, and every second it waits for a slow rank); if neither a span, the .end marker nor the
    .error marker appears while the beat is older than stale_s seconds (the distributor's process
    died without leaving .error), this rank raises instead of polling forever."""
    import os
    import time
    from . import misc
    pre = _spool_prefix(spool, job)
    d, base = os.path.split(pre)
    c = rank
    while True:
        t_wait = time.time()
        while True:
            if os.path.exists(pre + 'error'):
                with open(pre + 'error') as f:
                    raise RuntimeError('input distributor failed: ' + f.read())
            mine = [x for x in os.listdir(d) if x.startswith('%s%d_' % (base, c)) and x.endswith('.fq')]
            if mine:
                break
            if os.path.exists(pre + 'end'):
                with open(pre + 'end') as f:
                    if c >= int(f.read()):
                        return
                continue                       # the marker came after the span: look again
            if time.time() - t_wait > stale_s:
                try:
                    beat = os.path.getmtime(pre + 'beat')
                except OSError:
                    beat = t_wait
                if time.time() - beat > stale_s:
                    raise RuntimeError('input distributor silent for %.0f s (span %d of job %s never came)'
                                       % (time.time() - beat, c, job))
            time.sleep(poll)
        path = os.path.join(d, mine[0])
        alb = mine[0][len(base) + len(str(c)) + 1:-3]
        alb = None if alb == '-' else alb
        try:
            for j, b in enumerate(misc.read_batches(path, max_reads=max_reads)):
                yield (c, j), b, alb
        finally:
            os.remove(path)
        c += world


def trim_file_sharded(in_path, out_path, out_format='fastq', scoring_scheme_vals=(3, -6, -5, -2), end_size=150,
                      end_threshold=75.0, extra_end_trim=2, min_trim_size=4, middle_threshold=90.0,
                      extra_middle_trim_good_side=10, extra_middle_trim_bad_side=100, min_split_read_size=1000,
                      check_reads=10000, adapter_threshold=90.0, max_reads=100000, group=None, device=None,
                      trimmer_factory=None, barcode_dir=None, barcode_threshold=75.0, barcode_diff=5.0,
                      require_two_barcodes=False, untrimmed=False, discard_unassigned=False, inflate_dir=None,
                      spool_chunk_bytes=None):
    """The CLI's file-to-file path (porechop_abi.py:41-131: adapter-set search on the first
    check_reads records, end trim, middle scan, the fork's filter, trimmed output) on every rank of
    `group`, one GPU each:

      * adapter-set search: every rank reads the check records, aligns its shard of them and the
        per-sequence maxima are all-reduced once (find_matching_adapter_sets: the device buffer
        under RCCL);
      * trimming: a plain file is split into contiguous record ranges of about equal bytes (so
        bases), cut at record starts (misc.record_boundaries); each rank trims its range with a
        pipeline.FileTrimmer into its own part file, in order. A gzip file cannot be entered
        mid-stream, and an Albacore directory is many files: rank 0's distributor thread inflates
        the input once, in record-aligned spans handed round-robin to the ranks through spool files
        in inflate_dir (default: the output directory; it must be visible to every rank), at most
        SPOOL_DEPTH waiting per rank -- the ranks trim while it inflates (spool_distribute /
        spool_batches), recording the byte span of each batch they write;
      * output: rank 0 concatenates the parts in record order (the reference's output order) --
        the only other exchange is the span lists (spooled input), the job id and the read counts.

    With barcode_dir (-b) every rank writes its bins into a private directory, recording the
    byte span of each bin write, and rank 0 stitches every bin in record order; the barcoding
    kit direction comes from choose_barcoding_kit on the all-reduced set scores, as in the CLI.

    Returns the job's read counts (every rank). trimmer_factory(matching_sets, **options) builds
    the per-rank trimmer (FileTrimmer by default; the CPU tests pass an oracle-backed one)."""
    import io
    import os
    import shutil
    from . import misc
    dist = _dist()
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    # load_reads' check reads (porechop_abi.py:133-187): the first check_reads records of a file,
    # however many bases they hold; spread over the files of an Albacore directory
    check = misc.load_check_reads(in_path, check_reads) if check_reads > 0 else []
    dev = rank_device(device)
    # a fresh copy of the database: the search raises every set's best scores in place (the
    # reference's main() does that once per process; this function may run many times in one)
    matching = find_matching_adapter_sets(check, 0, end_size, scoring_scheme_vals, io.StringIO(), adapter_threshold, 1,
                                          adapter_sets=_adapters.fresh_adapters(), group=group, device=dev)
    matching = P.fix_up_1d2_sets(matching)
    fwd_rev = P.choose_barcoding_kit(matching, 0, io.StringIO()) if barcode_dir is not None else None
    matching = P.add_full_barcode_adapter_sets(matching)
    opts = dict(scoring_scheme_vals=scoring_scheme_vals, end_size=end_size, end_threshold=end_threshold,
                extra_end_trim=extra_end_trim, min_trim_size=min_trim_size, middle_threshold=middle_threshold,
                extra_middle_trim_good_side=extra_middle_trim_good_side,
                extra_middle_trim_bad_side=extra_middle_trim_bad_side, min_split_read_size=min_split_read_size)
    bdir = lambda r: os.path.join(barcode_dir, '.pcabi_rank%d' % r)
    if barcode_dir is not None:
        opts.update(barcode_dir=bdir(rank), forward_or_reverse_barcodes=fwd_rev, barcode_threshold=barcode_threshold,
                    barcode_diff=barcode_diff, require_two_barcodes=require_two_barcodes, untrimmed=untrimmed,
                    discard_unassigned=discard_unassigned)
    if trimmer_factory is None:
        from .pipeline import FileTrimmer
        trimmer_factory = FileTrimmer
        opts['device'] = dev
    ft = trimmer_factory(matching, **opts)
    d, base = os.path.split(os.path.abspath(out_path))
    part = lambda r: os.path.join(d, '.pcabi_part%d_%s' % (r, base))
    spooled = world > 1 and (os.path.isdir(in_path) or misc.get_compression_type(in_path) == 'gz')
    bounds = None if spooled else misc.record_boundaries(in_path, world)
    segments = None if (bounds is not None and barcode_dir is None) else []
    job = spool = distributor = None
    stop = None
    if spooled:
        import threading
        import uuid
        ids = [uuid.uuid4().hex if rank == 0 else None]
        dist.broadcast_object_list(ids, src=0, group=group)   # one spool namespace per job
        job, spool = ids[0], inflate_dir or d
        os.makedirs(spool, exist_ok=True)
        if rank == 0:
            stop = threading.Event()
            distributor = threading.Thread(target=spool_distribute, args=(in_path, spool, job, world),
                                           kwargs={'stop': stop, 'chunk_bytes': spool_chunk_bytes}, daemon=True)
            distributor.start()
    failed = False
    try:
        if spooled:
            counts = ft.trim_file(None, part(rank), out_format, max_reads, segments=segments,
                                  source=spool_batches(spool, job, rank, world, max_reads))
        elif bounds is not None:
            counts = ft.trim_file(in_path, part(rank), out_format, max_reads,
                                  byte_range=(bounds[rank], bounds[rank + 1]), segments=segments)
        else:
            counts = ft.trim_file(in_path, part(rank), out_format, max_reads, segments=segments)
    except BaseException as ex:
        failed = True
        if spooled:                           # the other ranks stop waiting for spans and raise too
            pre = _spool_prefix(spool, job)
            if not os.path.exists(pre + 'error'):
                with open(pre + 'error', 'w') as fo:
                    fo.write('rank %d: %s: %s' % (rank, type(ex).__name__, ex))
        raise
    finally:
        if hasattr(ft, 'close'):
            ft.close()
        if distributor is not None:
            stop.set()
            distributor.join()
        if failed and spooled:                # no hidden spool files left in the user's directory
            spool_fail_cleanup(spool, job, rank, world)
    if world > 1:
        spans = [None] * world
        dist.all_gather_object(spans, (segments, {k: v for k, v in counts.items() if k != 'bins'}), group=group)
    else:
        spans = [(segments, counts)]
    if rank == 0 and barcode_dir is not None:
        # every bin in record order: plain inputs by (rank, batch), gzip inputs by global batch
        order = sorted(((k, r) if bounds is None else (r, k), r, nm, a, e)
                       for r, (segs, _) in enumerate(spans) for k, nm, a, e in segs)
        outs = {}
        try:
            for _, r, nm, a, e in order:
                fmt_name = nm + '.' + out_format
                if fmt_name not in outs:
                    outs[fmt_name] = open(os.path.join(barcode_dir, fmt_name), 'wb')
                with open(os.path.join(bdir(r), fmt_name), 'rb') as f:
                    f.seek(a)
                    outs[fmt_name].write(f.read(e - a))
        finally:
            for f in outs.values():
                f.close()
        for r in range(world):
            shutil.rmtree(bdir(r), ignore_errors=True)
    elif rank == 0:
        with open(out_path, 'wb') as out:
            if bounds is not None:
                for r in range(world):
                    with open(part(r), 'rb') as f:
                        shutil.copyfileobj(f, out, 1 << 24)
            else:
                order = sorted((k, r, a, e) for r, (segs, _) in enumerate(spans) for k, a, e in segs)
                files = [open(part(r), 'rb') for r in range(world)]
                try:
                    for k, r, a, e in order:
                        files[r].seek(a)
                        out.write(files[r].read(e - a))
                finally:
                    for f in files:
                        f.close()
        for r in range(world):
            if os.path.exists(part(r)):
                os.remove(part(r))
    if world > 1:
        dist.barrier(group=group)
    if spooled and rank == 0:                 # markers (and anything a failed run left behind)
        pre = _spool_prefix(spool, job)
        sd, sb = os.path.split(pre)
        for f in os.listdir(sd):
            if f.startswith(sb):
                os.remove(os.path.join(sd, f))
    out = {k: sum(c[k] for _, c in spans) for k in ('reads_in', 'reads_kept')}
    out['reads_in_per_rank'] = [c['reads_in'] for _, c in spans]
    if barcode_dir is not None:
        out['bins'] = sorted(set(nm for segs, _ in spans for _, nm, _, _ in segs))
    return out

#!/usr/bin/env python3
"""Headline benchmark: reads/s trimmed, 100k synthetic ONT reads x 50 adapter sets (BASELINE.json).

One *step* = the end-trim hot path for one batch of reads, inputs resident in HBM:
    start windows (seq[:150]) -> tile layout    -> k_tile_windows
    start windows x start adapters              -> k_align (cross)  (nanopore_read.py:175-195)
    end windows (seq[-150:]) -> tile layout     -> k_tile_windows
    end windows x end adapters                  -> k_align (cross)  (nanopore_read.py:197-217)
    per-read trim decisions                     -> k_end_trim
for the first 50 non-"full sequence" adapter sets of the reference database
(porechop_abi/adapters.py:77-), scoring 3,-6,-5,-2, end_size 150, end_threshold 75,
extra_end_trim 2, min_trim_size 4 (reference defaults, arg_parser.py:178-208).

Multi-GPU: one process per GPU (torch.distributed.run); each rank trims its own 100k-read shard
(weak scaling, no data-path collective); the step time is the max over ranks (RCCL all-reduce
MAX of the rank times). value = reads all ranks trimmed / that time.

Also reported: roofline of the dominant kernel (k_align<24, true, TAGGED>: the 21-24 bp adapters,
~80% of the step; VALU-bound integer cell updates) from HIP events around its
launches, its HBM traffic from the committed rocprofv3 PMC pass (profiles/traffic.json), and the
reference SeqAn CPU path (oracle/_ref, compiled from the reference sources) timed on a bounded
sample on this host's cores.

At N = 1 the same line carries BASELINE.json's other configurations per GPU as sub-records
(run_other_configs): the production schedule, the host-buffer path, middle scan at 8 kb and 20 kb,
barcode demux, the configs[1] shape, file-to-file e2e, check_compatibility and approx_counter,
each with its own oracle spot check and CPU baseline (--sub 0 skips them, --only-subs picks).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12   # int32 lane-ops/s: 256 CU x 4 SIMD32 x 2.4 GHz
HBM_PEAK_GBS = 8000.0
OPS_PER_CELL = 10                               # algorithmic int ops per cell
SCORING = (3, -6, -5, -2)                       # reference default (arg_parser.py:178-180)
# the default scheme's 21-24 bp bucket runs the run-tagged layout (pcabi_dp.h pk::LayT, KIND 6)
DOM_KERNEL = 'k_align<24, true, 6> (run-tagged packed core, 21-24 bp adapters, affine)'


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--reads', type=int, default=100000, help='reads per GPU')
    ap.add_argument('--sets', type=int, default=50)
    ap.add_argument('--end-size', type=int, default=150)
    ap.add_argument('--mean-len', type=int, default=8000)
    ap.add_argument('--e2e-batch', type=int, default=12500,
                    help='e2e: reads per batch (the next batch is parsed while one is trimmed and written)')
    ap.add_argument('--cpu-sample', type=int, default=12000, help='reads in the CPU-baseline sample (0 = skip)')
    ap.add_argument('--cpu-threads', type=int, default=0, help='0 = min(16, cpus available)')
    ap.add_argument('--check', type=int, default=256, help='reads checked against the oracle after timing')
    ap.add_argument('--workload', choices=['endtrim', 'middle', 'barcodes', 'e2e', 'compat', 'kmer'],
                    default='endtrim',
                    help='endtrim: the headline metric (default); middle: end trim + middle-adapter scan '
                         '(BASELINE.json configs[2]); barcodes: end trim + barcode demultiplexing against '
                         '96 barcode sets (configs[3]); e2e: FASTQ file -> native parse -> end trim + middle '
                         'scan on the GPU -> fork filter -> native trimmed FASTQ output (the CLI path); compat: '
                         'the ab-initio all-vs-all check_compatibility matrix; kmer: the ab-initio k-mer counter '
                         '(approx_counter) on 40k sampled read ends')
    ap.add_argument('--compat-seqs', type=int, default=3000, help='sequences of the compat workload')
    ap.add_argument('--barcodes', type=int, default=96, help='barcode sets of the barcodes workload')
    ap.add_argument('--kit', choices=['pcr96', 'native12', 'rapid12'], default='pcr96',
                    help='barcodes workload: pcr96 = Barcode 1..96 (forward) sets; native12 = native '
                         'barcoding, Barcode 1..12 (reverse) + their 68/63 bp full-sequence adapters; rapid12 = '
                         'Rapid + RBK004, Barcode 1..12 (forward) + their 111 bp full rapid sequences')
    ap.add_argument('--middle-threshold', type=float, default=90.0)
    ap.add_argument('--middle-check', type=int, default=1000, help='middle: reads checked against the oracle loop')
    ap.add_argument('--e2e-check', type=int, default=150,
                    help='e2e: head reads whose written bytes are checked against the oracle-driven reference writer')
    ap.add_argument('--drivers-check', type=int, default=200,
                    help='drivers: reads whose decisions are compared with the same drivers over the oracle')
    ap.add_argument('--check-phase-check', type=int, default=400,
                    help='check_phase: check reads whose device reduction is compared with the oracle')
    ap.add_argument('--rj-check-overlap', type=int, default=1,
                    help='reference_job: 1 = the set search\'s two sides side by side (stream2; r04 A/B: 5.13 vs '
                         '5.23 ms per step); 0 = one after the other (each side\'s dominant launch then has the GPU '
                         'to itself, the roofline\'s events)')
    ap.add_argument('--rj-multi', type=int, default=1,
                    help='reference_job: 1 (default, r06) = the set search of both read ends in one '
                         'pcabi_align_cross_multi_dev call, and the kept-set end trim likewise (grouped launches); 0 = '
                         'per-side calls as --rj-check-overlap / --rj-end-streams say (r05)')
    ap.add_argument('--rj-end-streams', type=int, default=1,
                    help='reference_job: 1 = each kept adapter\'s end-trim cross product on a stream of its own '
                         '(r04x: 4.69-4.71 vs 4.78-4.84 ms per step); 0 = each side\'s table on one stream')
    ap.add_argument('--rj-side-streams', type=int, default=0,
                    help='reference_job: the library\'s side streams (pcabi_stream_side_streams on its streams) during the job; 0 '
                         '(default: it runs two caller streams at once) or 1')
    ap.add_argument('--head-side-streams', type=int, default=0,
                    help='headline schedule: the library\'s side streams while both sides\' smaller buckets run on two '
                         'caller streams at once; 0 (default, r04r: 7.61 vs 7.68 ms) or 1')
    ap.add_argument('--rest-overlap', type=int, default=5,
                    help='headline schedule: 5 (default, r06) = both read ends in ONE pcabi_align_cross_multi_dev call '
                         '(every run-tagged bucket of both sides in one grouped launch, the packed ones in another '
                         'beside it); 4 = each side\'s dominant launch alone, then both sides\' smaller buckets in one '
                         'multi call; 3 = after both dominant launches, both sides\' smaller buckets dealt onto the two '
                         'caller streams by cost; 2 = each on its own stream; 1 = the two sides\' calls side by side '
                         '(r05); 0 = after each side\'s dominant launch')
    ap.add_argument('--group-side', type=int, default=1,
                    help='headline schedule 5: the multi call\'s grouped launches side by side on the library\'s side '
                         'streams (1, default) or one after the other on the caller\'s stream (0: the dominant launch '
                         'then has the GPU to itself)')
    ap.add_argument('--overlap-steps', type=int, default=1,
                    help='headline schedule 5: 1 (default, r06) = consecutive steps overlap their memory-bound '
                         'prologue and epilogue with the align phase: step k+1\'s tile transposes and step k\'s end '
                         'trim run on a second stream (double-buffered tiles and results) while the main stream '
                         'aligns; every step still does all of its own work. 0 = one step after the other')
    ap.add_argument('--hw-queues', type=int, default=0,
                    help='GPU_MAX_HW_QUEUES for this process when the environment does not set it (0: HIP default, '
                         '4; r04 A/B with 8: headline 8.05 vs 7.61 ms, reference job 5.85 vs 5.23 ms)')
    ap.add_argument('--only-subs', default='', help='comma-separated sub-record names to run (default: all)')
    ap.add_argument('--ab', default='',
                    help='middle workloads: NAME=v0,v1 alternates an environment switch of the library between '
                         'timed steps and reports the middle scan time per value (A/B within one process)')
    ap.add_argument('--sub', type=int, default=1,
                    help='endtrim at N=1: also time the middle workload (configs[2]) and the host-buffer path '
                         '(H2D + kernels + D2H) as sub-records of the same JSON line')
    ap.add_argument('--dist-backend', default='nccl', help='nccl (RCCL over xGMI, default) or gloo (rehearsal of '
                                                           'several ranks sharing one GPU)')
    return ap.parse_args()


def main():
    args = parse()
    print('GPU_MAX_HW_QUEUES in the environment: %s' % os.environ.get('GPU_MAX_HW_QUEUES', 'unset'), file=sys.stderr)
    if args.hw_queues > 0 and 'GPU_MAX_HW_QUEUES' not in os.environ:
        # hardware queues per process (HIP's default 4): the headline's smaller buckets run on one
        # stream each (--rest-overlap 2), and streams beyond the queue count share queues
        os.environ['GPU_MAX_HW_QUEUES'] = str(min(args.hw_queues, 32))
    rank = int(os.environ.get('RANK', '0'))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    import torch  # single HIP runtime for torch (RCCL) and libpcabi (see _lib.py)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == 'nccl':
            torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend)
        if args.dist_backend != 'nccl':
            local = local % max(1, torch.cuda.device_count())
    from custom_porechop_abi_amd import _lib, adapters as A, synth
    from custom_porechop_abi_amd.engine import encode_adapters
    L = _lib.lib()
    _lib.check(L.pcabi_dev_set(local), 'pcabi_dev_set')
    args.local_device = local
    ctx = (rank, world, dist, torch, L, _lib, A, synth, encode_adapters)
    if args.workload == 'middle':
        out = run_middle(args, *ctx)
    elif args.workload == 'compat':
        out = run_compat(args, rank, world, dist, torch, L, _lib)
    elif args.workload == 'kmer':
        out = run_kmer(args, rank, world, dist, torch, L, _lib, synth)
    elif args.workload == 'e2e':
        out = run_e2e(args, *ctx)
    else:
        out = run_endtrim(args, *ctx)
        if world > 1 and args.workload == 'endtrim' and args.sub:
            # the path's one collective (the adapter-set search's MAX all-reduce), timed at every N
            # with every rank taking part; at N = 1 it is one of run_other_configs' sub-records
            cp = run_check_phase(args, *ctx)
            if out is not None:
                for k in ('n_gpus', 'higher_is_better', 'scaling', 'vs_baseline'):
                    cp.pop(k, None)
                out['check_phase'] = cp
        if out is not None and world == 1 and args.sub and args.workload == 'endtrim':
            out.update(run_other_configs(args, ctx))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def run_endtrim(args, rank, world, dist, torch, L, _lib, A, synth, encode_adapters):
    """The headline (BASELINE.json metric): end trim of 100k reads/GPU x 50 adapter sets, or the
    barcode demux workload (configs[3] shape per GPU) with --workload barcodes."""
    local = args.local_device
    # ---- workload (host) ----
    barcodes = args.workload == 'barcodes'
    kit_n = 2 if args.kit == 'rapid12' else 1      # kit adapter sets ahead of the barcode sets
    if barcodes:
        # BASELINE.json configs[3]: demultiplexing against 96 barcode sets ('Barcode k (forward)',
        # porechop_abi/adapters.py) plus the ligation kit adapters, forward orientation
        allsets = A.fresh_adapters()
        if args.kit == 'native12':
            # porechop_abi.py:332-356 adds the full native sequences for every found barcode
            nb = min(args.barcodes, 12)
            sets = [a for a in allsets if a.name == 'SQK-NSK007'] + \
                [a for a in allsets if a.name.startswith('Barcode ') and a.name.endswith('(reverse)')][:nb] + \
                [A.make_full_native_barcode_adapter(i) for i in range(1, nb + 1)]
            bc_dir = 'reverse'
        elif args.kit == 'rapid12':
            # porechop_abi.py:348-354: Rapid + RBK004 found -> the new full rapid sequences (111 bp)
            nb = min(args.barcodes, 12)
            sets = [a for a in allsets if a.name in ('Rapid', 'RBK004_upstream')] + \
                [a for a in allsets if a.name.startswith('Barcode ') and a.name.endswith('(forward)')][:nb] + \
                [A.make_new_full_rapid_barcode_adapter(i) for i in range(1, nb + 1)]
            bc_dir = 'forward'
        else:
            sets = [a for a in allsets if a.name == 'SQK-NSK007'] + \
                [a for a in allsets if a.name.startswith('Barcode ') and a.name.endswith('(forward)')][:args.barcodes]
            bc_dir = 'forward'
    else:
        sets = [a for a in A.fresh_adapters() if '(full sequence)' not in a.name][:args.sets]
    # adapters of the dominant register bucket (21..24 bp -> k_align<24, *, PACKED>, the table's
    # largest bucket, timed by pcabi_align_cross_dev_marked's events) first; the trim decision is
    # a max over adapters and does not depend on their order (the barcode dict order is kept
    # through bc slots)
    dom = lambda x: 20 < len(x) <= 24
    start_sets = [a for a in sets if a.start_sequence]
    end_sets = [a for a in sets if a.end_sequence]
    # the other adapters grouped by register bucket (rows = length rounded up to 4), so each bucket is
    # one contiguous table (the headline's per-bucket streams)
    rank_of = lambda x: (not dom(x), 0 if dom(x) else (len(x) + 3) // 4)
    order_s = sorted(range(len(start_sets)), key=lambda k: rank_of(start_sets[k].start_sequence[1]))
    order_e = sorted(range(len(end_sets)), key=lambda k: rank_of(end_sets[k].end_sequence[1]))
    start_adps = [start_sets[k].start_sequence[1] for k in order_s]
    end_adps = [end_sets[k].end_sequence[1] for k in order_e]
    pos_s, pos_e = np.argsort(order_s).astype(np.int32), np.argsort(order_e).astype(np.int32)
    t0 = time.time()
    truth = None
    if barcodes:
        carried = [a for a in sets[kit_n:] if '(full sequence)' in a.name] or sets[kit_n:]
        reads, truth = synth.make_barcoded_reads(args.reads, [(a.start_sequence[1], a.end_sequence[1] if a.end_sequence
                                                               else '') for a in carried],
                                                 args.mean_len, seed=12345 + rank, keep=args.end_size)
    else:
        reads = synth.make_reads(args.reads, args.mean_len, seed=12345 + rank, keep=args.end_size)
    buf, s_off, s_len, e_off, e_len = synth.pack_end_windows(reads, args.end_size)
    gen_s = time.time() - t0
    n = args.reads

    # ---- device-resident inputs ----
    vp = ctypes.c_void_p

    def dalloc(nbytes):
        p = vp()
        _lib.check(L.pcabi_dev_malloc(ctypes.byref(p), max(int(nbytes), 16)), 'malloc')
        return p

    def h2d(arr):
        arr = np.ascontiguousarray(arr)
        p = dalloc(arr.nbytes)
        _lib.check(L.pcabi_dev_h2d(p, arr.ctypes.data_as(vp), arr.nbytes), 'h2d')
        return p

    def table(lst):
        t = vp()
        if lst:
            c, o, l = encode_adapters(lst)
            _lib.check(L.pcabi_adapters_create_scored(c.ctypes.data_as(vp), o.ctypes.data_as(vp),
                                                      l.ctypes.data_as(vp), len(lst), *SCORING, ctypes.byref(t)),
                       'adapters_create')
        return t, len(lst)

    d_codes = h2d(buf)
    d_soff, d_slen, d_eoff, d_elen = h2d(s_off), h2d(s_len), h2d(e_off), h2d(e_len)
    n_sa, n_ea = len(start_adps), len(end_adps)
    s_stride, e_stride = n_sa * n, n_ea * n
    d_sres = dalloc(4 * 8 * s_stride)
    d_eres = dalloc(4 * 8 * e_stride)
    d_st, d_et = dalloc(4 * n), dalloc(4 * n)
    stream = vp()
    _lib.check(L.pcabi_stream_create(ctypes.byref(stream)), 'stream')
    sc = SCORING

    # tile layout: computed once from the host window lengths; the device
    # re-tiles the windows inside every step
    sides = []
    for lens, d_off, d_len, adps, d_res, stride in ((s_len, d_soff, d_slen, start_adps, d_sres, s_stride),
                                                    (e_len, d_eoff, d_elen, end_adps, d_eres, e_stride)):
        toff = np.zeros((n + 255) // 256 + 1, np.int64)
        nd = L.pcabi_tile_layout(lens.ctypes.data_as(vp), n, toff.ctypes.data_as(vp))
        if nd < 0:
            raise _lib.PcabiError('tile layout failed')
        n_dom = sum(1 for x in adps if dom(x))
        groups, group_first = [], []                # (table, result rows) per register bucket of the rest
        k0 = n_dom
        while k0 < len(adps):
            k1 = k0
            while k1 < len(adps) and (len(adps[k1]) + 3) // 4 == (len(adps[k0]) + 3) // 4:
                k1 += 1
            groups.append((table(adps[k0:k1]), vp(d_res.value + 4 * k0 * n)))
            group_first.append(k0)
            k0 = k1
        sides.append(dict(lens=lens, d_off=d_off, d_len=d_len, d_toff=h2d(toff), d_tiles=dalloc(4 * nd),
                          mq=int(np.diff(toff).max() // 256), dom=table(adps[:n_dom]), rest=table(adps[n_dom:]),
                          all=table(adps), d_res=d_res, d_res_rest=vp(d_res.value + 4 * n_dom * n), stride=stride,
                          groups=groups, group_first=group_first, adps=adps))

    ev = []
    for _ in range(4 * args.steps + 4):
        e = vp()
        _lib.check(L.pcabi_event_create(ctypes.byref(e)), 'event')
        ev.append(e)

    # the headline schedule's second caller stream: the two sides' smaller buckets run side by side
    # after both dominant launches (each side's own call on its stream; the library's side streams are
    # off while the two streams run: see two_streams below)
    stream2 = vp()
    _lib.check(L.pcabi_stream_create(ctypes.byref(stream2)), 'stream')
    ev_fork, ev_join = vp(), vp()
    _lib.check(L.pcabi_event_create(ctypes.byref(ev_fork)), 'event')
    _lib.check(L.pcabi_event_create(ctypes.byref(ev_join)), 'event')

    # --rest-overlap 4: both sides' smaller buckets in ONE pcabi_align_cross_multi_dev call (grouped
    # launches per core family); 5: both sides' whole tables in one call (the dominant buckets grouped
    # with the other run-tagged ones: one launch for both read ends, its events the roofline's)
    def regions(key, res_key):
        return _lib.cross_regions([(sd['d_tiles'], sd['d_toff'], sd['d_len'], n, int(sd['lens'].max()), sd[key][0],
                                    sd[res_key], sd['stride']) for sd in sides if sd[key][1]])
    rest_regions = regions('rest', 'd_res_rest') if args.rest_overlap == 4 else None
    all_regions = regions('all', 'd_res') if args.rest_overlap == 5 else None

    n_groups = sum(len(sd['groups']) for sd in sides) if args.rest_overlap == 2 else 0
    g_streams, g_join = [], []
    for _ in range(n_groups):
        gs, ge = vp(), vp()
        _lib.check(L.pcabi_stream_create(ctypes.byref(gs)), 'stream')
        _lib.check(L.pcabi_event_create(ctypes.byref(ge)), 'event')
        g_streams.append(gs)
        g_join.append(ge)

    def align_groups():
        # every smaller bucket of both sides on its own stream, after both dominant launches
        L.pcabi_event_record(ev_fork, stream)
        j = 0
        for sd in sides:
            mx = int(sd['lens'].max())
            for (tab, cnt), d_res in sd['groups']:
                gs = g_streams[j]
                L.pcabi_stream_wait_event(gs, ev_fork)
                _lib.check(L.pcabi_align_cross_dev(sd['d_tiles'], sd['d_toff'], sd['d_len'], n, mx, tab, *sc, d_res,
                                                   sd['stride'], gs), 'align')
                L.pcabi_event_record(g_join[j], gs)
                j += 1
        for e in g_join:
            L.pcabi_stream_wait_event(stream, e)

    # --rest-overlap 3: both sides' smaller buckets dealt onto the two caller streams, largest first
    # onto the less loaded one (cost = adapters x rows), so neither stream ends long after the other
    balanced = [[], []]
    if args.rest_overlap == 3:
        jobs = []
        for i, sd in enumerate(sides):
            for ((tab, cnt), d_res), k0 in zip(sd['groups'], sd['group_first']):
                jobs.append((cnt * ((len(sd['adps'][k0]) + 3) // 4 * 4), i, tab, d_res))
        jobs.sort(key=lambda x: -x[0])
        load = [0, 0]
        for cost, i, tab, d_res in jobs:
            j = 0 if load[0] <= load[1] else 1
            load[j] += cost
            balanced[j].append((i, tab, d_res))

    def align_balanced():
        L.pcabi_event_record(ev_fork, stream)
        L.pcabi_stream_wait_event(stream2, ev_fork)
        for st, lst in ((stream, balanced[0]), (stream2, balanced[1])):
            for i, tab, d_res in lst:
                sd = sides[i]
                _lib.check(L.pcabi_align_cross_dev(sd['d_tiles'], sd['d_toff'], sd['d_len'], n, int(sd['lens'].max()),
                                                   tab, *sc, d_res, sd['stride'], st), 'align')
        L.pcabi_event_record(ev_join, stream2)
        L.pcabi_stream_wait_event(stream, ev_join)

    def align_rest(sd, st):
        tab, cnt = sd['rest']
        if cnt:
            _lib.check(L.pcabi_align_cross_dev(sd['d_tiles'], sd['d_toff'], sd['d_len'], n, int(sd['lens'].max()), tab,
                                               *sc, sd['d_res_rest'], sd['stride'], st), 'align')

    def align_side(sd, e0=None, e1=None, fused=False, rest=True):
        _lib.check(L.pcabi_tile_windows_dev(d_codes, sd['d_off'], sd['d_len'], n, sd['d_toff'], sd['mq'],
                                            sd['d_tiles'], stream), 'tile')
        mx = int(sd['lens'].max())
        if fused:
            # the production schedule (the drivers' one cross product per side): the dominant
            # bucket on `stream`, the other buckets beside it on the side streams
            tab, cnt = sd['all']
            if cnt:
                _lib.check(L.pcabi_align_cross_dev_marked(sd['d_tiles'], sd['d_toff'], sd['d_len'], n, mx, tab, *sc,
                                                          sd['d_res'], sd['stride'], stream, e0, e1), 'align')
            return
        # headline schedule: the dominant bucket's launch alone on the GPU (so e0 / e1 time the
        # kernel itself, the roofline), then the other buckets side by side
        for key, d_res in (('dom', sd['d_res']), ('rest', sd['d_res_rest'])):
            tab, cnt = sd[key]
            if not cnt or (key == 'rest' and not rest):
                continue
            if key == 'dom' and e0 is not None:
                L.pcabi_event_record(e0, stream)
            _lib.check(L.pcabi_align_cross_dev(sd['d_tiles'], sd['d_toff'], sd['d_len'], n, mx, tab, *sc, d_res,
                                               sd['stride'], stream), 'align')
            if key == 'dom' and e1 is not None:
                L.pcabi_event_record(e1, stream)

    bc = None
    if barcodes:
        from custom_porechop_abi_amd.porechop_abi import barcode_slots
        ids = {}
        sa_, sn_ = barcode_slots(start_sets, bc_dir, ids)
        ea_, en_ = barcode_slots(end_sets, bc_dir, ids)
        bc = dict(s_adp=h2d(pos_s[sa_]), s_name=h2d(sn_), ns=len(sa_), e_adp=h2d(pos_e[ea_]), e_name=h2d(en_),
                  ne=len(ea_), d_call=dalloc(4 * n), names={v: k for k, v in ids.items()}, dir=bc_dir)

    def epilogue():
        _lib.check(L.pcabi_end_trim_dev(d_sres, s_stride, n_sa, d_eres, e_stride, n_ea, n, args.end_size,
                                        2, 75.0, 4, d_st, d_et, None, None, stream), 'end_trim')
        if bc is not None:
            # determine_barcode, reference defaults: barcode_threshold 75, barcode_diff 5
            _lib.check(L.pcabi_barcode_call_dev(d_sres, s_stride, bc['s_adp'], bc['s_name'], bc['ns'], d_eres,
                                                e_stride, bc['e_adp'], bc['e_name'], bc['ne'], n, 75.0, 5.0, 0,
                                                bc['d_call'], None, stream), 'barcode_call')

    # The headline configuration times its dominant launch alone (the roofline is that kernel's
    # own); every other configuration runs the production schedule (one cross product per side,
    # the events around its largest bucket, which then shares the GPU with the small buckets).
    headline = not barcodes and n == 100000 and len(sets) == 50 and args.end_size == 150
    timed_fused = not headline

    # --overlap-steps (schedule 5, headline): two buffer sets (tiles and results) so that step k+1's
    # tile transposes and step k's end trim run on `aux` while `stream` runs the align phase. Events:
    # tile_done[s] (set s's tiles written), align_done[s] (its align read them and wrote its results),
    # trim_done[s] (its end trim read the results).
    pipelined = args.overlap_steps and args.rest_overlap == 5 and headline
    pipe = None
    if pipelined:
        for sd in sides:
            sd['d_tiles2'] = dalloc(4 * int(L.pcabi_tile_layout(sd['lens'].ctypes.data_as(vp), n,
                                                                   np.zeros((n + 255) // 256 + 1, np.int64).ctypes.data_as(vp))))
            sd['d_res2'] = dalloc(4 * 8 * sd['stride'])
        pipe = dict(set=0, ahead=False, aux=vp(), regions=[all_regions, _lib.cross_regions(
            [(sd['d_tiles2'], sd['d_toff'], sd['d_len'], n, int(sd['lens'].max()), sd['all'][0], sd['d_res2'],
              sd['stride']) for sd in sides if sd['all'][1]])],
                    res=[(d_sres, d_eres), (sides[0]['d_res2'], sides[1]['d_res2'])],
                    tiles=[[sd['d_tiles'] for sd in sides], [sd['d_tiles2'] for sd in sides]],
                    ev={k: [vp(), vp()] for k in ('tile', 'align', 'trim')}, used={k: [False, False] for k in ('tile', 'align', 'trim')})
        _lib.check(L.pcabi_stream_create(ctypes.byref(pipe['aux'])), 'stream')
        for k in pipe['ev']:
            for e_ in pipe['ev'][k]:
                _lib.check(L.pcabi_event_create(ctypes.byref(e_)), 'event')

    def pipe_record(kind, s_, st):
        L.pcabi_event_record(pipe['ev'][kind][s_], st)
        pipe['used'][kind][s_] = True

    def pipe_wait(st, kind, s_):
        if pipe['used'][kind][s_]:
            L.pcabi_stream_wait_event(st, pipe['ev'][kind][s_])

    def pipe_tiles(s_):
        # set s_'s tiles on aux, once the align that last read them is done
        pipe_wait(pipe['aux'], 'align', s_)
        for sd, d_t in zip(sides, pipe['tiles'][s_]):
            _lib.check(L.pcabi_tile_windows_dev(d_codes, sd['d_off'], sd['d_len'], n, sd['d_toff'], sd['mq'], d_t,
                                                pipe['aux']), 'tile')
        pipe_record('tile', s_, pipe['aux'])

    def step_pipelined(e, last):
        s_ = pipe['set']
        if not pipe['ahead']:
            pipe_tiles(s_)
        pipe_wait(stream, 'tile', s_)
        pipe_wait(stream, 'trim', s_)                # set s_'s results: read by the end trim two steps ago
        if e[2] is not None:
            L.pcabi_event_record(e[2], stream)
        _lib.check(L.pcabi_align_cross_multi_dev(pipe['regions'][s_], len(pipe['regions'][s_]), *sc, stream, e[0], e[1]),
                   'align')
        if e[3] is not None:
            L.pcabi_event_record(e[3], stream)
        pipe_record('align', s_, stream)
        # the next step's tiles beside this align, then this step's end trim after it
        pipe['ahead'] = not last
        if not last:
            pipe_tiles(1 - s_)
        pipe_wait(pipe['aux'], 'align', s_)
        sres, eres = pipe['res'][s_]
        _lib.check(L.pcabi_end_trim_dev(sres, s_stride, n_sa, eres, e_stride, n_ea, n, args.end_size,
                                        2, 75.0, 4, d_st, d_et, None, None, pipe['aux']), 'end_trim')
        pipe_record('trim', s_, pipe['aux'])
        pipe['set'] = 1 - s_

    def pipe_sync():
        if pipe is not None:
            L.pcabi_stream_sync(pipe['aux'])
            L.pcabi_stream_sync(stream)

    def step(k=None, fused=False, last=True):
        if pipe is not None and not fused and (k is not None or not timed_fused):
            step_pipelined((None,) * 4 if k is None else tuple(ev[4 * k + i] for i in range(4)), last)
            return
        fused = fused if k is None else timed_fused
        e = (None,) * 4 if k is None else tuple(ev[4 * k + i] for i in range(4))
        if not fused and args.rest_overlap == 5:
            for sd in sides:
                _lib.check(L.pcabi_tile_windows_dev(d_codes, sd['d_off'], sd['d_len'], n, sd['d_toff'], sd['mq'],
                                                    sd['d_tiles'], stream), 'tile')
            # e0 / e1: the grouped run-tagged launch (the roofline's kernel); e2 / e3: the whole call
            if e[2] is not None:
                L.pcabi_event_record(e[2], stream)
            _lib.check(L.pcabi_align_cross_multi_dev(all_regions, len(all_regions), *sc, stream, e[0], e[1]), 'align')
            if e[3] is not None:
                L.pcabi_event_record(e[3], stream)
            epilogue()
            return
        if fused or not args.rest_overlap:
            align_side(sides[0], e[0], e[1], fused=fused)
            align_side(sides[1], e[2], e[3], fused=fused)
        else:
            # headline schedule: each side's dominant launch alone (its events are the kernel's own
            # time), then both sides' smaller buckets together -- the start side's on `stream`, the
            # end side's on stream2 -- so the latency-bound single-adapter buckets (50 bp, 1.6 k
            # waves) overlap the other side's instead of leaving the GPU idle behind them
            align_side(sides[0], e[0], e[1], rest=False)
            align_side(sides[1], e[2], e[3], rest=False)
            if args.rest_overlap == 2:
                align_groups()
                epilogue()
                return
            if args.rest_overlap == 3:
                align_balanced()
                epilogue()
                return
            if args.rest_overlap == 4:
                _lib.check(L.pcabi_align_cross_multi_dev(rest_regions, len(rest_regions), *sc, stream, None, None),
                           'align')
                epilogue()
                return
            L.pcabi_event_record(ev_fork, stream)
            L.pcabi_stream_wait_event(stream2, ev_fork)
            align_rest(sides[0], stream)
            align_rest(sides[1], stream2)
            L.pcabi_event_record(ev_join, stream2)
            L.pcabi_stream_wait_event(stream, ev_join)
        epilogue()

    # the headline schedule runs both sides' smaller buckets on two caller streams at once: the
    # library's side streams go off on its two streams (pcabi_stream_side_streams; one cross product at a time,
    # as the production schedule, keeps them on)
    two_streams = not timed_fused and args.rest_overlap in (1, 3)
    if not timed_fused and args.rest_overlap in (4, 5):
        # one (grouped) call at a time: its launches side by side (or, --group-side 0, one after the other)
        L.pcabi_stream_side_streams(stream, 1 if args.rest_overlap == 4 or args.group_side else 0)
    # (per stream, r05: pcabi_stream_side_streams leaves every other caller of the library alone)
    if two_streams:
        for s_ in (stream, stream2):
            L.pcabi_stream_side_streams(s_, args.head_side_streams)
    for w_ in range(args.warmup):
        step(fused=timed_fused, last=w_ == args.warmup - 1)
    _lib.check(L.pcabi_stream_sync(stream), 'sync')
    pipe_sync()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize() if torch.cuda.is_available() else None
        L.pcabi_stream_sync(stream)

    barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k, last=k == args.steps - 1)
    L.pcabi_stream_sync(stream)
    pipe_sync()
    barrier()
    elapsed = time.perf_counter() - t0
    side_timed = args.head_side_streams if two_streams else L.pcabi_set_side_streams(-1)
    for s_ in (stream, stream2):
        L.pcabi_stream_side_streams(s_, -1)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device='cuda' if args.dist_backend == 'nccl' else 'cpu')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # dominant kernel: average launch duration, start and end launches separately
    dom_ms = [[], []]
    for k in range(args.steps):
        for side in (0, 1):
            ms = ctypes.c_float()
            _lib.check(L.pcabi_event_elapsed_ms(ctypes.byref(ms), ev[4 * k + 2 * side], ev[4 * k + 2 * side + 1]),
                       'elapsed')
            dom_ms[side].append(ms.value)
    phase_ms = None
    if args.rest_overlap == 5 and not timed_fused:
        phase_ms = float(np.mean(dom_ms[1]))      # the whole multi call (both grouped launches)
        dom_ms = [dom_ms[0], dom_ms[0]]           # one grouped launch for both sides
    dom_ms = [float(np.mean(x)) for x in dom_ms]

    # ---- algorithmic work (per GPU) ----
    s_len64, e_len64 = s_len.astype(np.int64), e_len.astype(np.int64)
    La = np.array([len(x) for x in start_adps], np.int64)
    Le = np.array([len(x) for x in end_adps], np.int64)
    cells = int(s_len64.sum() * La.sum() + e_len64.sum() * Le.sum())
    # dominant kernel, per launch (start launch and end launch averaged)
    dom_cells = [int(s_len64.sum() * La[[dom(x) for x in start_adps]].sum()),
                 int(e_len64.sum() * Le[[dom(x) for x in end_adps]].sum())]
    dom_bytes = [int(s_len64.sum() + La[[dom(x) for x in start_adps]].sum() + 32 * n * sum(map(dom, start_adps))),
                 int(e_len64.sum() + Le[[dom(x) for x in end_adps]].sum() + 32 * n * sum(map(dom, end_adps)))]
    launch_ms = float(np.mean(dom_ms))
    launch_cells = float(np.mean(dom_cells))
    launch_bytes = float(np.mean(dom_bytes))
    dom_kernel = DOM_KERNEL
    phase = None
    if args.rest_overlap == 5 and not timed_fused:
        # the grouped run-tagged launch: every <= 32-row bucket of both sides
        grp = lambda x: (len(x) + 3) // 4 * 4 <= 32
        launch_cells = float(s_len64.sum() * La[[grp(x) for x in start_adps]].sum() +
                             e_len64.sum() * Le[[grp(x) for x in end_adps]].sum())
        launch_bytes = float(s_len64.sum() + e_len64.sum() + 32 * n * (sum(map(grp, start_adps)) + sum(map(grp, end_adps))))
        launch_ms = dom_ms[0]
        dom_kernel = 'k_align_group<0> (run-tagged core, every <= 32-row bucket of both read ends in one launch)'
        # the align phase as a whole: both grouped launches (k_align_group<1>, the 36-52-row packed
        # buckets, runs beside <0> and inside its span), every cell of the step over the call's time
        phase = {'ms': round(phase_ms, 4), 'cells': cells,
                 'achieved': round(cells * OPS_PER_CELL / (phase_ms * 1e-3) / 1e12, 3),
                 'frac': round(cells * OPS_PER_CELL / (phase_ms * 1e-3) / 1e12 / VALU_PEAK_TOPS, 4),
                 'what': 'pcabi_align_cross_multi_dev over both read ends: k_align_group<0> and <1> (events around '
                         'the call)'}
    tops = launch_cells * OPS_PER_CELL / (launch_ms * 1e-3) / 1e12
    gbs = launch_bytes / (launch_ms * 1e-3) / 1e9
    step_ms = 1e3 * elapsed / args.steps

    # ---- correctness spot-check (outside the timed region) ----
    checked = None
    if args.check and rank == 0:
        checked = spot_check(L, _lib, d_sres, d_eres, d_st, d_et, s_stride, e_stride, n, n_sa, n_ea, reads,
                             start_adps, end_adps, args.end_size, min(args.check, n), sc, bc=bc,
                             bc_sets=(start_sets, end_sets, pos_s, pos_e))

    if checked is not None and bc is not None:
        # demultiplexing sanity: calls vs the barcode each synthetic read was built with
        call = np.empty(n, np.int32)
        _lib.check(L.pcabi_dev_d2h(call.ctypes.data_as(vp), bc['d_call'], call.nbytes), 'd2h')
        ids = {v: k for k, v in bc['names'].items()}
        want = np.array([ids.get(sets[kit_n + t].get_barcode_name(), -2) if t >= 0 else -1 for t in truth.tolist()])
        checked['calls_equal_synthetic_truth'] = round(float(np.mean(call == want)), 4)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        # bounded sample: ~1.2M reference alignments (~10 s on 16 host threads)
        k_cpu = max(1, min(args.cpu_sample, args.cpu_sample * 98 // max(1, n_sa + n_ea)))
        cpu = cpu_baseline(reads[:k_cpu], sets, args.end_size, sc, args.cpu_threads)

    subs = {}
    if rank == 0 and world == 1 and args.sub and not barcodes:
        # the same step in the production schedule: one cross product per side, the small buckets
        # overlapping the dominant launch (faster as a whole; the dominant launch then shares the
        # GPU, so the headline keeps it alone for the roofline)
        L.pcabi_stream_side_streams(stream, 1)     # one cross product at a time: side by side pays
        for _ in range(2):
            step(fused=True)
        L.pcabi_stream_sync(stream)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(fused=True)
        L.pcabi_stream_sync(stream)
        dt = (time.perf_counter() - t0) / args.steps
        L.pcabi_stream_side_streams(stream, -1)
        subs['per_side_schedule'] = {'value': round(n / dt, 1), 'unit': 'reads/s', 'ms_per_step': round(1e3 * dt, 4),
                                     'steps': args.steps, 'what': 'the headline step with one cross product per side '
                                     '(pcabi_align_cross_dev_marked, the r05 production schedule): register buckets side '
                                     'by side with the dominant one (side streams on); r06 production (the library\'s '
                                     'end decisions, pipeline.FileTrimmer) is the headline\'s multi call'}
        subs['host_path'] = run_host_path(args, L, _lib, buf, s_off, s_len, e_off, e_len, sides, d_sres, d_eres, d_st,
                                          d_et, n, n_sa, n_ea, stream, start_adps, end_adps)

    # the headline's extra streams go before the other configurations run (idle streams still take
    # hardware queues from the ones the library creates later)
    for st_ in [stream2] + g_streams + ([pipe['aux']] if pipe is not None else []):
        L.pcabi_stream_destroy(st_)

    if rank == 0:
        value = world * n * args.steps / elapsed
        prof = load_traffic()   # the PMC traffic record: the headline configuration's dominant launch
        if prof and not dom_kernel.startswith(str(prof.get('kernel'))):
            prof = None         # recorded for another layout of the dominant bucket
        out = {
            'metric': ('reads/sec trimmed + demultiplexed (ONT reads x %d barcode sets)' % (len(sets) - kit_n)
                       if barcodes and args.kit == 'pcr96' else
                       'reads/sec trimmed + demultiplexed (%s barcoding, %d barcodes + full sequences)'
                       % ('native' if args.kit == 'native12' else 'rapid', nb)
                       if barcodes
                       else 'reads/sec trimmed (100k ONT reads x 50 adapter pairs)' if n == 100000 and len(sets) == 50
                       else 'reads/sec trimmed (%d ONT reads x %d adapter sets)' % (n, len(sets))),
            'value': round(value, 1),
            'unit': 'reads/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(step_ms, 4),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'int32',
            'data': 'synthetic (seeded ONT-like reads, SURVEY.md §8d recipe; mean %d bp)' % args.mean_len,
            'config': {'workload': ('barcode demux (%s): %d reads/GPU x %d barcode sets + SQK-NSK007 (%d start + %d end '
                                    'adapters), start+end windows of %d bp, + per-read trim decisions and barcode '
                                    'calls (determine_barcode, threshold 75, diff 5)'
                                    % (args.kit, n, len(sets) - kit_n, n_sa, n_ea, args.end_size)) if barcodes else
                                   ('end-trim: %d reads/GPU x %d adapter sets (%d start + %d end adapters), '
                                    'start+end windows of %d bp, + per-read trim decisions'
                                    % (n, len(sets), n_sa, n_ea, args.end_size)),
                       'reads_per_gpu': n, 'adapter_sets': len(sets), 'end_size': args.end_size,
                       'scoring': list(sc), 'parallelism': 'dp%d (read shards)' % world,
                       'hw_queues': os.environ.get('GPU_MAX_HW_QUEUES', 'HIP default'),
                       'side_streams': side_timed,
                       'steps_overlap': ('each step\'s tile transposes and end trim on a second stream beside the '
                                         'neighbouring steps\' align phase (double-buffered tiles and results)'
                                         if pipe is not None else None)},
            'roofline': {'bound': 'valu', 'achieved': round(tops, 3), 'peak': round(VALU_PEAK_TOPS, 1),
                         'unit': 'Tops/s (int32 lane-ops)', 'frac': round(tops / VALU_PEAK_TOPS, 4),
                         'traffic': prof.get('traffic_bytes_per_launch') if prof and headline else None,
                         'kernel': dom_kernel,
                         'launch_ms': round(launch_ms, 4), 'cells_per_launch': int(launch_cells),
                         'schedule': ('production: one cross product per side, the dominant launch shares the GPU '
                                      'with the small buckets' if timed_fused else
                                      'both read ends in one multi call: the grouped run-tagged launch, the grouped '
                                      'packed launch beside it' if args.rest_overlap == 5 else 'dominant launch alone'),
                         'ops_per_cell': OPS_PER_CELL,
                         'traffic_source': prof.get('source') if prof and headline else None,
                         'align_phase': phase},
            'hbm': {'achieved': round(gbs, 2), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                    'frac': round(gbs / HBM_PEAK_GBS, 5), 'algorithmic_bytes_per_launch': int(launch_bytes),
                    'kernel': dom_kernel},
            'gcups_step': round(cells / (step_ms * 1e-3) / 1e9, 1),
            'cells_per_step': cells,
            'cpu_baseline': cpu,
            'gpu_vs_cpu': round(value / cpu['value'], 1) if cpu else None,
            'parity_spot_check': checked,
            'setup_s': round(gen_s, 2),
        }
        out.update(subs)
        return out
    return None


def run_other_configs(args, ctx):
    """The default run's sub-records (N = 1): BASELINE.json's other configs, per GPU, each with its
    own oracle spot check and CPU baseline, so one driver-timed line carries every workload.
    A sub-record that fails reports its error instead of taking the headline down."""
    rank, world, dist, torch, L, _lib, A, synth, encode_adapters = ctx

    def sub(**kw):
        s = argparse.Namespace(**vars(args))
        s.steps, s.warmup = max(5, args.steps // 2), 2
        for k, v in kw.items():
            setattr(s, k, v)
        return s

    runs = [
        # the adapter-set search (configs[1]'s check phase: 10k reads x 119 sets) and its MAX
        # all-reduce (here over one rank)
        ('check_phase', lambda: run_check_phase(sub(), rank, 1, None, torch, L, _lib, A, synth, encode_adapters)),
        # the reference-API path (porechop_abi.py's three drivers on 100k NanoporeRead objects)
        ('drivers', lambda: run_drivers(sub(steps=2), rank, 1, None, torch, L, _lib, A, synth, encode_adapters)),
        # the reference's own job shape: set search on the first 10k reads x 119 sets, then end trim
        # and middle scan of 100k reads with only the sets it keeps (porechop_abi.py:41-131)
        ('reference_job', lambda: run_reference_job(sub(), rank, 1, None, torch, L, _lib, A, synth,
                                                    encode_adapters)),
        # configs[2]: end trim + middle scan, 100k x 8 kb per GPU
        ('middle', lambda: run_middle(sub(workload='middle'), rank, 1, None, torch, L, _lib, A, synth,
                                      encode_adapters)),
        # configs[4] per GPU: 100k x 20 kb, middle scan on (CPU sample scaled to the read length)
        ('middle_20kb', lambda: run_middle(sub(workload='middle', mean_len=20000, steps=5,
                                               cpu_sample=args.cpu_sample * 2 // 5, middle_check=300),
                                           rank, 1, None, torch, L, _lib, A, synth, encode_adapters)),
        # configs[3] per GPU: 100k reads x 96 forward barcode sets + SQK-NSK007, demux calls
        ('barcodes', lambda: run_endtrim(sub(workload='barcodes', sub=0, cpu_sample=args.cpu_sample // 4), rank, 1,
                                         None, torch, L, _lib, A, synth, encode_adapters)),
        # configs[1] shape: a 10k-read batch against all 119 adapter sets
        ('config2_10k_119sets', lambda: run_endtrim(sub(workload='endtrim', sub=0, reads=10000, sets=119,
                                                        cpu_sample=args.cpu_sample // 4),
                                                    rank, 1, None, torch, L, _lib, A, synth, encode_adapters)),
        # the CLI path file to file (parse + trim + middle + write), 25k reads
        # 100k reads = 8 batches of 12.5k per step: the parse / device / write pipeline at its
        # steady state (r04 timed 2 batches per step, which never fills it)
        ('e2e', lambda: run_e2e(sub(workload='e2e', reads=100000, steps=4, warmup=1), rank, 1, None, torch, L, _lib, A,
                                synth, encode_adapters)),
        # SURVEY §8(f) 3 and 4
        ('compat', lambda: run_compat(sub(workload='compat', cpu_sample=args.cpu_sample // 4), rank, 1, None, torch,
                                      L, _lib)),
        ('kmer', lambda: run_kmer(sub(workload='kmer', steps=5, warmup=1), rank, 1, None, torch, L, _lib, synth)),
    ]
    subs = {}
    for name, fn in runs:
        if args.only_subs and name not in args.only_subs.split(','):
            continue
        t0 = time.perf_counter()
        try:
            rec = fn()
            for k in ('n_gpus', 'higher_is_better', 'scaling', 'vs_baseline'):
                rec.pop(k, None)
        except Exception as ex:   # reported, never fatal for the headline line
            rec = {'error': '%s: %s' % (type(ex).__name__, ex)}
        rec['sub_wall_s'] = round(time.perf_counter() - t0, 2)
        subs[name] = rec
        print('sub-record %s: %.1f s' % (name, rec['sub_wall_s']), file=sys.stderr, flush=True)
    return subs


def run_check_phase(args, rank, world, dist, torch, L, _lib, A, synth, encode_adapters, n_check=10000):
    """The adapter-set search (porechop_abi.py:200-245, nanopore_read.py:158-173), the path's one
    collective: the job's first n_check reads (every rank generates the same
    seeded set) against every non-"full sequence" set of the database (119 sets: their distinct
    start and end sequences), start / end windows of 150 bp. Rank r takes its contiguous shard
    of the check reads. One step, inputs resident in HBM:
        windows -> tiles -> k_align cross product -> k_best_full_id        (per sequence, on the device,
                                                                         into a torch tensor on the rank's GPU)
        dist.all_reduce(MAX) of the tensor (RCCL over xGMI; gloo: the host copy)
    value = check reads / step time (max over ranks). Parity: the maxima after the all-reduce are
    compared with the oracle's reduction over the same reads (the first --check-phase-check reads
    separately on the device, so the oracle's share stays bounded) and every rank must hold the
    same maxima."""
    from custom_porechop_abi_amd import porechop_abi as P
    vp = ctypes.c_void_p
    search = [a for a in A.fresh_adapters() if '(full sequence)' not in a.name]
    starts_u, _ = P._unique([a.start_sequence[1] for a in search if a.start_sequence])
    ends_u, _ = P._unique([a.end_sequence[1] for a in search if a.end_sequence])
    n_u = len(starts_u) + len(ends_u)
    E = args.end_size
    reads = synth.make_reads(n_check, args.mean_len, seed=4242, keep=E)
    lo, hi = n_check * rank // world, n_check * (rank + 1) // world
    mine = reads[lo:hi]
    n = len(mine)
    buf, s_off, s_len, e_off, e_len = synth.pack_end_windows(mine, E)

    def dalloc(nbytes):
        p = vp()
        _lib.check(L.pcabi_dev_malloc(ctypes.byref(p), max(int(nbytes), 16)), 'malloc')
        return p

    def h2d(arr):
        arr = np.ascontiguousarray(arr)
        p = dalloc(arr.nbytes)
        _lib.check(L.pcabi_dev_h2d(p, arr.ctypes.data_as(vp), arr.nbytes), 'h2d')
        return p

    def table(lst):
        t = vp()
        c, o, l = encode_adapters(lst)
        _lib.check(L.pcabi_adapters_create_scored(c.ctypes.data_as(vp), o.ctypes.data_as(vp), l.ctypes.data_as(vp),
                                                  len(lst), *SCORING, ctypes.byref(t)), 'adapters_create')
        return t

    stream = vp()
    _lib.check(L.pcabi_stream_create(ctypes.byref(stream)), 'stream')
    d_codes = h2d(buf)
    nccl = dist is not None and args.dist_backend == 'nccl'
    dev = torch.device('cuda', args.local_device) if nccl else None
    # the buffer the collective reduces: on the rank's GPU (RCCL), or a device buffer copied to
    # a host tensor (gloo)
    t_best = torch.zeros(n_u, dtype=torch.float64, device=dev) if nccl else torch.zeros(n_u, dtype=torch.float64)
    d_best = vp(t_best.data_ptr()) if nccl else dalloc(8 * n_u)
    sides = []
    for off, ln, adps, b0 in ((s_off, s_len, starts_u, 0), (e_off, e_len, ends_u, len(starts_u))):
        toff = np.zeros((n + 255) // 256 + 1, np.int64)
        nd = L.pcabi_tile_layout(ln.ctypes.data_as(vp), n, toff.ctypes.data_as(vp))
        sides.append(dict(d_off=h2d(off), d_len=h2d(ln), d_toff=h2d(toff), d_tiles=dalloc(4 * max(nd, 1)),
                          mq=int(np.diff(toff).max() // 256) if n else 0, mx=int(ln.max()) if n else 0,
                          tab=table(adps), n_adp=len(adps), d_res=dalloc(4 * 8 * len(adps) * max(n, 1)),
                          d_best=vp(d_best.value + 8 * b0)))

    def reduce_local(n_win):
        if nccl:
            t_best.zero_()
            torch.cuda.synchronize(dev)   # zeroed before the library's stream writes the tensor
        else:
            _lib.check(L.pcabi_dev_memset(d_best, 0, 8 * n_u), 'memset')
        for sd in sides:
            if n_win == 0:
                continue
            _lib.check(L.pcabi_tile_windows_dev(d_codes, sd['d_off'], sd['d_len'], n_win, sd['d_toff'], sd['mq'],
                                                sd['d_tiles'], stream), 'tile')
            _lib.check(L.pcabi_align_cross_dev(sd['d_tiles'], sd['d_toff'], sd['d_len'], n_win, sd['mx'], sd['tab'],
                                               *SCORING, sd['d_res'], sd['n_adp'] * n_win, stream), 'align')
            _lib.check(L.pcabi_best_full_identity_dev(sd['d_res'], sd['n_adp'] * n_win, n_win, sd['n_adp'],
                                                      sd['d_best'], stream), 'best')
        _lib.check(L.pcabi_stream_sync(stream), 'sync')

    def step():
        reduce_local(n)
        if not nccl:   # one process or gloo: the maxima through the host
            _lib.check(L.pcabi_dev_d2h(ctypes.c_void_p(t_best.data_ptr()), d_best, 8 * n_u), 'd2h')
        if dist is not None:
            dist.all_reduce(t_best, op=dist.ReduceOp.MAX)
        if nccl:
            torch.cuda.synchronize(dev)

    for _ in range(max(1, args.warmup)):
        step()
    if dist is not None:
        dist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if nccl else 'cpu')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    maxima = t_best.cpu().numpy().copy()
    agree = None
    if dist is not None:
        # every rank must hold the same reduced maxima
        g = torch.tensor(maxima, dtype=torch.float64, device=dev if nccl else 'cpu')
        g_min = g.clone()
        dist.all_reduce(g_min, op=dist.ReduceOp.MIN)
        agree = bool(torch.equal(g, g_min))
    checked = None
    k = min(getattr(args, 'check_phase_check', 400), n)
    if args.check and rank == 0 and k > 0:
        # the device reduction over the first k check reads of this rank vs the oracle's
        from tests import oracle_lib
        from custom_porechop_abi_amd.engine import pid6
        from multiprocessing.dummy import Pool as ThreadPool
        reduce_local(k)
        got = np.empty(n_u, np.float64)
        _lib.check(L.pcabi_dev_d2h(got.ctypes.data_as(vp), d_best if not nccl else vp(t_best.data_ptr()), 8 * n_u),
                   'd2h')
        heads = [synth.codes_to_str(r[0] if isinstance(r, tuple) else r[:E]) for r in mine[:k]]
        tails = [synth.codes_to_str(r[1] if isinstance(r, tuple) else r[-E:]) for r in mine[:k]]

        def one(job):
            wins, adps, a0 = job
            exp = oracle_lib.align_many(wins, adps, (np.zeros(len(adps), np.int64), np.arange(len(adps))), SCORING)
            return exp

        jobs = [([heads[i]], starts_u, i) for i in range(k)] + [([tails[i]], ends_u, i) for i in range(k)]
        with ThreadPool(min(16, len(os.sched_getaffinity(0)))) as pool:
            res = pool.map(one, jobs)
        exp = np.zeros(n_u, np.float64)
        for (wins, adps, _), r in zip(jobs, res):
            full = np.where(r[0] == -1, 0.0, pid6(r[5], r[7]))
            b0 = 0 if adps is starts_u else len(starts_u)
            exp[b0:b0 + len(adps)] = np.maximum(exp[b0:b0 + len(adps)], full)
        checked = {'reads_checked': k, 'sequences': n_u, 'maxima_identical': bool(np.array_equal(got, exp)),
                   'matching_sets_at_90': int(sum(1 for a in search
                                                  if max(maxima[starts_u.index(a.start_sequence[1])]
                                                         if a.start_sequence else 0.0,
                                                         maxima[len(starts_u) + ends_u.index(a.end_sequence[1])]
                                                         if a.end_sequence else 0.0) >= 90.0))}
    if rank == 0:
        step_ms = 1e3 * elapsed / args.steps
        cells = int(s_len.astype(np.int64).sum() * sum(map(len, starts_u)) +
                    e_len.astype(np.int64).sum() * sum(map(len, ends_u)))
        return {'metric': 'check reads/sec through the adapter-set search (%d reads x %d sets, MAX all-reduce)'
                          % (n_check, len(search)),
                'value': round(n_check * args.steps / elapsed, 1), 'unit': 'reads/s', 'n_gpus': world,
                'steps': args.steps, 'warmup': max(1, args.warmup), 'ms_per_step': round(step_ms, 4),
                'dtype': 'int32', 'data': 'synthetic (seeded ONT-like reads, mean %d bp)' % args.mean_len,
                'config': {'workload': 'adapter-set search: %d check reads sharded over %d rank(s) x %d sets (%d start + '
                                       '%d end sequences), windows of %d bp, per-sequence maxima on the device, '
                                       'all-reduce MAX (%s)' % (n_check, world, len(search), len(starts_u),
                                                                len(ends_u), E, args.dist_backend if dist else 'none'),
                           'reads_per_rank': n, 'collective_bytes': 8 * n_u},
                'gcups_rank0': round(cells / (step_ms * 1e-3) / 1e9, 1),
                'ranks_agree': agree, 'parity_spot_check': checked}
    return None


def run_reference_job(args, rank, world, dist, torch, L, _lib, A, synth, encode_adapters, n_check=10000):
    """The reference's job as its main() runs it (porechop_abi/porechop_abi.py:41-131), on 100k
    synthetic reads of mean 8 kb per GPU, inputs resident in HBM. One step:
      adapter-set search: the first 10k reads' start / end windows x the 119 sets' distinct
          sequences (k_align cross products -> k_best_full_id -> the maxima to the host)  (:200-245)
      host: sets with best start-or-end identity >= 90, fix_up_1d2_sets, add_full_barcode_adapter_sets
      end trim of every read with only the kept sets (k_align -> k_end_trim)          (:359-438)
      trimmed views + middle scan with the kept sets' middle list (queued device rounds) (:457-522)
    The kept sets' adapter tables and the scan's scratch are made on the first step and reused (a
    job makes them once). Events time each phase; the roofline is the step's dominant launch (the
    set search's largest register bucket). Parity: the set search's maxima == the oracle's on the
    first 400 check reads, the kept end windows == the oracle on the first 256 reads, the middle hits
    == the oracle's masked loop on the first 1000 reads."""
    from custom_porechop_abi_amd import porechop_abi as P
    from custom_porechop_abi_amd.engine import pid6
    vp = ctypes.c_void_p
    n, E, sc = args.reads, args.end_size, SCORING
    search = [a for a in A.fresh_adapters() if '(full sequence)' not in a.name]
    starts_u, _ = P._unique([a.start_sequence[1] for a in search if a.start_sequence])
    ends_u, _ = P._unique([a.end_sequence[1] for a in search if a.end_sequence])
    n_u = len(starts_u) + len(ends_u)
    t0 = time.time()
    reads = synth.make_reads(n, args.mean_len, seed=12345 + rank)
    lens = np.array([len(r) for r in reads], np.int64)
    offs = np.zeros(n, np.int64)
    offs[1:] = np.cumsum((lens + 3) & ~3)[:-1]
    pack = np.full(int(offs[-1] + lens[-1]) + 64, 4, np.uint8)
    for k, r in enumerate(reads):
        pack[offs[k]:offs[k] + lens[k]] = r
    s_len = np.minimum(lens, E).astype(np.int32)
    e_len = s_len.copy()
    s_off, e_off = offs.copy(), offs + lens - e_len
    gen_s = time.time() - t0
    n_chk = min(n_check, n)

    def dalloc(nbytes):
        p = vp()
        _lib.check(L.pcabi_dev_malloc(ctypes.byref(p), max(int(nbytes), 16)), 'malloc')
        return p

    def h2d(arr):
        arr = np.ascontiguousarray(arr)
        p = dalloc(arr.nbytes)
        _lib.check(L.pcabi_dev_h2d(p, arr.ctypes.data_as(vp), arr.nbytes), 'h2d')
        return p

    def table(lst):
        c, o, l = encode_adapters(lst)
        t = vp()
        _lib.check(L.pcabi_adapters_create_scored(c.ctypes.data_as(vp), o.ctypes.data_as(vp), l.ctypes.data_as(vp),
                                                  len(lst), *sc, ctypes.byref(t)), 'adapters_create')
        return t

    d_pack = h2d(pack)               # resident for every step (the middle scan leaves it intact)
    d_offs, d_lens = h2d(offs), h2d(lens.astype(np.int32))
    d_st, d_et = dalloc(4 * n), dalloc(4 * n)
    d_toff_mid, d_tlen_mid = dalloc(8 * n), dalloc(4 * n)
    d_best = dalloc(8 * n_u)
    stream, stream2 = vp(), vp()
    _lib.check(L.pcabi_stream_create(ctypes.byref(stream)), 'stream')
    _lib.check(L.pcabi_stream_create(ctypes.byref(stream2)), 'stream')
    # --rj-end-streams 1: each kept adapter's end-trim cross product on a stream of its own
    x_streams, x_join = [], []
    for _ in range(6 if args.rj_end_streams else 0):
        xs, xe = vp(), vp()
        _lib.check(L.pcabi_stream_create(ctypes.byref(xs)), 'stream')
        _lib.check(L.pcabi_event_create(ctypes.byref(xe)), 'event')
        x_streams.append(xs)
        x_join.append(xe)
    sides = []
    for w_off, w_len, u in ((s_off, s_len, starts_u), (e_off, e_len, ends_u)):
        toff = np.zeros((n + 255) // 256 + 1, np.int64)
        nd = L.pcabi_tile_layout(w_len.ctypes.data_as(vp), n, toff.ctypes.data_as(vp))
        sides.append(dict(d_off=h2d(w_off), d_len=h2d(w_len), d_toff=h2d(toff), d_tiles=dalloc(4 * nd),
                          mq=int(np.diff(toff).max() // 256), mx=int(w_len.max()), mx_chk=int(w_len[:n_chk].max()),
                          search=table(u), n_u=len(u), d_chk=dalloc(4 * 8 * len(u) * n_chk)))
    search_regions = _lib.cross_regions([(sd['d_tiles'], sd['d_toff'], sd['d_len'], n_chk, sd['mx_chk'], sd['search'],
                                          sd['d_chk'], sd['n_u'] * n_chk) for sd in sides])
    ev = [vp() for _ in range(11)]
    for e in ev:
        _lib.check(L.pcabi_event_create(ctypes.byref(e)), 'event')
    kept_cache = {}
    cap = max(4096, n)
    hits = np.zeros((6, cap), np.int32)
    stats = {'kept': None, 'hits': 0}
    acc = {}

    def kept_state(names, matching):
        if names not in kept_cache:
            st_ = [a.start_sequence[1] for a in matching if a.start_sequence]
            en_ = [a.end_sequence[1] for a in matching if a.end_sequence]
            mid = [x[1] for x in P.middle_adapter_list(matching)[0]]
            ks = dict(start=st_, end=en_, mid=mid, tabs=[table(x) if x else None for x in (st_, en_, mid)],
                      d_res=[dalloc(4 * 8 * max(1, len(x)) * n) for x in (st_, en_)], scan=vp(),
                      one=[[table([a]) for a in x] if args.rj_end_streams else [] for x in (st_, en_)])
            if mid:
                _lib.check(L.pcabi_scan_create(ks['tabs'][2], ctypes.byref(ks['scan'])), 'scan_create')
            ks['regions'] = _lib.cross_regions([(sd['d_tiles'], sd['d_toff'], sd['d_len'], n, sd['mx'], ks['tabs'][k],
                                                  ks['d_res'][k], len(x) * n)
                                                 for k, (sd, x) in enumerate(zip(sides, (st_, en_))) if x])
            kept_cache[names] = ks
        return kept_cache[names]

    srch_sets = [a for a in A.fresh_adapters() if '(full sequence)' not in a.name]

    def step():
        work = d_pack
        L.pcabi_event_record(ev[0], stream)
        _lib.check(L.pcabi_dev_memset(d_best, 0, 8 * n_u), 'memset')
        b0 = 0
        for k, sd in enumerate(sides):
            _lib.check(L.pcabi_tile_windows_dev(work, sd['d_off'], sd['d_len'], n, sd['d_toff'], sd['mq'],
                                                sd['d_tiles'], stream), 'tile')
        if args.rj_multi:
            # both read ends' set search in one call; events around the whole call (ev[2] / ev[3])
            L.pcabi_event_record(ev[2], stream)
            _lib.check(L.pcabi_align_cross_multi_dev(search_regions, len(search_regions), *sc, stream, None, None),
                       'align')
            L.pcabi_event_record(ev[3], stream)
            for k, sd in enumerate(sides):
                L.pcabi_event_record(ev[4 + k], stream)
                _lib.check(L.pcabi_best_full_identity_dev(sd['d_chk'], sd['n_u'] * n_chk, n_chk, sd['n_u'],
                                                          vp(d_best.value + 8 * b0), stream), 'best')
                b0 += sd['n_u']
        if args.rj_check_overlap and not args.rj_multi:
            L.pcabi_event_record(ev[9], stream)
            L.pcabi_stream_wait_event(stream2, ev[9])
        for k, sd in enumerate(sides if not args.rj_multi else []):
            st_k = stream2 if (args.rj_check_overlap and k == 1) else stream
            # the check reads are the first n_check reads: their windows are the first tiles
            _lib.check(L.pcabi_align_cross_dev_marked(sd['d_tiles'], sd['d_toff'], sd['d_len'], n_chk, sd['mx_chk'],
                                                      sd['search'], *sc, sd['d_chk'], sd['n_u'] * n_chk, st_k,
                                                      ev[2 + 2 * k], ev[3 + 2 * k]), 'align')
            _lib.check(L.pcabi_best_full_identity_dev(sd['d_chk'], sd['n_u'] * n_chk, n_chk, sd['n_u'],
                                                      vp(d_best.value + 8 * b0), st_k), 'best')
            b0 += sd['n_u']
        if args.rj_check_overlap and not args.rj_multi:
            L.pcabi_event_record(ev[9], stream2)
            L.pcabi_stream_wait_event(stream, ev[9])
        maxima = np.empty(n_u, np.float64)
        _lib.check(L.pcabi_dev_copy_async(maxima.ctypes.data_as(vp), d_best, 8 * n_u, 1, stream), 'd2h')
        _lib.check(L.pcabi_stream_sync(stream), 'sync')
        th = time.perf_counter()
        # the searched sets' scores start from zero each job (the adapter objects are made once, as
        # a long-running caller keeps them; fresh_adapters() per step cost ~0.15-0.4 ms of host time)
        srch = srch_sets
        for a in srch:
            a.best_start_score = a.best_end_score = 0.0
        P.apply_set_maxima(srch, maxima)
        matching = [a for a in srch if a.best_start_or_end_score() >= 90.0]
        matching = P.add_full_barcode_adapter_sets(P.fix_up_1d2_sets(matching))
        ks = kept_state(tuple(a.name for a in matching), matching)
        acc['host_ms'] = acc.get('host_ms', 0.0) + 1e3 * (time.perf_counter() - th)
        stats['kept'] = [a.name for a in matching]
        L.pcabi_event_record(ev[1], stream)
        # the two sides' few-adapter cross products side by side (start on `stream`, end on stream2):
        # with the kept sets each bucket holds one adapter (1,564 waves), too few to fill the chip alone
        L.pcabi_stream_wait_event(stream2, ev[1])
        if args.rj_multi:
            if len(ks['regions']):
                _lib.check(L.pcabi_align_cross_multi_dev(ks['regions'], len(ks['regions']), *sc, stream, None, None),
                           'align')
        elif args.rj_end_streams:
            j = 0
            for k, sd in enumerate(sides):
                adps = ks['start'] if k == 0 else ks['end']
                for a, tab in enumerate(ks['one'][k]):
                    xs = x_streams[j % len(x_streams)]
                    L.pcabi_stream_wait_event(xs, ev[1])
                    _lib.check(L.pcabi_align_cross_dev(sd['d_tiles'], sd['d_toff'], sd['d_len'], n, sd['mx'], tab, *sc,
                                                       vp(ks['d_res'][k].value + 4 * a * n), len(adps) * n, xs), 'align')
                    L.pcabi_event_record(x_join[j % len(x_join)], xs)
                    L.pcabi_stream_wait_event(stream, x_join[j % len(x_join)])
                    j += 1
        else:
            for k, sd in enumerate(sides):
                adps = ks['start'] if k == 0 else ks['end']
                if adps:
                    _lib.check(L.pcabi_align_cross_dev(sd['d_tiles'], sd['d_toff'], sd['d_len'], n, sd['mx'],
                                                       ks['tabs'][k], *sc, ks['d_res'][k], len(adps) * n,
                                                       stream if k == 0 else stream2), 'align')
        L.pcabi_event_record(ev[8], stream2)
        L.pcabi_stream_wait_event(stream, ev[8])
        L.pcabi_event_record(ev[10], stream)
        n_sa, n_ea = len(ks['start']), len(ks['end'])
        _lib.check(L.pcabi_end_trim_dev(ks['d_res'][0], n_sa * n, n_sa, ks['d_res'][1], n_ea * n, n_ea, n, E, 2, 75.0, 4,
                                        d_st, d_et, None, None, stream), 'end_trim')
        L.pcabi_event_record(ev[6], stream)
        nh = 0
        if ks['mid']:
            _lib.check(L.pcabi_trim_views_dev(d_offs, d_lens, d_st, d_et, n, d_toff_mid, d_tlen_mid, stream), 'views')
            nh = L.pcabi_middle_scan_dev(ks['scan'], work, d_toff_mid, d_tlen_mid, None, n, *sc, 90.0,
                                         hits.ctypes.data_as(vp), cap, stream)
            if nh < 0:
                _lib.check(int(nh), 'middle_scan')
        L.pcabi_event_record(ev[7], stream)
        _lib.check(L.pcabi_stream_sync(stream), 'sync')
        stats['hits'] = int(nh)
        for key, a, b in (('check_ms', 0, 1), ('end_trim_ms', 1, 6), ('middle_ms', 6, 7), ('check_dom_start_ms', 2, 3),
                          ('check_dom_end_ms', 4, 5), ('end_trim_align_ms', 1, 10)):
            ms = ctypes.c_float()
            _lib.check(L.pcabi_event_elapsed_ms(ctypes.byref(ms), ev[a], ev[b]), 'elapsed')
            acc[key] = acc.get(key, 0.0) + ms.value
        return matching

    # the job runs cross products on two caller streams at once (set search and end trim: both
    # sides side by side), so the library's side streams go off on its streams (pcabi_stream_side_streams, r04r:
    # 4.95 -> 4.66 ms per step): a side stream on the other caller stream's hardware queue waits
    # for its large launch
    for s_ in [stream, stream2] + x_streams:
        L.pcabi_stream_side_streams(s_, 0 if args.rj_side_streams == 0 else 1)
    if args.rj_multi:
        # one (multi) call at a time on `stream`: its grouped launches side by side
        L.pcabi_stream_side_streams(stream, 1)
    try:
        for _ in range(max(1, args.warmup)):
            step()
        _lib.check(L.pcabi_stream_sync(stream), 'sync')
        acc.clear()
        torch.cuda.synchronize() if torch.cuda.is_available() else None
        t0 = time.perf_counter()
        for k in range(args.steps):
            matching = step()
        elapsed = time.perf_counter() - t0
    finally:
        for s_ in [stream, stream2] + x_streams:
            L.pcabi_stream_side_streams(s_, -1)
    step_ms = 1e3 * elapsed / args.steps
    per = {k: round(v / args.steps, 4) for k, v in acc.items()}
    ks = kept_state(tuple(a.name for a in matching), matching)
    # the dominant launch: the set search's largest register bucket (start and end launches averaged);
    # --rj-multi: the set search's whole multi call (both read ends, every grouped launch)
    dom_ms = per['check_dom_start_ms'] if args.rj_multi else 0.5 * (per['check_dom_start_ms'] + per['check_dom_end_ms'])
    dom_cells = []
    for k, (w_len, u) in enumerate(((s_len, starts_u), (e_len, ends_u))):
        from collections import Counter
        rows = Counter((len(x) + 3) // 4 * 4 for x in u)
        big = max(rows, key=lambda r: rows[r] * r)   # the table's largest bucket by adapters x rows
        dom_cells.append(int(w_len[:n_chk].astype(np.int64).sum()) * sum(len(x) for x in u if (len(x) + 3) // 4 * 4 == big))
    # end trim with the kept sets: cells and rate (the few-adapter launches)
    end_cells = int(s_len.astype(np.int64).sum() * sum(map(len, ks['start'])) +
                    e_len.astype(np.int64).sum() * sum(map(len, ks['end'])))
    chk_cells = int(s_len[:n_chk].astype(np.int64).sum() * sum(map(len, starts_u)) +
                    e_len[:n_chk].astype(np.int64).sum() * sum(map(len, ends_u)))
    if args.rj_multi:
        dom_cells = [chk_cells, chk_cells]
    tops = float(np.mean(dom_cells)) * OPS_PER_CELL / (dom_ms * 1e-3) / 1e12
    checked = None
    if args.check and rank == 0:
        from tests import oracle_lib
        # set search maxima over the first 400 check reads vs the oracle's
        k = min(400, n_chk)
        heads = [synth.codes_to_str(r[:E]) for r in reads[:k]]
        tails = [synth.codes_to_str(r[-E:]) for r in reads[:k]]
        exp = np.zeros(n_u)
        for wins, u, b0 in ((heads, starts_u, 0), (tails, ends_u, len(starts_u))):
            r_ = oracle_lib.align_many(wins, u, (np.tile(np.arange(k), len(u)), np.repeat(np.arange(len(u)), k)), sc)
            full = np.where(r_[0] == -1, 0.0, pid6(r_[5], r_[7])).reshape(len(u), k)
            exp[b0:b0 + len(u)] = full.max(axis=1)
        got = np.zeros(n_u)
        for j, sd in enumerate(sides):
            res = np.empty((8, sd['n_u'] * n_chk), np.int32)
            _lib.check(L.pcabi_dev_d2h(res.ctypes.data_as(vp), sd['d_chk'], res.nbytes), 'd2h')
            res = res.reshape(8, sd['n_u'], n_chk)[:, :, :k].reshape(8, -1)
            full = np.where(res[0] == -1, 0.0, pid6(res[5], res[7])).reshape(sd['n_u'], k)
            got[(0 if j == 0 else len(starts_u)):][:sd['n_u']] = full.max(axis=1)
        trims = np.zeros((2, n), np.int32)
        _lib.check(L.pcabi_dev_d2h(trims[0].ctypes.data_as(vp), d_st, 4 * n), 'd2h')
        _lib.check(L.pcabi_dev_d2h(trims[1].ctypes.data_as(vp), d_et, 4 * n), 'd2h')
        ends_chk = spot_check(L, _lib, ks['d_res'][0], ks['d_res'][1], d_st, d_et, len(ks['start']) * n,
                              len(ks['end']) * n, n, len(ks['start']), len(ks['end']), reads, ks['start'], ks['end'],
                              E, min(256, n), sc)
        mid_chk = middle_spot_check(reads, trims, hits, stats['hits'], ks['mid'], sc, 90.0, min(1000, n)) \
            if ks['mid'] else None
        checked = {'set_search_maxima_identical_400_reads': bool(np.array_equal(got, exp)),
                   'end_windows': ends_chk, 'middle': mid_chk, 'input_pack_intact': pack_intact(L, _lib, d_pack, pack)}
    return {'metric': 'reads/sec through the reference job (set search on 10k reads x 119 sets, then end trim + '
                      'middle scan with the kept sets)',
            'value': round(n * args.steps / elapsed, 1), 'unit': 'reads/s', 'steps': args.steps,
            'ms_per_step': round(step_ms, 3), 'ms_per_phase': per, 'kept_sets': stats['kept'],
            'kept_adapters': {'start': len(ks['start']), 'end': len(ks['end']), 'middle': len(ks['mid'])},
            'middle_hits_per_step': stats['hits'],
            'cells_per_step': {'set_search': chk_cells, 'end_trim': end_cells},
            'end_trim_gcups': round(end_cells / (per['end_trim_ms'] * 1e-3) / 1e9, 1),
            # the kept sets' one-adapter launches (both sides side by side, events around them)
            'single_adapter_launches': {
                'bound': 'valu', 'cells': end_cells, 'ms': per['end_trim_align_ms'],
                'achieved': round(end_cells * OPS_PER_CELL / (per['end_trim_align_ms'] * 1e-3) / 1e12, 3),
                'peak': round(VALU_PEAK_TOPS, 1), 'unit': 'Tops/s (int32 lane-ops)',
                'frac': round(end_cells * OPS_PER_CELL / (per['end_trim_align_ms'] * 1e-3) / 1e12 / VALU_PEAK_TOPS, 4),
                'launches': ('both sides\' kept adapters in one pcabi_align_cross_multi_dev call (grouped launches), '
                             '%d + %d adapters' if args.rj_multi else 'one per register bucket and side, %d + %d adapters')
                            % (len(ks['start']), len(ks['end']))},
            'roofline': {'bound': 'valu', 'kernel': ('the set search\'s multi call (both read ends, every grouped launch; '
                                                     'events around the call)' if args.rj_multi else
                                                     'the set search\'s largest register bucket (k_align<24, true, 6>)'),
                         'achieved': round(tops, 3), 'peak': round(VALU_PEAK_TOPS, 1), 'unit': 'Tops/s (int32 lane-ops)',
                         'frac': round(tops / VALU_PEAK_TOPS, 4), 'launch_ms': round(dom_ms, 4),
                         'cells_per_launch': int(np.mean(dom_cells)), 'ops_per_cell': OPS_PER_CELL,
                         'schedule': ('one multi call for both read ends' if args.rj_multi else
                                      'both sides\' cross products side by side: the launch shares the GPU'
                                      if args.rj_check_overlap else 'each side\'s cross product alone')},
            'dtype': 'int32', 'data': 'synthetic (seeded ONT-like reads, mean %d bp)' % args.mean_len,
            'config': {'workload': 'reference job: set search (%d check reads x %d sets, %d + %d distinct sequences), '
                                   'end trim + middle scan of %d reads/GPU with the kept sets' % (
                                       n_chk, len(search), len(starts_u), len(ends_u), n),
                       'reads_per_gpu': n,
                       'inputs': 'one read pack resident in HBM for every step (the scan leaves it intact)'},
            'parity_spot_check': checked, 'setup_s': round(gen_s, 2)}


def run_drivers(args, rank, world, dist, torch, L, _lib, A, synth, encode_adapters):
    """The reference-API path INTEGRATION.md §2 hands maintainers: the three phase drivers of
    porechop_abi.py (find_matching_adapter_sets :200-245, find_adapters_at_read_ends :359-438,
    find_adapters_in_read_middles :457-522) with their own signatures, on NanoporeRead objects of
    100k synthetic reads (mean 8 kb) against the first 50 adapter sets. A step builds fresh
    NanoporeRead objects (untimed) and times the three drivers: the check phase on the first 10k
    reads against all sets, end trimming (device decisions: only trims and the recorded alignments
    come back, engine.end_decisions) and the middle scan (only hits come back). Decisions of the
    first --drivers-check reads are compared with the same drivers over the CPU oracle."""
    import io
    from custom_porechop_abi_amd import engine, porechop_abi as P
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    n, E, sc = args.reads, args.end_size, SCORING
    t0 = time.time()
    seqs = [synth.codes_to_str(r) for r in synth.make_reads(n, args.mean_len, seed=12345 + rank)]
    sets = [a for a in A.fresh_adapters() if '(full sequence)' not in a.name][:args.sets]
    gen_s = time.time() - t0
    sink = io.StringIO()
    d2h = {}
    real = engine.end_decisions

    eng_t = {}
    real_mid = engine.middle_scan_seqs

    def timed_mid(*a, **kw):                # the middle driver's library call (staging + scan)
        t = time.perf_counter()
        try:
            return real_mid(*a, **kw)
        finally:
            eng_t['middle_scan_seqs'] = eng_t.get('middle_scan_seqs', 0.0) + time.perf_counter() - t

    def counted(*a, **kw):                  # the end-trim driver's device -> host bytes
        t = time.perf_counter()
        st, et, sl, el, bcf = real(*a, **kw)
        eng_t['end_decisions'] = eng_t.get('end_decisions', 0.0) + time.perf_counter() - t
        # pcabi_end_decisions_host's transfer (windows < 32 k, < 32 k adapters): the trims, the two
        # alignment counts, per side 12 B per alignment (six int16 fields) + 2 B per read (counts),
        # the barcode identities
        n = len(st)
        d2h['bytes'] = (st.nbytes + et.nbytes + 16 + 12 * (sl.shape[1] + el.shape[1]) + 2 * 4 * ((n + 1) // 2)
                        + (bcf.nbytes if bcf is not None else 0))
        return st, et, sl, el, bcf

    def drivers(reads, times):
        ta = time.perf_counter()
        P.find_matching_adapter_sets(reads[:10000], 0, E, sc, sink, 90.0, 1, adapter_sets=A.fresh_adapters())
        tb = time.perf_counter()
        P.find_adapters_at_read_ends(reads, sets, 0, E, 2, 75.0, sc, sink, 4, 1, False, 75.0, 5.0, False, None)
        tc = time.perf_counter()
        P.find_adapters_in_read_middles(reads, sets, 0, 90.0, 10, 100, sc, sink, 1, False)
        td = time.perf_counter()
        for k, v in (('check', tb - ta), ('ends', tc - tb), ('middles', td - tc)):
            times[k] = times.get(k, 0.0) + v

    engine.end_decisions = counted
    engine.middle_scan_seqs = timed_mid
    try:
        drivers([NanoporeRead('r%d' % i, s, '') for i, s in enumerate(seqs[:2000])], {})   # warm-up
        eng_t.clear()
        times = {}
        build = 0.0
        for _ in range(args.steps):
            tb = time.perf_counter()
            reads = [NanoporeRead('r%d' % i, s, '') for i, s in enumerate(seqs)]
            build += time.perf_counter() - tb
            drivers(reads, times)
    finally:
        engine.end_decisions = real
        engine.middle_scan_seqs = real_mid
    total = sum(times.values()) / args.steps
    checked = None
    k = min(args.drivers_check, n)
    if args.check and k:
        # the same drivers over the CPU oracle (TEST INFRASTRUCTURE: the checker) on the first k
        # reads, decisions compared read by read
        from tests import oracle_lib
        got = reads[:k]
        sub = [NanoporeRead('r%d' % i, s, '') for i, s in enumerate(seqs[:k])]
        saved = {f: getattr(engine, f) for f in ('align', 'end_decisions', 'best_full_identity', 'middle_scan',
                                                 'middle_scan_seqs')}
        engine.align, engine.end_decisions = oracle_lib.align_windows, oracle_lib.end_decisions_windows
        engine.best_full_identity = oracle_lib.best_full_identity_windows
        engine.middle_scan = lambda v, a, s_, t, device=0: oracle_lib.middle_scan_threaded(v, a, s_, t)
        engine.middle_scan_seqs = oracle_lib.middle_scan_seqs_threaded
        try:
            P.find_adapters_at_read_ends(sub, sets, 0, E, 2, 75.0, sc, sink, 4, 1, False, 75.0, 5.0, False, None)
            P.find_adapters_in_read_middles(sub, sets, 0, 90.0, 10, 100, sc, sink, 1, False)
        finally:
            for f, v in saved.items():
                setattr(engine, f, v)

        def dec(r):
            return (r.start_trim_amount, r.end_trim_amount,
                    [(a[0].name,) + tuple(a[1:]) for a in r.start_adapter_alignments],
                    [(a[0].name,) + tuple(a[1:]) for a in r.end_adapter_alignments],
                    sorted(r.middle_adapter_positions), sorted(r.middle_trim_positions), r.middle_hit_str)
        bad = sum(1 for a, b in zip(got, sub) if dec(a) != dec(b))
        checked = {'reads_checked': k, 'mismatches': bad,
                   'recorded_alignments': sum(len(r.start_adapter_alignments) + len(r.end_adapter_alignments)
                                              for r in sub)}
    return {'metric': 'reads/sec through the reference-API phase drivers (NanoporeRead objects)',
            'value': round(n / total, 1), 'unit': 'reads/s', 'steps': args.steps, 'ms_per_step': round(1e3 * total, 2),
            'ms_per_driver': {k: round(1e3 * v / args.steps, 2) for k, v in times.items()},
            'nanopore_read_objects_ms': round(1e3 * build / args.steps, 1),
            # inside the drivers: the library calls (engine.end_decisions -- the windows gathered there --
            # and engine.middle_scan_seqs: host staging, PCIe and the scan)
            'library_call_ms': {k: round(1e3 * v / args.steps, 2) for k, v in eng_t.items()},
            'end_trim_d2h_bytes_per_100k_reads': int(d2h.get('bytes', 0) * 100000 / max(n, 1)),
            'dtype': 'int32', 'data': 'synthetic (seeded ONT-like reads, mean %d bp)' % args.mean_len,
            'config': {'workload': 'porechop_abi.find_matching_adapter_sets (first 10k reads x %d sets) + '
                                   'find_adapters_at_read_ends + find_adapters_in_read_middles on %d NanoporeRead '
                                   'objects x %d adapter sets' % (len([a for a in A.fresh_adapters()
                                                                       if '(full sequence)' not in a.name]), n,
                                                                  len(sets))},
            'parity_spot_check': checked, 'setup_s': round(gen_s, 2)}


def run_host_path(args, L, _lib, buf, s_off, s_len, e_off, e_len, sides, d_sres, d_eres, d_st, d_et, n, n_sa, n_ea,
                  stream, start_adps, end_adps):
    """The headline step from HOST buffers (SURVEY.md §8(d) "hot-path end to end": batched dispatch
    incl. H2D / D2H, no FASTQ parse / write): per step the packed windows (the reads' first and
    last 150 bases, pageable host memory) and their views go up, the tile layout is computed on
    the host, the same kernels run, and the per-read trim amounts come back ('decisions', what the
    file pipeline moves). 'results' = the batch ABI the Python drivers call (pcabi_align_host,
    start and end windows): every alignment's 8 result fields come back over PCIe."""
    vp = ctypes.c_void_p
    sc = SCORING
    dev = {}

    def dbuf(key, nbytes):
        if key not in dev:
            p = vp()
            _lib.check(L.pcabi_dev_malloc(ctypes.byref(p), max(int(nbytes), 16)), 'malloc')
            dev[key] = p
        return dev[key]

    def up(key, arr):
        arr = np.ascontiguousarray(arr)
        p = dbuf(key, arr.nbytes)
        _lib.check(L.pcabi_dev_copy_async(p, arr.ctypes.data_as(vp), arr.nbytes, 0, stream), 'h2d')
        return p

    trims = np.zeros((2, n), np.int32)
    views = ((s_off, s_len), (e_off, e_len))

    def step():
        d_codes = up('codes', buf)
        for k, (sd, (w_off, w_len)) in enumerate(zip(sides, views)):
            toff = np.zeros((n + 255) // 256 + 1, np.int64)
            L.pcabi_tile_layout(w_len.ctypes.data_as(vp), n, toff.ctypes.data_as(vp))
            d_off, d_len, d_toff = up('off%d' % k, w_off), up('len%d' % k, w_len), up('toff%d' % k, toff)
            _lib.check(L.pcabi_tile_windows_dev(d_codes, d_off, d_len, n, d_toff, int(np.diff(toff).max() // 256),
                                                sd['d_tiles'], stream), 'tile')
            mx = int(w_len.max())
            tab, cnt = sd['all']
            if cnt:
                _lib.check(L.pcabi_align_cross_dev(sd['d_tiles'], d_toff, d_len, n, mx, tab, *sc, sd['d_res'],
                                                   sd['stride'], stream), 'align')
        _lib.check(L.pcabi_end_trim_dev(d_sres, n_sa * n, n_sa, d_eres, n_ea * n, n_ea, n, args.end_size, 2, 75.0, 4,
                                        d_st, d_et, None, None, stream), 'end_trim')
        _lib.check(L.pcabi_dev_copy_async(trims[0].ctypes.data_as(vp), d_st, 4 * n, 1, stream), 'd2h')
        _lib.check(L.pcabi_dev_copy_async(trims[1].ctypes.data_as(vp), d_et, 4 * n, 1, stream), 'd2h')
        _lib.check(L.pcabi_stream_sync(stream), 'sync')

    for _ in range(2):
        step()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    dt_dec = (time.perf_counter() - t0) / args.steps
    h2d = buf.nbytes + 2 * (s_off.nbytes + s_len.nbytes) + 2 * 8 * ((n + 255) // 256 + 1)
    # the batch ABI with full results: pcabi_align_host, start and end windows
    from custom_porechop_abi_amd import engine
    res_bytes = 4 * 8 * n * (n_sa + n_ea)
    k_res = max(2, args.steps // 4)
    engine.align((buf, s_off, s_len), start_adps, sc)
    t0 = time.perf_counter()
    for _ in range(k_res):
        engine.align((buf, s_off, s_len), start_adps, sc)
        engine.align((buf, e_off, e_len), end_adps, sc)
    dt_res = (time.perf_counter() - t0) / k_res
    for p in dev.values():
        L.pcabi_dev_free(p)
    return {'decisions': {'value': round(n / dt_dec, 1), 'unit': 'reads/s', 'ms_per_step': round(1e3 * dt_dec, 3),
                          'steps': args.steps, 'h2d_bytes': int(h2d), 'd2h_bytes': 8 * n,
                          'what': 'host windows + views up, tile layout on the host, the headline kernels, '
                                  'trim amounts down (pageable host memory)'},
            'results': {'value': round(n / dt_res, 1), 'unit': 'reads/s', 'ms_per_step': round(1e3 * dt_res, 3),
                        'steps': k_res, 'd2h_bytes': int(res_bytes),
                        'what': 'pcabi_align_host (the Python drivers\' batch ABI) for the start and end windows: '
                                'every alignment\'s 8 int32 result fields back to the host'}}


def run_middle(args, rank, world, dist, torch, L, _lib, A, synth, encode_adapters):
    """BASELINE.json configs[2]: end trim + middle-adapter scan of whole synthetic reads (mean 8 kb)
    against the first 50 adapter sets. One step, inputs resident in HBM:
      pristine read pack -> working copy (the scan masks hits in place)
      start/end windows -> tiles -> k_align -> k_end_trim                (as the headline step)
      pcabi_trim_views_dev: trimmed-read views on the device (no host round trip)
      pcabi_middle_scan_dev: queued rounds on the device -- round 1 from exact k-mer
      seeds (k_seed_scan -> k_seed_expand -> banded k_seed_band -> k_cands -> device plan ->
      chunked candidate DP -> merges), then rounds over the reads that just hit, masked, until
      none hits; the host reads the round counts once per three rounds
    value = reads / step time (all ranks, max over ranks). Also the default bench's 'middle'
    sub-record (N = 1), with the oracle loop over the first --middle-check reads."""
    from custom_porechop_abi_amd.porechop_abi import middle_adapter_list
    vp = ctypes.c_void_p
    sets = [a for a in A.fresh_adapters() if '(full sequence)' not in a.name][:args.sets]
    start_adps = [a.start_sequence[1] for a in sets if a.start_sequence]
    end_adps = [a.end_sequence[1] for a in sets if a.end_sequence]
    mid_adps = [x[1] for x in middle_adapter_list(sets)[0]]
    n, E = args.reads, args.end_size
    t0 = time.time()
    reads = synth.make_reads(n, args.mean_len, seed=12345 + rank)
    lens = np.array([len(r) for r in reads], np.int64)
    offs = np.zeros(n, np.int64)
    offs[1:] = np.cumsum((lens + 3) & ~3)[:-1]
    pack = np.full(int(offs[-1] + lens[-1]) + 64, 4, np.uint8)
    for k, r in enumerate(reads):
        pack[offs[k]:offs[k] + lens[k]] = r
    s_len = np.minimum(lens, E).astype(np.int32)
    e_len = s_len.copy()
    s_off = offs.copy()
    e_off = offs + lens - e_len
    gen_s = time.time() - t0

    def dalloc(nbytes):
        p = vp()
        _lib.check(L.pcabi_dev_malloc(ctypes.byref(p), max(int(nbytes), 16)), 'malloc')
        return p

    def h2d(arr):
        arr = np.ascontiguousarray(arr)
        p = dalloc(arr.nbytes)
        _lib.check(L.pcabi_dev_h2d(p, arr.ctypes.data_as(vp), arr.nbytes), 'h2d')
        return p

    def table(lst):
        c, o, l = encode_adapters(lst)
        t = vp()
        _lib.check(L.pcabi_adapters_create_scored(c.ctypes.data_as(vp), o.ctypes.data_as(vp), l.ctypes.data_as(vp),
                                                  len(lst), *SCORING, ctypes.byref(t)), 'adapters_create')
        return t

    # the reads, resident in HBM for every step: the middle scan leaves them intact (it masks copies
    # of the reads that hit, as the reference masks a copy, nanopore_read.py:225,234)
    d_pack = h2d(pack)
    d_offs, d_lens = h2d(offs), h2d(lens.astype(np.int32))
    n_sa, n_ea = len(start_adps), len(end_adps)
    d_sres, d_eres = dalloc(4 * 8 * n_sa * n), dalloc(4 * 8 * n_ea * n)
    d_st, d_et = dalloc(4 * n), dalloc(4 * n)
    d_toff_mid, d_tlen_mid = dalloc(8 * n), dalloc(4 * n)
    stream = vp()
    _lib.check(L.pcabi_stream_create(ctypes.byref(stream)), 'stream')
    ev = [vp(), vp()]
    for e in ev:
        _lib.check(L.pcabi_event_create(ctypes.byref(e)), 'event')
    sc = SCORING
    sides = []
    for w_off, w_len, adps, d_res in ((s_off, s_len, start_adps, d_sres), (e_off, e_len, end_adps, d_eres)):
        toff = np.zeros((n + 255) // 256 + 1, np.int64)
        nd = L.pcabi_tile_layout(w_len.ctypes.data_as(vp), n, toff.ctypes.data_as(vp))
        sides.append(dict(d_off=h2d(w_off), d_len=h2d(w_len), d_toff=h2d(toff), d_tiles=dalloc(4 * nd),
                          mq=int(np.diff(toff).max() // 256), mx=int(w_len.max()), tab=table(adps), d_res=d_res,
                          stride=len(adps) * n))
    # both read ends' end-trim cross products in one pcabi_align_cross_multi_dev call (grouped
    # launches, as the headline's default schedule); --rest-overlap 0..4: one call per side
    end_regions = _lib.cross_regions([(sd['d_tiles'], sd['d_toff'], sd['d_len'], n, sd['mx'], sd['tab'], sd['d_res'],
                                       sd['stride']) for sd in sides]) if args.rest_overlap == 5 else None
    mid_tab = table(mid_adps)
    scan = vp()
    _lib.check(L.pcabi_scan_create(mid_tab, ctypes.byref(scan)), 'scan_create')
    cap = max(4096, n)
    hits = np.zeros((6, cap), np.int32)
    trims = np.zeros((2, n), np.int32)
    t_len = np.zeros(n, np.int32)
    stats = {}
    ab_name, ab_vals = (args.ab.split('=', 1)[0], args.ab.split('=', 1)[1].split(',')) if args.ab else ('', [])

    def step():
        work = d_pack
        for sd in sides:
            _lib.check(L.pcabi_tile_windows_dev(work, sd['d_off'], sd['d_len'], n, sd['d_toff'], sd['mq'],
                                                sd['d_tiles'], stream), 'tile')
            if end_regions is None:
                _lib.check(L.pcabi_align_cross_dev(sd['d_tiles'], sd['d_toff'], sd['d_len'], n, sd['mx'], sd['tab'],
                                                   *sc, sd['d_res'], sd['stride'], stream), 'align')
        if end_regions is not None:
            _lib.check(L.pcabi_align_cross_multi_dev(end_regions, len(end_regions), *sc, stream, None, None), 'align')
        _lib.check(L.pcabi_end_trim_dev(d_sres, n_sa * n, n_sa, d_eres, n_ea * n, n_ea, n, E, 2, 75.0, 4, d_st, d_et,
                                        None, None, stream), 'end_trim')
        _lib.check(L.pcabi_event_record(ev[0], stream), 'event')
        # NanoporeRead.get_seq_with_start_end_adapters_trimmed (nanopore_read.py:44-49), on the device
        _lib.check(L.pcabi_trim_views_dev(d_offs, d_lens, d_st, d_et, n, d_toff_mid, d_tlen_mid, stream), 'views')
        nh = L.pcabi_middle_scan_dev(scan, work, d_toff_mid, d_tlen_mid, None, n, *sc,
                                     args.middle_threshold, hits.ctypes.data_as(vp), cap, stream)
        if nh < 0:
            _lib.check(int(nh), 'middle_scan')
        _lib.check(L.pcabi_event_record(ev[1], stream), 'event')
        _lib.check(L.pcabi_stream_sync(stream), 'sync')
        ms = ctypes.c_float()
        _lib.check(L.pcabi_event_elapsed_ms(ctypes.byref(ms), ev[0], ev[1]), 'elapsed')
        stats['hits'] = int(nh)
        stats['middle_s'] = stats.get('middle_s', 0.0) + 1e-3 * ms.value
        if ab_name:
            stats.setdefault('ab', {}).setdefault(os.environ.get(ab_name, ''), []).append(round(ms.value, 4))

    for _ in range(args.warmup):
        step()
    _lib.check(L.pcabi_stream_sync(stream), 'sync')
    stats['middle_s'] = 0.0
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize() if torch.cuda.is_available() else None
    t0 = time.perf_counter()
    for k in range(args.steps):
        if ab_name:                        # --ab: the switch alternates between the timed steps
            os.environ[ab_name] = ab_vals[k % 2]
        step()
    L.pcabi_stream_sync(stream)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device='cuda' if args.dist_backend == 'nccl' else 'cpu')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # the last step's trims and views, for the checks and the cell counts (after the timed region)
    _lib.check(L.pcabi_dev_copy_async(trims[0].ctypes.data_as(vp), d_st, 4 * n, 1, stream), 'd2h')
    _lib.check(L.pcabi_dev_copy_async(trims[1].ctypes.data_as(vp), d_et, 4 * n, 1, stream), 'd2h')
    _lib.check(L.pcabi_dev_copy_async(t_len.ctypes.data_as(vp), d_tlen_mid, 4 * n, 1, stream), 'd2h')
    _lib.check(L.pcabi_stream_sync(stream), 'sync')

    # one more step (untimed) with the scan's per-phase profile on: every queued round synchronised
    # on its own, events around its phases, the units they processed -> per-kernel roofline
    phases = None
    if rank == 0:
        prof = np.zeros(26, np.float64)
        timed = dict(stats)
        rc = int(L.pcabi_scan_profile(scan, 1, None, 0))
        if rc >= 0:
            step()
            rc = int(L.pcabi_scan_profile(scan, 0, prof.ctypes.data_as(vp), 26))
        if rc < 0:
            _lib.check(rc, 'profile')
        stats.update(timed)
        phases = middle_phase_roofline(prof)
    checked = None
    if args.check and rank == 0:
        checked = middle_spot_check(reads, trims, hits, stats['hits'], mid_adps, sc, args.middle_threshold,
                                    min(args.middle_check, n))
        checked['input_pack_intact'] = pack_intact(L, _lib, d_pack, pack)
    Lm = np.array([len(x) for x in mid_adps], np.int64)
    cells_mid = int(t_len.astype(np.int64).sum() * Lm.sum())
    cells_end = int(s_len.astype(np.int64).sum() * sum(map(len, start_adps)) +
                    e_len.astype(np.int64).sum() * sum(map(len, end_adps)))
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cpu = cpu_baseline_middle(reads[:max(1, args.cpu_sample // 40)], trims, mid_adps, sc, args.middle_threshold,
                                  args.cpu_threads)
    if rank == 0:
        step_ms = 1e3 * elapsed / args.steps
        value = world * n * args.steps / elapsed
        out = {
            'metric': 'reads/sec trimmed + middle-adapter scan (ONT reads x 50 adapter sets)',
            'value': round(value, 1), 'unit': 'reads/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(step_ms, 3), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'int32',
            'data': 'synthetic (seeded ONT-like reads, SURVEY.md §8d recipe; mean %d bp)' % args.mean_len,
            'config': {'workload': 'end trim + middle scan: %d whole reads/GPU (mean %d bp) x %d adapter sets '
                                   '(%d start, %d end, %d middle adapters), threshold %.0f'
                                   % (n, args.mean_len, len(sets), n_sa, n_ea, len(mid_adps), args.middle_threshold),
                       'reads_per_gpu': n, 'adapter_sets': len(sets), 'scoring': list(sc),
                       'parallelism': 'dp%d (read shards)' % world,
                       'end_trim': ('both read ends in one pcabi_align_cross_multi_dev call' if end_regions is not None
                                    else 'one pcabi_align_cross_dev call per read end'),
                       'inputs': 'one read pack resident in HBM for every step (the scan leaves it intact)'},
            'middle_ms_per_step': round(1e3 * stats['middle_s'] / args.steps, 3),
            'middle_hits_per_step': stats['hits'],
            # --ab: the middle scan's event time per value of the alternated switch (median, all)
            'ab': {ab_name: {v: {'median_ms': float(np.median(x)), 'ms': x} for v, x in stats.get('ab', {}).items()}}
                  if ab_name else None,
            # the middle scan computes only the seeded band cells and its candidates' chunks, not
            # the whole-read cross product: only the end windows' cells are counted as computed
            'cells_per_step': {'end_windows': cells_end, 'middle_cross_product_not_computed': cells_mid},
            'gcups_end_windows': round(cells_end / (step_ms * 1e-3) / 1e9, 1),
            'cpu_baseline': cpu,
            'gpu_vs_cpu': round(value / cpu['value'], 1) if cpu else None,
            'parity_spot_check': checked,
            'middle_phases': phases,
            'setup_s': round(gen_s, 2),
        }
        return out
    return None


def middle_phase_roofline(prof):
    """pcabi_scan_profile's table (include/pcabi.h) -> per-phase time and, for the kernels with an
    algorithmic unit, their roofline (one profiled step: every queued round synchronised on its own):
      k_seed_scan   HBM: every base of the round's reads once (u8 codes) + 16 B per raw seed hit written;
      k_seed_expand HBM: 16 B per raw hit read + 16 B per band task written;
      candidate DP  VALU: cells (chunk columns x adapter rows) x OPS_PER_CELL int32 lane-ops;
      bands         VALU: the pinned classes' band cells (active lane-rows x (2E + 1), counted by the
                    profiled launches) x OPS_PER_CELL over the phase's time (which also holds the
                    edge tasks' band_best launches beside them: a lower bound on the pinned kernels'
                    own rate), and the lanes the passes kept busy.
    k_cands, the plan kernels and the rest (views, merges, masks: latency-bound launches): time only."""
    names = ['k_seed_scan', 'k_seed_expand', 'bands', 'k_cands', 'plan', 'candidate_dp', 'rest']
    ms = {k: float(prof[i]) for i, k in enumerate(names)}
    rounds, reads, bases, raw, b_in, b_edge, dp_tasks, dp_cells = (int(x) for x in prof[7:15])
    out = {'ms': {k: round(v, 4) for k, v in ms.items()}, 'round1_ms': round(float(prof[15]), 4),
           'rounds': rounds, 'reads_scanned': reads,
           'bases_scanned': bases, 'raw_seed_hits': raw, 'band_tasks': {'inside': b_in, 'edge': b_edge},
           'dp_tasks': dp_tasks, 'dp_cells': dp_cells, 'roofline': {}}

    def hbm(nbytes, t_ms, per_unit):
        if t_ms <= 0:
            return None
        gbs = nbytes / (t_ms * 1e-3) / 1e9
        return {'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': round(gbs / HBM_PEAK_GBS, 4), 'algorithmic_bytes': int(nbytes), 'per_unit': per_unit}
    out['roofline']['k_seed_scan'] = hbm(bases + 16 * raw, ms['k_seed_scan'],
                                         '1 B per base scanned + 16 B per raw hit written')
    out['roofline']['k_seed_expand'] = hbm(16 * raw + 16 * (b_in + b_edge), ms['k_seed_expand'],
                                           '16 B per raw hit read + 16 B per band task written')
    if len(prof) >= 26 and ms['bands'] > 0:
        band = [int(x) for x in prof[16:24]]
        es = [int(x) for x in prof[24:26]]
        cells = sum(band[4 * c + 1] * (2 * es[c] + 1) for c in range(2))
        tops = cells * OPS_PER_CELL / (ms['bands'] * 1e-3) / 1e12
        out['roofline']['bands'] = {
            'bound': 'valu', 'achieved': round(tops, 3), 'peak': round(VALU_PEAK_TOPS, 1),
            'unit': 'T int32 lane-ops/s', 'frac': round(tops / VALU_PEAK_TOPS, 4), 'band_cells': cells,
            'per_unit': '%d ops per band cell; cells = active lane-rows x (2E + 1)' % OPS_PER_CELL,
            'classes': [{'E': es[c], 'lane_rows_issued': band[4 * c], 'lane_rows_active': band[4 * c + 1],
                         'lanes_busy': round(band[4 * c + 1] / max(1, band[4 * c]), 3), 'tasks': band[4 * c + 2],
                         'rows_per_task': round(band[4 * c + 1] / max(1, band[4 * c + 2]), 2),
                         'passes': band[4 * c + 3]} for c in range(2)]}
    if ms['candidate_dp'] > 0:
        tops = dp_cells * OPS_PER_CELL / (ms['candidate_dp'] * 1e-3) / 1e12
        out['roofline']['candidate_dp'] = {'bound': 'valu', 'achieved': round(tops, 3),
                                           'peak': round(VALU_PEAK_TOPS, 1), 'unit': 'T int32 lane-ops/s',
                                           'frac': round(tops / VALU_PEAK_TOPS, 4),
                                           'per_unit': '%d ops per cell (SURVEY.md §8d)' % OPS_PER_CELL}
    return out


def run_compat(args, rank, world, dist, torch, L, _lib):
    """Ab-initio clustering link test (consensus.py:72-100 all_vs_all_matrix over
    compatibility.so::check_compatibility): every pair of --compat-seqs adapter-like sequences
    (20-60 bp, families of mutated variants, the shape the k-mer counting feeds it). One step =
    the whole flag matrix through pcabi_compat_all_vs_all_host (host buffers in, the n x n int32
    matrix out; every sequence against every sequence as one tiled cross product).
    value = pairs / s; cpu_baseline = the reference's own compatibility.so on a bounded sample of
    the same pairs, called like consensus.py does (one Python loop, one thread)."""
    from custom_porechop_abi_amd import consensus
    rng = np.random.default_rng(77 + rank)
    letters = np.array(list('ACGT'))
    seqs = []
    while len(seqs) < args.compat_seqs:
        base = ''.join(letters[rng.integers(0, 4, int(rng.integers(20, 61)))])
        for _ in range(int(rng.integers(1, 12))):
            s = list(base)
            for _ in range(int(rng.integers(0, 4))):
                k = int(rng.integers(0, len(s)))
                s[k] = letters[rng.integers(0, 4)]
            a = int(rng.integers(0, 4))
            seqs.append(''.join(s)[a:])
    seqs = seqs[:args.compat_seqs]
    n = len(seqs)
    iu, ju = np.triu_indices(n, 1)
    iu, ju = iu.astype(np.int32), ju.astype(np.int32)
    for _ in range(args.warmup):
        consensus.all_vs_all_flags(seqs, device=args.local_device)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        mat = consensus.all_vs_all_flags(seqs, device=args.local_device)
    elapsed = time.perf_counter() - t0
    flags = mat[iu, ju]
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device='cuda' if args.dist_backend == 'nccl' else 'cpu')
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    n_pairs = len(iu)
    checked = None
    cpu = None
    sample = np.random.default_rng(5).choice(n_pairs, size=min(n_pairs, 4000), replace=False)
    if rank == 0 and args.check:
        from tests import oracle_lib
        olib = oracle_lib.load()
        olib.pcabi_oracle_compat.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        olib.pcabi_oracle_compat.restype = ctypes.c_int
        bad = sum(int(olib.pcabi_oracle_compat(seqs[iu[k]].encode(), seqs[ju[k]].encode()) != flags[k])
                  for k in sample.tolist())
        checked = {'pairs_checked': int(len(sample)), 'mismatches': bad,
                   'flags_0_1_2': [int((flags == v).sum()) for v in range(3)]}
    ref = os.path.join(ROOT, 'oracle', '_ref', 'compatibility.so')
    if rank == 0 and world == 1 and args.cpu_sample > 0 and os.path.isfile(ref):
        clib = ctypes.CDLL(ref)
        clib.check_compatibility.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        clib.check_compatibility.restype = ctypes.c_int
        enc = [s.encode('utf-8') for s in seqs]
        k = min(n_pairs, args.cpu_sample * 30)
        t1 = time.perf_counter()
        for t in range(k):
            clib.check_compatibility(enc[iu[t]], enc[ju[t]])
        dt = time.perf_counter() - t1
        cpu = {'value': round(k / dt, 1), 'unit': 'pairs/s', 'cores': 1, 'kind': 'reference',
               'sample': '%d pairs of the same set, %.1f s, the reference compatibility.so called from one Python '
                         'loop as consensus.py:88-99 does' % (k, dt)}
    if rank == 0:
        value = world * n_pairs * args.steps / elapsed
        out = {'metric': 'check_compatibility pairs/sec (ab-initio all-vs-all link test)',
               'value': round(value, 1), 'unit': 'pairs/s', 'n_gpus': world, 'steps': args.steps,
               'warmup': args.warmup, 'ms_per_step': round(1e3 * elapsed / args.steps, 3), 'higher_is_better': True,
               'scaling': 'weak', 'vs_baseline': None, 'dtype': 'int32',
               'data': 'synthetic adapter-like sequences (20-60 bp families of mutated variants)',
               'config': {'workload': 'compat: all %d pairs of %d sequences (consensus.all_vs_all_flags), scoring '
                                      '2/-1/-1 linear, flags on the device, host buffers in / out' % (n_pairs, n),
                          'parallelism': 'dp%d' % world},
               'cpu_baseline': cpu, 'gpu_vs_cpu': round(value / cpu['value'], 1) if cpu else None,
               'parity_spot_check': checked}
        return out
    return None


def run_kmer(args, rank, world, dist, torch, L, _lib, synth):
    """The ab-initio k-mer counter (approx_counter.cpp, run by abinitio.py:392-440) with the
    reference's config (ab_initio.config: k 16, sl 100, sn 40000, lim 500, lc 1.0) on a
    synthetic FASTA of 40k reads: one step = one run of the program minus the file parse (the
    reads are already loaded): both read ends sampled, exact counts on the GPU (k_kmer_keys,
    radix sort, RLE, then sorted by count so only the k-mers the cut can keep leave the device),
    the 500 most frequent, approximate counts at <= 2 errors on the GPU
    (k_kmer_approx: 500 k-mers x 40k sequences of ~100 bp), ordering and export.
    cpu_baseline: the reference program itself (oracle/_ref/approx_counter, OpenMP on the host
    cores) on the same file, its wall time minus nothing (it parses the file too)."""
    import subprocess
    import tempfile
    from custom_porechop_abi_amd import approx_counter as AC, misc
    n = 40000
    tmp = tempfile.mkdtemp(prefix='pcabi_kmer_')
    path = os.path.join(tmp, 'reads.fasta')
    reads = synth.make_reads(n, 1500, seed=31 + rank)
    letters = np.frombuffer(b'ACGTN', np.uint8)
    with open(path, 'wb') as f:
        for k, r in enumerate(reads):
            f.write(b'>r%d\n' % k + letters[r].tobytes() + b'\n')
    batch = misc.load_batch(path)
    K, SL, LIM = 16, 100, 500
    lct = AC.adjust_threshold(1.0, 16, K)

    def step():
        out = []
        for bottom in (False, True):
            smp = AC.sample_sequences(batch, n, SL, bottom, seed=0)
            km, cn = AC.count_kmers_top(smp, K, lct, (), top=LIM, device=args.local_device)
            tk, tc = AC.most_frequent(km, cn, LIM, K)
            err = AC.error_count(smp, tk, K, device=args.local_device)
            out.append(AC.most_frequent(tk, err, LIM, K))
        return out

    for _ in range(args.warmup):
        step()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    elapsed = time.perf_counter() - t0
    cpu = None
    ref = os.path.join(ROOT, 'oracle', '_ref', 'approx_counter')
    checked = None
    if rank == 0 and args.cpu_sample > 0 and os.path.isfile(ref):
        nthr = args.cpu_threads or max(1, min(16, len(os.sched_getaffinity(0))))
        t1 = time.perf_counter()
        subprocess.run([ref, path, '-o', os.path.join(tmp, 'ref'), '-k', str(K), '-sl', str(SL), '-sn', str(n),
                        '-lim', str(LIM), '-nt', str(nthr), '-v', '0'], check=True, stdout=subprocess.DEVNULL,
                       stderr=subprocess.DEVNULL)
        dt = time.perf_counter() - t1
        cpu = {'value': round(1.0 / dt, 4), 'unit': 'runs/s', 'cores': nthr, 'kind': 'reference',
               'sample': 'one full run of the reference approx_counter (file parse included) on the same %d-read '
                         'file, %.2f s' % (n, dt)}
        # every read is sampled (sn = n), so the reference's output is deterministic: compare
        got = {}
        for which, (tk, tc) in zip(('start', 'end'), res):
            got[which] = ''.join('%s\t%d\n' % (AC.kmer_to_str(v, K), c) for v, c in zip(tk.tolist(), tc.tolist()))
        same = all(open(os.path.join(tmp, 'ref_0.' + w)).read() == got[w] for w in ('start', 'end'))
        checked = {'identical_to_reference_outputs': same}
    shutil_rm = __import__('shutil').rmtree
    shutil_rm(tmp, ignore_errors=True)
    if rank == 0:
        value = world * args.steps / elapsed
        out = {'metric': 'approx_counter runs/sec (ab-initio k-mer counts, 40k reads, k 16, both ends)',
               'value': round(value, 3), 'unit': 'runs/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
               'ms_per_step': round(1e3 * elapsed / args.steps, 2), 'higher_is_better': True, 'scaling': 'weak',
               'vs_baseline': None, 'dtype': 'int32 / uint64',
               'data': 'synthetic reads (SURVEY.md §8d recipe, mean 1.5 kb)',
               'config': {'workload': 'kmer: sample 40000 read starts and ends (100 bp), exact 16-mer counts, top 500, '
                                      'approximate counts at <= 2 edits, ordering (reference ab_initio.config)',
                          'parallelism': 'dp%d' % world},
               'cpu_baseline': cpu, 'gpu_vs_cpu': round(value / cpu['value'], 1) if cpu else None,
               'parity_spot_check': checked}
        return out
    return None


def write_probe(path, nbytes, repeat):
    """The output file system's write ceiling for the e2e output: nbytes from one contiguous,
    already faulted-in buffer through write() calls of 256 MB (the page-cache copy the trimmed-read
    writer also pays). 'burst': one fresh file of nbytes, best of three; 'sustained': `repeat` fresh
    files of nbytes back to back, as the timed e2e steps write them (dirty-page writeback and
    throttling included); 'rewrite': `repeat` writes of one path, each truncating the last (what the
    steps did through r05's first records: the truncation frees the previous file's cached pages).
    The e2e writer's busy time is compared against these."""
    buf = np.full(min(nbytes, 256 << 20), 65, np.uint8)
    mv = memoryview(buf)

    def one(p):
        fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        left = nbytes
        while left > 0:
            left -= os.write(fd, mv[:min(left, len(buf))])
        os.close(fd)

    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        one(path)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
        os.remove(path)
    t0 = time.perf_counter()
    for k in range(repeat):
        one('%s.%d' % (path, k))
    sus = (time.perf_counter() - t0) / repeat
    for k in range(repeat):
        os.remove('%s.%d' % (path, k))
    t0 = time.perf_counter()
    for _ in range(repeat):
        one(path)
    rew = (time.perf_counter() - t0) / repeat
    os.remove(path)
    return {'bytes': int(nbytes), 'burst_ms': round(1e3 * best, 2), 'burst_GB_per_s': round(nbytes / best / 1e9, 2),
            'sustained_ms': round(1e3 * sus, 2), 'sustained_GB_per_s': round(nbytes / sus / 1e9, 2),
            'sustained_files': repeat, 'rewrite_ms': round(1e3 * rew, 2),
            'rewrite_GB_per_s': round(nbytes / rew / 1e9, 2)}


def write_fastq(path, reads, seed):
    """Synthetic reads (Dna5 code arrays) as a FASTQ file with ONT-like headers and qualities."""
    rng = np.random.default_rng(seed)
    letters = np.frombuffer(b'ACGTN', np.uint8)
    with open(path, 'wb') as f:
        for k, r in enumerate(reads):
            q = (rng.integers(5, 40, len(r)) + 33).astype(np.uint8).tobytes()
            f.write(b'@read%d runid=synthetic ch=%d\n' % (k, k % 512) + letters[r].tobytes() + b'\n+\n' + q + b'\n')


def run_e2e(args, rank, world, dist, torch, L, _lib, A, synth, encode_adapters):
    """The CLI path end to end, file to file (porechop_abi.py:41-131 with the reference's defaults:
    end_size 150, end_threshold 75, extra_end_trim 2, min_trim_size 4, middle_threshold 90, extra
    middle trim 10 / 100, min_split_read_size 1000, the fork's start-and-end filter, FASTQ out),
    for the first 50 adapter sets (adapter-set discovery is excluded: it runs once on the check
    reads). One step:
      native parse of the FASTQ (pcabi_fastx_load) -> H2D of the packed codes + window views
      -> k_tile_windows / k_align / k_end_trim -> trims D2H -> middle scan of the trimmed reads
      (pcabi_middle_scan_dev) -> middle cut ranges (host, vectorised) -> native trimmed FASTQ
      writer (pcabi_reads_write) for the reads with start and end adapters.
    value = reads / step time; the breakdown says where the time goes."""
    from custom_porechop_abi_amd import misc
    from custom_porechop_abi_amd.porechop_abi import middle_adapter_list
    sets = [a for a in A.fresh_adapters() if '(full sequence)' not in a.name][:args.sets]
    start_adps = [a.start_sequence[1] for a in sets if a.start_sequence]
    end_adps = [a.end_sequence[1] for a in sets if a.end_sequence]
    mid_adps = [x[1] for x in middle_adapter_list(sets)[0]]
    n, E = args.reads, args.end_size
    tmp = os.environ.get('TMPDIR', '/tmp')
    in_path = os.path.join(tmp, 'pcabi_e2e_%d_%d.fastq' % (os.getpid(), rank))
    out_path = os.path.join(tmp, 'pcabi_e2e_%d_%d.out.fastq' % (os.getpid(), rank))
    t0 = time.time()
    reads = synth.make_reads(n, args.mean_len, seed=12345 + rank)
    write_fastq(in_path, reads, 99 + rank)
    in_bytes = os.path.getsize(in_path)
    k_cpu = max(1, args.cpu_sample // 80) if rank == 0 and world == 1 and args.cpu_sample > 0 else 0
    sample = reads[:k_cpu]
    del reads
    gen_s = time.time() - t0

    from custom_porechop_abi_amd.pipeline import FileTrimmer
    sc = SCORING
    n_sa, n_ea = len(start_adps), len(end_adps)
    ft = FileTrimmer(sets, sc, E, 75.0, 2, 4, args.middle_threshold, 10, 100, 1000, device=args.local_device)
    last = {}
    outs, done_outs = [], []

    def step():
        # every step writes a fresh output file, as a CLI run does: re-truncating one 1.4 GB file
        # each step made the writer also free the previous step's ~350 k cached pages (~150 ms per
        # step on the GPU box: bench write_probe, r04-r05 'sustained' vs 'burst'); the files are
        # removed after the timed steps
        ft.times = {}
        outs.append('%s.%d' % (out_path, len(done_outs) + len(outs)))
        last.update(ft.trim_file(in_path, outs[-1], 'fastq', max_reads=min(n, args.e2e_batch)))
        if getattr(ft, 'trace', None):
            t0 = min(x[2] for x in ft.trace)
            last['timeline'] = [[s_, k_, round(1e3 * (a_ - t0), 2), round(1e3 * (b_ - t0), 2)]
                                for s_, k_, a_, b_ in ft.trace]
        return dict(ft.times)

    for _ in range(args.warmup):
        step()
    for p in outs:                        # the warm-up's output, before the timed steps
        os.remove(p)
    done_outs += outs
    del outs[:]
    if dist is not None:
        dist.barrier()
    acc = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for k, v in step().items():
            acc[k] = acc.get(k, 0.0) + v
    elapsed = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device='cuda' if args.dist_backend == 'nccl' else 'cpu')
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    out_path = outs[-1]
    out_bytes = os.path.getsize(out_path)
    for p in outs[:-1]:
        os.remove(p)
    probe = write_probe(out_path + '.probe', out_bytes, args.steps + args.warmup) if rank == 0 else None
    checked = None
    if args.check and rank == 0:
        # the written bytes of the first reads against the reference's output rule on decisions the
        # ORACLE made: the reference-API drivers (porechop_abi.find_adapters_at_read_ends /
        # find_adapters_in_read_middles) with the oracle standing in for the kernels, the fork's
        # filter and NanoporeRead.get_fastq (nanopore_read.py:106-156, porechop_abi.py:535-668)
        got = misc.load_batch(out_path)
        checked = {'records_written': int(got.n), 'reads_in': last['reads_in'], 'reads_kept': last['reads_kept']}
        checked.update(e2e_output_check(in_path, out_path, sets, sc, E, args.middle_threshold,
                                        min(args.e2e_check, n)))
    for p in (in_path, out_path):
        try:
            os.remove(p)
        except OSError:
            pass
    cpu = None
    if k_cpu:
        # the reference's alignment work for the same reads (every end window x every adapter,
        # then the whole-read middle loop), on a bounded sample; its FASTQ parse and write are not
        # timed, so this is a lower bound on the reference CLI's time per read
        ce = cpu_baseline(sample, sets, E, sc, args.cpu_threads)
        cm = cpu_baseline_middle(sample, np.zeros((2, len(sample)), np.int32), mid_adps, sc, args.middle_threshold,
                                 args.cpu_threads)
        v = 1.0 / (1.0 / ce['value'] + 1.0 / cm['value'])
        cpu = {'value': round(v, 3), 'unit': 'reads/s', 'cores': ce['cores'], 'kind': ce['kind'],
               'sample': 'alignment work only (parse / write not timed): %s; then %s' % (ce['sample'], cm['sample'])}
    if rank == 0:
        step_s = elapsed / args.steps
        value = world * n * args.steps / elapsed
        out = {
            'metric': 'reads/sec end to end, FASTQ file -> trimmed FASTQ file (ONT reads x 50 adapter sets)',
            'value': round(value, 1), 'unit': 'reads/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(1e3 * step_s, 3), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'int32',
            'data': 'synthetic FASTQ (seeded ONT-like reads, SURVEY.md §8d recipe; mean %d bp)' % args.mean_len,
            'config': {'workload': 'e2e: %d reads/GPU FASTQ (%.0f MB) -> parse -> end trim (%d start + %d end '
                                   'adapters) -> middle scan (%d adapters, threshold %.0f) -> fork filter -> '
                                   'trimmed FASTQ' % (n, in_bytes / 1e6, n_sa, n_ea, len(mid_adps),
                                                      args.middle_threshold),
                       'reads_per_gpu': n, 'batch_reads': min(n, args.e2e_batch), 'adapter_sets': len(sets),
                       'scoring': list(sc), 'parallelism': 'dp%d (read shards)' % world},
            # 'read' / 'write' are the reader / writer threads' busy times, overlapped with the rest:
            # not in 'other'
            'breakdown_ms_per_step': dict({k: round(1e3 * v / args.steps, 2) for k, v in acc.items()},
                                          other=round(1e3 * (step_s - sum(v for k, v in acc.items()
                                                                          if k not in ('read', 'write'))
                                                             / args.steps), 2)),
            # the step against its slowest stage (steady state: the stages overlap fully)
            'step_vs_slowest_stage': round(step_s / max(1e-9, max(acc.get('read', 0.0), acc.get('write', 0.0),
                                                                  acc.get('end_trim', 0.0) + acc.get('middle', 0.0))
                                                        / args.steps), 3),
            'input_MB_per_s': round(in_bytes / step_s / 1e6, 1),
            'output_bytes': out_bytes,
            # the file system's own ceiling for this output: the same byte count from one buffer
            'write_probe': probe,
            'cpu_baseline': cpu,
            'gpu_vs_cpu': round(value / cpu['value'], 1) if cpu else None,
            'parity_spot_check': checked,
            'setup_s': round(gen_s, 2),
        }
        if 'timeline' in last:            # PCABI_PIPE_TRACE=1: the last step's (stage, batch, ms, ms)
            out['timeline'] = last['timeline']
        return out
    return None


def e2e_output_check(in_path, out_path, sets, sc, end_size, middle_threshold, k):
    """The first k input reads through the reference's drivers and writer with the oracle as the
    alignment engine (tests/oracle_lib: CPU restatements pinned to the reference's own build, the
    kernels swapped out for the duration), against the same reads' records at the head of the
    pipeline's output file, byte for byte."""
    import contextlib
    import io
    from custom_porechop_abi_amd import engine, misc, porechop_abi as P
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    from tests import oracle_lib
    b = misc.load_batch(in_path)
    reads = [NanoporeRead(b.name(i), b.sequence(i), b.quals(i)) for i in range(min(k, b.n))]
    swaps = {'align': oracle_lib.align_windows, 'end_decisions': oracle_lib.end_decisions_windows,
             'first_hits': oracle_lib.first_hits_windows,
             'middle_scan': lambda w, a, s_, t, device=0: oracle_lib.middle_scan_threaded(w, a, s_, t),
             'middle_scan_seqs': oracle_lib.middle_scan_seqs_threaded}
    saved = {name: getattr(engine, name) for name in swaps}
    t0 = time.perf_counter()
    try:
        for name, fn in swaps.items():
            setattr(engine, name, fn)
        sink = io.StringIO()
        with contextlib.redirect_stdout(sink):
            P.find_adapters_at_read_ends(reads, sets, 0, end_size, 2, 75.0, sc, sink, 4, 1, False, 75.0, 5.0, False,
                                         None)
            P.find_adapters_in_read_middles(reads, sets, 0, middle_threshold, 10, 100, sc, sink, 1, False)
    finally:
        for name, fn in saved.items():
            setattr(engine, name, fn)
    want = ''.join(r.get_fastq(1000, False) for r in reads if r.adapters_found()).encode()
    with open(out_path, 'rb') as f:
        head = f.read(len(want))
    return {'oracle_reads_checked': len(reads), 'oracle_bytes_compared': len(want), 'output_identical': head == want,
            'oracle_s': round(time.perf_counter() - t0, 2)}


def pack_intact(L, _lib, d_pack, pack):
    """The read pack on the device after the timed steps is byte-identical to the one uploaded:
    the middle scan masks copies, not the caller's reads (nanopore_read.py:225,234)."""
    back = np.empty_like(pack)
    _lib.check(L.pcabi_dev_d2h(back.ctypes.data_as(ctypes.c_void_p), d_pack, pack.nbytes), 'd2h')
    return bool(np.array_equal(back, pack))


def middle_spot_check(reads, trims, hits, n_hits, mid_adps, sc, thr, k):
    """First k reads: trimmed sequence (from the device's trim amounts) through the reference's
    middle loop restated on the oracle (tests/oracle_lib.middle_scan_threaded: the C loop, reads
    over the host threads) vs the device hits, every round."""
    from tests import oracle_lib
    from custom_porechop_abi_amd import synth
    from custom_porechop_abi_amd.engine import SeqPack
    seqs = []
    for i in range(k):
        r = synth.codes_to_str(reads[i])
        st, et = int(trims[0][i]), int(trims[1][i])
        seqs.append(r[st:len(r) - et] if st or et else r)
    pack = SeqPack(seqs)
    exp = oracle_lib.middle_scan_threaded(pack.views(np.zeros(k, np.int64), pack.lengths), mid_adps, sc, thr)
    got = hits[:, :min(n_hits, hits.shape[1])]
    got = got[:, got[0] < k]
    og = np.lexsort((np.arange(got.shape[1]), got[0]))
    oe = np.lexsort((np.arange(exp.shape[1]), exp[0]))
    same = got.shape == exp.shape and bool(np.array_equal(got[:, og], exp[:, oe]))
    return {'reads_checked': k, 'hits': int(exp.shape[1]), 'identical': same}


def cpu_baseline_middle(reads, trims, mid_adps, sc, thr, threads):
    """The reference CPU path for the middle scan on a bounded sample: each trimmed read's loop of
    nanopore_read.find_middle_adapters (nanopore_read.py:236-246) through the reference's own
    adapterAlignment (oracle/_ref/cpp_functions.so), reads fanned out over a ThreadPool."""
    from multiprocessing.dummy import Pool as ThreadPool
    from custom_porechop_abi_amd import synth
    ref = os.path.join(ROOT, 'oracle', '_ref', 'cpp_functions.so')
    kind = 'reference'
    if os.path.isfile(ref):
        lib = ctypes.CDLL(ref)
        fn, fr = lib.adapterAlignment, lib.freeCString
    else:
        from tests import oracle_lib
        lib = oracle_lib.load()
        fn, fr = lib.pcabi_oracle_adapter_alignment, lib.pcabi_oracle_free
        kind = 'port'
    fn.argtypes = [ctypes.c_char_p, ctypes.c_char_p] + [ctypes.c_int] * 4
    fn.restype = ctypes.c_void_p
    fr.argtypes = [ctypes.c_void_p]
    seqs = []
    for i, r in enumerate(reads):
        s = synth.codes_to_str(r)
        st, et = int(trims[0][i]), int(trims[1][i])
        seqs.append(s[st:len(s) - et] if st or et else s)
    adps = [a.encode() for a in mid_adps]

    def one(seq):
        masked = seq
        n = 0
        for a in adps:
            while True:
                p = fn(masked.encode(), a, *sc)
                t = ctypes.cast(p, ctypes.c_char_p).value.decode()
                fr(p)
                f = t.split(',')
                if int(f[0]) == -1 or float(f[6]) < thr:
                    break
                rs, re_ = int(f[0]), int(f[1]) + 1
                masked = masked[:rs] + '-' * (re_ - rs) + masked[re_:]
                n += 1
        return n

    threads = threads or min(16, len(os.sched_getaffinity(0)))
    t0 = time.perf_counter()
    with ThreadPool(threads) as pool:
        pool.map(one, seqs)
    wall = time.perf_counter() - t0
    return {'value': round(len(seqs) / wall, 3), 'unit': 'reads/s', 'cores': threads, 'kind': kind,
            'sample': '%d whole trimmed reads x %d middle adapters (find_middle_adapters loop), %.1f s wall, '
                      'ThreadPool(%d) over ctypes adapterAlignment' % (len(seqs), len(adps), wall, threads)}


def spot_check(L, _lib, d_sres, d_eres, d_st, d_et, s_stride, e_stride, n, n_sa, n_ea, reads, start_adps,
               end_adps, E, k, sc, bc=None, bc_sets=None):
    """Compare the first k reads' raw alignment fields with the oracle (and, for the barcodes
    workload, the device barcode calls with NanoporeRead.determine_barcode over the oracle's
    identities, dicts filled in set order as find_start_trim / find_end_trim do)."""
    from tests import oracle_lib
    from custom_porechop_abi_amd import synth
    vp = ctypes.c_void_p
    sres = np.empty((8, s_stride), np.int32)
    eres = np.empty((8, e_stride), np.int32)
    _lib.check(L.pcabi_dev_d2h(sres.ctypes.data_as(vp), d_sres, sres.nbytes), 'd2h')
    _lib.check(L.pcabi_dev_d2h(eres.ctypes.data_as(vp), d_eres, eres.nbytes), 'd2h')
    heads, tails = [], []
    for r in reads[:k]:
        if isinstance(r, tuple):
            heads.append(synth.codes_to_str(r[0]))
            tails.append(synth.codes_to_str(r[1]))
        else:
            heads.append(synth.codes_to_str(r[:E]))
            tails.append(synth.codes_to_str(r[-E:]))
    bad = 0
    exps = []
    for wins, adps, res, nad in ((heads, start_adps, sres, n_sa), (tails, end_adps, eres, n_ea)):
        pr = np.tile(np.arange(k), nad)
        pa = np.repeat(np.arange(nad), k)
        exp = oracle_lib.align_many(wins, adps, (pr, pa), sc)
        got = res.reshape(8, nad, n)[:, :, :k].reshape(8, -1)
        bad += int(np.sum(np.any(got != exp, axis=0)))
        exps.append(exp)
    out = {'pairs_checked': int(k * (n_sa + n_ea)), 'mismatches': bad}
    if bc is not None:
        from custom_porechop_abi_amd.nanopore_read import NanoporeRead
        call = np.empty(n, np.int32)
        _lib.check(L.pcabi_dev_d2h(call.ctypes.data_as(vp), bc['d_call'], call.nbytes), 'd2h')
        start_sets, end_sets, pos_s, pos_e = bc_sets
        bad_calls = 0
        for r in range(k):
            read = NanoporeRead('r', 'A', '')
            for sets_, pos, exp, d in ((start_sets, pos_s, exps[0], read.start_barcode_scores),
                                       (end_sets, pos_e, exps[1], read.end_barcode_scores)):
                for j, a in enumerate(sets_):
                    if a.is_barcode() and a.barcode_direction() == bc['dir']:
                        i = int(pos[j]) * k + r
                        d[a.get_barcode_name()] = 0.0 if exp[0, i] == -1 else float('%f' % (100.0 * exp[5, i] / exp[7, i]))
            read.determine_barcode(75.0, 5.0, False)
            bad_calls += int(read.barcode_call != bc['names'].get(int(call[r]), 'none'))
        out.update({'barcode_calls_checked': k, 'barcode_call_mismatches': bad_calls,
                    'barcoded_fraction': round(float(np.mean(call != -1)), 4)})
    return out


def cpu_baseline(reads, sets, E, sc, threads):
    """The reference CPU path on a bounded sample: for every read, every adapter set's start and
    end window through the reference's own adapterAlignment (oracle/_ref/cpp_functions.so, built
    from /root/reference sources by oracle/Makefile) called via ctypes exactly as
    porechop_abi/cpp_function_wrappers.py does, fanned out over a ThreadPool like
    porechop_abi.py:418-432. Falls back to the oracle port if the reference build is absent."""
    from multiprocessing.dummy import Pool as ThreadPool
    from custom_porechop_abi_amd import synth
    ref = os.path.join(ROOT, 'oracle', '_ref', 'cpp_functions.so')
    kind = 'reference'
    if os.path.isfile(ref):
        lib = ctypes.CDLL(ref)
        fn, fr = lib.adapterAlignment, lib.freeCString
    else:
        from tests import oracle_lib
        lib = oracle_lib.load()
        fn, fr = lib.pcabi_oracle_adapter_alignment, lib.pcabi_oracle_free
        kind = 'port'
    fn.argtypes = [ctypes.c_char_p, ctypes.c_char_p] + [ctypes.c_int] * 4
    fn.restype = ctypes.c_void_p
    fr.argtypes = [ctypes.c_void_p]
    jobs = []
    for r in reads:
        if isinstance(r, tuple):
            h, t = synth.codes_to_str(r[0]), synth.codes_to_str(r[1])
        else:
            h, t = synth.codes_to_str(r[:E]), synth.codes_to_str(r[-E:])
        jobs.append((h.encode(), t.encode()))
    starts = [a.start_sequence[1].encode() for a in sets if a.start_sequence]
    ends = [a.end_sequence[1].encode() for a in sets if a.end_sequence]

    def one(job):
        h, t = job
        best = 0
        for a in starts:
            p = fn(h, a, *sc)
            s = ctypes.cast(p, ctypes.c_char_p).value
            fr(p)
            best += len(s)
        for a in ends:
            p = fn(t, a, *sc)
            s = ctypes.cast(p, ctypes.c_char_p).value
            fr(p)
            best += len(s)
        return best

    avail = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else os.cpu_count()
    nthr = threads or max(1, min(16, avail))
    t0 = time.perf_counter()
    with ThreadPool(nthr) as pool:
        list(pool.imap(one, jobs, chunksize=4))
    dt = time.perf_counter() - t0
    return {'value': round(len(jobs) / dt, 2), 'unit': 'reads/s', 'cores': nthr, 'kind': kind,
            'sample': '%d reads x %d+%d adapters (%d alignments), %.1f s wall, ThreadPool(%d) over ctypes '
                      'adapterAlignment' % (len(jobs), len(starts), len(ends), len(jobs) * (len(starts) + len(ends)),
                                            dt, nthr)}


def load_traffic():
    """HBM bytes per step from the committed rocprofv3 PMC pass (profiles/), if present."""
    p = os.path.join(ROOT, 'profiles', 'traffic.json')
    if os.path.isfile(p):
        try:
            return json.load(open(p))
        except Exception:
            return None
    return None


if __name__ == '__main__':
    main()

#!/bin/bash
# GPU-box script for round 6: the stages named in STAGES (default "replay"), each under its own time
# limit, stopping at the first failure. Output under gpurun_out/$TAG.
#   replay   tools/replay_k24 (dominant-kernel replays + issue-rate probes, in-kernel clock)
#   tests    pytest -m gpu (TESTS, default the whole suite)
#   head     the headline bench line without sub-records (BENCH_ARGS)
#   bench    the default bench line (every sub-record)
#   prof     rocprofv3 kernel-trace summaries: headline, reference job, middle 8 kb / 20 kb
#   mid      bench --workload middle at 8 kb and 20 kb (MID_ARGS)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06}
mkdir -p $OUT
cd $R
for st in ${STAGES:-replay}; do
  case $st in
    replay)
      timeout -k 10 180 tools/replay_k24 ${REPS:-20} > $OUT/replay.jsonl 2> $OUT/replay.err || { echo "replay failed rc=$?"; tail -5 $OUT/replay.err; exit 1; }
      cut -c1-330 $OUT/replay.jsonl ;;
    tests)
      timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu ${TESTS:-tests} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest_gpu.log; exit 1; }
      tail -2 $OUT/pytest_gpu.log ;;
    head)
      timeout -k 10 300 python bench.py --sub 0 ${BENCH_ARGS:-} > $OUT/bench_head.json 2> $OUT/bench_head.err || { echo "bench head failed rc=$?"; tail -20 $OUT/bench_head.err; exit 1; }
      cut -c1-700 $OUT/bench_head.json ;;
    bench)
      timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench_default.err; exit 1; }
      python - $OUT/bench_default.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(json.dumps({k: d.get(k) for k in ('value', 'ms_per_step', 'roofline')}))
for k in ('reference_job', 'middle', 'middle_20kb', 'per_side_schedule', 'barcodes', 'config2_10k_119sets', 'drivers', 'check_phase', 'e2e'):
    v = d.get(k) or {}
    print(k, json.dumps({x: v.get(x) for x in ('value', 'ms_per_step', 'middle_ms_per_step', 'ms_per_phase', 'error', 'parity_spot_check', 'step_vs_slowest_stage')})[:900])
PY
      ;;
    mid)
      for L in 8000 20000; do
        timeout -k 10 300 python bench.py --workload middle --mean-len $L ${MID_ARGS:-} > $OUT/mid_$L.json 2> $OUT/mid_$L.err || { echo "mid $L failed rc=$?"; tail -20 $OUT/mid_$L.err; exit 1; }
        python -c "import json,sys; d=json.load(open(sys.argv[1])); print($L, d.get('ms_per_step'), json.dumps(d.get('middle_phases', {}))[:1500])" $OUT/mid_$L.json
      done ;;
    prof)
      export TMPDIR=/tmp
      ( cd /tmp &&
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_head -o run -- python3 $R/bench.py --sub 0 --steps 5 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_head.json 2> $OUT/prof_head.err &&
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_rj -o run -- python3 $R/bench.py --only-subs reference_job --steps 3 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_rj.json 2> $OUT/prof_rj.err &&
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mid8 -o run -- python3 $R/bench.py --workload middle --steps 3 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_mid8.json 2> $OUT/prof_mid8.err &&
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mid20 -o run -- python3 $R/bench.py --workload middle --mean-len 20000 --steps 3 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_mid20.json 2> $OUT/prof_mid20.err ) || { echo "rocprof failed rc=$?"; exit 1; }
      head -12 $OUT/prof_head/run_kernel_stats.csv | cut -d, -f1-4 ;;
    poison)
      timeout -k 10 400 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py -k poisoned > $OUT/poison.log 2>&1 || { echo "poisoned test failed rc=$?"; tail -30 $OUT/poison.log; exit 1; }
      tail -2 $OUT/poison.log
      # the same cases against a library with c1b7048's fix reverted (perf_variants/r05bug.so): the
      # 0x3f poison is expected to fail it
      for b in 1 0x3f; do
        PCABI_POISON=$b PCABI_LIB=$R/perf_variants/r05bug.so timeout -k 10 400 python -u tests/poisoned_middle.py > $OUT/poison_r05bug_$b.log 2>&1
        echo "r05bug variant, poison $b: rc=$? (nonzero expected for 0x7f)"; tail -3 $OUT/poison_r05bug_$b.log
      done ;;
    trace)
      # kernel trace (per-dispatch begin / end) of the headline bench (TRACE_ARGS), for timelines
      export TMPDIR=/tmp
      ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --sub 0 --steps 3 --warmup 1 --cpu-sample 0 --check 0 ${TRACE_ARGS:-} > $OUT/trace.json 2> $OUT/trace.err ) || { echo "trace failed rc=$?"; tail -5 $OUT/trace.err; exit 1; }
      ls $OUT/trace ;;
    midab)
      # in-process A/B of a library switch over the middle workloads: AB="NAME=v0,v1"
      for L in 8000 20000; do
        timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps ${AB_STEPS:-20} --warmup 2 --ab "$AB" ${MID_ARGS:-} > $OUT/midab_$L.json 2> $OUT/midab_$L.err || { echo "midab $L failed rc=$?"; tail -20 $OUT/midab_$L.err; exit 1; }
        python -c "import json,sys; d=json.load(open(sys.argv[1])); print($L, d.get('middle_ms_per_step'), {k: {v: x['median_ms'] for v, x in y.items()} for k, y in (d.get('ab') or {}).items()}, d.get('parity_spot_check'))" $OUT/midab_$L.json
      done ;;
    e2e)
      for th in ${E2E_THREADS:-16}; do
        PCABI_PIPE_TRACE=1 PCABI_IO_THREADS=$th timeout -k 10 300 python bench.py --workload e2e --reads 100000 --steps 2 --warmup 1 ${E2E_ARGS:-} > $OUT/e2e_t$th.json 2> $OUT/e2e_t$th.err || { echo "e2e failed rc=$?"; tail -20 $OUT/e2e_t$th.err; exit 1; }
        python -c "import json,sys; d=json.load(open(sys.argv[1])); print('io threads $th', d['ms_per_step'], d['step_vs_slowest_stage'], d['breakdown_ms_per_step'], d['parity_spot_check']['output_identical'])" $OUT/e2e_t$th.json
      done ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done

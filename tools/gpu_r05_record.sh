#!/bin/bash
# GPU-box script for the r05 performance record: the GPU test suite, the default bench line (every
# sub-record), rocprofv3 kernel-trace summaries of the headline bench, the reference job and the
# 8 kb / 20 kb middle workloads, and PMC passes of the dominant kernel -- each step time-limited,
# stopping at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r05final}
mkdir -p $OUT
cd $R
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 900 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench_default.err; exit 1; }
python - $OUT/bench_default.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(json.dumps({k: d.get(k) for k in ('value', 'ms_per_step', 'roofline')}))
for k in ('reference_job', 'middle', 'middle_20kb', 'fused_schedule', 'barcodes', 'config2_10k_119sets', 'drivers', 'check_phase', 'e2e'):
    v = d.get(k) or {}
    print(k, json.dumps({x: v.get(x) for x in ('value', 'ms_per_step', 'middle_ms_per_step', 'ms_per_phase', 'error', 'parity_spot_check')})[:900])
PY
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_head -o run -- python3 $R/bench.py --sub 0 --steps 5 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_head.json 2> $OUT/prof_head.err || { echo "rocprof head failed rc=$?"; tail -20 $OUT/prof_head.err; exit 1; }
echo rocprof head ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_rj -o run -- python3 $R/bench.py --only-subs reference_job --steps 3 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_rj.json 2> $OUT/prof_rj.err || { echo "rocprof rj failed rc=$?"; tail -20 $OUT/prof_rj.err; exit 1; }
echo rocprof rj ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mid8 -o run -- python3 $R/bench.py --workload middle --steps 3 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_mid8.json 2> $OUT/prof_mid8.err || { echo "rocprof mid8 failed rc=$?"; tail -20 $OUT/prof_mid8.err; exit 1; }
echo rocprof mid8 ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mid20 -o run -- python3 $R/bench.py --workload middle --mean-len 20000 --steps 3 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_mid20.json 2> $OUT/prof_mid20.err || { echo "rocprof mid20 failed rc=$?"; tail -20 $OUT/prof_mid20.err; exit 1; }
echo rocprof mid20 ok
KRE="${KRE:-k_align<24, true, 6>}"
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "$KRE" --output-format csv -d $OUT/pmc$i -o run -- python3 $R/bench.py --sub 0 --steps 2 --warmup 1 --cpu-sample 0 --check 0 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
  echo "pmc pass $i ok: $pmc"
done

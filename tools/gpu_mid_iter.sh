#!/bin/bash
# GPU-box script for middle-scan iterations: the middle-scan GPU tests, the middle benches, then a
# kernel trace of the 8 kb middle workload (rocprofv3 --kernel-trace --stats). Stops at the first
# failure. Outputs under gpurun_out/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_long.py tests/test_gpu_freegap.py tests/test_pipeline.py} > $OUT/pytest_mid.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest_mid.log; exit 1; }
tail -2 $OUT/pytest_mid.log
timeout -k 10 300 python bench.py --only-subs middle,middle_20kb --steps 10 ${ARGS:-} > $OUT/bench_mid.json 2> $OUT/bench_mid.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench_mid.err; exit 1; }
python - $OUT/bench_mid.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ('middle', 'middle_20kb'):
    m = d[k]
    print(k, m['value'], 'ms/step', m['ms_per_step'], 'middle_ms', m['middle_ms_per_step'], 'parity', m['parity_spot_check'])
PY
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_it8000 -o run -- python3 $R/bench.py --workload middle --mean-len 8000 --steps 5 --warmup 1 --cpu-sample 0 --check 0 ${ARGS:-} > $OUT/prof_it8000.json 2> $OUT/prof_it8000.err || { echo "trace failed rc=$?"; tail -20 $OUT/prof_it8000.err; exit 1; }
echo trace ok

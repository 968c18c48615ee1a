#!/bin/bash
# r06: the device plan's balanced wave targets (PCABI_MIDDLE_PLAN_BALANCE=1: a bucket with more than
# the mean of the DP cells takes proportionally more waves) vs one target for every bucket (=0): the
# middle-scan GPU tests with it on, then alternating middle benches at 8 kb (separate processes) and
# one pair at 20 kb
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06bal}
mkdir -p $OUT
cd $R
PCABI_MIDDLE_PLAN_BALANCE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_gpu_parity.py > $OUT/pytest_middle.log 2>&1 || { echo "middle tests failed rc=$?"; tail -30 $OUT/pytest_middle.log; exit 1; }
tail -1 $OUT/pytest_middle.log
run() {  # $1 = LATE value, $2 = mean length, $3 = tag
  PCABI_MIDDLE_PLAN_BALANCE=$1 timeout -k 10 300 python bench.py --workload middle --mean-len $2 --steps 20 --warmup 2 --cpu-sample 0 > $OUT/mid_$3.json 2> $OUT/mid_$3.err || { echo "bench $3 failed rc=$?"; tail -20 $OUT/mid_$3.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); m=d.get('middle_phases',{}); print('$3', d.get('middle_ms_per_step'), m.get('ms',{}), m.get('round1_ms'), d.get('middle_hits_per_step'), d.get('parity_spot_check'))" $OUT/mid_$3.json
}
for k in 1 2 3; do
  run 1 8000 8k_bal1_$k || exit 1
  run 0 8000 8k_bal0_$k || exit 1
done
run 1 20000 20k_bal1 || exit 1
run 0 20000 20k_bal0 || exit 1

#!/bin/bash
# GPU-box script: the GPU test suite, then the headline bench (no sub-records) with each schedule
# variant in HEAD_ARGS (';'-separated bench.py argument strings), then a fuzz run; stops at the first
# failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
i=0
IFS=';' read -ra VS <<< "${HEAD_ARGS:---rest-overlap 0;--rest-overlap 1}"
for v in "${VS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --sub 0 --cpu-sample 0 $v > $OUT/ab_$i.json 2> $OUT/ab_$i.err || { echo "bench $v failed"; tail -20 $OUT/ab_$i.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d['parity_spot_check'])" $OUT/ab_$i.json "$v"
done
if [ "${FUZZ:-0}" != "0" ]; then
  timeout -k 10 $((FUZZ + 60)) python -u tools/gpu_fuzz.py $FUZZ 11 > $OUT/fuzz.log 2>&1
  tail -2 $OUT/fuzz.log
fi

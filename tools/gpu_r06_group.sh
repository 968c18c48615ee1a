#!/bin/bash
# r06: grouped cross launches -- their parity test, then the headline under each schedule (A/B)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06g}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_group.py > $OUT/pytest_group.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest_group.log; exit 1; }
tail -2 $OUT/pytest_group.log
for m in ${MODES:-1 4 5}; do
  timeout -k 10 300 python bench.py --sub 0 --cpu-sample 0 --rest-overlap $m ${BENCH_ARGS:-} > $OUT/head_m$m.json 2> $OUT/head_m$m.err || { echo "bench mode $m failed rc=$?"; tail -20 $OUT/head_m$m.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('mode', $m, d['ms_per_step'], r['launch_ms'], r['frac'], r['kernel'][:40], d['parity_spot_check'])" $OUT/head_m$m.json
done

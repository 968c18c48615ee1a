#!/bin/bash
# Serial rounds from round 2 (the new default): the middle GPU tests, then the 8 kb and 20 kb
# middle workloads twice each and the default bench line.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05au
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests -k "middle or seed or window or round or overflow or shadow" > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for L in 8000 20000 8000 20000; do
timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 10 --warmup 2 --cpu-sample 0 > $OUT/mid$L.json 2> $OUT/mid$L.err || { echo "mid failed rc=$?"; tail -20 $OUT/mid$L.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: d.get(k) for k in ('value','ms_per_step','middle_ms_per_step')}, d['middle_phases']['ms'], d['parity_spot_check'])" $OUT/mid$L.json $L
done

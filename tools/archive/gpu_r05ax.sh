#!/bin/bash
# k_cands / k_bound_reset without per-lane 64-bit division: the middle GPU tests, the 8 kb / 20 kb
# middle workloads, and a kernel-stats profile of the 8 kb one.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05ax
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests -k "middle or seed or window or round or overflow or shadow or drivers" > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for L in 8000 20000; do
timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 10 --warmup 2 --cpu-sample 0 > $OUT/mid$L.json 2> $OUT/mid$L.err || { echo "mid failed rc=$?"; tail -20 $OUT/mid$L.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: d.get(k) for k in ('value','ms_per_step','middle_ms_per_step')}, d['middle_phases']['ms'])" $OUT/mid$L.json $L
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mid8 -o run -- python3 $R/bench.py --workload middle --steps 3 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_mid8.json 2> $OUT/prof_mid8.err || { echo "rocprof failed rc=$?"; tail -20 $OUT/prof_mid8.err; exit 1; }
echo rocprof ok

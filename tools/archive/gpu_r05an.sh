#!/bin/bash
# e2e batch size: 12500 (default) against 6250 and 8334 reads per batch, twice each.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05an
mkdir -p $OUT
cd $R
for b in 12500 6250 8334 12500 6250 8334; do
timeout -k 10 300 python bench.py --only-subs e2e --cpu-sample 0 --e2e-batch $b > $OUT/e2e_$b.json 2> $OUT/e2e_$b.err || { echo "bench failed rc=$?"; tail -20 $OUT/e2e_$b.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])).get('e2e',{}); print(sys.argv[2], {k: d.get(k) for k in ('value','ms_per_step','step_vs_slowest_stage','breakdown_ms_per_step')})" $OUT/e2e_$b.json $b
done

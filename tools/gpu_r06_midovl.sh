#!/bin/bash
# r06: the middle workloads (8 kb, 20 kb) with the overlapped-steps figure (`overlapped`: step k+1's
# end trim on a second stream beside step k's middle scan)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06midovl}
mkdir -p $OUT
cd $R
for L in 8000 20000; do
  timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 20 --warmup 2 --cpu-sample 0 > $OUT/mid_$L.json 2> $OUT/mid_$L.err || { echo "bench $L failed rc=$?"; tail -20 $OUT/mid_$L.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print($L, d['ms_per_step'], d['middle_ms_per_step'], d['middle_hits_per_step'], d['overlapped'], d['parity_spot_check'])" $OUT/mid_$L.json
done

#!/bin/bash
# r06: the headline with consecutive steps overlapped (--overlap-steps 1: the next step's tile
# transposes and this step's end trim on a second stream, double-buffered) vs one step after the
# other (0), three alternating pairs with the oracle spot check on; then the e2e queue depth A/B
# (tools/gpu_r06_depth.sh)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06overlap}
mkdir -p $OUT
cd $R
for k in 1 2 3; do
  for o in 1 0; do
    timeout -k 10 200 python bench.py --sub 0 --cpu-sample 0 --check 2000 --steps 30 --overlap-steps $o > $OUT/head_o${o}_$k.json 2> $OUT/head_o${o}_$k.err || { echo "head o$o failed rc=$?"; tail -20 $OUT/head_o${o}_$k.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('overlap', $o, d['ms_per_step'], r['launch_ms'], r['frac'], r['align_phase']['ms'], d['parity_spot_check'])" $OUT/head_o${o}_$k.json
  done
done
TAG=${TAG:-r06overlap} bash tools/gpu_r06_depth.sh

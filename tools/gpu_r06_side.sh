#!/bin/bash
# r06: the grouped headline with its launches side by side (--group-side 1) or one after the other (0),
# alternating on one box
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06side}
mkdir -p $OUT
cd $R
for k in 1 2 3; do
  for g in 1 0; do
    timeout -k 10 200 python bench.py --sub 0 --cpu-sample 0 --check 0 --steps 30 --group-side $g > $OUT/head_g${g}_$k.json 2> $OUT/head_g${g}_$k.err || { echo "head g$g failed rc=$?"; tail -20 $OUT/head_g${g}_$k.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('group_side', $g, d['ms_per_step'], r['launch_ms'], r['frac'], r['align_phase']['ms'], r['align_phase']['frac'])" $OUT/head_g${g}_$k.json
  done
done

#!/bin/bash
# GPU-box script (r04): the headline's smaller buckets dealt onto the two caller streams by cost
# (--rest-overlap 3) against each side's call on its own stream (1), side streams off for both.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04u
mkdir -p $OUT
cd $R
for V in 1 3 1 3 1 3; do
  timeout -k 10 300 python bench.py --sub 0 --rest-overlap $V --steps 20 --warmup 3 --cpu-sample 0 --check 64 > $OUT/head_ro$V.json 2> $OUT/head_ro$V.err || { echo "head $V failed rc=$?"; tail -20 $OUT/head_ro$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/head_ro$V.json')); print('head rest-overlap=$V', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['config']['side_streams'], d['parity_spot_check'])"
done

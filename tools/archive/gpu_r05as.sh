#!/bin/bash
# Headline and middle with and without side streams (PCABI_FORK 1 default, 0 = every launch on the caller's stream),
# alternating, two runs each (GPU_MAX_HW_QUEUES stays the box default: 8 measured slower for the middle, r05ar).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05as
mkdir -p $OUT
cd $R
for q in 1 0 1 0; do
PCABI_FORK=$q timeout -k 10 300 python bench.py --sub 0 --steps 20 --warmup 3 --cpu-sample 0 --check 0 > $OUT/head_f$q.json 2> $OUT/head_f$q.err || { echo "head failed rc=$?"; tail -20 $OUT/head_f$q.err; exit 1; }
PCABI_FORK=$q timeout -k 10 300 python bench.py --workload middle --mean-len 20000 --steps 10 --warmup 2 --cpu-sample 0 --check 0 > $OUT/mid20_f$q.json 2> $OUT/mid20_f$q.err || { echo "mid failed rc=$?"; tail -20 $OUT/mid20_f$q.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); m=json.load(open(sys.argv[2])); print('fork', sys.argv[3], 'head ms', d['ms_per_step'], 'mid20 ms', m['middle_ms_per_step'], m['ms_per_step'])" $OUT/head_f$q.json $OUT/mid20_f$q.json $q
done

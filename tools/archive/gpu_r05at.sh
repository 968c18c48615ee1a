#!/bin/bash
# In-process A/B of PCABI_MIDDLE_SERIAL_FROM (the round from which band classes and candidate-DP
# buckets run one after the other on the scan's stream): 0 (every round) / 1 / 2 (default), 8 kb and 20 kb.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05at
mkdir -p $OUT
cd $R
for L in 8000 20000; do
for ab in 0,2 1,2 0,1; do
timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 24 --warmup 2 --cpu-sample 0 --check 0 --ab PCABI_MIDDLE_SERIAL_FROM=$ab > $OUT/ab_${L}_$ab.json 2> $OUT/ab_${L}_$ab.err || { echo "ab failed rc=$?"; tail -20 $OUT/ab_${L}_$ab.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ab'])" $OUT/ab_${L}_$ab.json $L $ab
done
done

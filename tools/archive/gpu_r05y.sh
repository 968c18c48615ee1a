#!/bin/bash
# r05y: in-process A/Bs of the middle scan (bench --ab alternates the switch between timed steps):
# graph-replayed rounds, the chunk row split, the first batch's rounds; 8 kb and 20 kb reads.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05y
mkdir -p $OUT
cd $R
for ml in 8000 20000; do
  for ab in PCABI_MIDDLE_GRAPHS=0,1 PCABI_CHUNK_SPLIT=0,2 PCABI_MIDDLE_BATCH1=2,3; do
    nm=$(echo $ab | cut -d= -f1)
    timeout -k 10 300 python bench.py --workload middle --mean-len $ml --steps 24 --warmup 3 --sub 0 --cpu-sample 0 --check 0 --middle-check 0 --ab $ab > $OUT/ab_${nm}_$ml.json 2> $OUT/ab_${nm}_$ml.err || { echo "ab $ab $ml failed"; tail -20 $OUT/ab_${nm}_$ml.err; exit 1; }
    python -c "
import json; d=json.load(open('$OUT/ab_${nm}_$ml.json'))
ab=d['ab']; k=list(ab)[0]
print('$ml', k, {v: x['median_ms'] for v, x in ab[k].items()})
"
  done
done

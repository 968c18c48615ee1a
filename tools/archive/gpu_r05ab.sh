#!/bin/bash
# r05ab: in-process A/B of the candidate windows at 8 kb and 20 kb (PCABI_MIDDLE_WINDOWS 0 / 1).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05ab
mkdir -p $OUT
cd $R
for ml in 8000 12000 20000; do
  timeout -k 10 300 python bench.py --workload middle --mean-len $ml --steps 24 --warmup 3 --sub 0 --cpu-sample 0 --check 0 --middle-check 0 --ab PCABI_MIDDLE_WINDOWS=0,1 > $OUT/ab_win_$ml.json 2> $OUT/ab_win_$ml.err || { echo "ab $ml failed"; tail -20 $OUT/ab_win_$ml.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/ab_win_$ml.json'))
ab=d['ab']; k=list(ab)[0]
print('$ml', k, {v: x['median_ms'] for v, x in ab[k].items() if v})
"
done

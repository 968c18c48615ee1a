#!/bin/bash
# r05ah: in-process A/B of the device plan's wave target (PCABI_MIDDLE_PLAN_WAVES) at 8 and 20 kb.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05ah
mkdir -p $OUT
cd $R
for ml in 8000 20000; do
  for ab in PCABI_MIDDLE_PLAN_WAVES=2048,4096 PCABI_MIDDLE_PLAN_WAVES=8192,4096; do
    nm=$(echo $ab | tr '=,' '__')
    timeout -k 10 300 python bench.py --workload middle --mean-len $ml --steps 24 --warmup 3 --sub 0 --cpu-sample 0 --check 0 --middle-check 0 --ab $ab > $OUT/ab_${nm}_$ml.json 2> $OUT/ab_${nm}_$ml.err || { echo "ab $ml failed"; tail -20 $OUT/ab_${nm}_$ml.err; exit 1; }
    python -c "
import json; d=json.load(open('$OUT/ab_${nm}_$ml.json'))
ab=d['ab']; k=list(ab)[0]
print('$ml', '$ab', {v: x['median_ms'] for v, x in ab[k].items() if v})
"
  done
done

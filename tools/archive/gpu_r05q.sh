#!/bin/bash
# r05q: device plan's wave target (PCABI_MIDDLE_PLAN_WAVES) with 32-column chunks available:
# middle / 20 kb sub-records per setting.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05q
mkdir -p $OUT
cd $R
for w in 1024 2048 4096 1024 2048 4096; do
  PCABI_MIDDLE_PLAN_WAVES=$w timeout -k 10 600 python bench.py --only-subs middle,middle_20kb --cpu-sample 0 --middle-check 200 > $OUT/w$w.json 2> $OUT/w$w.err || { echo "bench $w failed"; tail -20 $OUT/w$w.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/w$w.json'))
for k in ('middle','middle_20kb'): print('$w', k, d[k]['ms_per_step'], d[k]['middle_ms_per_step'], d[k]['parity_spot_check']['identical'], d[k]['middle_phases']['ms']['candidate_dp'], d[k]['middle_phases']['ms']['plan'])
"
done

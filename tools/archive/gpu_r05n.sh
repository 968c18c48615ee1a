#!/bin/bash
# r05n: middle-scan queue A/B (side streams with a CU mask each; 8 hardware queues) and the 20 kb
# rounds' candidate counts (PCABI_DEBUG=1).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05n
mkdir -p $OUT
cd $R
PCABI_DEBUG=1 timeout -k 10 300 python bench.py --workload middle --mean-len 20000 --steps 1 --warmup 1 --sub 0 --cpu-sample 0 --check 0 --middle-check 0 > $OUT/debug.json 2> $OUT/debug.err || { echo "debug failed"; tail -20 $OUT/debug.err; exit 1; }
grep "middle round" $OUT/debug.err | tail -12
mid() {  # name env...
  env "${@:2}" timeout -k 10 600 python bench.py --only-subs middle,middle_20kb --cpu-sample 0 > $OUT/mid_$1.json 2> $OUT/mid_$1.err || { echo "bench $1 failed"; tail -20 $OUT/mid_$1.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/mid_$1.json'))
for k in ('middle','middle_20kb'): print('$1', k, d[k]['ms_per_step'], d[k]['middle_ms_per_step'], d[k]['middle_phases']['ms'])
"
}
mid base X=0 && mid cumask PCABI_SIDE_CUMASK=1 && mid q8 GPU_MAX_HW_QUEUES=8 && mid base2 X=0

#!/bin/bash
# r05r: the middle scan at 20 kb and 8 kb on the current code -- per-round debug counts
# (PCABI_DEBUG=1), then rocprofv3 kernel traces + stats of each (per-dispatch durations of the
# candidate-DP chunk launches).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05r
mkdir -p $OUT
cd $R
PCABI_DEBUG=1 timeout -k 10 300 python bench.py --workload middle --mean-len 20000 --steps 1 --warmup 1 --sub 0 --cpu-sample 0 --check 0 --middle-check 0 > $OUT/debug20.json 2> $OUT/debug20.err || { echo "debug failed"; tail -20 $OUT/debug20.err; exit 1; }
grep "pcabi\]" $OUT/debug20.err | tail -14
export TMPDIR=/tmp
for ml in 20000 8000; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof$ml -o run -- python3 $R/bench.py --workload middle --mean-len $ml --steps 3 --warmup 1 --sub 0 --cpu-sample 0 --check 0 --middle-check 0 > $OUT/prof$ml.json 2> $OUT/prof$ml.err) || { echo "prof $ml failed"; tail -20 $OUT/prof$ml.err; exit 1; }
  echo "prof $ml ok"
done

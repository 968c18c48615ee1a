#!/bin/bash
# r05p: 20 kb rounds' candidate counts, certificate flags and plan waves (PCABI_DEBUG=1).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05p
mkdir -p $OUT
cd $R
PCABI_DEBUG=1 timeout -k 10 300 python bench.py --workload middle --mean-len 20000 --steps 1 --warmup 1 --sub 0 --cpu-sample 0 --check 0 --middle-check 0 > $OUT/debug.json 2> $OUT/debug.err || { echo "debug failed"; tail -20 $OUT/debug.err; exit 1; }
grep "pcabi\]" $OUT/debug.err | tail -14

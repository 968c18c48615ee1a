#!/bin/bash
# GPU-box script: kernel trace (timestamps) of a short bench run: ARGS="--workload compat" bash tools/gpu_trace.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_x -o run -- python3 $R/bench.py $ARGS --steps 2 --warmup 1 --cpu-sample 0 --check 0 > $OUT/trace_x.log 2>&1 || { echo "trace failed rc=$?"; tail -20 $OUT/trace_x.log; exit 1; }
find $OUT/trace_x -name '*trace.csv'

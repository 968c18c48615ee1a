#!/bin/bash
# GPU-box script: kernel trace (timestamps) of one middle-scan step, for the per-round timeline.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_mid -o run -- python3 $R/bench.py --workload middle --steps 1 --warmup 1 --cpu-sample 0 --check 0 > $OUT/trace_mid.log 2>&1 || { echo "trace failed rc=$?"; tail -20 $OUT/trace_mid.log; exit 1; }
find $OUT/trace_mid -name '*kernel_trace.csv'

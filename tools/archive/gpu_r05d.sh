#!/bin/bash
# r05d: kernel traces (timestamps) of one middle-scan step at 20 kb and 8 kb (per-round timeline).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05d
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for L in 20000 8000; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_mid$L -o run -- python3 $R/bench.py --workload middle --mean-len $L --steps 2 --warmup 1 --cpu-sample 0 --check 0 > $OUT/trace_mid$L.log 2>&1 || { echo "trace failed rc=$?"; tail -20 $OUT/trace_mid$L.log; exit 1; }
done
echo traces ok

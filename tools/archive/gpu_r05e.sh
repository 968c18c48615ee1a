#!/bin/bash
# r05e: host-side time marks of the middle scan (PCABI_HOSTPROF=1) at 20 kb and 8 kb.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05e
mkdir -p $OUT
cd $R
for L in 20000 8000; do
PCABI_HOSTPROF=1 timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 4 --warmup 1 --cpu-sample 0 --check 0 > $OUT/mid$L.json 2> $OUT/mid$L.err || { echo "bench failed rc=$?"; tail -20 $OUT/mid$L.err; exit 1; }
grep hostprof $OUT/mid$L.err | tail -12
done

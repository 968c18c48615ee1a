#!/bin/bash
# GPU-box script: every perf_variants/*.so on the headline bench (ms per step) and under
# rocprofv3 --kernel-trace --stats (per-kernel averages), one process each; stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/variants
mkdir -p $OUT
cd $R
BENCH_ARGS="--sub 0 --cpu-sample 0 --check 64 ${BENCH_ARGS:-}" bash tools/gpu_variants.sh || exit 1
export TMPDIR=/tmp
for so in $R/perf_variants/*.so; do
  n=$(basename $so .so)
  cd /tmp
  PCABI_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$n -o run -- python3 $R/bench.py --sub 0 --steps 5 --warmup 1 --cpu-sample 0 --check 0 ${BENCH_ARGS:-} > $OUT/prof_$n.log 2>&1 || { echo "prof $n failed"; tail -5 $OUT/prof_$n.log; exit 1; }
  echo "== $n"; head -8 $OUT/prof_$n/run_kernel_stats.csv | cut -d, -f1-4
done

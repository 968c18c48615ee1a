#!/bin/bash
# GPU-box script: the GPU test suite (TESTS, default all), then the headline bench without
# sub-records and a kernel-stats profile of it; each step time-limited, stop at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --sub 0 ${BENCH_ARGS:-} > $OUT/bench_q.json 2> $OUT/bench_q.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench_q.err; exit 1; }
cat $OUT/bench_q.json | cut -c1-600
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_q -o run -- python3 $R/bench.py --sub 0 --steps 5 --warmup 1 --cpu-sample 0 --check 0 ${BENCH_ARGS:-} > $OUT/prof_q.json 2> $OUT/prof_q.err || { echo "rocprof failed rc=$?"; tail -20 $OUT/prof_q.err; exit 1; }
head -12 $OUT/prof_q/run_kernel_stats.csv | cut -d, -f1-5

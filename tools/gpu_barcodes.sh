#!/bin/bash
# GPU-box script: barcode-call parity tests, then the barcodes workload (BASELINE.json configs[3])
# bench + rocprofv3 kernel stats. Each GPU step has its own time limit; stop at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_barcode_call.py} > $OUT/pytest_bc.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest_bc.log; exit 1; }
tail -3 $OUT/pytest_bc.log
timeout -k 10 600 python bench.py --workload barcodes ${BENCH_ARGS:-} > $OUT/bench_barcodes.json 2> $OUT/bench_barcodes.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench_barcodes.err; exit 1; }
cat $OUT/bench_barcodes.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bc -o run -- python3 $R/bench.py --workload barcodes --steps 5 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_bc.log 2>&1 || { echo "rocprof failed rc=$?"; tail -20 $OUT/prof_bc.log; exit 1; }
find $OUT/prof_bc -name '*kernel_stats.csv'

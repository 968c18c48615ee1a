#!/bin/bash
# r05a: input-preserving middle scan -- the middle-path GPU tests, then the middle / 20 kb /
# reference-job sub-records of the default bench (one resident read pack per workload).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05a
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_pipeline.py > $OUT/pytest_mid.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest_mid.log; exit 1; }
tail -3 $OUT/pytest_mid.log
timeout -k 10 600 python bench.py --only-subs middle,middle_20kb,reference_job > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench.err; exit 1; }
echo bench ok

#!/bin/bash
# r05 baseline: the GPU test suite and the default bench line on the r04 code.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05base
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench.err; exit 1; }
echo bench ok

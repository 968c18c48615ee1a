#!/bin/bash
# GPU-box script: parity tests, then bench + rocprof (each step time-limited; stop on failure).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest aborted rc=$rc"; exit 1; fi
if [ $rc -ne 0 ]; then echo "pytest failures rc=$rc (continuing to bench)"; fi
bash tools/gpu_bench.sh

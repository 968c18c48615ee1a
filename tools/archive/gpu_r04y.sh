#!/bin/bash
# GPU-box script (r04): the whole GPU suite on the round's final code.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04y
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()"

#!/bin/bash
# r05ae: the round-graph replay test (library stream) and the middle-path suite.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05ae
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
grep -c PASSED $OUT/pytest.log
grep 'round_graphs' $OUT/pytest.log

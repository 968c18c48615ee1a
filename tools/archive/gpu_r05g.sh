#!/bin/bash
# r05g: the middle scan with a first batch of two rounds (default) against three (PCABI_MIDDLE_BATCH1=3),
# 20 kb and 8 kb, after the middle-path GPU tests.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05g
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_pipeline.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for B in 2 3; do
PCABI_MIDDLE_BATCH1=$B timeout -k 10 600 python bench.py --only-subs middle,middle_20kb --cpu-sample 0 > $OUT/mid_b$B.json 2> $OUT/mid_b$B.err || { echo "bench failed rc=$?"; tail -20 $OUT/mid_b$B.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/mid_b$B.json'))
for k in ('middle','middle_20kb'): print('batch1=$B', k, d[k]['ms_per_step'], d[k]['middle_ms_per_step'], d[k]['parity_spot_check'])
"
done

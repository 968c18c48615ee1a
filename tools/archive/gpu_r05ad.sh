#!/bin/bash
# r05ad: seed scan in 1024-thread blocks (32 waves per CU) against the r04 512-thread blocks
# (PCABI_SCAN_THREADS=512), two processes each, middle / 20 kb sub-records; the bytemap test.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05ad
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py -k "bytemap or overflow or windows" > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for t in 1024 512 1024 512; do
  PCABI_SCAN_THREADS=$t timeout -k 10 600 python bench.py --only-subs middle,middle_20kb --cpu-sample 0 --middle-check 300 > $OUT/mid_$t.json 2> $OUT/mid_$t.err || { echo "bench mid failed rc=$?"; tail -20 $OUT/mid_$t.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/mid_$t.json'))
for k in ('middle','middle_20kb'): print('tpb=$t', k, d[k]['ms_per_step'], d[k]['middle_ms_per_step'], d[k]['parity_spot_check']['identical'], d[k]['middle_phases']['ms']['k_seed_scan'], d[k]['middle_phases']['ms']['k_seed_expand'])
"
done

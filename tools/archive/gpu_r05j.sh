#!/bin/bash
# r05j: band kernels with per-lane task switching (default) vs one task per pass (PCABI_BAND_SWITCH=0):
# lane statistics (experiment build), middle-path tests, middle / 20 kb sub-records for both.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05j
mkdir -p $OUT
cd $R
for SW in 0 1; do
for L in 20000 8000; do
PCABI_BAND_SWITCH=$SW PCABI_LIB=perf_variants/bandstats.so timeout -k 10 300 python tools/band_stats.py $L > $OUT/stats_sw${SW}_$L.txt 2>&1 || { echo "stats failed"; tail -5 $OUT/stats_sw${SW}_$L.txt; exit 1; }
echo "switch=$SW len=$L"; cat $OUT/stats_sw${SW}_$L.txt
done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_pipeline.py > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for SW in 1 0 1; do
PCABI_BAND_SWITCH=$SW timeout -k 10 600 python bench.py --only-subs middle,middle_20kb --cpu-sample 0 > $OUT/mid_sw$SW.json 2> $OUT/mid_sw$SW.err || { echo "bench failed rc=$?"; tail -20 $OUT/mid_sw$SW.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/mid_sw$SW.json'))
for k in ('middle','middle_20kb'): print('switch=$SW', k, d[k]['ms_per_step'], d[k]['middle_ms_per_step'], d[k]['parity_spot_check']['identical'], d[k]['middle_phases']['ms'])
"
done

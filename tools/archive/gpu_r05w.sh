#!/bin/bash
# r05w: e2e with the reader's populate-ahead helper (+ timeline); io / pipeline GPU tests; chunk
# row-split A/B on the middle / 20 kb sub-records (PCABI_CHUNK_SPLIT 0 / 2 / 4); cProfile of the
# reference-API drivers.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05w
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pipeline.py tests/test_io.py > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
PCABI_PIPE_TRACE=1 timeout -k 10 300 python bench.py --only-subs e2e --cpu-sample 0 > $OUT/e2e.json 2> $OUT/e2e.err || { echo "e2e failed rc=$?"; tail -20 $OUT/e2e.err; exit 1; }
python -c "
import json; v=json.load(open('$OUT/e2e.json'))['e2e']
print('e2e', v.get('value'), v.get('ms_per_step'), v.get('breakdown_ms_per_step'), v.get('parity_spot_check'), v.get('error'))
"
for sp in 0 2 4 0; do
  PCABI_CHUNK_SPLIT=$sp timeout -k 10 600 python bench.py --only-subs middle,middle_20kb --cpu-sample 0 --middle-check 200 > $OUT/mid_s$sp.json 2> $OUT/mid_s$sp.err || { echo "bench mid failed rc=$?"; tail -20 $OUT/mid_s$sp.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/mid_s$sp.json'))
for k in ('middle','middle_20kb'): print('split=$sp', k, d[k]['ms_per_step'], d[k]['middle_ms_per_step'], d[k]['parity_spot_check']['identical'], d[k]['middle_phases']['ms']['candidate_dp'])
"
done
timeout -k 10 300 python tools/profile_drivers.py > $OUT/drivers_prof.txt 2>&1 || { echo "drivers prof failed"; tail -20 $OUT/drivers_prof.txt; exit 1; }
grep '==' $OUT/drivers_prof.txt

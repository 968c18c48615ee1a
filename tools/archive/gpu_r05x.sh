#!/bin/bash
# r05x: later middle rounds replayed from captured graphs + the two-lane chunk split by default:
# middle-path / parity / pipeline GPU tests; PCABI_MIDDLE_GRAPHS 1 / 0 on the middle / 20 kb /
# reference-job sub-records; the drivers sub-record (pid6 table).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05x
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_gpu_parity.py tests/test_pipeline.py tests/test_drivers.py > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for g in 1 0 1 0; do
  PCABI_MIDDLE_GRAPHS=$g timeout -k 10 600 python bench.py --only-subs middle,middle_20kb,reference_job --cpu-sample 0 --middle-check 300 > $OUT/mid_g$g.json 2> $OUT/mid_g$g.err || { echo "bench mid failed rc=$?"; tail -20 $OUT/mid_g$g.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/mid_g$g.json'))
for k in ('middle','middle_20kb'): print('graphs=$g', k, d[k]['ms_per_step'], d[k]['middle_ms_per_step'], d[k]['parity_spot_check']['identical'], d[k]['middle_phases']['ms'])
r=d['reference_job']; print('graphs=$g reference_job', r.get('ms_per_step'), r['ms_per_phase']['middle_ms'])
"
done
timeout -k 10 300 python bench.py --only-subs drivers --cpu-sample 0 > $OUT/drivers.json 2> $OUT/drivers.err || { echo "drivers failed rc=$?"; tail -20 $OUT/drivers.err; exit 1; }
python -c "
import json; v=json.load(open('$OUT/drivers.json'))['drivers']
print('drivers', v.get('value'), v.get('ms_per_driver'), v.get('parity_spot_check'))
"

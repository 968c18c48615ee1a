#!/bin/bash
# r05o: 32-column chunks in the device plans: middle-path tests, middle / 20 kb sub-records (x2).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05o
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_pipeline.py > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
timeout -k 10 600 python bench.py --only-subs middle,middle_20kb,reference_job --cpu-sample 0 > $OUT/mid$i.json 2> $OUT/mid$i.err || { echo "bench failed rc=$?"; tail -20 $OUT/mid$i.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/mid$i.json'))
for k in ('middle','middle_20kb'): print(k, d[k]['ms_per_step'], d[k]['middle_ms_per_step'], d[k]['parity_spot_check']['identical'], d[k]['middle_phases']['ms'], d[k]['middle_phases']['roofline']['candidate_dp']['frac'])
r=d['reference_job']; print('reference_job', r.get('ms_per_step'), r.get('value'))
"
done

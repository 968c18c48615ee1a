#!/bin/bash
# r05u: pair-map seed scan (one LDS read per two positions) + lazy file map / progressive page
# release / exact batch buffers: middle-path, pipeline and io GPU tests; middle / 20 kb / e2e
# sub-records (e2e timeline); kernel stats of the 20 kb middle workload.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05u
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_pipeline.py tests/test_io.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python bench.py --only-subs middle,middle_20kb,reference_job --cpu-sample 0 > $OUT/mid.json 2> $OUT/mid.err || { echo "bench mid failed rc=$?"; tail -20 $OUT/mid.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/mid.json'))
for k in ('middle','middle_20kb'): print(k, d[k]['ms_per_step'], d[k]['middle_ms_per_step'], d[k]['parity_spot_check'], d[k]['middle_phases']['ms'], d[k]['middle_phases']['roofline']['k_seed_scan']['frac'])
r=d['reference_job']; print('reference_job', r.get('ms_per_step'), r.get('ms_per_phase'))
"
PCABI_PIPE_TRACE=1 timeout -k 10 300 python bench.py --only-subs e2e --cpu-sample 0 > $OUT/e2e.json 2> $OUT/e2e.err || { echo "e2e failed rc=$?"; tail -20 $OUT/e2e.err; exit 1; }
python -c "
import json; v=json.load(open('$OUT/e2e.json'))['e2e']
print('e2e', v.get('value'), v.get('ms_per_step'), v.get('breakdown_ms_per_step'), v.get('parity_spot_check'), v.get('error'))
"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof20000 -o run -- python3 $R/bench.py --workload middle --mean-len 20000 --steps 3 --warmup 1 --sub 0 --cpu-sample 0 --check 0 --middle-check 0 > $OUT/prof20000.json 2> $OUT/prof20000.err) || { echo "prof failed"; tail -20 $OUT/prof20000.err; exit 1; }
echo prof ok

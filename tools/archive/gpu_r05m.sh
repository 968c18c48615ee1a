#!/bin/bash
# r05m: band-class roofline (per-wave counters), e2e pipeline knobs (batch size, queue depth, GIL
# switch interval).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05m
mkdir -p $OUT
cd $R
if [ -z "${E2E_ONLY:-}" ]; then
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py -k "profile or expand or bytemap" > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/band_stats.py 20000 > $OUT/band_stats.txt 2>&1 || { echo "band stats failed"; tail -5 $OUT/band_stats.txt; exit 1; }
cat $OUT/band_stats.txt
timeout -k 10 600 python bench.py --only-subs middle,middle_20kb --cpu-sample 0 > $OUT/mid.json 2> $OUT/mid.err || { echo "bench mid failed rc=$?"; tail -20 $OUT/mid.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/mid.json'))
for k in ('middle','middle_20kb'): print(k, d[k]['ms_per_step'], d[k]['middle_ms_per_step'], d[k]['middle_phases']['ms'], json.dumps(d[k]['middle_phases']['roofline'].get('bands')))
"
fi
run_e2e() {  # name batch depth [switch]
  PCABI_PIPE_DEPTH=$3 timeout -k 10 300 python -c "
import sys, runpy
if '${4:-}': sys.setswitchinterval(float('${4:-}'))
sys.argv = ['bench.py', '--only-subs', 'e2e', '--cpu-sample', '0', '--e2e-batch', '$2', '--e2e-check', '20']
runpy.run_path('bench.py', run_name='__main__')
" > $OUT/e2e_$1.json 2> $OUT/e2e_$1.err || { echo "e2e $1 failed"; tail -20 $OUT/e2e_$1.err; exit 1; }
  python -c "
import json; v=json.load(open('$OUT/e2e_$1.json'))['e2e']
print('$1', v['value'], v['ms_per_step'], v['breakdown_ms_per_step'], v['step_vs_slowest_stage'])
"
}
run_e2e b6250d2 6250 2 && run_e2e b6250d4 6250 4 && run_e2e b4000d4 4000 4 && run_e2e b6250d4s 6250 4 0.0005 && run_e2e b12500d4 12500 4

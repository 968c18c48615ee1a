#!/bin/bash
# GPU-box script (r04): middle-scan parity (seeds, windows, overflow paths), middle 8 / 20 kb with the
# scan profile, a kernel trace of the 8 kb step (timed steps, no profile step: --check 0 skips none of it).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04d
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_gpu_parity.py -k "middle or seed or windows or overflow or scan" > $OUT/pytest_mid.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" $OUT/pytest_mid.log | head -20; tail -30 $OUT/pytest_mid.log; exit 1; }
tail -2 $OUT/pytest_mid.log
timeout -k 10 300 python bench.py --sub 0 --steps 20 --warmup 3 --cpu-sample 0 > $OUT/head.json 2> $OUT/head.err || { echo "head failed rc=$?"; tail -20 $OUT/head.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/head.json')); print('head', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d.get('parity_spot_check'))"
for L in 8000 20000; do
  timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 8 --warmup 2 --cpu-sample 0 > $OUT/mid_$L.json 2> $OUT/mid_$L.err || { echo "mid $L failed rc=$?"; tail -20 $OUT/mid_$L.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/mid_$L.json')); p=d['middle_phases']; print('mid $L', d['value'], d['ms_per_step'], d['middle_ms_per_step'], json.dumps(p['ms']), p['round1_ms'], d['parity_spot_check'])"
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_head -o run -- python3 $R/bench.py --sub 0 --steps 5 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_head.json 2> $OUT/prof_head.err || { echo "rocprof head failed rc=$?"; tail -20 $OUT/prof_head.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mid8 -o run -- python3 $R/bench.py --workload middle --steps 3 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_mid8.json 2> $OUT/prof_mid8.err || { echo "rocprof failed rc=$?"; tail -20 $OUT/prof_mid8.err; exit 1; }
python3 - $OUT <<'PY'
import csv, sys, os
rows = list(csv.DictReader(open(os.path.join(sys.argv[1], 'prof_mid8', 'run_kernel_stats.csv'))))
for r in rows[:24]:
    print('%-66s %5s %9.1f us' % (r['Name'][:66], r['Calls'], float(r['AverageNs']) / 1e3))
PY

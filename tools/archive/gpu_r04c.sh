#!/bin/bash
# GPU-box script (r04): the whole GPU suite, the headline (split threshold, k_end_trim), middle 8 / 20 kb
# with the scan profile, a kernel trace of the 8 kb middle step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04c
mkdir -p $OUT
cd $R
timeout -k 10 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error|error" $OUT/pytest_gpu.log | head -20; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --sub 0 --steps 20 --warmup 3 --cpu-sample 0 > $OUT/head_$i.json 2> $OUT/head_$i.err || { echo "bench failed rc=$?"; tail -20 $OUT/head_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/head_$i.json')); print('head', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d.get('parity_spot_check'))"
done
for L in 8000 20000; do
  timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 8 --warmup 2 --cpu-sample 0 > $OUT/mid_$L.json 2> $OUT/mid_$L.err || { echo "mid $L failed rc=$?"; tail -20 $OUT/mid_$L.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/mid_$L.json')); print('mid $L', d['value'], d['ms_per_step'], d['middle_ms_per_step'], json.dumps(d['middle_phases']), d['parity_spot_check'])"
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mid8 -o run -- python3 $R/bench.py --workload middle --steps 3 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_mid8.json 2> $OUT/prof_mid8.err || { echo "rocprof failed rc=$?"; tail -20 $OUT/prof_mid8.err; exit 1; }
python3 - $OUT <<'PY'
import csv, sys, os
rows = list(csv.DictReader(open(os.path.join(sys.argv[1], 'prof_mid8', 'run_kernel_stats.csv'))))
for r in rows[:30]:
    print('%-66s %5s %9.1f us' % (r['Name'][:66], r['Calls'], float(r['AverageNs']) / 1e3))
PY

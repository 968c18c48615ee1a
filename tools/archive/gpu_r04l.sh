#!/bin/bash
# GPU-box script (r04): middle parity after the tiled segment scan and with the one-pass expansion,
# the middle step two-pass vs one-pass expansion, and kernel-trace summaries of both.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04l
mkdir -p $OUT
cd $R
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_gpu_parity.py -k "middle or seed or windows or overflow or scan" > $OUT/pytest_mid.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" $OUT/pytest_mid.log | head -20; tail -30 $OUT/pytest_mid.log; exit 1; }
tail -2 $OUT/pytest_mid.log
for V in base e1 base e1; do
  case $V in base) E="PCABI_NOOP=1";; e1) E="PCABI_EXPAND_PASSES=1";; esac
  env $E timeout -k 10 300 python bench.py --workload middle --steps 8 --warmup 2 --cpu-sample 0 > $OUT/mid_$V.json 2> $OUT/mid_$V.err || { echo "mid $V failed rc=$?"; tail -20 $OUT/mid_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/mid_$V.json')); print('mid $V', d['middle_ms_per_step'], json.dumps(d['middle_phases']['ms']), d['parity_spot_check']['identical'])"
done
env PCABI_EXPAND_PASSES=1 timeout -k 10 300 python bench.py --workload middle --mean-len 20000 --steps 6 --warmup 2 --cpu-sample 0 > $OUT/mid20_e1.json 2> $OUT/mid20_e1.err || { echo "mid20 e1 failed rc=$?"; tail -20 $OUT/mid20_e1.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/mid20_e1.json')); print('mid20 e1', d['middle_ms_per_step'], json.dumps(d['middle_phases']['ms']), d['parity_spot_check']['identical'])"
export TMPDIR=/tmp
cd /tmp
for V in base e1; do
  case $V in base) X=0;; e1) X=1;; esac
  PCABI_EXPAND_PASSES=$X timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mid8_$V -o run -- python3 $R/bench.py --workload middle --steps 3 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_mid8_$V.json 2> $OUT/prof_mid8_$V.err || { echo "rocprof mid8 $V failed rc=$?"; tail -20 $OUT/prof_mid8_$V.err; exit 1; }
  echo rocprof mid8 $V ok
  python3 - $OUT/prof_mid8_$V <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)
rows = list(csv.DictReader(open(f[0])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print('  %-60s calls %6s avg %9.1f us total %9.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3, float(r['TotalDurationNs']) / 1e3))
for r in rows:
    if any(k in r['Name'] for k in ('k_seg_cum', 'k_merge_best', 'k_seed_expand', 'k_round')):
        print('  * %-58s calls %6s avg %9.1f us' % (r['Name'][:58], r['Calls'], float(r['AverageNs']) / 1e3))
PY
done

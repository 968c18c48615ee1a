#!/bin/bash
# GPU-box script (r04): A/B of the row-split core on the headline and the reference job
# (PCABI_SPLIT=0 off, unset = auto, 2 = always two lanes), kernel-stats profiles of the headline both ways.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04b
mkdir -p $OUT
cd $R
for S in 0 auto 2 0 auto; do
  if [ "$S" = auto ]; then unset PCABI_SPLIT; else export PCABI_SPLIT=$S; fi
  timeout -k 10 300 python bench.py --sub 0 --steps 20 --warmup 3 --cpu-sample 0 --check 0 > $OUT/head_$S.json 2> $OUT/head_$S.err || { echo "bench $S failed rc=$?"; tail -20 $OUT/head_$S.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/head_$S.json')); print('split=$S', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
done
for S in 0 auto; do
  if [ "$S" = auto ]; then unset PCABI_SPLIT; else export PCABI_SPLIT=$S; fi
  timeout -k 10 300 python bench.py --only-subs reference_job --steps 6 --warmup 2 --cpu-sample 0 --check 0 > $OUT/rj_$S.json 2> $OUT/rj_$S.err || { echo "rj $S failed rc=$?"; tail -20 $OUT/rj_$S.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/rj_$S.json'))['reference_job']; print('rj split=$S', d['value'], d['ms_per_step'], d['ms_per_phase'])"
done
export TMPDIR=/tmp
cd /tmp
for S in 0 auto; do
  if [ "$S" = auto ]; then unset PCABI_SPLIT; else export PCABI_SPLIT=$S; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_head_$S -o run -- python3 $R/bench.py --sub 0 --steps 5 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_head_$S.json 2> $OUT/prof_head_$S.err || { echo "rocprof $S failed rc=$?"; tail -20 $OUT/prof_head_$S.err; exit 1; }
done
python3 - $OUT <<'PY'
import csv, sys, os
for S in ('0', 'auto'):
    rows = list(csv.DictReader(open(os.path.join(sys.argv[1], 'prof_head_%s' % S, 'run_kernel_stats.csv'))))
    print('== split', S)
    for r in rows[:14]:
        print('%-66s %5s %9.1f us' % (r['Name'][:66], r['Calls'], float(r['AverageNs']) / 1e3))
PY

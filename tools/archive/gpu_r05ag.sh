#!/bin/bash
# r05ag: e2e against the interpreter's GIL switch interval (5 ms default, 1 ms, 0.5 ms), twice each.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05ag
mkdir -p $OUT
cd $R
for sw in 0.005 0.001 0.0005 0.005 0.001 0.0005; do
  timeout -k 10 300 python -c "
import sys, runpy
sys.setswitchinterval($sw)
sys.argv = ['bench.py', '--only-subs', 'e2e', '--cpu-sample', '0']
runpy.run_path('bench.py', run_name='__main__')
" > $OUT/e2e_$sw.json 2> $OUT/e2e_$sw.err || { echo "e2e $sw failed"; tail -20 $OUT/e2e_$sw.err; exit 1; }
  python -c "
import json; v=json.load(open('$OUT/e2e_$sw.json'))['e2e']
print('switch $sw', v.get('value'), v.get('ms_per_step'), v.get('breakdown_ms_per_step'), v.get('error'))
"
done

#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05bc
mkdir -p $OUT
cd $R
for h in 3 2 3 2; do
PCABI_EXPAND_HITS=$h timeout -k 10 200 python bench.py --only-subs reference_job --cpu-sample 0 --check 0 > $OUT/rj_$h.json 2> $OUT/rj_$h.err || { echo "rj failed"; tail -5 $OUT/rj_$h.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1]))['reference_job']; print('hits', sys.argv[2], d['ms_per_step'], d['ms_per_phase']['middle_ms'])" $OUT/rj_$h.json $h
done

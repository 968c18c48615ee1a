#!/bin/bash
# GPU-box script (r04): the reference job's end trim with each kept adapter on a stream of its own.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04x
mkdir -p $OUT
cd $R
for V in 0 1 0 1 0 1; do
  timeout -k 10 300 python bench.py --only-subs reference_job --rj-end-streams $V --steps 8 --warmup 2 --cpu-sample 0 > $OUT/rj_$V.json 2> $OUT/rj_$V.err || { echo "rj $V failed rc=$?"; tail -20 $OUT/rj_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/rj_$V.json'))['reference_job']; print('rj end-streams=$V', d['ms_per_step'], json.dumps(d['ms_per_phase']), d['single_adapter_launches']['frac'], d['parity_spot_check']['end_windows'])"
done

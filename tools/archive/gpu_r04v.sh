#!/bin/bash
# GPU-box script (r04): the >= 36-row buckets of a few adapters in 2 lanes per window
# (PCABI_SPLIT_WIDE=1) on the headline, the reference job and the middle step's end trim.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04v
mkdir -p $OUT
cd $R
for V in base wide base wide; do
  case $V in base) E="PCABI_NOOP=1";; wide) E="PCABI_SPLIT_WIDE=1";; esac
  env $E timeout -k 10 300 python bench.py --sub 0 --steps 20 --warmup 3 --cpu-sample 0 --check 64 > $OUT/head_$V.json 2> $OUT/head_$V.err || { echo "head $V failed rc=$?"; tail -20 $OUT/head_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/head_$V.json')); print('head $V', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['parity_spot_check'])"
  env $E timeout -k 10 300 python bench.py --only-subs reference_job,fused_schedule --steps 6 --warmup 2 --cpu-sample 0 > $OUT/rj_$V.json 2> $OUT/rj_$V.err || { echo "rj $V failed rc=$?"; tail -20 $OUT/rj_$V.err; exit 1; }
  python -c "import json; D=json.load(open('$OUT/rj_$V.json')); d=D['reference_job']; print('rj $V', d['ms_per_step'], json.dumps(d['ms_per_phase']), d['single_adapter_launches']['frac'], d['parity_spot_check']['end_windows']); print('fused $V', D.get('fused_schedule', {}).get('ms_per_step'))"
done

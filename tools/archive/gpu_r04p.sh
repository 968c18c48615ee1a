#!/bin/bash
# GPU-box script (r04): the reference job with its kept sets' small tables merged to at most N
# register buckets (PCABI_SMALL_TABLE_BUCKETS, tables of <= 4 adapters): default vs 1 vs 2.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04p
mkdir -p $OUT
cd $R
for V in base 1 2 base 1 2; do
  case $V in base) E="PCABI_NOOP=1";; *) E="PCABI_SMALL_TABLE_BUCKETS=$V";; esac
  env $E timeout -k 10 300 python bench.py --only-subs reference_job --steps 6 --warmup 2 --cpu-sample 0 > $OUT/rj_$V.json 2> $OUT/rj_$V.err || { echo "rj $V failed rc=$?"; tail -20 $OUT/rj_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/rj_$V.json'))['reference_job']; print('rj $V', d['ms_per_step'], json.dumps(d['ms_per_phase']), d['single_adapter_launches']['frac'], d['parity_spot_check'])"
done

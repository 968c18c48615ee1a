#!/bin/bash
# GPU-box script (r04): headline A/B of the bucket-merge limit (PCABI_MAX_FAST_BUCKETS), and the
# reference job with both sides' kept-set launches side by side.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04i
mkdir -p $OUT
cd $R
for M in 4 3 2 1 4 2; do
  PCABI_MAX_FAST_BUCKETS=$M timeout -k 10 300 python bench.py --sub 0 --steps 20 --warmup 3 --cpu-sample 0 --check 0 > $OUT/head_$M.json 2> $OUT/head_$M.err || { echo "head $M failed rc=$?"; tail -20 $OUT/head_$M.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/head_$M.json')); print('maxfast=$M', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
done
timeout -k 10 300 python bench.py --only-subs reference_job --steps 6 --warmup 2 --cpu-sample 0 > $OUT/rj.json 2> $OUT/rj.err || { echo "rj failed rc=$?"; tail -20 $OUT/rj.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/rj.json'))['reference_job']; print('rj', d['value'], d['ms_per_step'], d['ms_per_phase'], d['single_adapter_launches'], d['parity_spot_check'])"

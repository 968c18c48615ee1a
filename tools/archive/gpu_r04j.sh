#!/bin/bash
# GPU-box script (r04): the reference job's single-adapter end-trim launches under the row split
# (PCABI_SPLIT unset / 2 / 4) with both sides side by side, and a kernel trace of it.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04j
mkdir -p $OUT
cd $R
for S in auto 2 4 auto; do
  if [ "$S" = auto ]; then unset PCABI_SPLIT; else export PCABI_SPLIT=$S; fi
  timeout -k 10 300 python bench.py --only-subs reference_job --steps 8 --warmup 2 --cpu-sample 0 --check 0 > $OUT/rj_$S.json 2> $OUT/rj_$S.err || { echo "rj $S failed rc=$?"; tail -20 $OUT/rj_$S.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/rj_$S.json'))['reference_job']; print('split=$S', d['ms_per_step'], d['ms_per_phase'], d['single_adapter_launches']['frac'])"
done
unset PCABI_SPLIT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_rj -o run -- python3 $R/bench.py --only-subs reference_job --steps 3 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_rj.json 2> $OUT/prof_rj.err || { echo "rocprof failed rc=$?"; tail -20 $OUT/prof_rj.err; exit 1; }
echo traced

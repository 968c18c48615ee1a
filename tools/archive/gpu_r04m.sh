#!/bin/bash
# GPU-box script (r04): the reference job's middle scan (4 kept adapters, ~4.5 k true hits per 100 k
# reads) with candidate windows off / on, and a kernel trace of the job with them on.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04m
mkdir -p $OUT
cd $R
timeout -k 10 60 tools/launch_bench > $OUT/launch_bench.txt 2>&1 || { echo "launch_bench failed rc=$?"; cat $OUT/launch_bench.txt; exit 1; }
cat $OUT/launch_bench.txt
timeout -k 10 60 tools/queue_probe > $OUT/queue_probe.txt 2>&1 || { echo "queue_probe failed rc=$?"; cat $OUT/queue_probe.txt; exit 1; }
cat $OUT/queue_probe.txt
for W in 0 1 0 1; do
  PCABI_MIDDLE_WINDOWS=$W timeout -k 10 300 python bench.py --only-subs reference_job --steps 6 --warmup 2 --cpu-sample 0 > $OUT/rj_w$W.json 2> $OUT/rj_w$W.err || { echo "rj w$W failed rc=$?"; tail -20 $OUT/rj_w$W.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/rj_w$W.json'))['reference_job']; print('rj windows=$W', d['ms_per_step'], json.dumps(d['ms_per_phase']), d['parity_spot_check']['middle'])"
done
for W in 0 1; do
  PCABI_MIDDLE_WINDOWS=$W timeout -k 10 300 python bench.py --workload middle --steps 8 --warmup 2 --cpu-sample 0 > $OUT/mid_w$W.json 2> $OUT/mid_w$W.err || { echo "mid w$W failed rc=$?"; tail -20 $OUT/mid_w$W.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/mid_w$W.json')); print('mid windows=$W', d['middle_ms_per_step'], json.dumps(d['middle_phases']['ms']), d['parity_spot_check']['identical'])"
done
export TMPDIR=/tmp
cd /tmp
PCABI_MIDDLE_WINDOWS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_rj_w1 -o run -- python3 $R/bench.py --only-subs reference_job --steps 3 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_rj_w1.json 2> $OUT/prof_rj_w1.err || { echo "rocprof rj failed rc=$?"; tail -20 $OUT/prof_rj_w1.err; exit 1; }
echo rocprof rj w1 ok

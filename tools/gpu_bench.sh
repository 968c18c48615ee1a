#!/bin/bash
# GPU-box script: headline bench + rocprofv3 kernel trace (stats). Each GPU step has its own
# time limit; the script stops at the first failing GPU step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
if [ "${PROFILE:-1}" = "1" ]; then
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed rc=$?"; tail -20 $OUT/prof.err; exit 1; }
  find $OUT/prof -name "*stats*" | head
fi

#!/bin/bash
# GPU-box script: middle-scan workload (BASELINE.json configs[2]) bench + rocprofv3 kernel stats.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python bench.py --workload middle --reads ${MID_READS:-100000} --steps ${MID_STEPS:-3} --warmup 1 > $OUT/bench_middle.json 2> $OUT/bench_middle.err || { echo "middle bench failed"; tail -5 $OUT/bench_middle.err; exit 1; }
cat $OUT/bench_middle.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_middle -o run -- python3 $R/bench.py --workload middle --reads ${MID_READS:-100000} --steps 2 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_middle.log 2>&1 || { echo "middle profile failed"; tail -5 $OUT/prof_middle.log; exit 1; }
find $OUT/prof_middle -name '*kernel_stats.csv'

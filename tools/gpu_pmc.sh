#!/bin/bash
# GPU-box script: rocprofv3 PMC passes over the headline bench (each pass its own run, counters
# only with --kernel-trace; never combined with sys/runtime traces).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
ARGS="--steps 2 --warmup 1 --cpu-sample 0 --check 0 ${BENCH_ARGS:-}"
i=0
for set in "${PMC_SETS[@]:-}"; do :; done
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok: $line"
done < ${PMC_FILE:-$R/tools/pmc_sets.txt}

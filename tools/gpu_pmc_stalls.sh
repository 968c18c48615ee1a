#!/bin/bash
# GPU-box script: stall breakdown of one kernel (KRE regex) over the headline bench, one rocprofv3
# --pmc pass per counter set (each <= 8 SQ counters, --kernel-trace only), plus the counter list.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/stalls
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $line --kernel-include-regex "${KRE:-k_align<24, true}" --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --check 0 ${BENCH_ARGS:-} > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok: $line"
done < ${PMC_FILE:-$R/tools/pmc_stalls.txt}

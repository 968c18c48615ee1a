#!/bin/bash
# r05k: PMC stall breakdown of the middle scan's kernels at 20 kb (one rocprofv3 --pmc pass per
# counter set, --kernel-trace only), one-task-per-pass bands (default) and, pass 1 only, switching.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05k
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
KRE='k_seed|k_align_chunk|k_cands|k_certify|k_plan|k_round|k_mask'
ARGS="--workload middle --mean-len 20000 --steps 2 --warmup 1 --sub 0 --cpu-sample 0 --check 0 --middle-check 0"
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $line GRBM_GUI_ACTIVE --kernel-include-regex "$KRE" --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok: $line"
done < $R/tools/pmc_stalls.txt
PCABI_BAND_SWITCH=1 timeout -s KILL 120 rocprofv3 --pmc $(head -1 $R/tools/pmc_stalls.txt) GRBM_GUI_ACTIVE --kernel-include-regex "k_seed_band" --output-format csv -d $OUT/sw1 -o run -- python3 $R/bench.py $ARGS > $OUT/sw1.log 2>&1 || { echo "pmc sw failed"; tail -5 $OUT/sw1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $R/bench.py $ARGS > $OUT/kt.log 2>&1 || { echo "kt failed"; tail -5 $OUT/kt.log; exit 1; }
find $OUT -name '*.csv' | head -30

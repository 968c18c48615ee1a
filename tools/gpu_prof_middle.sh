#!/bin/bash
# GPU-box script: the middle-scan workloads' kernel statistics (rocprofv3 --kernel-trace --stats,
# 8 kb and 20 kb reads), then PMC passes over the seed-scan kernels (each pass its own run, one
# counter group, --kernel-include-regex; never combined with other traces). Stops at the first
# failure. Outputs under gpurun_out/prof_mid*.
#   KRE   kernels of the PMC passes (default: k_seed_scan|k_seed_expand|k_seed_band)
#   ARGS  extra bench.py arguments
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
KRE="${KRE:-k_seed_scan|k_seed_expand|k_seed_band}"
for ml in 8000 20000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mid$ml -o run -- python3 $R/bench.py --workload middle --mean-len $ml --steps 5 --warmup 1 --cpu-sample 0 --check 0 ${ARGS:-} > $OUT/prof_mid$ml.json 2> $OUT/prof_mid$ml.err || { echo "stats $ml failed rc=$?"; tail -20 $OUT/prof_mid$ml.err; exit 1; }
  echo "stats $ml ok"
done
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "$KRE" --output-format csv -d $OUT/prof_midpmc$i -o run -- python3 $R/bench.py --workload middle --steps 1 --warmup 1 --cpu-sample 0 --check 0 ${ARGS:-} > $OUT/prof_midpmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/prof_midpmc$i.log; exit 1; }
  echo "pmc pass $i ok: $pmc"
done

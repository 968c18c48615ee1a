#!/bin/bash
# GPU-box script: one rocprofv3 --pmc pass over a bench command for the kernels matching $KRE.
# usage: KRE=k_seed_scan PMC="SQ_WAVES SQ_INSTS_VALU ..." ARGS="--workload middle --steps 1 --warmup 0" bash tools/gpu_pmc_kernel.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-include-regex "$KRE" --output-format csv -d $OUT/pmc_k -o run -- python3 $R/bench.py $ARGS --cpu-sample 0 --check 0 > $OUT/pmc_k.log 2>&1 || { echo "pmc failed rc=$?"; tail -20 $OUT/pmc_k.log; exit 1; }
find $OUT/pmc_k -name '*counter_collection.csv'

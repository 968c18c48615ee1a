#!/bin/bash
# r06: where the middle scan's host time goes (PCABI_HOSTPROF marks), and PMC passes over the
# middle workload comparing the candidate-DP chunk kernel (per-lane gathered reads) with the
# end trim's cross kernel (tile reads)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06cpmc}
mkdir -p $OUT
cd $R
PCABI_HOSTPROF=1 timeout -k 10 300 python bench.py --workload middle --steps 6 --warmup 2 --cpu-sample 0 --check 0 > $OUT/mid8.json 2> $OUT/mid8.err || { echo "hostprof run failed rc=$?"; tail -5 $OUT/mid8.err; exit 1; }
grep hostprof $OUT/mid8.err | tail -8
export TMPDIR=/tmp
cd /tmp
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-trace --kernel-include-regex "k_align" --output-format csv -d $OUT/pmc/p$i -o run -- python3 $R/bench.py --workload middle --steps 2 --warmup 1 --cpu-sample 0 --check 0 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed rc=$?"; tail -5 $OUT/pmc$i.log; exit 1; }
  echo "pmc pass $i ok"
done
cd $R
python tools/pmc_report.py $OUT/pmc "k_align_chunk<28" "k_align<24" > $OUT/pmc_report.txt 2>&1; cat $OUT/pmc_report.txt | head -60

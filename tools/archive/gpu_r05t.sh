#!/bin/bash
# r05t: e2e with a fresh output file per step (+ timeline, write probe); the drivers sub-record;
# PCABI_MIDDLE_BATCH1 2 vs 3 on the middle / 20 kb sub-records; SQ / LDS counters of the seed
# kernels at 20 kb (one counter group per pass).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05t
mkdir -p $OUT
cd $R
PCABI_PIPE_TRACE=1 timeout -k 10 300 python bench.py --only-subs e2e,drivers --cpu-sample 0 > $OUT/e2e.json 2> $OUT/e2e.err || { echo "e2e failed rc=$?"; tail -20 $OUT/e2e.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/e2e.json')); v=d['e2e']
print('e2e', v.get('value'), v.get('ms_per_step'), v.get('breakdown_ms_per_step'), v.get('write_probe'), v.get('parity_spot_check'), v.get('error'))
v=d['drivers']; print('drivers', v.get('value'), v.get('ms_per_driver'), v.get('parity_spot_check'))
"
for b in 2 3 2 3; do
  PCABI_MIDDLE_BATCH1=$b timeout -k 10 600 python bench.py --only-subs middle,middle_20kb --cpu-sample 0 --middle-check 200 > $OUT/mid_b$b.json 2> $OUT/mid_b$b.err || { echo "bench mid failed rc=$?"; tail -20 $OUT/mid_b$b.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/mid_b$b.json'))
for k in ('middle','middle_20kb'): print('batch1=$b', k, d[k]['ms_per_step'], d[k]['middle_ms_per_step'], d[k]['parity_spot_check']['identical'])
"
done
export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "k_seed" --output-format csv -d $OUT/pmc$i -o run -- python3 $R/bench.py --workload middle --mean-len 20000 --steps 1 --warmup 1 --sub 0 --cpu-sample 0 --check 0 --middle-check 0 > $OUT/pmc$i.log 2>&1) || { echo "pmc $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
  echo "pmc $i ok"
done

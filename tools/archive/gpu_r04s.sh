#!/bin/bash
# GPU-box script (r04): the cell-mix issue-rate benchmark, then no-fork (PCABI_FORK=0) against the
# side-stream fork on the middle (8 / 20 kb), barcode and file-to-file workloads.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04s
mkdir -p $OUT
cd $R
#timeout -k 10 120 tools/cellmix_bench > $OUT/cellmix.txt 2>&1 || { echo "cellmix failed rc=$?"; cat $OUT/cellmix.txt; exit 1; }
#cat $OUT/cellmix.txt
for V in base nofork base nofork; do
  case $V in base) E="PCABI_FORK=1";; nofork) E="PCABI_FORK=0";; esac
  env $E timeout -k 10 300 python bench.py --workload middle --steps 8 --warmup 2 --cpu-sample 0 > $OUT/mid_$V.json 2> $OUT/mid_$V.err || { echo "mid $V failed rc=$?"; tail -20 $OUT/mid_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/mid_$V.json')); print('mid $V', d['ms_per_step'], d['middle_ms_per_step'], d['parity_spot_check']['identical'])"
  env $E timeout -k 10 300 python bench.py --workload middle --mean-len 20000 --steps 6 --warmup 2 --cpu-sample 0 --check 0 > $OUT/mid20_$V.json 2> $OUT/mid20_$V.err || { echo "mid20 $V failed rc=$?"; tail -20 $OUT/mid20_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/mid20_$V.json')); print('mid20 $V', d['ms_per_step'], d['middle_ms_per_step'])"
  env $E timeout -k 10 300 python bench.py --workload barcodes --steps 10 --warmup 2 --cpu-sample 0 --check 0 > $OUT/bc_$V.json 2> $OUT/bc_$V.err || { echo "bc $V failed rc=$?"; tail -20 $OUT/bc_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bc_$V.json')); print('barcodes $V', d['value'], d['ms_per_step'])"
  env $E timeout -k 10 300 python bench.py --only-subs config2_10k_119sets,check_phase --steps 10 --warmup 2 --cpu-sample 0 --check 0 > $OUT/c2_$V.json 2> $OUT/c2_$V.err || { echo "c2 $V failed rc=$?"; tail -20 $OUT/c2_$V.err; exit 1; }
  python -c "import json; D=json.load(open('$OUT/c2_$V.json')); print('config2 $V', D.get('config2_10k_119sets', {}).get('ms_per_step'), 'check_phase', D.get('check_phase', {}).get('ms_per_step'))"
done

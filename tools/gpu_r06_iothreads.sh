#!/bin/bash
# r06: the file pipeline's host threads per parse or write (PCABI_IO_THREADS, default min(16, cores)
# on the e2e workload, alternating 16 / 8 / 12, two rounds
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06iothr}
mkdir -p $OUT
cd $R
for k in 1 2 3; do
  for d in ${THREADS:-16 8 12}; do
    PCABI_IO_THREADS=$d timeout -k 10 300 python bench.py --workload e2e --reads 100000 --steps 3 --warmup 1 --cpu-sample 0 > $OUT/e2e_d${d}_$k.json 2> $OUT/e2e_d${d}_$k.err || { echo "e2e d$d failed rc=$?"; tail -20 $OUT/e2e_d${d}_$k.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('threads $d', d['ms_per_step'], d.get('step_vs_slowest_stage'), d.get('breakdown_ms_per_step'), (d.get('parity_spot_check') or {}).get('output_identical'))" $OUT/e2e_d${d}_$k.json
  done
done

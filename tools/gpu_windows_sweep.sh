#!/bin/bash
# GPU-box script: the middle workload at several mean read lengths with candidate windows off / on
# (PCABI_MIDDLE_WINDOWS), one bench process each, for the length-based switch.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/wsweep
mkdir -p $OUT
cd $R
for len in ${LENS:-8000 12000 16000 20000}; do
  for w in 0 1; do
    PCABI_MIDDLE_WINDOWS=$w timeout -k 10 240 python -u bench.py --workload middle --mean-len $len --sub 0 \
      --cpu-sample 0 --check 64 --steps ${STEPS:-10} --warmup 2 > $OUT/m${len}_w$w.json 2> $OUT/m${len}_w$w.err \
      || { echo "bench len=$len windows=$w failed rc=$?"; tail -5 $OUT/m${len}_w$w.err; exit 1; }
    echo "len=$len windows=$w: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('breakdown_ms_per_step', d.get('middle_scan_ms')))" $OUT/m${len}_w$w.json)"
  done
done

#!/bin/bash
# r06: the pinned bands' row cap (k_seed_band_pin in two launches: PCABI_PIN_ROW_CAP rows, then the
# survivors from the start; default 16) vs one launch (PCABI_PIN_ROW_CAP=0): the GPU suite with the
# cap on (and the poisoned-scratch tests), then alternating middle benches at 8 kb and 20 kb
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06rowcap}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 || { echo "GPU suite failed rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
run() {  # $1 = row cap, $2 = mean length, $3 = tag
  PCABI_PIN_ROW_CAP=$1 timeout -k 10 300 python bench.py --workload middle --mean-len $2 --steps 20 --warmup 2 --cpu-sample 0 > $OUT/mid_$3.json 2> $OUT/mid_$3.err || { echo "bench $3 failed rc=$?"; tail -20 $OUT/mid_$3.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); m=d.get('middle_phases',{}); print('$3', d.get('middle_ms_per_step'), m.get('ms',{}).get('bands'), m.get('round1_ms'), d.get('middle_hits_per_step'), d.get('parity_spot_check'))" $OUT/mid_$3.json
}
for k in 1 2; do
  run 16 8000 8k_cap16_$k || exit 1
  run 0 8000 8k_cap0_$k || exit 1
  run 16 20000 20k_cap16_$k || exit 1
  run 0 20000 20k_cap0_$k || exit 1
done
run 10 8000 8k_cap10 || exit 1
run 10 20000 20k_cap10 || exit 1

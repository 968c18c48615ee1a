#!/bin/bash
# r06: the device plan's wave target (PCABI_MIDDLE_PLAN_WAVES, default 4096) below the default:
# 4096 / 2048 / 1024 in separate processes (each keeps its round graphs), alternating, at 8 kb and
# 20 kb. (r06 balance_ab: MORE waves for the largest bucket was 0.25 ms slower at 8 kb.)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06waves}
mkdir -p $OUT
cd $R
run() {  # $1 = target, $2 = mean length, $3 = tag
  PCABI_MIDDLE_PLAN_WAVES=$1 timeout -k 10 300 python bench.py --workload middle --mean-len $2 --steps 20 --warmup 2 --cpu-sample 0 > $OUT/mid_$3.json 2> $OUT/mid_$3.err || { echo "bench $3 failed rc=$?"; tail -20 $OUT/mid_$3.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); m=d.get('middle_phases',{}); print('$3', d.get('middle_ms_per_step'), m.get('ms',{}).get('candidate_dp'), m.get('round1_ms'), d.get('middle_hits_per_step'), d.get('parity_spot_check'))" $OUT/mid_$3.json
}
for k in 1 2; do
  for w in 4096 2048 1024; do
    run $w 8000 8k_w${w}_$k || exit 1
  done
done
for w in 4096 2048 1024; do
  run $w 20000 20k_w$w || exit 1
done

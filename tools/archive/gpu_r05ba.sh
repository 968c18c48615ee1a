#!/bin/bash
# Round 2's candidate-DP buckets side by side while its bands run serial: in-process A/B of
# PCABI_MIDDLE_DP_SERIAL_FROM 1 (default at 8 kb) / 2 / 3, 8 kb, twice.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05ba
mkdir -p $OUT
cd $R
for ab in 1,2 1,3 2,3; do
timeout -k 10 300 python bench.py --workload middle --steps 24 --warmup 2 --cpu-sample 0 --check 0 --ab PCABI_MIDDLE_DP_SERIAL_FROM=$ab > $OUT/ab_$ab.json 2> $OUT/ab_$ab.err || { echo "ab failed rc=$?"; tail -20 $OUT/ab_$ab.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: v['median_ms'] for k, v in d['ab']['PCABI_MIDDLE_DP_SERIAL_FROM'].items()})" $OUT/ab_$ab.json $ab
done

#!/bin/bash
# Round 1's fork granularity, in-process A/B at 8 kb and 20 kb: the candidate-DP buckets serial or
# side by side (PCABI_MIDDLE_DP_SERIAL_FROM 0 / 1) with the bands side by side (default) and with
# the bands serial too (PCABI_MIDDLE_SERIAL_FROM=0).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05aw
mkdir -p $OUT
cd $R
for L in 8000 20000; do
timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 24 --warmup 2 --cpu-sample 0 --check 0 --ab PCABI_MIDDLE_DP_SERIAL_FROM=0,1 > $OUT/ab_bandsfork_$L.json 2> $OUT/ab_bandsfork_$L.err || { echo "ab failed rc=$?"; tail -20 $OUT/ab_bandsfork_$L.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'bands fork', {k: v['median_ms'] for k, v in d['ab']['PCABI_MIDDLE_DP_SERIAL_FROM'].items()})" $OUT/ab_bandsfork_$L.json $L
PCABI_MIDDLE_SERIAL_FROM=0 timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 24 --warmup 2 --cpu-sample 0 --check 0 --ab PCABI_MIDDLE_DP_SERIAL_FROM=0,1 > $OUT/ab_bandsserial_$L.json 2> $OUT/ab_bandsserial_$L.err || { echo "ab failed rc=$?"; tail -20 $OUT/ab_bandsserial_$L.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'bands serial', {k: v['median_ms'] for k, v in d['ab']['PCABI_MIDDLE_DP_SERIAL_FROM'].items()})" $OUT/ab_bandsserial_$L.json $L
done

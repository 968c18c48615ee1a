#!/bin/bash
# time every perf_variants/*.so on the headline bench (kernel ms/step), one process each
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/variants
for so in perf_variants/*.so; do
  n=$(basename $so .so)
  PCABI_LIB=$R/$so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 --check 64 ${BENCH_ARGS:-} > gpurun_out/variants/$n.json 2> gpurun_out/variants/$n.err || { echo "$n failed"; tail -3 gpurun_out/variants/$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/variants/$n.json')); print('$n', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('launch_ms'), d.get('middle_ms_per_step'), d['parity_spot_check'])"
done

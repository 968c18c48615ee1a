#!/bin/bash
# Kernel statistics of every perf_variants/*.so on one bench workload: rocprofv3 --kernel-trace
# --stats per variant, then the average duration of the kernels matching KRE.
#   KRE="k_seed_scan" ARGS="--workload middle --steps 3 --warmup 1" bash tools/gpu_kstat_variants.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/kvar
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for so in $R/perf_variants/*.so; do
  n=$(basename $so .so)
  PCABI_LIB=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o run -- python3 $R/bench.py ${ARGS:---workload middle --steps 3 --warmup 1} --cpu-sample 0 --check 0 > $OUT/$n.log 2>&1 || { echo "$n failed"; tail -3 $OUT/$n.log; exit 1; }
  python3 - $OUT/$n "${KRE:-k_seed}" $n <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if sys.argv[2] in r['Name']:
        print(sys.argv[3], r['Name'].split('(')[0][-40:], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us avg')
PY
done

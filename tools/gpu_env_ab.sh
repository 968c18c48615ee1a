#!/bin/bash
# A/B of an environment switch on one bench workload: rocprofv3 --kernel-trace --stats per setting,
# then the per-call durations of the kernels matching KRE.
#   VAR=PCABI_SEED_SCAN16 VALUES="1 0" KRE=k_seed_scan ARGS="--workload middle --steps 2 --warmup 1" bash tools/gpu_env_ab.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/envab
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for v in ${VALUES:-1 0}; do
  env $VAR=$v true
  export $VAR=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- python3 $R/bench.py ${ARGS:---workload middle --steps 2 --warmup 1} --cpu-sample 0 --check 0 > $OUT/$v.log 2>&1 || { echo "$VAR=$v failed"; tail -3 $OUT/$v.log; exit 1; }
  python3 - $OUT/$v "${KRE:-k_seed}" "$VAR=$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in csv.DictReader(open(f)))
print(sys.argv[3], [round((e - s) / 1e3) for s, e, n in rows if sys.argv[2] in n])
PY
done

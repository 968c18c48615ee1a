#!/bin/bash
# GPU-box script (r04): 8 kb middle step under candidate windows on/off and chunk-plan wave targets.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04h
mkdir -p $OUT
cd $R
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload middle --steps 10 --warmup 2 --cpu-sample 0 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed rc=$?"; tail -20 $OUT/$name.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); p=d['middle_phases']; print('$name', d['middle_ms_per_step'], json.dumps(p['ms']), p['dp_cells'], d['parity_spot_check']['identical'])"
}
run base PCABI_NOOP=1
run win1 PCABI_MIDDLE_WINDOWS=1
run pw8k PCABI_MIDDLE_PLAN_WAVES=8192
run pw2k PCABI_MIDDLE_PLAN_WAVES=2048
run base2 PCABI_NOOP=1
run win1b PCABI_MIDDLE_WINDOWS=1

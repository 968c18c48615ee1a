#!/bin/bash
# r06: (1) the poisoned-scratch guard against a library with the r05 memset fix reverted
# (perf_variants/r05bug.so, tools/make_r05bug.sh: the 0x3F poison is expected to fail it, 0xFF to pass);
# (2) the device plan's wave target A/B on the middle workloads (MID_AB)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06misc}
mkdir -p $OUT
cd $R
for b in 1 0x3f; do
  PCABI_POISON=$b PCABI_LIB=$R/perf_variants/r05bug.so timeout -k 10 300 python -u tests/poisoned_middle.py > $OUT/r05bug_$b.log 2>&1; rc=$?
  echo "r05bug library, poison $b: rc=$rc"; tail -3 $OUT/r05bug_$b.log
  if [ $rc -ge 124 ]; then echo "stopping: rc $rc"; exit 1; fi
done
[ "${SKIP_MIDAB:-0}" = "1" ] && exit 0
for L in 8000 20000; do
  timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 20 --warmup 2 --ab "${MID_AB:-PCABI_MIDDLE_PLAN_WAVES=4096,8192,12288}" > $OUT/midab_$L.json 2> $OUT/midab_$L.err || { echo "midab $L failed rc=$?"; tail -20 $OUT/midab_$L.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print($L, d.get('middle_ms_per_step'), {k: {v: x['median_ms'] for v, x in y.items()} for k, y in (d.get('ab') or {}).items()}, d.get('parity_spot_check'))" $OUT/midab_$L.json
done

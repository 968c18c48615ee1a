#!/bin/bash
# r06: the multi call's issue order -- the largest grouped launch first (the library) vs the side
# streams' launches first (perf_variants/smallfirst.so: TU=pcabi_engine tools/build_variant.sh
# smallfirst -DPCABI_GROUP_ISSUE_SMALL_FIRST=1, a one-off edit of pcabi_align_cross_multi_dev not
# kept in the source) -- on the headline, three alternating pairs
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06order}
mkdir -p $OUT
cd $R
for k in 1 2 3; do
  for v in large small; do
    if [ $v = large ]; then lib=$R/custom_porechop_abi_amd/libpcabi.so; else lib=$R/perf_variants/smallfirst.so; fi
    PCABI_LIB=$lib timeout -k 10 200 python bench.py --sub 0 --cpu-sample 0 --check 2000 --steps 30 > $OUT/head_${v}_$k.json 2> $OUT/head_${v}_$k.err || { echo "head $v failed rc=$?"; tail -20 $OUT/head_${v}_$k.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('$v', d['ms_per_step'], r['launch_ms'], r['align_phase']['ms'], d['parity_spot_check'])" $OUT/head_${v}_$k.json
  done
done

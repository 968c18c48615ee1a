#!/bin/bash
# r06: the 20 kb rounds' certified-out whole reads (the second, whole-read plan) on the one-lane
# chunk core, grouped (perf_variants/wholens.so: TU=pcabi_engine tools/build_variant.sh wholens
# -DPCABI_WHOLE_NOSPLIT=1, a one-off edit not kept in the source) vs the row-split core (the library,
# r05y/z), three alternating pairs at 20 kb
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06wholens}
mkdir -p $OUT
cd $R
run() {
  PCABI_LIB=$1 timeout -k 10 300 python bench.py --workload middle --mean-len 20000 --steps 20 --warmup 2 --cpu-sample 0 > $OUT/mid_$2.json 2> $OUT/mid_$2.err || { echo "bench $2 failed rc=$?"; tail -20 $OUT/mid_$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); m=d.get('middle_phases',{}); print('$2', d.get('middle_ms_per_step'), m.get('ms',{}).get('candidate_dp'), m.get('round1_ms'), d.get('middle_hits_per_step'), d.get('parity_spot_check'))" $OUT/mid_$2.json
}
for k in 1 2 3; do
  run $R/perf_variants/wholens.so ns_$k || exit 1
  run $R/custom_porechop_abi_amd/libpcabi.so split_$k || exit 1
done

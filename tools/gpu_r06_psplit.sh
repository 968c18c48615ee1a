#!/bin/bash
# r06: the whole-read rounds' packed candidate-DP buckets (36+ rows) on the row-split core, two
# lanes per chunk task (perf_variants/psplit.so: TU=pcabi_engine tools/build_variant.sh psplit
# -DPCABI_PACKED_SPLIT=1, a one-off edit not kept in the source) vs one lane (the library): middle-scan
# GPU tests with it, alternating middle benches at 8 kb, one pair at 20 kb, and the reference job
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06psplit}
mkdir -p $OUT
cd $R
PCABI_LIB=$R/perf_variants/psplit.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_gpu_parity.py > $OUT/pytest_middle.log 2>&1 || { echo "middle tests failed rc=$?"; tail -30 $OUT/pytest_middle.log; exit 1; }
tail -1 $OUT/pytest_middle.log
run() {  # $1 = library, $2 = mean length, $3 = tag
  PCABI_LIB=$1 timeout -k 10 300 python bench.py --workload middle --mean-len $2 --steps 20 --warmup 2 --cpu-sample 0 > $OUT/mid_$3.json 2> $OUT/mid_$3.err || { echo "bench $3 failed rc=$?"; tail -20 $OUT/mid_$3.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); m=d.get('middle_phases',{}); print('$3', d.get('middle_ms_per_step'), m.get('ms',{}).get('candidate_dp'), m.get('ms',{}).get('rest'), m.get('round1_ms'), d.get('middle_hits_per_step'), d.get('parity_spot_check'))" $OUT/mid_$3.json
}
LIB=$R/custom_porechop_abi_amd/libpcabi.so
NO=$R/perf_variants/psplit.so
for k in 1 2 3; do
  run $LIB 8000 8k_lib_$k || exit 1
  run $NO 8000 8k_psplit_$k || exit 1
done
run $LIB 20000 20k_lib || exit 1
run $NO 20000 20k_psplit || exit 1
for v in lib psplit; do
  if [ $v = lib ]; then lib=$LIB; else lib=$NO; fi
  PCABI_LIB=$lib timeout -k 10 300 python bench.py --only-subs reference_job --sub 1 --steps 10 --cpu-sample 0 > $OUT/rj_$v.json 2> $OUT/rj_$v.err || { echo "rj $v failed rc=$?"; tail -20 $OUT/rj_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); d=d.get('reference_job', d); print('rj $v', d['ms_per_step'], d['ms_per_phase'].get('middle_ms'))" $OUT/rj_$v.json
done

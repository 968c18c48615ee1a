#!/bin/bash
# r06: the candidate DP's run-tagged buckets (<= 28 rows) as one grouped launch (k_align_chunk_group,
# PCABI_CHUNK_GROUP=1, the built library at 5 waves per SIMD; perf_variants/cg4.so: the same kernel
# without the wave bound, 4 waves) vs one launch per bucket (PCABI_CHUNK_GROUP=0): the middle-scan
# GPU tests with it on, then alternating middle benches at 8 kb (separate processes) and 20 kb
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06cgroup}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_gpu_parity.py > $OUT/pytest_middle.log 2>&1 || { echo "middle tests failed rc=$?"; tail -30 $OUT/pytest_middle.log; exit 1; }
tail -1 $OUT/pytest_middle.log
run() {  # $1 = group on/off, $2 = library, $3 = mean length, $4 = tag
  PCABI_CHUNK_GROUP=$1 PCABI_LIB=$2 timeout -k 10 300 python bench.py --workload middle --mean-len $3 --steps 20 --warmup 2 --cpu-sample 0 > $OUT/mid_$4.json 2> $OUT/mid_$4.err || { echo "bench $4 failed rc=$?"; tail -20 $OUT/mid_$4.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); m=d.get('middle_phases',{}); print('$4', d.get('middle_ms_per_step'), m.get('ms',{}).get('candidate_dp'), m.get('ms',{}).get('rest'), m.get('round1_ms'), d.get('middle_hits_per_step'), d.get('parity_spot_check'))" $OUT/mid_$4.json
}
LIB=$R/custom_porechop_abi_amd/libpcabi.so
CG4=$R/perf_variants/cg4.so
for k in 1 2 3; do
  run 1 $LIB 8000 8k_on_$k || exit 1
  run 0 $LIB 8000 8k_off_$k || exit 1
  run 1 $CG4 8000 8k_cg4_$k || exit 1
done
run 1 $LIB 20000 20k_on || exit 1
run 0 $LIB 20000 20k_off || exit 1

#!/bin/bash
# r06: the packed grouped class split in two (36..48 rows at 4 waves per SIMD, 52..64 at 3: the built
# library) against one packed class for 36..64 (perf_variants/nosplit.so: TU="pcabi_engine
# pcabi_k_group" tools/build_variant.sh nosplit -DPCABI_GROUP_SPLIT=0): the grouped-launch parity
# tests, then the headline alternating on one box, and one middle bench (its end trim now one multi call)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06split}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_group.py > $OUT/pytest_group.log 2>&1 || { echo "group tests failed rc=$?"; tail -30 $OUT/pytest_group.log; exit 1; }
tail -1 $OUT/pytest_group.log
for k in 1 2 3; do
  for v in split nosplit; do
    if [ $v = split ]; then lib=$R/custom_porechop_abi_amd/libpcabi.so; else lib=$R/perf_variants/nosplit.so; fi
    PCABI_LIB=$lib timeout -k 10 200 python bench.py --sub 0 --cpu-sample 0 --check 0 --steps 30 > $OUT/head_${v}_$k.json 2> $OUT/head_${v}_$k.err || { echo "head $v failed rc=$?"; tail -20 $OUT/head_${v}_$k.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('$v', d['ms_per_step'], r['launch_ms'], r['frac'], r['align_phase']['ms'], r['align_phase']['frac'])" $OUT/head_${v}_$k.json
  done
done
timeout -k 10 300 python bench.py --workload middle --steps 10 --warmup 2 --cpu-sample 0 > $OUT/mid8.json 2> $OUT/mid8.err || { echo "middle failed rc=$?"; tail -20 $OUT/mid8.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('middle', d['ms_per_step'], d['middle_ms_per_step'], d['config']['end_trim'], d.get('parity_spot_check'))" $OUT/mid8.json

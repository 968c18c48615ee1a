#!/bin/bash
# r06: the candidate-DP chunk kernels' 16-byte gathered reads (PCABI_GATHER16=1, the built library)
# vs per-column dword reads (perf_variants/nogather.so: TU="pcabi_k_chunk pcabi_k_split_chunk"
# tools/build_variant.sh nogather -DPCABI_GATHER16=0): the middle-scan GPU tests, then alternating
# middle benches at 8 kb and 20 kb
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06gather}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py > $OUT/pytest_middle.log 2>&1 || { echo "middle tests failed rc=$?"; tail -30 $OUT/pytest_middle.log; exit 1; }
tail -2 $OUT/pytest_middle.log
for rep in 1 2 3; do
  for L in 8000 20000; do
    for v in gather nogather; do
      if [ $v = gather ]; then lib=$R/custom_porechop_abi_amd/libpcabi.so; else lib=$R/perf_variants/nogather.so; fi
      PCABI_LIB=$lib timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 20 --warmup 2 --cpu-sample 0 > $OUT/mid_${L}_${v}_$rep.json 2> $OUT/mid_${L}_${v}_$rep.err || { echo "bench $L $v failed rc=$?"; tail -20 $OUT/mid_${L}_${v}_$rep.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); m=d.get('middle_phases',{}); print('$rep $L $v', d.get('middle_ms_per_step'), m.get('ms',{}).get('candidate_dp'), m.get('round1_ms'), d.get('parity_spot_check'))" $OUT/mid_${L}_${v}_$rep.json
    done
  done
done

#!/bin/bash
# GPU-box script (r04): hardware queues per process (GPU_MAX_HW_QUEUES 4, the box default, vs 8)
# on the headline, the reference job and the middle step; chunk kernels at 6 waves per SIMD.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04k
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_gpu_parity.py -k "middle or seed or windows or overflow or scan" > $OUT/pytest_mid.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" $OUT/pytest_mid.log | head -20; tail -30 $OUT/pytest_mid.log; exit 1; }
tail -2 $OUT/pytest_mid.log
for Q in 4 8 4 8; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --sub 0 --steps 20 --warmup 3 --cpu-sample 0 --check 0 > $OUT/head_q$Q.json 2> $OUT/head_q$Q.err || { echo "head $Q failed rc=$?"; tail -20 $OUT/head_q$Q.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/head_q$Q.json')); print('head q=$Q', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --only-subs reference_job --steps 6 --warmup 2 --cpu-sample 0 --check 0 > $OUT/rj_q$Q.json 2> $OUT/rj_q$Q.err || { echo "rj $Q failed rc=$?"; tail -20 $OUT/rj_q$Q.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/rj_q$Q.json'))['reference_job']; print('rj q=$Q', d['ms_per_step'], d['ms_per_phase']['end_trim_align_ms'], d['ms_per_phase']['check_ms'], d['ms_per_phase']['middle_ms'], d['single_adapter_launches']['frac'])"
done
for Q in 4 8; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --workload middle --steps 8 --warmup 2 --cpu-sample 0 --check 0 > $OUT/mid_q$Q.json 2> $OUT/mid_q$Q.err || { echo "mid $Q failed rc=$?"; tail -20 $OUT/mid_q$Q.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/mid_q$Q.json')); print('mid q=$Q', d['ms_per_step'], d['middle_ms_per_step'], json.dumps(d['middle_phases']['ms']))"
done
for W in 1 6; do
  PCABI_CHUNK_WAVES=$W timeout -k 10 300 python bench.py --workload middle --steps 8 --warmup 2 --cpu-sample 0 > $OUT/mid_w$W.json 2> $OUT/mid_w$W.err || { echo "mid w$W failed rc=$?"; tail -20 $OUT/mid_w$W.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/mid_w$W.json')); print('mid chunkwaves=$W', d['middle_ms_per_step'], json.dumps(d['middle_phases']['ms']), d['parity_spot_check']['identical'])"
done
for O in 0 1 0 1; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --only-subs reference_job --rj-check-overlap $O --steps 6 --warmup 2 --cpu-sample 0 --check 0 > $OUT/rj_o$O.json 2> $OUT/rj_o$O.err || { echo "rj o$O failed rc=$?"; tail -20 $OUT/rj_o$O.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/rj_o$O.json'))['reference_job']; print('rj q8 overlap=$O', d['ms_per_step'], d['ms_per_phase']['check_ms'], d['ms_per_phase']['end_trim_align_ms'], d['single_adapter_launches']['frac'])"
done

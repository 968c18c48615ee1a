#!/bin/bash
# GPU-box script (r04): middle parity (the chunk-split path included), then A/B runs: hardware
# queues per process (4, the box default, vs 8) on the headline and the reference job; the middle
# step's chunk DP one lane per task vs 6 waves per SIMD vs the row split (K = 2, 4).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04k
mkdir -p $OUT
cd $R
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_gpu_parity.py -k "middle or seed or windows or overflow or scan or split" > $OUT/pytest_mid.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" $OUT/pytest_mid.log | head -20; tail -30 $OUT/pytest_mid.log; exit 1; }
tail -2 $OUT/pytest_mid.log
for V in base e1 w6 s2 s4 base e1 s2; do
  case $V in base) E="PCABI_NOOP=1";; e1) E="PCABI_EXPAND_PASSES=1";; w6) E="PCABI_CHUNK_WAVES=6";; s2) E="PCABI_CHUNK_SPLIT=2";; s4) E="PCABI_CHUNK_SPLIT=4";; esac
  env $E timeout -k 10 300 python bench.py --workload middle --steps 8 --warmup 2 --cpu-sample 0 > $OUT/mid_$V.json 2> $OUT/mid_$V.err || { echo "mid $V failed rc=$?"; tail -20 $OUT/mid_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/mid_$V.json')); print('mid $V', d['middle_ms_per_step'], json.dumps(d['middle_phases']['ms']), d['parity_spot_check']['identical'])"
done
for Q in 4 8 4 8; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --sub 0 --steps 20 --warmup 3 --cpu-sample 0 --check 0 > $OUT/head_q$Q.json 2> $OUT/head_q$Q.err || { echo "head $Q failed rc=$?"; tail -20 $OUT/head_q$Q.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/head_q$Q.json')); print('head q=$Q', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
done
for Q in 4 8; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --only-subs reference_job --steps 6 --warmup 2 --cpu-sample 0 --check 0 > $OUT/rj_q$Q.json 2> $OUT/rj_q$Q.err || { echo "rj $Q failed rc=$?"; tail -20 $OUT/rj_q$Q.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/rj_q$Q.json'))['reference_job']; print('rj q=$Q', d['ms_per_step'], d['ms_per_phase']['end_trim_align_ms'], d['ms_per_phase']['check_ms'], d['ms_per_phase']['middle_ms'], d['single_adapter_launches']['frac'])"
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --only-subs reference_job --rj-check-overlap 1 --steps 6 --warmup 2 --cpu-sample 0 --check 0 > $OUT/rj_o_q$Q.json 2> $OUT/rj_o_q$Q.err || { echo "rj o $Q failed rc=$?"; tail -20 $OUT/rj_o_q$Q.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/rj_o_q$Q.json'))['reference_job']; print('rj overlap q=$Q', d['ms_per_step'], d['ms_per_phase']['check_ms'])"
done

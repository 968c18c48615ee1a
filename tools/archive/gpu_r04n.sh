#!/bin/bash
# GPU-box script (r04): one-wave chunk blocks (PCABI_CHUNK_WPB=1) parity and A/B on the middle step,
# and the reference job with it; CU-masked side streams (PCABI_SIDE_CUMASK=1) on the headline and the
# reference job.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04n
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py -k "one_wave or one_pass" > $OUT/pytest_wpb.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" $OUT/pytest_wpb.log | head -20; tail -30 $OUT/pytest_wpb.log; exit 1; }
tail -2 $OUT/pytest_wpb.log
for V in base wpb1 base wpb1; do
  case $V in base) E="PCABI_NOOP=1";; wpb1) E="PCABI_CHUNK_WPB=1";; esac
  env $E timeout -k 10 300 python bench.py --workload middle --steps 8 --warmup 2 --cpu-sample 0 > $OUT/mid_$V.json 2> $OUT/mid_$V.err || { echo "mid $V failed rc=$?"; tail -20 $OUT/mid_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/mid_$V.json')); print('mid $V', d['middle_ms_per_step'], json.dumps(d['middle_phases']['ms']), d['parity_spot_check']['identical'])"
done
env PCABI_CHUNK_WPB=1 timeout -k 10 300 python bench.py --only-subs reference_job --steps 6 --warmup 2 --cpu-sample 0 > $OUT/rj_wpb1.json 2> $OUT/rj_wpb1.err || { echo "rj wpb1 failed rc=$?"; tail -20 $OUT/rj_wpb1.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/rj_wpb1.json'))['reference_job']; print('rj wpb1', d['ms_per_step'], json.dumps(d['ms_per_phase']))"
for V in base cm base cm; do
  case $V in base) E="PCABI_NOOP=1";; cm) E="PCABI_SIDE_CUMASK=1";; esac
  env $E timeout -k 10 300 python bench.py --sub 0 --steps 20 --warmup 3 --cpu-sample 0 --check 0 > $OUT/head_$V.json 2> $OUT/head_$V.err || { echo "head $V failed rc=$?"; tail -20 $OUT/head_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/head_$V.json')); print('head $V', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
  env $E timeout -k 10 300 python bench.py --only-subs reference_job --steps 6 --warmup 2 --cpu-sample 0 --check 0 > $OUT/rj_$V.json 2> $OUT/rj_$V.err || { echo "rj $V failed rc=$?"; tail -20 $OUT/rj_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/rj_$V.json'))['reference_job']; print('rj $V', d['ms_per_step'], json.dumps(d['ms_per_phase']), d['single_adapter_launches']['frac'])"
done

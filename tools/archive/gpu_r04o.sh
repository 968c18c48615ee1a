#!/bin/bash
# GPU-box script (r04): chunk-block parity (one-wave default, four-wave switch), then hardware
# queues per process 1 / 2 / 3 / 4 on the headline, the reference job and the 8 kb middle step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04o
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_drivers.py -k "one_wave or one_pass or chunk or drivers" > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for Q in 2 4 3 1 2 4; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --sub 0 --steps 20 --warmup 3 --cpu-sample 0 --check 0 > $OUT/head_q$Q.json 2> $OUT/head_q$Q.err || { echo "head $Q failed rc=$?"; tail -20 $OUT/head_q$Q.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/head_q$Q.json')); print('head q=$Q', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --only-subs reference_job --steps 6 --warmup 2 --cpu-sample 0 --check 0 > $OUT/rj_q$Q.json 2> $OUT/rj_q$Q.err || { echo "rj $Q failed rc=$?"; tail -20 $OUT/rj_q$Q.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/rj_q$Q.json'))['reference_job']; print('rj q=$Q', d['ms_per_step'], json.dumps(d['ms_per_phase']), d['single_adapter_launches']['frac'])"
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --workload middle --steps 8 --warmup 2 --cpu-sample 0 --check 0 > $OUT/mid_q$Q.json 2> $OUT/mid_q$Q.err || { echo "mid $Q failed rc=$?"; tail -20 $OUT/mid_q$Q.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/mid_q$Q.json')); print('mid q=$Q', d['value'], d['ms_per_step'], d['middle_ms_per_step'])"
done
bash tools/gpu_r04p.sh
bash tools/gpu_r04q.sh

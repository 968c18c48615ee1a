#!/bin/bash
# r05b: (1) input-preserving middle scan -- middle-path GPU tests, middle / 20 kb / reference-job
# sub-records; (2) the dominant kernel's replay microbenchmark (tools/replay_k24) by events and under
# rocprofv3 PMC, next to the same PMC passes of the real kernel in the headline bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05b
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_pipeline.py > $OUT/pytest_mid.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest_mid.log; exit 1; }
tail -3 $OUT/pytest_mid.log
timeout -k 10 600 python bench.py --only-subs middle,middle_20kb,reference_job > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench.err; exit 1; }
echo bench ok
timeout -k 10 120 tools/replay_k24 > $OUT/replay.json 2> $OUT/replay.err || { echo "replay failed rc=$?"; cat $OUT/replay.err; exit 1; }
cat $OUT/replay.json
export TMPDIR=/tmp
cd /tmp
i=0
for pmc in "SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $OUT/rp_pmc$i -o run -- $R/tools/replay_k24 17986 150 5 > $OUT/rp_pmc$i.log 2>&1 || { echo "replay pmc pass $i failed"; tail -5 $OUT/rp_pmc$i.log; exit 1; }
  echo "replay pmc pass $i ok"
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "k_align<24, true" --output-format csv -d $OUT/kp_pmc$i -o run -- python3 $R/bench.py --sub 0 --steps 2 --warmup 1 --cpu-sample 0 --check 0 > $OUT/kp_pmc$i.log 2>&1 || { echo "kernel pmc pass $i failed"; tail -5 $OUT/kp_pmc$i.log; exit 1; }
  echo "kernel pmc pass $i ok"
done

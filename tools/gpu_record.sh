#!/bin/bash
# GPU-box script for a performance record: the GPU test suite, the default bench line, a
# rocprofv3 kernel-trace summary of the headline bench, and PMC passes (HBM traffic, stalls) of the
# dominant kernel -- each step time-limited, stopping at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench.err; exit 1; }
echo bench ok
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --sub 0 --steps 5 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed rc=$?"; tail -20 $OUT/prof.err; exit 1; }
echo rocprof ok
KRE="${KRE:-k_align<24, true}"
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "$KRE" --output-format csv -d $OUT/pmc$i -o run -- python3 $R/bench.py --sub 0 --steps 2 --warmup 1 --cpu-sample 0 --check 0 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
  echo "pmc pass $i ok: $pmc"
done

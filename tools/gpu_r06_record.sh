#!/bin/bash
# GPU-box script for the r06 performance record: the GPU test suite (SKIP_TESTS=1 skips it), the
# default bench line (every sub-record), rocprofv3 kernel-trace summaries of the headline bench, the
# reference job and the 8 kb / 20 kb middle workloads, and PMC passes (each its own run, counters
# with --kernel-trace only) of the headline's grouped run-tagged launch -- each step time-limited,
# stopping at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06final}
mkdir -p $OUT
cd $R
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 900 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench_default.err; exit 1; }
  python tools/bench_summary.py $OUT/bench_default.json
fi
export TMPDIR=/tmp
cd /tmp
for spec in "head|--sub 0 --steps 5 --warmup 1" "rj|--only-subs reference_job --steps 3 --warmup 1" "mid8|--workload middle --steps 3 --warmup 1" "mid20|--workload middle --mean-len 20000 --steps 3 --warmup 1"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$name -o run -- python3 $R/bench.py $args --cpu-sample 0 --check 0 > $OUT/prof_$name.json 2> $OUT/prof_$name.err || { echo "rocprof $name failed rc=$?"; tail -20 $OUT/prof_$name.err; exit 1; }
  echo rocprof $name ok
done
KRE="${KRE:-k_align_group<0>}"
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "$KRE" --kernel-trace --output-format csv -d $OUT/pmc/p$i -o run -- python3 $R/bench.py --sub 0 --steps 2 --warmup 1 --cpu-sample 0 --check 0 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
  echo "pmc pass $i ok: $pmc"
done
cd $R
python tools/pmc_report.py $OUT/pmc "$KRE" > $OUT/pmc_report.txt 2>&1 && cat $OUT/pmc_report.txt

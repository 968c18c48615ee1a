#!/bin/bash
# GPU-box script: the whole GPU test suite, then the benches named in BENCHES (bench.py argument
# strings separated by ';'), each with its own time limit; stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
i=0
IFS=';' read -ra BS <<< "${BENCHES:-}"
for b in "${BS[@]}"; do
  i=$((i+1))
  timeout -k 10 600 python bench.py $b > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { echo "bench $i failed rc=$?: $b"; tail -20 $OUT/bench_$i.err; exit 1; }
  echo "bench $i: $b"; cat $OUT/bench_$i.json
done
if [ -n "${PROF:-}" ]; then
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_x -o run -- python3 $R/bench.py $PROF --cpu-sample 0 --check 0 > $OUT/prof_x.log 2>&1 || { echo "rocprof failed rc=$?"; tail -20 $OUT/prof_x.log; exit 1; }
  find $OUT/prof_x -name '*kernel_stats.csv'
fi

#!/bin/bash
# Graph replay of the serial rounds: the middle GPU tests (graph replay parity included), then an
# in-process A/B PCABI_MIDDLE_GRAPHS=1,0 at 8 kb and 20 kb.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05av
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests -k "middle or seed or window or round or overflow or shadow or graph" > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for L in 8000 20000; do
timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 24 --warmup 2 --cpu-sample 0 --check 0 --ab PCABI_MIDDLE_GRAPHS=1,0 > $OUT/ab_$L.json 2> $OUT/ab_$L.err || { echo "ab failed rc=$?"; tail -20 $OUT/ab_$L.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: v['median_ms'] for k, v in d['ab']['PCABI_MIDDLE_GRAPHS'].items()})" $OUT/ab_$L.json $L
done

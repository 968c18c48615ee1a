#!/bin/bash
# r05f: k_align_tile (cross mode of the packed / run-tagged cores, 8 waves per SIMD at 24 rows):
# the whole GPU suite, the headline line alone, and the middle scan's host marks.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05f
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --sub 0 > $OUT/head.json 2> $OUT/head.err || { echo "bench failed rc=$?"; tail -20 $OUT/head.err; exit 1; }
cat $OUT/head.json | python -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['value'], d['roofline'])"
for L in 20000 8000; do
PCABI_HOSTPROF=1 timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 4 --warmup 1 --cpu-sample 0 --check 0 > $OUT/mid$L.json 2> $OUT/mid$L.err || { echo "bench failed rc=$?"; tail -20 $OUT/mid$L.err; exit 1; }
grep hostprof $OUT/mid$L.err | tail -8
done
PCABI_DEBUG=1 timeout -k 10 300 python bench.py --workload middle --mean-len 20000 --steps 1 --warmup 1 --cpu-sample 0 --check 0 > $OUT/dbg20.json 2> $OUT/dbg20.err || { echo "debug bench failed rc=$?"; tail -20 $OUT/dbg20.err; exit 1; }
grep "pcabi\]" $OUT/dbg20.err | tail -30

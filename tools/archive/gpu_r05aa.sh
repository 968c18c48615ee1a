#!/bin/bash
# r05aa: single-pass reader line scan + split by round mode: io / pipeline / middle-path GPU tests,
# e2e (timeline), in-process A/B of the split hint (x) against 0 / 2 at 8 and 20 kb.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05aa
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_io.py tests/test_pipeline.py tests/test_gpu_middle_paths.py tests/test_verbose_output.py > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
PCABI_PIPE_TRACE=1 timeout -k 10 300 python bench.py --only-subs e2e --cpu-sample 0 > $OUT/e2e.json 2> $OUT/e2e.err || { echo "e2e failed rc=$?"; tail -20 $OUT/e2e.err; exit 1; }
python -c "
import json; v=json.load(open('$OUT/e2e.json'))['e2e']
print('e2e', v.get('value'), v.get('ms_per_step'), v.get('breakdown_ms_per_step'), v.get('parity_spot_check'), v.get('error'))
"
for ml in 8000 20000; do
  for ab in PCABI_CHUNK_SPLIT=0,x PCABI_CHUNK_SPLIT=2,x; do
    timeout -k 10 300 python bench.py --workload middle --mean-len $ml --steps 24 --warmup 3 --sub 0 --cpu-sample 0 --check 0 --middle-check 0 --ab $ab > $OUT/ab_$ml.json 2> $OUT/ab_$ml.err || { echo "ab $ml failed"; tail -20 $OUT/ab_$ml.err; exit 1; }
    python -c "
import json; d=json.load(open('$OUT/ab_$ml.json'))
ab=d['ab']; k=list(ab)[0]
print('$ml', '$ab', {v: x['median_ms'] for v, x in ab[k].items() if v})
"
  done
done

#!/bin/bash
# r05ac: small first batch + device-buffer headroom in the pipeline (e2e at 12.5 k and 6.25 k
# reads per batch, timelines); round graphs captured on a key's second sight (middle-path tests,
# windows A/B at 8 / 12 / 20 kb with graphs off).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05ac
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pipeline.py tests/test_gpu_middle_paths.py tests/test_shards.py > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for b in 12500 6250; do
  PCABI_PIPE_TRACE=1 timeout -k 10 300 python bench.py --only-subs e2e --cpu-sample 0 --e2e-batch $b > $OUT/e2e_$b.json 2> $OUT/e2e_$b.err || { echo "e2e failed rc=$?"; tail -20 $OUT/e2e_$b.err; exit 1; }
  python -c "
import json; v=json.load(open('$OUT/e2e_$b.json'))['e2e']
print('e2e $b', v.get('value'), v.get('ms_per_step'), v.get('breakdown_ms_per_step'), v.get('parity_spot_check', {}).get('output_identical'), v.get('error'))
"
done
for ml in 8000 14000 20000; do
  PCABI_MIDDLE_GRAPHS=0 timeout -k 10 300 python bench.py --workload middle --mean-len $ml --steps 24 --warmup 3 --sub 0 --cpu-sample 0 --check 0 --middle-check 0 --ab PCABI_MIDDLE_WINDOWS=0,1 > $OUT/ab_win_$ml.json 2> $OUT/ab_win_$ml.err || { echo "ab $ml failed"; tail -20 $OUT/ab_win_$ml.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/ab_win_$ml.json'))
ab=d['ab']; k=list(ab)[0]
print('$ml', k, {v: x['median_ms'] for v, x in ab[k].items() if v})
"
done

#!/bin/bash
# r06: band kernel v3 (lane refill, transposed read slots) parity and A/B; the grouped headline
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06v3}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_group.py > $OUT/pytest_group.log 2>&1 || { echo "group tests failed rc=$?"; tail -30 $OUT/pytest_group.log; exit 1; }
tail -1 $OUT/pytest_group.log
PCABI_BAND_V3=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_gpu_parity.py tests/test_gpu_long.py -k "middle or seed or scan or window or round or chunk or poison" > $OUT/pytest_v3.log 2>&1 || { echo "v3 tests failed rc=$?"; tail -30 $OUT/pytest_v3.log; exit 1; }
tail -1 $OUT/pytest_v3.log
for L in 8000 20000; do
  timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 20 --warmup 2 --ab "PCABI_BAND_V3=0,1" > $OUT/midab_$L.json 2> $OUT/midab_$L.err || { echo "midab $L failed rc=$?"; tail -20 $OUT/midab_$L.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print($L, d.get('middle_ms_per_step'), {k: {v: x['median_ms'] for v, x in y.items()} for k, y in (d.get('ab') or {}).items()}, d.get('parity_spot_check'))" $OUT/midab_$L.json
done
timeout -k 10 300 python bench.py --sub 0 --cpu-sample 0 > $OUT/head.json 2> $OUT/head.err || { echo "head failed rc=$?"; tail -20 $OUT/head.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('head', d['ms_per_step'], r['launch_ms'], r['frac'], r['align_phase'], d['parity_spot_check'])" $OUT/head.json

#!/bin/bash
# r06: the tile transpose and end-trim epilogue rewrite -- parity (tiled cross products, end decisions,
# drivers, pipeline) and the headline
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06epi}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_drivers.py tests/test_pipeline.py tests/test_gpu_group.py > $OUT/pytest_epi.log 2>&1 || { echo "epi tests failed rc=$?"; tail -30 $OUT/pytest_epi.log; exit 1; }
tail -1 $OUT/pytest_epi.log
for k in 1 2; do
  timeout -k 10 200 python bench.py --sub 0 --cpu-sample 0 --steps 30 > $OUT/head_$k.json 2> $OUT/head_$k.err || { echo "head failed rc=$?"; tail -20 $OUT/head_$k.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('head', d['ms_per_step'], r['launch_ms'], r['frac'], r['align_phase']['ms'], d['parity_spot_check'])" $OUT/head_$k.json
done

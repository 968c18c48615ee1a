#!/bin/bash
# End-trim driver without the set expansion / sort for distinct adapters: the driver GPU tests, then
# the drivers sub-record twice.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05ay
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_drivers.py tests/test_verbose_output.py tests/test_shards.py > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
timeout -k 10 300 python bench.py --only-subs drivers --cpu-sample 0 > $OUT/drivers$i.json 2> $OUT/drivers$i.err || { echo "bench failed rc=$?"; tail -20 $OUT/drivers$i.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])).get('drivers',{}); print({k: d.get(k) for k in ('value','ms_per_step','ms_per_driver','library_call_ms','parity_spot_check')})" $OUT/drivers$i.json
done

#!/bin/bash
# Staging pipeline + seed-scan occupancy check: the middle / host-string GPU tests, the drivers
# sub-record twice, the 8 kb / 20 kb middle workloads, and a kernel trace of the 20 kb one.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05ai
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests -k "host_string or seqs or drivers or middle or seed" > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
timeout -k 10 300 python bench.py --only-subs drivers --cpu-sample 0 > $OUT/drivers$i.json 2> $OUT/drivers$i.err || { echo "bench failed rc=$?"; tail -20 $OUT/drivers$i.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])).get('drivers',{}); print({k: d.get(k) for k in ('value','ms_per_driver','library_call_ms','parity_spot_check')})" $OUT/drivers$i.json
done
for L in 8000 20000; do
timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 10 --warmup 2 --cpu-sample 0 > $OUT/mid$L.json 2> $OUT/mid$L.err || { echo "mid failed rc=$?"; tail -20 $OUT/mid$L.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: d.get(k) for k in ('value','ms_per_step','middle_ms_per_step')})" $OUT/mid$L.json $L
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mid20 -o run -- python3 $R/bench.py --workload middle --mean-len 20000 --steps 3 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_mid20.json 2> $OUT/prof_mid20.err || { echo "rocprof mid20 failed rc=$?"; tail -20 $OUT/prof_mid20.err; exit 1; }
echo rocprof ok

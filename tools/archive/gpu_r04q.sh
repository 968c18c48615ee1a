#!/bin/bash
# GPU-box script (r04): the reference-API drivers after the native host passes -- the drivers
# sub-record and a cProfile of the end-trim and middle drivers.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04q
mkdir -p $OUT
cd $R
timeout -k 10 400 python bench.py --only-subs drivers --steps 3 --warmup 1 --cpu-sample 0 > $OUT/drivers.json 2> $OUT/drivers.err || { echo "drivers failed rc=$?"; tail -20 $OUT/drivers.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/drivers.json'))['drivers']; print('drivers', d['value'], d['ms_per_driver'], d['nanopore_read_objects_ms'], d['parity_spot_check'])"
timeout -k 10 400 python tools/profile_drivers.py > $OUT/drivers_cprofile.txt 2>&1 || { echo "profile failed rc=$?"; tail -20 $OUT/drivers_cprofile.txt; exit 1; }
grep -E "^== " $OUT/drivers_cprofile.txt

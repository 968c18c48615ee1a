#!/bin/bash
# End-decisions phase marks (PCABI_END_PROF) under the drivers profile, then the drivers sub-record twice.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05al
mkdir -p $OUT
cd $R
PCABI_END_PROF=1 timeout -k 10 300 python tools/prof_drivers.py > $OUT/prof.txt 2> $OUT/prof.err || { echo "prof failed"; tail -5 $OUT/prof.err; exit 1; }
grep plain $OUT/prof.txt
tail -12 $OUT/prof.err
for i in 1 2; do
timeout -k 10 300 python bench.py --only-subs drivers --cpu-sample 0 > $OUT/drivers$i.json 2> $OUT/drivers$i.err || { echo "bench failed rc=$?"; tail -20 $OUT/drivers$i.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])).get('drivers',{}); print({k: d.get(k) for k in ('value','ms_per_driver','library_call_ms','parity_spot_check')})" $OUT/drivers$i.json
done

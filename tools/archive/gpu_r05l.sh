#!/bin/bash
# r05l: host-string middle scan (pcabi_middle_scan_seqs) + GC pause in append_rows: tests, the
# reference-API drivers, e2e with the reader's busy time (12.5k and 6.25k-read batches).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05l
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_drivers.py tests/test_abi.py tests/test_pipeline.py > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python tools/band_stats.py 20000 > $OUT/band_stats.txt 2>&1 || { echo "band stats failed"; tail -5 $OUT/band_stats.txt; exit 1; }
cat $OUT/band_stats.txt
timeout -k 10 600 python bench.py --only-subs middle,middle_20kb --cpu-sample 0 > $OUT/mid.json 2> $OUT/mid.err || { echo "bench mid failed rc=$?"; tail -20 $OUT/mid.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/mid.json'))
for k in ('middle','middle_20kb'): print(k, d[k]['ms_per_step'], d[k]['middle_ms_per_step'], d[k]['parity_spot_check']['identical'], d[k]['middle_phases']['ms'], json.dumps(d[k]['middle_phases']['roofline'].get('bands')))
"
timeout -k 10 600 python bench.py --only-subs drivers,e2e --cpu-sample 0 > $OUT/subs.json 2> $OUT/subs.err || { echo "bench failed rc=$?"; tail -20 $OUT/subs.err; exit 1; }
timeout -k 10 600 python bench.py --only-subs e2e --cpu-sample 0 --e2e-batch 6250 > $OUT/e2e_6250.json 2> $OUT/e2e_6250.err || { echo "bench failed rc=$?"; tail -20 $OUT/e2e_6250.err; exit 1; }
python - <<PY
import json
for f in ('$OUT/subs.json', '$OUT/e2e_6250.json'):
    d = json.load(open(f))
    for k in ('drivers', 'e2e'):
        if k in d:
            v = d[k]
            print(f, k, v['value'], v['ms_per_step'], v.get('ms_per_driver'), v.get('breakdown_ms_per_step'), v.get('step_vs_slowest_stage'), v.get('parity_spot_check'))
PY

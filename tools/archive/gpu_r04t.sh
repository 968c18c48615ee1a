#!/bin/bash
# GPU-box script (r04): side-stream switch parity, then the default bench line (every sub-record).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04t
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "tiled_cross" > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 900 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench_default.err; exit 1; }
python - $OUT/bench_default.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(json.dumps({k: d.get(k) for k in ('value', 'ms_per_step')}), d['config'].get('side_streams'), d['roofline']['frac'])
for k in ('reference_job', 'middle', 'middle_20kb', 'fused_schedule', 'barcodes', 'config2_10k_119sets', 'drivers', 'check_phase', 'e2e'):
    v = d.get(k) or {}
    print(k, json.dumps({x: v.get(x) for x in ('value', 'ms_per_step', 'middle_ms_per_step', 'ms_per_phase', 'error')})[:500])
    if k == 'reference_job':
        print('  single_adapter frac', (v.get('single_adapter_launches') or {}).get('frac'), 'parity', v.get('parity_spot_check'))
PY

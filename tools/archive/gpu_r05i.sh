#!/bin/bash
# r05i: per-stream side streams, pinned batch buffers, the 8-batch e2e with its oracle-driven
# output check; then the band-lane statistics (experiment build).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05i
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_pipeline.py tests/test_io.py > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for P in 1 0; do
PCABI_PIN_BATCHES=$P timeout -k 10 600 python bench.py --only-subs e2e > $OUT/e2e_pin$P.json 2> $OUT/e2e_pin$P.err || { echo "bench failed rc=$?"; tail -20 $OUT/e2e_pin$P.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/e2e_pin$P.json'))['e2e']
print('pin=$P', d['value'], d['ms_per_step'], d['breakdown_ms_per_step'], d['parity_spot_check'], d['write_probe'])
"
done
PCABI_LIB=perf_variants/bandstats.so timeout -k 10 300 python tools/band_stats.py 20000 && PCABI_LIB=perf_variants/bandstats.so timeout -k 10 300 python tools/band_stats.py 8000

#!/bin/bash
# r05af: batch blocks with headroom (the block cache reuses them across batches), populate-ahead
# that never lags the reader: io / pipeline GPU tests, e2e twice (timelines, reader marks).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05af
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_io.py tests/test_pipeline.py > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  PCABI_IOPROF=$((i - 1)) PCABI_PIPE_TRACE=1 timeout -k 10 300 python bench.py --only-subs e2e --cpu-sample 0 > $OUT/e2e_$i.json 2> $OUT/e2e_$i.err || { echo "e2e failed rc=$?"; tail -20 $OUT/e2e_$i.err; exit 1; }
  python -c "
import json; v=json.load(open('$OUT/e2e_$i.json'))['e2e']
print('e2e $i', v.get('value'), v.get('ms_per_step'), v.get('breakdown_ms_per_step'), v.get('parity_spot_check', {}).get('output_identical'), v.get('error'))
"
done
grep 'pcabi io' $OUT/e2e_2.err | tail -12

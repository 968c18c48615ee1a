#!/bin/bash
# GPU-box script (r04): middle parity after the edge-band exit, then the 8 kb middle step under a few
# expansion grids (PCABI_EXPAND_BLOCKS) with kernel traces.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04e
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_gpu_parity.py -k "middle or seed or windows or overflow or scan" > $OUT/pytest_mid.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" $OUT/pytest_mid.log | head -20; tail -30 $OUT/pytest_mid.log; exit 1; }
tail -2 $OUT/pytest_mid.log
for EB in 0 256 512; do
  if [ "$EB" = 0 ]; then unset PCABI_EXPAND_BLOCKS; else export PCABI_EXPAND_BLOCKS=$EB; fi
  timeout -k 10 300 python bench.py --workload middle --steps 8 --warmup 2 --cpu-sample 0 > $OUT/mid8_$EB.json 2> $OUT/mid8_$EB.err || { echo "mid $EB failed rc=$?"; tail -20 $OUT/mid8_$EB.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/mid8_$EB.json')); p=d['middle_phases']; print('mid8 eb=$EB', d['value'], d['ms_per_step'], d['middle_ms_per_step'], json.dumps(p['ms']), p['round1_ms'], d['parity_spot_check'])"
done
unset PCABI_EXPAND_BLOCKS
timeout -k 10 300 python bench.py --workload middle --mean-len 20000 --steps 8 --warmup 2 --cpu-sample 0 > $OUT/mid20.json 2> $OUT/mid20.err || { echo "mid20 failed rc=$?"; tail -20 $OUT/mid20.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/mid20.json')); p=d['middle_phases']; print('mid20', d['value'], d['ms_per_step'], d['middle_ms_per_step'], json.dumps(p['ms']), p['round1_ms'], d['parity_spot_check'])"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mid8 -o run -- python3 $R/bench.py --workload middle --steps 3 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_mid8.json 2> $OUT/prof_mid8.err || { echo "rocprof failed rc=$?"; tail -20 $OUT/prof_mid8.err; exit 1; }
echo done

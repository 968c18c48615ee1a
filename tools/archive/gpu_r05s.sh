#!/bin/bash
# r05s: band bounds below T left unwritten (no atomic per failed probe hit): middle-path tests,
# middle / 20 kb sub-records; FETCH_SIZE / WRITE_SIZE of the band kernels at 20 kb; the e2e
# pipeline's timeline (PCABI_PIPE_TRACE=1).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05s
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python bench.py --only-subs middle,middle_20kb --cpu-sample 0 > $OUT/mid.json 2> $OUT/mid.err || { echo "bench mid failed rc=$?"; tail -20 $OUT/mid.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/mid.json'))
for k in ('middle','middle_20kb'): print(k, d[k]['ms_per_step'], d[k]['middle_ms_per_step'], d[k]['parity_spot_check'], d[k]['middle_phases']['ms'])
"
PCABI_PIPE_TRACE=1 timeout -k 10 300 python bench.py --only-subs e2e --cpu-sample 0 > $OUT/e2e.json 2> $OUT/e2e.err || { echo "e2e failed rc=$?"; tail -20 $OUT/e2e.err; exit 1; }
python -c "
import json; v=json.load(open('$OUT/e2e.json'))['e2e']
print('e2e', v['value'], v['ms_per_step'], v['breakdown_ms_per_step'])
"
export TMPDIR=/tmp
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "k_seed" --output-format csv -d $OUT/pmc$i -o run -- python3 $R/bench.py --workload middle --mean-len 20000 --steps 1 --warmup 1 --sub 0 --cpu-sample 0 --check 0 --middle-check 0 > $OUT/pmc$i.log 2>&1) || { echo "pmc $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
  echo "pmc $i ok"
done

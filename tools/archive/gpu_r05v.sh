#!/bin/bash
# r05v: dword-interleaved band slots + triple-buffered seed scan: middle-path / parity GPU tests,
# middle / 20 kb / reference-job sub-records, kernel stats of the 20 kb middle workload.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05v
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
timeout -k 10 600 python bench.py --only-subs middle,middle_20kb,reference_job --cpu-sample 0 > $OUT/mid$i.json 2> $OUT/mid$i.err || { echo "bench mid failed rc=$?"; tail -20 $OUT/mid$i.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/mid$i.json'))
for k in ('middle','middle_20kb'): print(k, d[k]['ms_per_step'], d[k]['middle_ms_per_step'], d[k]['parity_spot_check'], d[k]['middle_phases']['ms'], d[k]['middle_phases']['roofline']['k_seed_scan']['frac'])
r=d['reference_job']; print('reference_job', r.get('ms_per_step'), r.get('ms_per_phase'))
"
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof20000 -o run -- python3 $R/bench.py --workload middle --mean-len 20000 --steps 3 --warmup 1 --sub 0 --cpu-sample 0 --check 0 --middle-check 0 > $OUT/prof20000.json 2> $OUT/prof20000.err) || { echo "prof failed"; tail -20 $OUT/prof20000.err; exit 1; }
echo prof ok

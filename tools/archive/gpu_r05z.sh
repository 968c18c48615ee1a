#!/bin/bash
# r05z: the whole GPU suite and the default bench line on the current code (two-lane split only
# for the whole-read plan, adaptive first batch, graph-replayed rounds, reader populate-ahead);
# in-process A/B of the split hint against a split everywhere; e2e at 6250-read batches.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05z
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench.json'))
print('headline', d['value'], d['ms_per_step'], d['roofline']['frac'])
for k in ('middle','middle_20kb'): print(k, d[k].get('ms_per_step'), d[k].get('middle_ms_per_step'), d[k].get('parity_spot_check'))
for k in ('reference_job','e2e','drivers','barcodes','config2_10k_119sets','check_phase','compat','kmer'): print(k, d[k].get('value'), d[k].get('ms_per_step'), d[k].get('error'))
"
for ml in 8000 20000; do
  timeout -k 10 300 python bench.py --workload middle --mean-len $ml --steps 24 --warmup 3 --sub 0 --cpu-sample 0 --check 0 --middle-check 0 --ab PCABI_CHUNK_SPLIT=2,x > $OUT/ab_split_$ml.json 2> $OUT/ab_split_$ml.err || { echo "ab $ml failed"; tail -20 $OUT/ab_split_$ml.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/ab_split_$ml.json'))
ab=d['ab']; k=list(ab)[0]
print('$ml', k, {v: x['median_ms'] for v, x in ab[k].items()})
"
done
PCABI_PIPE_TRACE=1 timeout -k 10 300 python bench.py --only-subs e2e --cpu-sample 0 --e2e-batch 6250 > $OUT/e2e_6250.json 2> $OUT/e2e_6250.err || { echo "e2e failed rc=$?"; tail -20 $OUT/e2e_6250.err; exit 1; }
python -c "
import json; v=json.load(open('$OUT/e2e_6250.json'))['e2e']
print('e2e 6250', v.get('value'), v.get('ms_per_step'), v.get('breakdown_ms_per_step'), v.get('error'))
"

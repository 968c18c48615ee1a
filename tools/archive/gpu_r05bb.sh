#!/bin/bash
# Expansion with three hits per thread and pass (64 VGPRs, two blocks per CU): the seed GPU tests
# with PCABI_EXPAND_HITS=3, then in-process A/B 3,2 at 8 kb and 20 kb.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05bb
mkdir -p $OUT
cd $R
PCABI_EXPAND_HITS=3 timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests -k "middle or seed or overflow" > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for L in 8000 20000; do
timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 24 --warmup 2 --cpu-sample 0 --check 0 --ab PCABI_EXPAND_HITS=3,2 > $OUT/ab_$L.json 2> $OUT/ab_$L.err || { echo "ab failed rc=$?"; tail -20 $OUT/ab_$L.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k: v['median_ms'] for k, v in d['ab']['PCABI_EXPAND_HITS'].items()})" $OUT/ab_$L.json $L
done

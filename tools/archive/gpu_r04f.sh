#!/bin/bash
# GPU-box script (r04): PMC passes on the seed band kernels of the 8 kb middle step (why an edge-band
# launch of a few thousand tasks takes ~55 us).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04f
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py tests/test_gpu_parity.py -k "middle or seed or windows or overflow or scan" > $OUT/pytest_mid.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" $OUT/pytest_mid.log | head -20; tail -30 $OUT/pytest_mid.log; exit 1; }
tail -2 $OUT/pytest_mid.log
for L in 8000 20000; do
  timeout -k 10 300 python bench.py --workload middle --mean-len $L --steps 8 --warmup 2 --cpu-sample 0 > $OUT/mid_$L.json 2> $OUT/mid_$L.err || { echo "mid $L failed rc=$?"; tail -20 $OUT/mid_$L.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/mid_$L.json')); p=d['middle_phases']; print('mid $L', d['value'], d['ms_per_step'], d['middle_ms_per_step'], json.dumps(p['ms']), p['round1_ms'], d['parity_spot_check'])"
done
export TMPDIR=/tmp
cd /tmp
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "k_seed_band|k_seed_expand|k_align_chunk|k_seed_scan" --output-format csv -d $OUT/pmc$i -o run -- python3 $R/bench.py --workload middle --steps 2 --warmup 1 --cpu-sample 0 --check 0 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
  echo "pmc pass $i ok"
done
python3 - $OUT <<'PY'
import csv, sys, os, glob, collections
for f in sorted(glob.glob(os.path.join(sys.argv[1], 'pmc*', '*counter_collection.csv'))):
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        agg[r['Kernel_Name'][:40]][r['Counter_Name']].append(float(r['Counter_Value']))
    print('==', f)
    for k, d in agg.items():
        print(k, {c: round(sum(v) / len(v), 1) for c, v in d.items()})
PY

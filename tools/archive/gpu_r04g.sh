#!/bin/bash
# GPU-box script (r04): the default bench line (every sub-record), then PMC passes on the middle
# step's chunk DP and seed scan.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04g
mkdir -p $OUT
cd $R
timeout -k 10 900 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench_default.err; exit 1; }
python - $OUT/bench_default.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(json.dumps({k: d.get(k) for k in ('value', 'ms_per_step')}), json.dumps(d.get('roofline'))[:300])
for k, v in d.items():
    if isinstance(v, dict) and ('value' in v or 'ms_per_step' in v) and k not in ('roofline',):
        print(k, json.dumps({x: v.get(x) for x in ('value', 'ms_per_step', 'middle_ms_per_step', 'ms_per_phase', 'error', 'parity_spot_check')})[:700])
PY
export TMPDIR=/tmp
cd /tmp
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "k_align_chunk|k_seed_scan" --output-format csv -d $OUT/pmc$i -o run -- python3 $R/bench.py --workload middle --steps 2 --warmup 1 --cpu-sample 0 --check 0 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
  echo "pmc pass $i ok"
done
python3 - $OUT <<'PY'
import csv, sys, os, glob, collections
for f in sorted(glob.glob(os.path.join(sys.argv[1], 'pmc*', '*counter_collection.csv'))):
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        agg[r['Kernel_Name'][:44]][r['Counter_Name']].append(float(r['Counter_Value']))
    print('==', f)
    for k, d in agg.items():
        print(k, {c: (round(max(v), 1), len(v)) for c, v in d.items()})
PY

#!/bin/bash
# GPU-box script (r04): staged per-step inputs (--stage-inputs 1) against the per-step device copy
# on the middle workload and the reference job, then the default bench line.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04z
mkdir -p $OUT
cd $R
for V in 0 1 0 1; do
  timeout -k 10 300 python bench.py --workload middle --stage-inputs $V --steps 8 --warmup 2 --cpu-sample 0 > $OUT/mid_$V.json 2> $OUT/mid_$V.err || { echo "mid $V failed rc=$?"; tail -20 $OUT/mid_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/mid_$V.json')); print('mid stage=$V', d['value'], d['ms_per_step'], d['middle_ms_per_step'], d['parity_spot_check']['identical'])"
  timeout -k 10 300 python bench.py --only-subs reference_job --stage-inputs $V --steps 8 --warmup 2 --cpu-sample 0 > $OUT/rj_$V.json 2> $OUT/rj_$V.err || { echo "rj $V failed rc=$?"; tail -20 $OUT/rj_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/rj_$V.json'))['reference_job']; print('rj stage=$V', d['ms_per_step'], json.dumps(d['ms_per_phase']), d['parity_spot_check']['middle'])"
done
timeout -k 10 900 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench_default.err; exit 1; }
python - $OUT/bench_default.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(json.dumps({k: d.get(k) for k in ('value', 'ms_per_step')}), d['roofline']['frac'])
for k in ('reference_job', 'middle', 'middle_20kb', 'fused_schedule', 'barcodes', 'drivers', 'e2e'):
    v = d.get(k) or {}
    print(k, json.dumps({x: v.get(x) for x in ('value', 'ms_per_step', 'middle_ms_per_step', 'error')})[:300])
PY

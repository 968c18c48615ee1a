set -u
for w in 4096 8192 16384 32768; do
  PCABI_MIDDLE_PLAN_WAVES=$w timeout -k 10 200 python bench.py --workload middle --steps 10 --warmup 2 --cpu-sample 0 --check 300 > gpurun_out/sw_$w.json 2> gpurun_out/sw_$w.err || { echo "sweep $w failed"; tail -5 gpurun_out/sw_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sw_$w.json')); print('$w', d['value'], d['ms_per_step'], d['middle_ms_per_step'], d['parity_spot_check'])"
done

set -u
bash tools/gpu_record.sh || exit 1
for w in "--workload middle" "--workload middle --mean-len 20000 --steps 5 --warmup 1" "--workload barcodes" "--workload barcodes --kit native12" "--workload barcodes --kit rapid12" "--reads 10000 --sets 119 --sub 0"; do
  n=$(echo "$w" | tr -c 'a-z0-9' '_')
  timeout -k 10 400 python bench.py $w > gpurun_out/w$n.json 2> gpurun_out/w$n.err || { echo "workload $w failed"; tail -5 gpurun_out/w$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/w$n.json')); print('$w', d['value'], d['ms_per_step'], (d.get('cpu_baseline') or {}).get('value'), d.get('parity_spot_check'))"
done

set -u
timeout -k 10 400 python bench.py --workload middle --mean-len 20000 --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/mid20k.json 2> gpurun_out/mid20k.err || { tail -20 gpurun_out/mid20k.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/mid20k.json')); print(d['value'], d['ms_per_step'], d['middle_ms_per_step'], d['parity_spot_check'])"
timeout -k 10 400 python bench.py --workload e2e --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { tail -20 gpurun_out/e2e.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/e2e.json')); print(json.dumps(d)[:1500])"

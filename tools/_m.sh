set -u
timeout -k 10 400 python bench.py --cpu-sample 0 > gpurun_out/b0.json 2> gpurun_out/b0.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/b0.json')); m=d['middle']; print('nocpu', d['value'], m['value'], m['ms_per_step'], m['middle_ms_per_step'])"
timeout -k 10 400 python bench.py > gpurun_out/b1.json 2> gpurun_out/b1.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/b1.json')); m=d['middle']; print('default', d['value'], m['value'], m['ms_per_step'], m['middle_ms_per_step'])"
timeout -k 10 400 python bench.py --workload middle --cpu-sample 0 > gpurun_out/b2.json 2> gpurun_out/b2.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/b2.json')); print('standalone', d['value'], d['ms_per_step'], d['middle_ms_per_step'])"

#!/bin/bash
# r06: (1) the N > 1 bench path rehearsed with 2 ranks sharing the box's GPU (gloo for the timing
# all-reduce): the overlapped headline steps under torch.distributed.run; (2) the reference job with
# its adapter objects made once (scores reset per job)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06n2}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --cpu-sample 0 > $OUT/bench_n2.json 2> $OUT/bench_n2.err || { echo "n2 failed rc=$?"; tail -20 $OUT/bench_n2.err; exit 1; }
cut -c1-300 $OUT/bench_n2.json
for k in 1 2; do
  timeout -k 10 300 python bench.py --only-subs reference_job --steps 10 --cpu-sample 0 > $OUT/rj_$k.json 2> $OUT/rj_$k.err || { echo "rj failed rc=$?"; tail -20 $OUT/rj_$k.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); d=d.get('reference_job', d); print('rj', d['ms_per_step'], d['ms_per_phase'], d.get('parity_spot_check'))" $OUT/rj_$k.json | cut -c1-500
done

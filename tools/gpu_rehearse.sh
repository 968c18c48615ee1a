#!/bin/bash
# Multi-rank rehearsal of bench.py on a ONE-GPU box: N ranks share cuda:0 over gloo (the
# driver's 8-GPU scaling runs use one GPU per rank over RCCL); checks that the N > 1 code path
# (shards, barrier, max-over-ranks clock, one JSON line from rank 0) runs end to end.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for n in ${RANKS:-2 4}; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 2 --dist-backend gloo ${BENCH_ARGS:-} \
      > gpurun_out/rehearse_n$n.json 2> gpurun_out/rehearse_n$n.err || { echo "n=$n failed"; tail -5 gpurun_out/rehearse_n$n.err; exit 1; }
  echo "n=$n: $(tail -1 gpurun_out/rehearse_n$n.json)"
done

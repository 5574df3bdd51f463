#!/bin/bash
# Rehearsal of `bench.py --gpus N` on the one-GPU box: N ranks share the GPU
# through host-staged collectives (SEZKP_BENCH_HOST_COMM=1; RCCL refuses two
# ranks on one GPU), so the N > 1 code path (replicas, the `sharded` proof
# checked against the single-GPU bytes, dist_ntt) runs end to end.
set -euo pipefail
mkdir -p gpurun_out
for n in 2 4; do
  SEZKP_BENCH_HOST_COMM=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29530 + n)) bench.py --gpus $n --steps 5 --warmup 2 \
    --detail gpurun_out/rehearse$n.detail.json > gpurun_out/rehearse$n.log 2> gpurun_out/rehearse$n.err
  echo "rehearse $n ok"
done

#!/bin/bash
# A/B of the HIP hardware-queue count per process (GPU_MAX_HW_QUEUES, default
# 4 on the box) against proofs in flight: each context has a main and a side
# stream (plus a copy stream once it stages), and streams map to hardware
# queues round-robin, so with 3+ contexts streams share queues.
set -euo pipefail
mkdir -p gpurun_out/abq
B="python -u bench.py --steps 200 --no-cpu-baseline --no-worst-case --no-configs --dntt-log-n 0"
for q in 4 8 12 16; do
  for k in 3 4; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 $B --inflight $k > gpurun_out/abq/q${q}_k${k}.json 2> gpurun_out/abq/q${q}_k${k}.err
    echo "q=$q k=$k done"
  done
done

#!/bin/bash
# A/B of the staged-upload settings on the host_to_proof headline (100 steps):
# base, SEZKP_IMAGE_ON_MAIN=1, GPU_MAX_HW_QUEUES=8; two rounds, alternating.
set -e
mkdir -p gpurun_out
B="python3 bench.py --steps 100 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --dntt-log-n 0"
for i in 1 2; do
  timeout -k 10 200 $B > gpurun_out/ab_stage_base_$i.json 2>/dev/null
  SEZKP_IMAGE_ON_MAIN=1 timeout -k 10 200 $B > gpurun_out/ab_stage_main_$i.json 2>/dev/null
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $B > gpurun_out/ab_stage_q8_$i.json 2>/dev/null
done
echo done

#!/bin/bash
# A/B: small FRI layers inside the forest launch (default) vs their own
# kernel on the side stream (SEZKP_TAIL_SEPARATE=1): single-proof stage split.
set -e
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/ab_tail.jsonl
  SEZKP_TAIL_SEPARATE=1 timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/ab_tail.jsonl
done
echo done

#!/bin/bash
# Sharded INTT schedule A/B on the per-rank cost model (bench sharded_predicted):
# the distributed INTT (default) against SEZKP_REPLICATED_INTT=1.
set -euo pipefail
mkdir -p gpurun_out
B="python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-host-to-proof --dntt-log-n 0"
timeout -k 10 300 $B --detail gpurun_out/intt_dist.json > gpurun_out/intt_dist.log 2>&1
timeout -k 10 300 env SEZKP_REPLICATED_INTT=1 $B --detail gpurun_out/intt_rep.json > gpurun_out/intt_rep.log 2>&1
echo "intt ab ok"

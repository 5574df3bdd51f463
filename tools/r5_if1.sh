#!/bin/bash
# Kernel stats of the single-proof pass (bench --inflight 1) under rocprofv3.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/prof_if1
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
  python3 bench.py --inflight 1 --steps 20 --no-cpu-baseline --no-configs --no-worst-case --no-host-to-proof --no-host-rows --no-sharded --dntt-log-n 0 --detail gpurun_out/prof_if1/detail.json > $O/if1.log 2>&1
echo "if1 ok"

#!/bin/bash
# Short default-shape bench (stage times, throughput) + single-proof kernel stats.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 100 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-sharded --detail gpurun_out/quick_detail.json > gpurun_out/quick.log 2> gpurun_out/quick.err
echo "bench ok"
bash tools/r5_if1.sh

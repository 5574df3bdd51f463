#!/bin/bash
# Host -> device copy paths: bandwidth probe (SDMA engines vs blit kernels,
# 1-3 concurrent streams), then the default bench with HSA_ENABLE_SDMA=0 as
# the B side (staged uploads through blit kernels).
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 python3 tools/h2d_probe.py 67 10 > gpurun_out/h2d_probe.txt 2>/dev/null
HSA_ENABLE_SDMA=0 timeout -k 10 60 python3 tools/h2d_probe.py 67 10 >> gpurun_out/h2d_probe.txt 2>/dev/null
B="python3 bench.py --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --dntt-log-n 0 --steps 100"
for i in 1 2; do
  timeout -k 10 200 $B > gpurun_out/sdma_base_$i.json 2>/dev/null
  HSA_ENABLE_SDMA=0 timeout -k 10 200 $B > gpurun_out/sdma_blit_$i.json 2>/dev/null
done
echo done

#!/bin/bash
# Register-transposed trace image for tau = 8 (k_trace_image8) against the
# byte-wise kernel (SEZKP_TRACE_IMAGE_BYTES=1): parity (every upload and
# staged upload builds the image), kernel time, and the host -> proof bench.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ti_tests.log 2>&1
for v in 0 1; do
  SEZKP_TRACE_IMAGE_BYTES=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ti$v -o run -- python3 tools/stage_probe.py 21 3 > /dev/null 2>&1
done
B="python3 bench.py --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --dntt-log-n 0 --steps 100"
for i in 1 2; do
  timeout -k 10 200 $B > gpurun_out/ti_new_$i.json 2>/dev/null
  SEZKP_TRACE_IMAGE_BYTES=1 timeout -k 10 200 $B > gpurun_out/ti_old_$i.json 2>/dev/null
done
echo done

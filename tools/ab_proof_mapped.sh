#!/bin/bash
# Proof body written by the path kernels into mapped host memory (default)
# against the device image + D2H copies (SEZKP_PROOF_D2H=1): parity, single
# proof latency, and the host -> proof bench.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernel_abi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pm_tests.log 2>&1
for v in 0 1 0 1; do
  SEZKP_PROOF_D2H=$v timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/ab_proof_mapped.jsonl
done
B="python3 bench.py --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --dntt-log-n 0 --steps 100"
for i in 1 2; do
  timeout -k 10 200 $B > gpurun_out/pm_new_$i.json 2>/dev/null
  SEZKP_PROOF_D2H=1 timeout -k 10 200 $B > gpurun_out/pm_old_$i.json 2>/dev/null
done
echo done

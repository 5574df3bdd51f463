#!/bin/bash
# A/B (4 MB is the default since): staged trace uploads as one copy per array vs copies of <= 4
# or 8 MB (SEZKP_UPLOAD_CHUNK_MB), so the proofs' D2H copies on the same copy
# engine wait for one chunk instead of a whole upload; alternating bench lines.
set -euo pipefail
mkdir -p gpurun_out
SEZKP_UPLOAD_CHUNK_MB=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "stage" > gpurun_out/upload_chunk_tests.log 2>&1
echo tests-ok
B="python3 bench.py --no-cpu-baseline --no-configs --dntt-log-n 0 --steps 100"
for v in 0 4 8 0 4 8 0 4 8; do
  echo -n "$v " >> gpurun_out/ab_upload_chunk.txt
  SEZKP_UPLOAD_CHUNK_MB=$v timeout -k 10 200 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['trace_resident']['value'], d['single_proof']['ms_per_proof'])" >> gpurun_out/ab_upload_chunk.txt
done
echo done

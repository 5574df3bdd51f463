#!/bin/bash
# A/B (run while SEZKP_REQ_MAPPED=1 was the variant; it is the default since):
# query requests read by the kernels from mapped host memory
# (SEZKP_REQ_MAPPED=1) vs one small H2D copy per proof (default), which can
# queue behind a staged trace upload on the copy engine. Parity under the
# switch, then alternating default bench lines (value = host -> proof).
set -euo pipefail
mkdir -p gpurun_out
SEZKP_REQ_MAPPED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "synthetic or headline or stage or async or golden" > gpurun_out/reqmapped_tests.log 2>&1
echo tests-ok
B="python3 bench.py --no-cpu-baseline --no-configs --dntt-log-n 0 --steps 100"
for v in 0 1 0 1 0 1; do
  echo -n "$v " >> gpurun_out/ab_req_mapped.txt
  SEZKP_REQ_MAPPED=$v timeout -k 10 200 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['trace_resident']['value'], d['single_proof']['ms_per_proof'])" >> gpurun_out/ab_req_mapped.txt
done
echo done

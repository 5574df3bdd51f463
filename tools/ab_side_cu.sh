#!/bin/bash
# A/B (measured round 3: single proof ~50 us shorter, trace-resident in flight
# 2% lower; off): side stream on every CU (default) vs on every 4th / 2nd CU
# (SEZKP_SIDE_CU_EVERY, a CU-masked stream): parity subset under the mask,
# single-proof stage split, rocprof kernel stats, alternating bench lines.
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SEZKP_SIDE_CU_EVERY=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "synthetic or dictionary or headline or golden or stage" > gpurun_out/side_cu_tests.log 2>&1
echo tests-ok
for v in 0 4 2 0 4 2; do
  echo -n "$v " >> gpurun_out/ab_side_cu.jsonl
  SEZKP_SIDE_CU_EVERY=$v timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/ab_side_cu.jsonl
done
for v in 0 4; do
  SEZKP_SIDE_CU_EVERY=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sidecu$v -o run -- python3 tools/stage_probe.py 21 10 > /dev/null 2>&1
done
B="python3 bench.py --no-cpu-baseline --no-configs --dntt-log-n 0 --steps 100"
for v in 0 4 0 4 0 4; do
  echo -n "$v " >> gpurun_out/ab_side_cu_bench.txt
  SEZKP_SIDE_CU_EVERY=$v timeout -k 10 200 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['trace_resident']['value'], d['single_proof']['ms_per_proof'], d['stages_ms']['col_commit'], d['stages_ms']['total'])" >> gpurun_out/ab_side_cu_bench.txt
done
echo done

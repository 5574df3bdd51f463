#!/bin/bash
# A/B: side-stream columns (tables, dense, piecewise) started right after
# expand, beside the whole dictionary chain (default) vs after the dictionary
# tables, beside the commit kernel only (SEZKP_SIDE_AT=2), or after the plan
# (SEZKP_SIDE_AT=1; first run: 0 vs 2, second: 0 vs 1 vs 2): parity
# under the switch, single-proof stage split, rocprof kernel stats per side,
# alternating in-flight bench lines.
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SEZKP_SIDE_AT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "synthetic or dictionary or random or headline or golden" > gpurun_out/side_after_tests.log 2>&1
echo tests-ok
for v in 0 1 2 0 1 2; do
  echo -n "$v " >> gpurun_out/ab_side_after.jsonl
  SEZKP_SIDE_AT=$v timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/ab_side_after.jsonl
done
for v in 0 1 2; do
  SEZKP_SIDE_AT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_side$v -o run -- python3 tools/stage_probe.py 21 10 > /dev/null 2>&1
done
B="python3 bench.py --no-cpu-baseline --no-configs --dntt-log-n 0 --steps 100"
for v in 0 1 0 1 0 1; do
  echo -n "$v " >> gpurun_out/ab_side_after_bench.txt
  SEZKP_SIDE_AT=$v timeout -k 10 200 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['trace_resident']['value'], d['single_proof']['ms_per_proof'], d['stages_ms']['col_commit'], d['stages_ms']['total'])" >> gpurun_out/ab_side_after_bench.txt
done
echo done

#!/bin/bash
# A/B: the piecewise columns' U tables (k_col_tables) on the side stream
# beside expand (SEZKP_TABLES_EARLY=1, the default while this ran; off since:
# slower) vs after expand, beside the dictionary chain's head
# (SEZKP_TABLES_EARLY=0): the full GPU suite with it on, single-proof
# stage split, rocprof kernel stats per side, alternating bench lines.
set -euo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tables_early_tests.log 2>&1
echo tests-ok
for v in 1 0 1 0; do
  echo -n "$v " >> gpurun_out/ab_tables_early.jsonl
  SEZKP_TABLES_EARLY=$v timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/ab_tables_early.jsonl
done
for v in 1 0; do
  SEZKP_TABLES_EARLY=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tables$v -o run -- python3 tools/stage_probe.py 21 10 > /dev/null 2>&1
done
B="python3 bench.py --no-cpu-baseline --no-configs --dntt-log-n 0 --steps 100"
for v in 1 0 1 0 1 0; do
  echo -n "$v " >> gpurun_out/ab_tables_early_bench.txt
  SEZKP_TABLES_EARLY=$v timeout -k 10 200 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['trace_resident']['value'], d['single_proof']['ms_per_proof'], d['stages_ms']['expand'] + d['stages_ms']['col_commit'], d['stages_ms']['total'])" >> gpurun_out/ab_tables_early_bench.txt
done
echo done

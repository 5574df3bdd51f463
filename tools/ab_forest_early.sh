#!/bin/bash
# A/B: the FRI forest's first-fold-pass layers hashed on the side stream
# beside the later fold passes (SEZKP_FOREST_EARLY=1; the default while this
# ran, off since: slower) vs one forest launch after the whole
# fold chain (SEZKP_FOREST_EARLY=0): the full GPU suite at the new default,
# single-proof stage split, alternating in-flight bench lines.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/forest_early_tests.log 2>&1
echo tests-ok
for v in 1 0 1 0; do
  echo -n "$v " >> gpurun_out/ab_forest_early.jsonl
  SEZKP_FOREST_EARLY=$v timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/ab_forest_early.jsonl
done
B="python3 bench.py --no-cpu-baseline --no-configs --dntt-log-n 0 --steps 100"
for v in 1 0 1 0 1 0; do
  echo -n "$v " >> gpurun_out/ab_forest_early_bench.txt
  SEZKP_FOREST_EARLY=$v timeout -k 10 200 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['trace_resident']['value'], d['single_proof']['ms_per_proof'], d['stages_ms']['fri_fold_trees'], d['stages_ms']['total'])" >> gpurun_out/ab_forest_early_bench.txt
done
echo done

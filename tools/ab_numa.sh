#!/bin/bash
# A/B (bound is the default since): bench process bound to the GPU's NUMA-local CPUs (SEZKP_BENCH_NUMA=1)
# vs the scheduler's choice (default), alternating default-length lines.
set -euo pipefail
mkdir -p gpurun_out
for v in 0 1 0 1 0 1; do
  echo -n "$v " >> gpurun_out/ab_numa.txt
  SEZKP_BENCH_NUMA=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-configs --dntt-log-n 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['trace_resident']['value'], d['single_proof']['ms_per_proof'], d.get('numa'))" >> gpurun_out/ab_numa.txt
done
echo done

#!/bin/bash
# Round-3 latency changes (measured: FRI paths beside the openings SLOWER, 2.44
# vs 2.39 ms of device time, reverted; mapped roots -2% host -> proof, kept off):
# the full GPU suite at the then defaults (FRI paths
# beside the openings, planner without scratch), then alternating bench lines:
# default / SEZKP_PATHS_SERIAL=1 (paths after the openings) / SEZKP_MAPPED_ROOTS=1.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_lat3.log 2>&1
echo tests-ok
B="python3 bench.py --no-cpu-baseline --no-configs --dntt-log-n 0 --steps 100"
for i in 1 2 3; do
  for v in base SEZKP_PATHS_SERIAL=1 SEZKP_MAPPED_ROOTS=1; do
    echo -n "$v " >> gpurun_out/ab_latency3.txt
    if [ $v = base ]; then E=""; else E=$v; fi
    env $E timeout -k 10 200 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms']; print(d['value'], d['trace_resident']['value'], d['single_proof']['ms_per_proof'], s['col_openings'], s['fri_paths'], s['total'])" >> gpurun_out/ab_latency3.txt
  done
done
echo done

#!/bin/bash
# Three default-length bench lines back to back on one box (headline spread);
# configs / CPU baseline / dist_ntt skipped to keep the call short.
set -euo pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-configs --dntt-log-n 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['trace_resident']['value'], d['ms_per_proof'], d['halves_ms_per_proof'], d['single_proof']['ms_per_proof'])" >> gpurun_out/bench_repeat_r03.txt
done
echo done

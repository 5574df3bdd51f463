#!/bin/bash
# Three default-length bench lines back to back on one box (the headline's
# spread); configs, CPU baseline, worst cases, host rows, the sharded model and
# dist_ntt skipped to keep the call short. One line per run: value,
# host_to_proof value, ms per proof in flight, one proof at a time (ms).
set -euo pipefail
mkdir -p gpurun_out
O=gpurun_out/bench_repeat_r06.txt
: > $O
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-sharded \
    --dntt-log-n 0 --detail gpurun_out/bench_repeat_$i.json > gpurun_out/bench_repeat_$i.log 2>/dev/null
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['host_to_proof']['value'], d['ms_per_proof'], d['single_proof']['ms_per_proof'])" gpurun_out/bench_repeat_$i.log >> $O
  echo "run $i ok"
done
echo done

#!/bin/bash
# A/B of an environment toggle on the default bench, alternating runs:
#   bash tools/ab_env.sh VAR [rounds]   -> gpurun_out/ab_{base,var}_<i>.json
set -e
V=$1; R=${2:-2}
B="python3 bench.py --no-cpu-baseline --no-configs --dntt-log-n 0"
for i in $(seq 1 $R); do
  timeout -k 10 200 $B > gpurun_out/ab_base_$i.json 2>/dev/null
  env $V=1 timeout -k 10 200 $B > gpurun_out/ab_var_$i.json 2>/dev/null
done
echo done

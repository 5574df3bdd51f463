#!/bin/bash
# A/B of an environment setting on the default bench, alternating runs:
#   bash tools/ab_env.sh VAR=VALUE [rounds]   -> gpurun_out/ab_{base,var}_<i>.json
set -e
V=$1; R=${2:-2}
case "$V" in *=*) ;; *) V="$V=1" ;; esac
B="python3 bench.py --no-cpu-baseline --no-configs --dntt-log-n 0"
for i in $(seq 1 $R); do
  timeout -k 10 200 $B > gpurun_out/ab_base_$i.json 2>/dev/null
  env $V timeout -k 10 200 $B > gpurun_out/ab_var_$i.json 2>/dev/null
done
echo done

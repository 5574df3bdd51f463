#!/bin/bash
set -euo pipefail
O=gpurun_out/kab
mkdir -p $O
B="python3 bench.py --steps 80 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-host-to-proof --no-sharded --dntt-log-n 0"
: > $O/ab.txt
for rep in 1 2 3; do
  for k in 3 4 2; do
    v=$(timeout -k 10 200 $B --inflight $k --detail $O/d.json 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9,3), round(d['ms_per_proof'],4))")
    echo "k$k $v" >> $O/ab.txt
  done
done
echo k ab done

#!/bin/bash
set -euo pipefail
O=gpurun_out/depth
mkdir -p $O
B="python3 bench.py --steps 60 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-host-to-proof --no-sharded --dntt-log-n 0"
: > $O/ab.txt
for rep in 1 2; do
  for cfg in "q4 k3" "q4 k6" "q8 k3" "q8 k6" "q8 k4"; do
    q=${cfg%% *}; k=${cfg##*k}
    v=$(GPU_MAX_HW_QUEUES=${q#q} timeout -k 10 200 $B --inflight $k --detail $O/d.json 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9,3), round(d['ms_per_proof'],4) if 'ms_per_proof' in d else '')")
    echo "$cfg $v" >> $O/ab.txt
  done
  v=$(SEZKP_BENCH_HOST_COMM=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 60 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-host-to-proof --no-sharded --dntt-log-n 0 --detail $O/d2.json 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9,3))")
  echo "2proc k3 $v" >> $O/ab.txt
done
echo depth done

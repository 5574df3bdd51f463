# deeper pipelines with more hardware queues in one process: (queues, contexts in flight)
set -uo pipefail
O=gpurun_out/r4v
mkdir -p $O
Q="bench.py --steps 100 --warmup 3 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-sharded"
for i in 1 2; do
  for c in "4 3" "16 4" "16 6" "8 4" "16 3"; do
    set -- $c
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 200 python3 $Q --inflight $2 > $O/q$1k$2.$i.json 2> $O/q$1k$2.$i.err || exit 1
    echo "q$1k$2.$i $(python3 -c "import json;d=json.loads(open('$O/q$1k$2.$i.json').read().strip().splitlines()[-1]);print(d['value']/1e9, d['trace_resident']['value']/1e9)")"
  done
done

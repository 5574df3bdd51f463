# hardware queues after the staging fix: GPU_MAX_HW_QUEUES 4 (HIP default on the box) vs 8, alternating
set -uo pipefail
O=gpurun_out/r4t
mkdir -p $O
Q="bench.py --steps 100 --warmup 3 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-sharded"
for i in 1 2 3; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 $Q > $O/q$q.$i.json 2> $O/q$q.$i.err || exit 1
    echo "q$q.$i $(python3 -c "import json;d=json.loads(open('$O/q$q.$i.json').read().strip().splitlines()[-1]);print(d['value']/1e9, d['trace_resident']['value']/1e9, d['single_proof']['ms_per_proof'])")"
  done
done

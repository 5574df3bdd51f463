# in-flight depth A/B at the round-4 code: 3 (default) vs 4 vs 2 contexts, alternating
set -uo pipefail
O=gpurun_out/r4n
mkdir -p $O
Q="bench.py --steps 100 --warmup 3 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-sharded"
for i in 1 2; do
  for k in 3 4 2; do
    timeout -k 10 200 python3 $Q --inflight $k > $O/k$k.$i.json 2> $O/k$k.$i.err || exit 1
    echo "k$k.$i $(python3 -c "import json;d=json.loads(open('$O/k$k.$i.json').read().strip().splitlines()[-1]);print(d['value']/1e9, d['trace_resident']['value']/1e9)")"
  done
done

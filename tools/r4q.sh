# A/B probe: the 13 timed stage events of a proof (default) vs none
# (SEZKP_AB_NO_STAGE_EVENTS=1): single-proof latency and in-flight value
set -uo pipefail
O=gpurun_out/r4q
mkdir -p $O
Q="bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-sharded"
for i in 1 2 3; do
  for v in ev noev; do
    if [ $v = noev ]; then export SEZKP_AB_NO_STAGE_EVENTS=1; else unset SEZKP_AB_NO_STAGE_EVENTS; fi
    timeout -k 10 200 python3 $Q > $O/$v$i.json 2> $O/$v$i.err || exit 1
    echo "$v$i $(python3 -c "import json;d=json.loads(open('$O/$v$i.json').read().strip().splitlines()[-1]);print(d['value']/1e9, d['trace_resident']['value']/1e9, d['single_proof']['ms_per_proof'])")"
  done
done

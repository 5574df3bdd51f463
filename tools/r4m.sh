# A/B: challenge record + betas through kernel arguments (new) vs SDMA copies (old)
set -uo pipefail
O=gpurun_out/r4m
mkdir -p $O
L=streaming-zero-knowledge-proofs_amd/lib/libsezkp_stark.so
Q="bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-sharded"
for i in 1 2 3; do
  for v in new old; do
    cp ab/lib$v.so $L || exit 1
    timeout -k 10 200 python3 $Q > $O/$v$i.json 2> $O/$v$i.err || exit 1
    echo "$v$i $(python3 -c "import json,sys;d=json.loads(open('$O/$v$i.json').read().strip().splitlines()[-1]);print(d['value']/1e9, d.get('trace_resident',{}).get('value',0)/1e9, d['single_proof']['ms_per_proof'])")"
  done
done
cp ab/libnew.so $L

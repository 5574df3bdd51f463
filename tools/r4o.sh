# staged uploads with the transposition moved from the copy stream to the
# prover stream (new) vs round-4 HEAD (old): staging parity tests, then
# alternating bench runs
set -uo pipefail
O=gpurun_out/r4o
mkdir -p $O
L=streaming-zero-knowledge-proofs_amd/lib/libsezkp_stark.so
cp ab/libnew.so $L || exit 1
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "stag or upload" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
Q="bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-sharded"
for i in 1 2 3; do
  for v in new old; do
    cp ab/lib$v.so $L || exit 1
    timeout -k 10 200 python3 $Q > $O/$v$i.json 2> $O/$v$i.err || exit 1
    echo "$v$i $(python3 -c "import json;d=json.loads(open('$O/$v$i.json').read().strip().splitlines()[-1]);print(d['value']/1e9, d['trace_resident']['value']/1e9, d['single_proof']['ms_per_proof'])")"
  done
done
cp ab/libnew.so $L

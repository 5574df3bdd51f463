#!/bin/bash
# A/B of in-flight stalls: per config, 5 bench runs with the completion
# timeline; prints value and the 12-proof windows (ms per proof).
set -e
run() {
  local tag="$1"; shift
  for i in 1 2 3 4 5; do
    env "$@" SEZKP_BENCH_TIMELINE=1 timeout -k 10 100 python bench.py --no-cpu-baseline --no-configs --dntt-log-n 0 > gpurun_out/ab.log 2>&1
    grep "^{" gpurun_out/ab.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); t=d['done_ms']
w=[round((t[min(k+11,len(t)-1)]-(t[k-1] if k else 0))/12,2) for k in range(0,len(t),12)]
print('$tag', round(d['value']/1e9,3), 'stalls', sum(1 for x in w[1:] if x > 2.45), w)"
  done
}
run default X=1
run one_stream SEZKP_ONE_STREAM=1
run hwq8 GPU_MAX_HW_QUEUES=8

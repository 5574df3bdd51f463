# kernel trace of one proof at a time (one context in flight, trace resident):
# where the single-proof latency goes between kernels
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/if1 -o run -- python3 bench.py --inflight 1 --steps 40 --warmup 3 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-sharded --no-host-to-proof --dntt-log-n 0 > $O/if1.log 2>&1 || exit 1
echo done

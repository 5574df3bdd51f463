# device vs host transcript: kernel traces (single proof) and the in-flight
# pipeline with more hardware queues
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
B="bench.py --inflight 1 --steps 10 --warmup 2 --no-cpu-baseline --no-configs --no-worst-case --no-host-to-proof --no-host-rows --dntt-log-n 0"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dev_if1 -o run -- python3 $B > $O/dev_if1.log 2>&1 || exit 1
SEZKP_HOST_TRANSCRIPT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/host_if1 -o run -- python3 $B > $O/host_if1.log 2>&1 || exit 1
Q="bench.py --steps 100 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --dntt-log-n 0"
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 $Q > $O/dev_q$q.log 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=$q SEZKP_HOST_TRANSCRIPT=1 timeout -k 10 200 python3 $Q > $O/host_q$q.log 2>&1 || exit 1
done
echo done

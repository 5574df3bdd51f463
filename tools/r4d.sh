# device vs host transcript: kernel traces (single proof) and the in-flight
# pipeline with more hardware queues
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_transcript.py tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
B="bench.py --inflight 1 --steps 10 --warmup 2 --no-cpu-baseline --no-configs --no-worst-case --no-host-to-proof --no-host-rows --dntt-log-n 0 --no-sharded"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dev_if1 -o run -- python3 $B > $O/dev_if1.log 2>&1 || exit 1
SEZKP_HOST_TRANSCRIPT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/host_if1 -o run -- python3 $B > $O/host_if1.log 2>&1 || exit 1
Q="bench.py --steps 100 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --dntt-log-n 0"
timeout -k 10 300 python3 $Q > $O/dev_pred.log 2>&1 || exit 1
Q="$Q --no-sharded"
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 $Q > $O/dev_q$q.log 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=$q SEZKP_HOST_TRANSCRIPT=1 timeout -k 10 200 python3 $Q > $O/host_q$q.log 2>&1 || exit 1
done
echo done

set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/gpu_tests.log | head -30; exit 1; }
echo tests ok
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/solo8 -o run -- python3 tools/solo_trace.py 8 0 21 > $O/solo8.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-worst-case --no-host-rows > $O/bench.log 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
SEZKP_DEVICE_TRANSCRIPT=1 timeout -k 10 200 python3 bench.py --inflight 1 --steps 10 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-sharded --dntt-log-n 0 > $O/bench_devtr.log 2> $O/bench_devtr.err || { tail -5 $O/bench_devtr.err; exit 1; }
SEZKP_DEVICE_TRANSCRIPT=1 timeout -k 10 300 python3 bench.py --steps 20 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --dntt-log-n 0 > $O/bench_devtr_pred.log 2> $O/bench_devtr_pred.err || { tail -5 $O/bench_devtr_pred.err; exit 1; }
Q="bench.py --steps 100 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-sharded --dntt-log-n 0"
for i in 1 2; do
  timeout -k 10 200 python3 $Q > $O/stage_dev$i.log 2>&1 || exit 1
  SEZKP_STAGE_HOST_WAIT=1 timeout -k 10 200 python3 $Q > $O/stage_host$i.log 2>&1 || exit 1
done
echo done

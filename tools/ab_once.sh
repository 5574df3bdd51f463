set -euo pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "dict or golden or headline or random or synthetic" > gpurun_out/xcd_tests.log 2>&1
timeout -k 10 200 python -u bench.py --steps 200 --no-cpu-baseline --no-worst-case --no-configs --dntt-log-n 0 > gpurun_out/bench_xcd.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/xcdfetch -o run -- python3 bench.py --inflight 1 --steps 3 --warmup 1 --no-cpu-baseline --no-configs --no-worst-case --no-host-to-proof --dntt-log-n 0 > gpurun_out/xcdfetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xcdstats -o run -- python3 bench.py --inflight 1 --steps 20 --no-cpu-baseline --no-configs --no-worst-case --no-host-to-proof --dntt-log-n 0 > gpurun_out/xcdstats.log 2>&1

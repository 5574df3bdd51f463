set -euo pipefail
mkdir -p gpurun_out/r4c
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r4c/gpu_tests.log 2>&1 && echo tests ok || { echo TESTS FAILED; grep -E "FAILED|Error" gpurun_out/r4c/gpu_tests.log | head -30; }
timeout -k 10 300 python -u bench.py --steps 50 --no-cpu-baseline --no-host-rows --no-worst-case --dntt-log-n 0 > gpurun_out/r4c/bench.log 2> gpurun_out/r4c/bench.err && echo bench ok
SEZKP_HOST_TRANSCRIPT=1 timeout -k 10 300 python -u bench.py --steps 50 --no-cpu-baseline --no-host-rows --no-worst-case --no-configs --dntt-log-n 0 > gpurun_out/r4c/bench_hosttr.log 2> gpurun_out/r4c/bench_hosttr.err && echo bench_hosttr ok

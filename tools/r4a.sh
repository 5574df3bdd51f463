set -euo pipefail
mkdir -p gpurun_out/r4a
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r4a/gpu_tests.log 2>&1 && echo tests ok || { echo TESTS FAILED; tail -30 gpurun_out/r4a/gpu_tests.log; exit 1; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-host-rows > gpurun_out/r4a/bench.log 2> gpurun_out/r4a/bench.err && echo bench ok

set -euo pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 300 python -u -m pytest tests/test_gpu_transcript.py -v --timeout 120 --timeout-method thread > gpurun_out/r4b/t_transcript.log 2>&1 && echo transcript ok || { echo TRANSCRIPT FAILED; tail -40 gpurun_out/r4b/t_transcript.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r4b/gpu_tests.log 2>&1 && echo tests ok || { echo TESTS FAILED; grep -E "FAILED|Error" gpurun_out/r4b/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python -u bench.py --steps 50 --no-cpu-baseline --no-host-rows --no-worst-case --dntt-log-n 0 > gpurun_out/r4b/bench.log 2> gpurun_out/r4b/bench.err && echo bench ok

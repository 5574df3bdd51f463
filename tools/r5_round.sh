#!/bin/bash
# Round-5 GPU pass (run from the repo root on the GPU box): the -m gpu suite,
# then the default bench. Each step has its own time limit; the first failure
# ends the script.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "tests ok"
timeout -k 10 500 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err
echo "bench ok"

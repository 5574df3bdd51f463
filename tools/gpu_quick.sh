#!/bin/bash
# Quick GPU pass: the -m gpu suite, then a short single-GPU bench without the
# CPU baseline / configs / worst case / host rows (stage times, throughput).
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "tests ok"
timeout -k 10 300 python -u bench.py --steps 100 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --detail gpurun_out/quick_detail.json > gpurun_out/quick.log 2> gpurun_out/quick.err
echo "bench ok"

#!/bin/bash
# One GPU call that produces the round's evidence (run from the repo root on
# the GPU box): the -m gpu suite, the default bench line, and the rocprofv3
# kernel-stats / PMC passes of tools/profile_round.sh. Each step has its own
# time limit; the first failure ends the script.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "tests ok"
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err
echo "bench ok"
bash tools/profile_round.sh

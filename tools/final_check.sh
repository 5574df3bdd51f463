#!/bin/bash
# Round-end check on the GPU box: the -m gpu suite and smoke().
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "tests ok"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo "smoke ok"

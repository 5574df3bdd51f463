#!/bin/bash
# Round-6 final evidence, part 1 (GPU box, repo root): the -m gpu suite, the
# default bench line (the driver's command) with its detail file. Each step
# has its own limit; the first failure ends the script.
set -euo pipefail
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests ok"
timeout -k 10 600 python -u bench.py --detail $O/bench_detail.json > $O/bench_default.json 2> $O/bench_default.err
echo "bench ok"

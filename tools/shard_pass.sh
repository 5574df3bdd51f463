#!/bin/bash
# Sharded pass: the sharded GPU tests and the dictionary parity tests, then a
# short bench with the per-rank cost model (sharded_predicted) in its detail.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_sharded.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/shard_tests.log 2>&1
echo "sharded tests ok"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "dict or random or headline or synthetic" > gpurun_out/dict_tests.log 2>&1
echo "dict tests ok"
timeout -k 10 300 python -u bench.py --steps 30 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-host-to-proof --detail gpurun_out/shard_detail.json > gpurun_out/shard_bench.log 2> gpurun_out/shard_bench.err
echo "bench ok"

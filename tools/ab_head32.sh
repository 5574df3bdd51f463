#!/bin/bash
# head column as int32 (block-local positions) instead of int64: parity of
# every path that reads it (expand, composition, dictionary / delta commit,
# openings), then the single-proof stage split and the pipeline bench.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernel_abi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/h32_tests.log 2>&1
timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/h32_probe.jsonl
timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/h32_probe.jsonl
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_h32 -o run -- python3 tools/stage_probe.py 21 10 > /dev/null 2>&1
B="python3 bench.py --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --dntt-log-n 0 --steps 100"
timeout -k 10 200 $B > gpurun_out/h32_bench_1.json 2>/dev/null
timeout -k 10 200 $B > gpurun_out/h32_bench_2.json 2>/dev/null
echo done

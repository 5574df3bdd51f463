#!/bin/bash
# Round-3 A/Bs: upper tree levels in one launch per pass set
# (SEZKP_TREE_CONT=0: one launch per upper pass) and the balanced-XCD
# dictionary commit (SEZKP_DICT_XCD=2) against the linear grid.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernel_abi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1
SEZKP_DICT_XCD=2 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -k "dict or golden or headline" > gpurun_out/r3b_tests_xcd2.log 2>&1
for v in 1 0 1 0; do
  SEZKP_TREE_CONT=$v timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/ab_r3b_cont.jsonl
done
for v in 2 0 2 0; do
  SEZKP_DICT_XCD=$v timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/ab_r3b_xcd.jsonl
done
for v in 2 0; do
  SEZKP_DICT_XCD=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3b_xcd$v -o run -- python3 tools/stage_probe.py 21 10 > /dev/null 2>&1
  SEZKP_DICT_XCD=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fetch_r3b_xcd$v -o run -- python3 tools/stage_probe.py 21 3 > /dev/null 2>&1
done
echo done

#!/bin/bash
# Diagnose the in-launch upper-level continuation: mode 0 (upper-job
# launches), 1 (full continuation), 2 (hand-off + counter only, upper jobs
# still launched), 3 (store drain + barrier only); plus host-side marks.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -k "golden or headline" > gpurun_out/tcm_tests.log 2>&1
for v in 0 1 2 3 0 1 2 3; do
  SEZKP_TREE_CONT=$v timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/ab_tree_cont_modes.jsonl
done
SEZKP_HOST_TRACE=1 SEZKP_TREE_CONT=0 timeout -k 10 120 python3 tools/stage_probe.py 21 10 > /dev/null 2> gpurun_out/host_trace.txt
SEZKP_TREE_CONT=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_htrace -o run -- python3 tools/stage_probe.py 21 10 > /dev/null 2>&1
echo done

#!/bin/bash
# Upper tree levels finished inside the layer launches (SEZKP_TREE_CONT=0:
# separate upper-job passes): parity, single-proof stage split per side,
# kernel stats per side.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernel_abi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/treecont_tests.log 2>&1
for v in 1 0 1 0; do
  SEZKP_TREE_CONT=$v timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/ab_tree_cont2.jsonl
done
for v in 1 0; do
  SEZKP_TREE_CONT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tree_cont2_$v -o run -- python3 tools/stage_probe.py 21 10 > /dev/null 2>&1
done
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-configs --no-worst-case --dntt-log-n 0 > gpurun_out/treecont2_bench.json 2> gpurun_out/treecont_bench.err
SEZKP_TREE_CONT=0 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-configs --no-worst-case --dntt-log-n 0 > gpurun_out/treecont2_bench0.json 2> gpurun_out/treecont_bench0.err
echo done

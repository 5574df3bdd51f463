#!/bin/bash
# A/B of the dictionary planner's gather-miss price (SEZKP_DICT_MISS_PEN, q8:
# 0 = tables chosen by entries + nodes only; 160 = wflag at K = 3 (8 KB
# table) instead of K = 4 (2 MB); 256 = also wsym at K = 1): dictionary
# parity tests under the penalty, single-proof stage split and in-flight
# bench per side, rocprofv3 kernel stats per side.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
SEZKP_DICT_MISS_PEN=256 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "synthetic or dictionary or random or headline" > gpurun_out/dictpen_tests.log 2>&1
echo tests-ok
for v in 0 160 256 0 160 256; do
  echo -n "$v " >> gpurun_out/ab_dict_pen.jsonl
  SEZKP_DICT_MISS_PEN=$v timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/ab_dict_pen.jsonl
done
B="python3 bench.py --no-cpu-baseline --no-configs --dntt-log-n 0 --steps 100"
for v in 0 256 160 0 256 160; do
  echo -n "$v " >> gpurun_out/ab_dict_pen_bench.txt
  SEZKP_DICT_MISS_PEN=$v timeout -k 10 200 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['trace_resident']['value'], d['single_proof']['ms_per_proof'], d['stages_ms']['col_commit'])" >> gpurun_out/ab_dict_pen_bench.txt
done
for v in 0 256; do
  SEZKP_DICT_MISS_PEN=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dict_pen$v -o run -- python3 tools/stage_probe.py 21 10 > /dev/null 2>&1
done
echo done

#!/bin/bash
# A/B of the XCD-interleaved dictionary commit order (SEZKP_DICT_XCD=0 is the
# round-2 grid): single-proof stage split + rocprofv3 kernel stats per side.
set -e
mkdir -p gpurun_out
for v in 0 1 0 1; do
  SEZKP_DICT_XCD=$v timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/ab_dict_xcd.jsonl
done
for v in 0 1; do
  SEZKP_DICT_XCD=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dict_xcd$v -o run -- python3 tools/stage_probe.py 21 10 > /dev/null 2>&1
done
echo done

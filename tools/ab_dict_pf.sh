#!/bin/bash
# A/B of the software-pipelined dictionary gathers (SEZKP_DICT_PF=0 is the
# rolled round-2 loop): dictionary parity tests, single-proof stage split per
# side, rocprofv3 kernel stats per side, FETCH_SIZE of the new default.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "dict or golden or headline" > gpurun_out/dictpf_tests.log 2>&1
for v in 1 0 1 0; do
  SEZKP_DICT_PF=$v timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/ab_dict_pf.jsonl
done
for v in 1 0; do
  SEZKP_DICT_PF=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dict_pf$v -o run -- python3 tools/stage_probe.py 21 10 > /dev/null 2>&1
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/dictpf_fetch -o run -- python3 tools/stage_probe.py 21 3 > /dev/null 2>&1
echo done

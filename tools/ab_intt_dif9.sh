#!/bin/bash
# A/B (9 + 12 is the default since): the prover's 2^21-point INTT as 9 + 12 stages (k_ntt_dif9 + X16,
# SEZKP_NTT_DIF9X16=1) vs three 7-stage passes: the headline-size parity test
# under the switch, single-proof stage split per side, alternating bench lines.
set -euo pipefail
mkdir -p gpurun_out
SEZKP_NTT_DIF9X16=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "headline or ntt_large" > gpurun_out/intt_dif9_tests.log 2>&1
echo tests-ok
for v in 0 1 0 1; do
  echo -n "$v " >> gpurun_out/ab_intt_dif9.jsonl
  SEZKP_NTT_DIF9X16=$v timeout -k 10 120 python3 tools/stage_probe.py 21 20 >> gpurun_out/ab_intt_dif9.jsonl
done
B="python3 bench.py --no-cpu-baseline --no-configs --dntt-log-n 0 --steps 100"
for v in 0 1 0 1 0 1; do
  echo -n "$v " >> gpurun_out/ab_intt_dif9_bench.txt
  SEZKP_NTT_DIF9X16=$v timeout -k 10 200 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['trace_resident']['value'], d['single_proof']['ms_per_proof'], d['stages_ms']['intt'])" >> gpurun_out/ab_intt_dif9_bench.txt
done
echo done

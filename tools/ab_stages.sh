#!/bin/bash
# A/B of lib/ against ab_lib/alt.so on per-stage device times: one proof at a
# time on one GPU (P = 1) and one rank of an 8-GPU sharded proof alone on the
# GPU (P = 8, the per-rank cost model), two alternating rounds; parity tests
# ($1: -k expression, "" = skip) on lib/ first.
set -euo pipefail
O=gpurun_out/${AB_OUT:-abst}
mkdir -p $O
L=streaming-zero-knowledge-proofs_amd/lib/libsezkp_stark.so
cp $L /tmp/lib_main.so
if [ -n "${1:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "$1" > $O/tests.log 2>&1
  echo "tests ok"
fi
for rep in 1 2; do
  for arm in main alt; do
    # AB_ALT_ENV="VAR=value": the alt arm is lib/ itself with that variable set
    if [ $arm = main ] || [ -n "${AB_ALT_ENV:-}" ]; then cp /tmp/lib_main.so $L; else cp ab_lib/alt.so $L; fi
    for P in 1 8; do
      if [ $arm = alt ] && [ -n "${AB_ALT_ENV:-}" ]; then
        env ${AB_ALT_ENV} timeout -k 10 120 python3 tools/solo_trace.py $P 0 21 > $O/${arm}${rep}_p$P.json 2> $O/${arm}${rep}_p$P.err
      else
        timeout -k 10 120 python3 tools/solo_trace.py $P 0 21 > $O/${arm}${rep}_p$P.json 2> $O/${arm}${rep}_p$P.err
      fi
    done
  done
done
cp /tmp/lib_main.so $L
python3 tools/ab_stages_report.py $O > $O/report.txt
echo "ab stages done"

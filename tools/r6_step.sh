#!/bin/bash
# Round-6 working pass on the GPU box: named tests (-k expression $1, "" = skip),
# the config-2 probe, a short headline bench. Each GPU step has its own limit;
# the first failure ends the script.
set -euo pipefail
O=gpurun_out/${R6_OUT:-r6}
mkdir -p $O
if [ -n "${1:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$1" > $O/tests.log 2>&1
  echo "tests ok"
fi
timeout -k 10 120 python -u tools/c2_probe.py 20 400 > $O/c2.txt 2>&1
echo "c2 ok"
timeout -k 10 300 python -u bench.py --steps 100 --no-cpu-baseline --no-worst-case --no-host-rows --detail $O/detail.json > $O/bench.json 2> $O/bench.err
echo "bench ok"

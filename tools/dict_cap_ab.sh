#!/bin/bash
# Dictionary table-size cap A/B (SEZKP_DICT_TAB_CAP: the largest table above
# level 0, in entries): dictionary parity tests at small caps, then per cap and
# round the single-proof kernel stats (rocprofv3) and the in-flight bench value.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/dictcap
mkdir -p $O
for cap in 16 4096; do
  SEZKP_DICT_TAB_CAP=$cap timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "dict or random or headline or golden" > $O/tests_$cap.log 2>&1
  echo "tests cap $cap ok"
done
P="python3 bench.py --inflight 1 --steps 12 --no-cpu-baseline --no-configs --no-worst-case --no-host-to-proof --no-host-rows --no-sharded --dntt-log-n 0"
B="python3 bench.py --steps 45 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-host-to-proof --no-sharded --dntt-log-n 0"
for rep in 1 2; do
  for cap in ${CAPS:-65536 16384 4096 1024}; do
    SEZKP_DICT_TAB_CAP=$cap timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c${cap}_$rep -o run -- $P --detail $O/c${cap}_${rep}_if1.json > $O/c${cap}_${rep}_if1.log 2>&1
    SEZKP_DICT_TAB_CAP=$cap timeout -k 10 200 $B --detail $O/c${cap}_${rep}_bench.json > $O/c${cap}_${rep}_bench.log 2>&1
    echo "cap $cap rep $rep ok"
  done
done
echo "dict cap ab done"

#!/bin/bash
# A/B of lib/ against ab_lib/alt.so (the same sources built with one switch
# flipped, swapped into lib/ on the box): the dictionary parity tests on lib/,
# then per arm and round the single-proof kernel stats (rocprofv3) and the
# in-flight bench value, alternating.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/libab
mkdir -p $O
L=streaming-zero-knowledge-proofs_amd/lib/libsezkp_stark.so
cp $L /tmp/lib_main.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dict or random or synthetic or headline or golden" > $O/tests.log 2>&1
echo "tests ok"
P="python3 bench.py --inflight 1 --steps 20 --no-cpu-baseline --no-configs --no-worst-case --no-host-to-proof --no-host-rows --no-sharded --dntt-log-n 0"
B="python3 bench.py --steps 60 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-host-to-proof --no-sharded --dntt-log-n 0"
for rep in 1 2; do
  for arm in main alt; do
    if [ $arm = main ]; then cp /tmp/lib_main.so $L; else cp ab_lib/alt.so $L; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${arm}$rep -o run -- $P --detail $O/${arm}${rep}_if1.json > $O/${arm}${rep}_if1.log 2>&1
    timeout -k 10 300 $B --detail $O/${arm}${rep}_bench.json > $O/${arm}${rep}_bench.log 2>&1
  done
done
cp /tmp/lib_main.so $L
echo "lib ab done"

#!/bin/bash
# Config 2 A/B step: NTT parity tests, then the 2^20 round-trip probe and its kernel stats.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/c2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k ntt --timeout 120 --timeout-method thread > $O/ntt_tests.log 2>&1
echo "ntt tests ok"
timeout -k 10 120 python3 tools/c2_probe.py 20 500 > $O/probe.log 2>&1
timeout -k 10 120 python3 tools/c2_probe.py 20 500 >> $O/probe.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- python3 tools/c2_probe.py 20 100 > $O/ks.log 2>&1
echo c2 done

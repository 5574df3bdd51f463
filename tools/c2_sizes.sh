#!/bin/bash
# Small-NTT diagnosis (run under rocprofv3 --kernel-trace): round trips at
# 2^12..2^20, so the per-kernel durations show how a pass's time grows with
# its workgroup count
set -e
for n in 12 14 16 17 18 19 20; do timeout -k 5 60 python3 tools/c2_probe.py $n 30; done

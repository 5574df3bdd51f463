#!/bin/bash
# Workgroups per CU for the small (latency-bound) NTT grids: SEZKP_NTT_SPREAD
# adds dynamic LDS to every pass of <= 1024 tiles (45000 B: one workgroup per
# CU; 20000 B: two), fwd + inv round trips (tools/c2_probe.py)
# (Measured round 3, profiles/r03/ab/ab_ntt_spread.txt: even. The switch was
# removed from ntt.hip afterwards; re-add it to repeat the run.)
set -e
for n in 20 19 18 22; do
  for sp in 0 45000 20000; do
    echo -n "spread $sp "; SEZKP_NTT_SPREAD=$sp timeout -k 5 60 python3 tools/c2_probe.py $n 100 2>/dev/null
  done
done

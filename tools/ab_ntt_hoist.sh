#!/bin/bash
# A/B of the NTT passes' load hoisting (round 3): ab_libs/base = the library
# before, lib/ = after; fwd + inv round trips through sezkp_gl_ntt
# (tools/c2_probe.py), alternating, two runs per side.
# (Measured round 3, profiles/r03/ab/ab_ntt_hoist.txt: even; the hoisted
# kernel was not kept. ab_libs/ is a local build, not in git.)
set -e
for n in 20 19 22 24 26; do
  for rep in 1 2; do
    echo -n "base $n "; SEZKP_PROBE_LIB=ab_libs/base/libsezkp_stark.so timeout -k 5 60 python3 tools/c2_probe.py $n 100 2>/dev/null
    echo -n "new  $n "; timeout -k 5 60 python3 tools/c2_probe.py $n 100 2>/dev/null
  done
done

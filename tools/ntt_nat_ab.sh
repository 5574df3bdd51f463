#!/bin/bash
# Natural-order NTT forms, fwd + inv round trip per size (tools/c2_probe.py):
#   dit  = DIT with a gathered first pass (default, round 3)
#   dif  = SEZKP_NTT_NAT_DIT=0: DIF with the transposed last pass (2^23..2^26)
#          or the L2-merged natural store (2^19..2^22)
#   brev = both off (SEZKP_NTT_NAT_TR=0 too): bit-reversal pass from 2^23
set -e
for n in 19 20 21 22 23 24 25 26; do
  echo -n "dit  "; timeout -k 5 60 python3 tools/c2_probe.py $n 40 2>/dev/null
  echo -n "dif  "; SEZKP_NTT_NAT_DIT=0 timeout -k 5 60 python3 tools/c2_probe.py $n 40 2>/dev/null
  if [ $n -ge 23 ]; then echo -n "brev "; SEZKP_NTT_NAT_DIT=0 SEZKP_NTT_NAT_TR=0 timeout -k 5 60 python3 tools/c2_probe.py $n 40 2>/dev/null; fi
done

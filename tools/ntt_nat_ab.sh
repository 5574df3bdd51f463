set -e
for n in 21 22 23 24 25 26; do
  for v in 0 1; do
    echo -n "NAT_TR=$v "; SEZKP_NTT_NAT_TR=$v timeout -k 5 60 python3 tools/c2_probe.py $n 40
  done
done

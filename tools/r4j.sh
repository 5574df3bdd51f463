set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/fs -o run -- python3 tools/fs_probe.py > $O/fs.log 2>&1 || exit 1
Q="bench.py --steps 100 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-sharded --dntt-log-n 0"
for i in 1 2; do
  timeout -k 10 200 python3 $Q > $O/if3_$i.log 2>&1 || exit 1
  timeout -k 10 200 python3 $Q --inflight 4 > $O/if4_$i.log 2>&1 || exit 1
done
echo done

# kernel timelines of one solo sharded rank (P = 8) and of the single-GPU proof
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/solo8 -o run -- python3 tools/solo_trace.py 8 0 21 > $O/solo8.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/single -o run -- python3 tools/solo_trace.py 1 0 21 > $O/single.log 2>&1 || exit 1
echo done

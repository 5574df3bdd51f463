# in-flight pipeline traces, staged (host -> proof) vs resident: kernels and
# memory copies, to find where the staged pipeline loses
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O
Q="bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-configs --no-worst-case --no-host-rows --no-sharded --dntt-log-n 0"
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/staged -o run -- python3 $Q > $O/staged.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/resident -o run -- python3 $Q --no-host-to-proof > $O/resident.log 2>&1 || exit 1
echo done

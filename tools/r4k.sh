set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
SEZKP_DEVICE_TRANSCRIPT=1 SEZKP_HOST_TRACE=1 timeout -k 10 120 python3 tools/solo_trace.py 1 0 21 > $O/devtr_single.log 2>&1 || exit 1
SEZKP_DEVICE_TRANSCRIPT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_transcript.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
echo done

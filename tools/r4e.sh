# radix-8 DIF passes (config 2 + the prover's INTT) and the device-transcript
# A/B: full GPU suite, NTT round-trip A/B, kernel traces, bench variants
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/gpu_tests.log | head -30; exit 1; }
for i in 1 2; do
  echo "r8" >> $O/c2_ab.txt
  timeout -k 10 60 python3 tools/c2_probe.py 20 300 >> $O/c2_ab.txt 2>&1 || exit 1
  echo "ntt4" >> $O/c2_ab.txt
  SEZKP_NTT_R8=0 timeout -k 10 60 python3 tools/c2_probe.py 20 300 >> $O/c2_ab.txt 2>&1 || exit 1
done
timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2prof -o run -- python3 tools/c2_probe.py 20 30 > $O/c2prof.log 2>&1 || exit 1
B="bench.py --inflight 1 --steps 10 --warmup 2 --no-cpu-baseline --no-configs --no-worst-case --no-host-to-proof --no-host-rows --dntt-log-n 0 --no-sharded"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dev_if1 -o run -- python3 $B > $O/dev_if1.log 2>&1 || exit 1
SEZKP_HOST_TRANSCRIPT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/host_if1 -o run -- python3 $B > $O/host_if1.log 2>&1 || exit 1
Q="bench.py --steps 100 --no-cpu-baseline --no-worst-case --no-host-rows --dntt-log-n 0"
timeout -k 10 400 python3 $Q > $O/dev_pred.log 2>&1 || exit 1
Q="$Q --no-sharded --no-configs"
SEZKP_NTT_R8=0 timeout -k 10 200 python3 $Q > $O/dev_ntt4.log 2>&1 || exit 1
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 $Q > $O/dev_q$q.log 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=$q SEZKP_HOST_TRANSCRIPT=1 timeout -k 10 200 python3 $Q > $O/host_q$q.log 2>&1 || exit 1
done
echo done

set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernel_abi.py -x -q --timeout 300 --timeout-method thread -k "ntt or coset or lde or headline" > gpurun_out/ntt_tests.log 2>&1
timeout -k 10 200 python -u bench.py --steps 100 --no-cpu-baseline --no-worst-case --no-host-to-proof --dntt-log-n 26 > gpurun_out/bench_narrow.log 2>&1
SEZKP_NTT_NO_NARROW=1 timeout -k 10 200 python -u bench.py --steps 100 --no-cpu-baseline --no-worst-case --no-host-to-proof --dntt-log-n 26 > gpurun_out/bench_nonarrow.log 2>&1

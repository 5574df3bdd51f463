# after making the stage events opt-in: GPU suite, default bench line, and the
# --gpus 2 rehearsal (two ranks on the one GPU, host-staged collectives) of the
# sharded measurement path
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/gpu_tests.log | head -30; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 500 python3 bench.py > $O/bench_default.log 2> $O/bench_default.err || { echo BENCH FAILED; tail -20 $O/bench_default.err; exit 1; }
echo bench ok
SEZKP_BENCH_HOST_COMM=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > $O/rehearse2.log 2> $O/rehearse2.err || { echo REHEARSAL FAILED; tail -20 $O/rehearse2.err; exit 1; }
echo done

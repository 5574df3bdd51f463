# bench.py --gpus 4 rehearsal: four ranks on the one GPU, host-staged collectives
set -uo pipefail
O=gpurun_out/r4u
mkdir -p $O
SEZKP_BENCH_HOST_COMM=1 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 4 --steps 5 --warmup 2 > $O/rehearse4.log 2> $O/rehearse4.err || { echo REHEARSAL FAILED; tail -30 $O/rehearse4.err; exit 1; }
echo done

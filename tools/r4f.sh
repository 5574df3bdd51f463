# host-transcript default + radix-8 2^20 passes: full GPU suite, default
# bench line, config 5 sliced ingest at P = 8 (host collectives, one GPU)
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 500 python3 bench.py > $O/bench_default.log 2> $O/bench_default.err || { echo BENCH FAILED; tail -20 $O/bench_default.err; exit 1; }
echo bench ok
timeout -k 10 600 python3 tools/c5_run.py 22 8 > $O/c5.log 2>&1 || { echo C5 FAILED; tail -20 $O/c5.log; exit 1; }
echo done

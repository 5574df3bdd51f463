# round-4 final measurements: GPU suite, default bench line, profile round
# (kernel stats + PMC passes), config-5 sliced ingest at P = 8
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r4final4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/gpu_tests.log | head -30; exit 1; }
echo tests ok
timeout -k 10 500 python3 bench.py > $O/bench_default.log 2> $O/bench_default.err || { echo BENCH FAILED; tail -20 $O/bench_default.err; exit 1; }
echo bench ok
bash tools/profile_round.sh > $O/profile_round.log 2>&1 || { echo PROFILE FAILED; tail -20 $O/profile_round.log; exit 1; }
echo profile ok
timeout -k 10 600 python3 tools/c5_run.py 22 8 > $O/c5.log 2>&1 || { echo C5 FAILED; tail -20 $O/c5.log; exit 1; }
echo done

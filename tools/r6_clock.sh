#!/bin/bash
# Round 6: the held clock of the kernels (GRBM_GUI_ACTIVE / 8 / wall, per
# MI355X_MICROARCH.md "DVFS give-back") with one proof at a time and with the
# bench's 3 proofs in flight, and kernel stats of one rank of an 8-GPU sharded
# proof alone on the GPU (the per-rank cost model) and of the single-GPU proof.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/${R6_OUT:-clock}
mkdir -p $O
C="SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
B="python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-configs --no-worst-case --no-host-to-proof --no-host-rows --no-sharded --dntt-log-n 0"
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $O/valu_if1 -o run -- $B --inflight 1 --detail $O/if1.json > $O/valu_if1.log 2>&1
echo "if1 ok"
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $O/valu_if3 -o run -- $B --detail $O/if3.json > $O/valu_if3.log 2>&1
echo "if3 ok"
python3 tools/pmc_clock.py $O/valu_if1 $O/valu_if3 > $O/clock.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/solo8 -o run -- python3 tools/solo_trace.py 8 0 21 > $O/solo8.json 2> $O/solo8.err
echo "solo8 ok"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/solo1 -o run -- python3 tools/solo_trace.py 1 0 21 > $O/solo1.json 2> $O/solo1.err
echo "solo1 ok"

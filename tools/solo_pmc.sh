#!/bin/bash
# PMC of one P = 8 rank alone (tools/solo_trace.py): clock, VALU issue and
# wave-cycle split of its kernels, to compare the small trees with the
# single-GPU ones.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/solo_pmc
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O/waits8 -o run -- python3 tools/solo_trace.py 8 0 21 > $O/waits8.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $O/clk8 -o run -- \
  python3 tools/solo_trace.py 8 0 21 > $O/clk8.log 2>&1
python3 tools/pmc_table.py $(find $O/waits8 -name "*counter_collection.csv") > $O/waits8.txt
python3 tools/pmc_clock.py $O/clk8 > $O/clock8.txt
echo solo pmc ok

#!/bin/bash
# The rocprofv3 runs behind profiles/ (run on the GPU box from the repo root):
#   1. kernel stats of the single-proof pass (bench --inflight 1): the
#      k_layer16 average the bench's live roofline is checked against
#   2. kernel stats of the default bench (3 proofs in flight)
#   3. one PMC pass of VALU/LDS issue counters (tools/pmc_valu.py)
#   4. FETCH_SIZE and WRITE_SIZE in separate passes (tools/pmc_summary.py)
#   5. one PMC pass of wave-cycle split counters (tools/pmc_table.py)
#   6. config 2 (the 2^20 NTT round trip): kernel stats and PMC passes (tools/c2_pmc.sh)
# Each step has its own time limit; the first failure ends the script.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
B="python3 bench.py --inflight 1 --steps 3 --warmup 1 --no-cpu-baseline --no-configs --no-worst-case --no-host-to-proof --no-host-rows --no-sharded --dntt-log-n 0 --detail $O/pmc.detail.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/if1 -o run -- \
  python3 bench.py --inflight 1 --steps 20 --no-cpu-baseline --no-configs --no-worst-case --no-host-to-proof --no-host-rows --no-sharded --dntt-log-n 0 --detail $O/if1.detail.json > $O/if1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/default -o run -- \
  python3 bench.py --no-cpu-baseline --no-sharded --detail $O/default.detail.json > $O/default.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU \
  SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/valu -o run -- $B > $O/valu.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d $O/waits -o run -- $B > $O/waits.log 2>&1
python3 tools/pmc_summary.py $O/fetch $O/write $O/valu > $O/pmc_summary.json
python3 tools/pmc_table.py $(find $O/waits -name "*counter_collection.csv") > $O/pmc_waits.txt
python3 tools/pmc_valu.py $O/valu/run_counter_collection.csv > $O/pmc_valu.txt
bash tools/c2_pmc.sh
echo profile_round done

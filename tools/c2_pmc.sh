#!/bin/bash
# Config 2 (2^20 NTT round trip): kernel stats and issue/stall PMC passes.
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/c2
mkdir -p $O
timeout -k 10 120 python3 tools/c2_probe.py 20 500 > $O/probe.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- python3 tools/c2_probe.py 20 100 > $O/ks.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  --output-format csv -d $O/p1 -o run -- python3 tools/c2_probe.py 20 10 > $O/p1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU \
  --output-format csv -d $O/p2 -o run -- python3 tools/c2_probe.py 20 10 > $O/p2.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o run -- python3 tools/c2_probe.py 20 10 > $O/p3.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p4 -o run -- python3 tools/c2_probe.py 20 10 > $O/p4.log 2>&1
python3 tools/pmc_table.py $(find $O/p1 $O/p2 $O/p3 $O/p4 -name "*counter_collection.csv") --match k_ntt > $O/pmc_table.txt
echo c2 pmc done

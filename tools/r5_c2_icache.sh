#!/bin/bash
# Config 2: instruction-fetch counters of the 2^20 passes (is the unrolled
# straight-line code fetch-bound on a cold instruction cache?).
set -euo pipefail
export TMPDIR=/tmp
O=gpurun_out/c2
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -iE "ICACHE|IFETCH|SQC_" $O/counters.txt | head -60 > $O/counters_if.txt || true
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $O/if1 -o run -- python3 tools/c2_probe.py 20 10 > $O/if1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d $O/if2 -o run -- python3 tools/c2_probe.py 20 10 > $O/if2.log 2>&1
python3 tools/pmc_table.py $(find $O/if1 $O/if2 -name "*counter_collection.csv") --match k_ntt > $O/icache_table.txt
echo icache done

#!/bin/bash
# Round-6 final evidence, part 2: smoke(), tools/profile_round.sh (kernel stats, PMC
# passes, config 2) and the held-clock passes of tools/r6_clock.sh.
set -euo pipefail
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/final_smoke.log 2>&1
echo "smoke ok"
bash tools/profile_round.sh
R6_OUT=clock_final bash tools/r6_clock.sh
echo "final2 ok"

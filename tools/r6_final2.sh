#!/bin/bash
# Round-6 final evidence, part 2: tools/profile_round.sh (kernel stats, PMC
# passes, config 2) and the held-clock passes of tools/r6_clock.sh.
set -euo pipefail
bash tools/profile_round.sh
R6_OUT=clock_final bash tools/r6_clock.sh
echo "final2 ok"

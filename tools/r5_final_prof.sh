#!/bin/bash
# Final round-5 profiles: tools/profile_round.sh, then the config-2 PMC passes.
set -euo pipefail
bash tools/profile_round.sh
bash tools/r5_c2_pmc.sh

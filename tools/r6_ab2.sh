#!/bin/bash
# Two stage A/Bs in one call (tools/ab_stages.sh with AB_ALT_ENV): the
# dictionary commit split across two streams (alt = SEZKP_DICT_SPLIT=0, the
# single-stream order) and, for the sharded FRI, the small-layer tail launched
# after the forest (alt = SEZKP_AB_TAIL_AFTER=1). Dictionary parity first.
set -euo pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "dict or random or headline or golden or staged or zero" > gpurun_out/ab2_tests.log 2>&1
echo "tests ok"
AB_ALT_ENV="SEZKP_DICT_SPLIT=0" AB_OUT=ab_split timeout -k 10 500 bash tools/ab_stages.sh ""
AB_ALT_ENV="SEZKP_AB_TAIL_AFTER=1" AB_OUT=ab_tail timeout -k 10 500 bash tools/ab_stages.sh ""
echo "ab2 done"

#!/bin/bash
# Small-NTT diagnosis: round trips at 2^12..2^20, one kernel trace per size,
# so the per-kernel durations show how a pass's time grows with its workgroup
# count. The loop runs here; rocprofv3 wraps the probe program itself (the
# program directly after `--`, no shell hop). Usage (GPU box, repo root):
#   bash tools/c2_sizes.sh [out_dir]
set -euo pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/c2_sizes}
mkdir -p "$O"
for n in 12 14 16 17 18 19 20; do
  timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/n$n" -o run -- \
    python3 tools/c2_probe.py $n 30 > "$O/n$n.log" 2>&1
done

#!/usr/bin/env python3
"""One rank of a P-rank sharded proof alone on one GPU (comm "solo", the
per-rank cost model of bench.py's sharded_predicted), T = 2^log_t: stage times
of a few proofs; run under `rocprofv3 --kernel-trace` for its kernel timeline.
Usage: tools/solo_trace.py [P] [rank] [log_t]"""
import os as _os
_os.environ.setdefault("SEZKP_STAGE_EVENTS", "1")  # device stage times (timed events)
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "streaming-zero-knowledge-proofs_amd"))
import torch  # noqa: E402,F401  (one HIP runtime: torch first)
from sezkp_amd import ProverContext, ShardedProverContext, reference_blocks  # noqa: E402


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    rank = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    log_t = int(sys.argv[3]) if len(sys.argv) > 3 else 21
    blocks = reference_blocks(1 << log_t, 512, 8)
    root = blocks.manifest_root()
    ctx = ShardedProverContext(rank, P, device=0, comm="solo") if P > 1 else ProverContext(0)
    ctx.upload(blocks)
    for _ in range(3):
        ctx.prove_view(root)
    walls, st = [], {}
    for _ in range(5):
        t0 = time.perf_counter()
        ctx.prove_view(root)
        walls.append((time.perf_counter() - t0) * 1e3)
        for k, v in ctx.stage_times_ms().items():
            st[k] = st.get(k, 0.0) + v / 5
    print(json.dumps({"P": P, "rank": rank, "wall_ms": walls, "stages_ms": {k: round(v, 4) for k, v in st.items()}}))
    ctx.close()


if __name__ == "__main__":
    main()

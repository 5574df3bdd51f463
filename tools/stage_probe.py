"""Single-proof stage split on the headline trace (T = 2^21, tau = 8): one
context, `reps` proofs one at a time, the mean of sezkp_ctx_stage_times per
stage. Run it twice under an environment switch for an A/B, or under
`rocprofv3 --kernel-trace --stats` for per-kernel durations:
  python3 tools/stage_probe.py [log_t] [reps]"""
import os as _os
_os.environ.setdefault("SEZKP_STAGE_EVENTS", "1")  # device stage times (timed events)
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "streaming-zero-knowledge-proofs_amd"))


def main():
    log_t = int(sys.argv[1]) if len(sys.argv) > 1 else 21
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    import torch  # noqa: F401  (one HIP runtime: torch first)
    from sezkp_amd import ProverContext, reference_blocks
    bl = reference_blocks(1 << log_t, 512, 8, 42)
    root = bl.manifest_root()
    c = ProverContext(0)
    c.upload(bl)
    for _ in range(3):
        c.prove_view(root)
    acc = {}
    t0 = time.perf_counter()
    for _ in range(reps):
        c.prove_view(root)
        for k, v in c.stage_times_ms().items():
            acc[k] = acc.get(k, 0.0) + v / reps
    wall = (time.perf_counter() - t0) / reps * 1e3
    env = {k: v for k, v in os.environ.items() if k.startswith("SEZKP_")}
    print(json.dumps({"log_t": log_t, "reps": reps, "wall_ms_per_proof": wall, "env": env,
                      "stages_ms": {k: round(v, 4) for k, v in acc.items()}}))
    c.close()


if __name__ == "__main__":
    main()

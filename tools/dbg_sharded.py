#!/usr/bin/env python3
"""Sharded prove on ONE GPU with P ranks (host collectives over gloo) or
RCCL (--comm rccl; needs P GPUs): every rank's proof must equal the oracle's.

    python tools/dbg_sharded.py --world 2 --log-t 13 --tau 2
"""
import os as _os
_os.environ.setdefault("SEZKP_STAGE_EVENTS", "1")  # device stage times (timed events)
import argparse
import hashlib
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "streaming-zero-knowledge-proofs_amd"), os.path.join(ROOT, "oracle")]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import sezkp_amd
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        blocks = sezkp_amd.synthetic_blocks(1 << args.log_t, args.b, args.tau, args.seed)
        root = blocks.manifest_root()
        dev = rank if (args.comm == "rccl" and not args.same_device) else 0
        ctx = sezkp_amd.ShardedProverContext(rank, world, device=dev, comm=args.comm)
        ctx.upload(blocks)
        t0 = time.perf_counter()
        art = ctx.prove(root)
        dt = time.perf_counter() - t0
        again = ctx.prove(root).proof_bytes == art.proof_bytes
        q.put((rank, hashlib.sha256(art.proof_bytes).hexdigest(), len(art.proof_bytes), dt, again,
               ctx.stage_times_ms()))
        ctx.close()
    except Exception as e:  # report, do not hang the parent
        import traceback
        traceback.print_exc()
        q.put((rank, f"ERR {e}", 0, 0, False, {}))
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--log-t", type=int, default=13)
    ap.add_argument("--b", type=int, default=512)
    ap.add_argument("--tau", type=int, default=2)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--comm", default="host")
    ap.add_argument("--no-oracle", action="store_true")
    ap.add_argument("--same-device", action="store_true", help="all ranks on GPU 0 (RCCL may refuse)")
    args = ap.parse_args()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=worker, args=(r, args.world, port, args, q)) for r in range(args.world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=600) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    want = None
    if not args.no_oracle:
        import oracle_ctypes as O
        import sezkp_amd
        blocks = sezkp_amd.synthetic_blocks(1 << args.log_t, args.b, args.tau, args.seed)
        want = hashlib.sha256(O.prove_v1(blocks, blocks.manifest_root())).hexdigest()
    ok = all(r[1] == (want or res[0][1]) and r[4] for r in res)
    for r in res:
        print(f"rank {r[0]}: {r[1][:16]} len={r[2]} {r[3]*1e3:.2f} ms repeat_ok={r[4]}")
    print("oracle:", (want or "skipped")[:16])
    print("ok" if ok else "MISMATCH")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()

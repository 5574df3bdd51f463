"""Multi-GPU `prove` launcher (BASELINE config 5: a streaming prove from a
blocks.jsonl sharded over the GPUs of one node).

    python -m sezkp_amd.launch prove --blocks blocks.jsonl --manifest manifest.cbor \\
        --out proof.cbor [--stream] [--gpus 8] [--comm rccl|host] [--assume-committed]

Mirrors `sezkp-cli prove --backend stark` (crates/sezkp-cli/src/main.rs:429-527):
the manifest precheck (main.rs:454-457) unless --assume-committed, then ONE
proof over all GPUs (`ShardedProverContext`: one process per GPU, RCCL over
xGMI inside the library), written by rank 0 as the CBOR ProofArtifact
(io.rs:176-183). Unlike the reference's stark path (io.rs:78-88), .jsonl/.ndjson
block files are accepted (io_jsonl.rs:43-84), as config 5 requires; their
precheck uses the streaming Frontier root as the reference's
verify_block_file_against_manifest does (sezkp-merkle lib.rs:302-330).
--gpus 1 runs the single-GPU context. --comm host runs every rank on GPU 0
with host-staged collectives (tests).

With several GPUs a .jsonl/.ndjson file is read in slices (sezkp_amd.ingest):
each rank decodes the metadata of 1/P of the lines, the metadata and the
manifest leaf hashes are allgathered (rank 0 reduces the leaves to the root
and broadcasts the precheck verdict), and each rank fully decodes and uploads
only the lines of the blocks over its own rows plus the halo row
(--full-ingest: every rank decodes the whole file, as before).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _read_manifest(path: str):
    """Manifest file {root: [32 uints], n_leaves} (sezkp-merkle commit output),
    .cbor or .json -> (root, n_leaves)."""
    import ctypes as C
    from ._lib import check, lib
    raw = open(path, "rb").read()
    root = C.create_string_buffer(32)
    n = C.c_uint32()
    err = C.create_string_buffer(512)
    check(lib.sezkp_manifest_decode(raw, len(raw), int(path.lower().endswith(".json")), root, C.byref(n), err, 512),
          err)
    return root.raw, n.value


def _precheck(blocks, path: str, root: bytes, n_leaves: int) -> None:
    """verify_block_file_against_manifest (sezkp-merkle lib.rs:302-337): the
    Frontier root for .jsonl/.ndjson files, the batch root otherwise, then the
    leaf count."""
    got = blocks.file_root(path)
    if got != root:
        raise RuntimeError(f"blocks/manifest mismatch: root mismatch: manifest={root.hex()}, recomputed={got.hex()}")
    if blocks.n_blocks != n_leaves:
        raise RuntimeError(f"blocks/manifest mismatch: leaf count mismatch: manifest={n_leaves}, "
                           f"recomputed={blocks.n_blocks}")


def _is_jsonl(path: str) -> bool:
    return path.rsplit(".", 1)[-1].lower() in ("jsonl", "ndjson") if "." in path else False


def _worker(rank: int, world: int, port: int, args, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # this rank's share of the host threads for block decoding (codec.cpp decode_threads)
    if "SEZKP_HOST_THREADS" not in os.environ:
        cpus = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
        os.environ["SEZKP_HOST_THREADS"] = str(max(1, cpus // world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from . import ShardedProverContext
        from .blocks import BlockSoA
        t0 = time.perf_counter()
        root, n_leaves = _read_manifest(args.manifest)
        dev = 0 if args.comm == "host" else rank
        if _is_jsonl(args.blocks) and not args.full_ingest:
            from .ingest import TorchComm, sliced_ingest
            ing = sliced_ingest(args.blocks, rank, world, TorchComm(), None if args.assume_committed else root,
                                n_leaves, frontier=True)
            t_load = time.perf_counter() - t0
            ctx = ShardedProverContext(rank, world, device=dev, comm=args.comm)
            ctx.upload_rows(ing["blocks"], ing["row0"], ing["nrows"])
        else:
            blocks = BlockSoA.from_file(args.blocks)
            t_load = time.perf_counter() - t0
            if not args.assume_committed:
                _precheck(blocks, args.blocks, root, n_leaves)
            ctx = ShardedProverContext(rank, world, device=dev, comm=args.comm)
            ctx.upload(blocks)
        t1 = time.perf_counter()
        art = ctx.prove(root, streaming=args.stream)
        t_prove = time.perf_counter() - t1
        if rank == 0:
            with open(args.out, "wb") as f:
                f.write(art.to_cbor())
        ctx.close()
        q.put((rank, None, len(art.proof_bytes), t_load, t_prove))
    except Exception as e:  # reported by the parent
        q.put((rank, f"{type(e).__name__}: {e}", 0, 0.0, 0.0))
    finally:
        dist.destroy_process_group()


def _stop(ps) -> None:
    """Terminate, then kill, every worker still alive (a rank blocked in a
    collective whose peer failed never returns on its own)."""
    for p in ps:
        if p.is_alive():
            p.terminate()
    for p in ps:
        p.join(timeout=10)
        if p.is_alive():
            p.kill()
            p.join(timeout=10)


def _collect(ps, q, timeout: float):
    """Results one by one. The first error, a worker that died without
    reporting, or the overall timeout stops the remaining ranks.
    Returns (sorted results, None) or (partial results, error message)."""
    import queue
    res = []
    deadline = time.monotonic() + timeout
    while len(res) < len(ps):
        left = deadline - time.monotonic()
        if left <= 0:
            _stop(ps)
            return res, f"timeout after {timeout:.0f} s ({len(res)} of {len(ps)} ranks reported)"
        try:
            r = q.get(timeout=min(1.0, left))
        except queue.Empty:
            reported = {x[0] for x in res}
            dead = [i for i, p in enumerate(ps) if i not in reported and not p.is_alive()]
            if dead:
                _stop(ps)
                return res, f"rank {dead[0]} exited with code {ps[dead[0]].exitcode} without a result"
            continue
        res.append(r)
        if r[1]:
            _stop(ps)
            return res, f"rank {r[0]}: {r[1]}"
    for p in ps:
        p.join(timeout=60)
    return sorted(res), None


def prove(args) -> int:
    if not args.out.lower().endswith(".cbor"):
        print("error: --out must be a .cbor artifact", file=sys.stderr)
        return 2
    if args.gpus == 1 and args.comm == "rccl":
        from . import ProverContext
        from .blocks import BlockSoA
        blocks = BlockSoA.from_file(args.blocks)
        root, n_leaves = _read_manifest(args.manifest)
        if not args.assume_committed:
            try:
                _precheck(blocks, args.blocks, root, n_leaves)
            except RuntimeError as e:
                print(f"error: {e}", file=sys.stderr)
                return 1
        ctx = ProverContext(0)
        ctx.upload(blocks)
        art = ctx.prove(root, streaming=args.stream)
        open(args.out, "wb").write(art.to_cbor())
        print(json.dumps({"gpus": 1, "proof_bytes": len(art.proof_bytes)}))
        return 0
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, args.gpus, port, args, q), daemon=True) for r in range(args.gpus)]
    for p in ps:
        p.start()
    res, err = _collect(ps, q, args.timeout)
    if err:
        print(f"error: {err}", file=sys.stderr)
        return 1
    print(json.dumps({"gpus": args.gpus, "comm": args.comm, "proof_bytes": res[0][2],
                      "load_s": [round(x[3], 3) for x in res], "prove_s": [round(x[4], 4) for x in res]}))
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m sezkp_amd.launch")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("prove")
    p.add_argument("--backend", default="stark", choices=["stark"])
    p.add_argument("--blocks", required=True)
    p.add_argument("--manifest", required=True)
    p.add_argument("--out", required=True)
    p.add_argument("--stream", action="store_true")
    p.add_argument("--assume-committed", action="store_true")
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--comm", default="rccl", choices=["rccl", "host"])
    p.add_argument("--timeout", type=float, default=1800.0)
    p.add_argument("--full-ingest", action="store_true",
                   help="every rank decodes the whole block file (default for .jsonl with --gpus > 1: sliced)")
    args = ap.parse_args(argv)
    return prove(args)


if __name__ == "__main__":
    sys.exit(main())

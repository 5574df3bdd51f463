"""Sliced ingest of a JSONL blocks file for a sharded prove (BASELINE config 5).

The reference streams `blocks.jsonl` line by line with bounded memory
(`stream_block_summaries_jsonl`, crates/sezkp-core/src/io_jsonl.rs:84) into
the O(log n) Frontier (crates/sezkp-merkle/src/lib.rs:173-207, 302-330). Here
each of the P ranks reads only its share of the file:

1. each rank decodes the lines that start in bytes [len g/P, len (g+1)/P)
   in full (fields, steps, byte offset per line), while a warm-up collective
   sets up the transport;
2. the metadata (fields + step counts) and manifest leaf hashes are
   allgathered, so every rank knows every block's rows; rank 0 reduces the
   leaves to the Frontier / batch root and broadcasts the precheck verdict
   (main.rs:454-457);
3. each rank's rows plus the halo (sezkp_shard_rows) lie over nearly the same
   lines as its byte range (rows and bytes per block are near uniform): it
   takes them from its own decode and decodes only the few lines beyond it,
   then uploads that slice (sezkp_ctx_upload_rows).

`comm` provides allgather_object(obj) -> list and broadcast_object(obj) -> obj
(torch.distributed over gloo in the launcher; a stub in the CPU tests).
"""
from __future__ import annotations

import os
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from .blocks import BlockSoA, merkle_root_of_leaves, shard_rows


class TorchComm:
    """allgather / broadcast of Python objects over a torch.distributed group."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist, self.group = dist, group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)

    def allgather_object(self, obj):
        out = [None] * self.world
        self.dist.all_gather_object(out, obj, group=self.group)
        return out

    def broadcast_object(self, obj):
        box = [obj]
        self.dist.broadcast_object_list(box, src=0, group=self.group)
        return box[0]

    def warm(self, nbytes: int) -> None:
        """One allgather of nbytes per rank: gloo's first large transfer
        costs ~0.1-0.5 s, paid here while the decode runs."""
        import torch
        out = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.world)]
        self.dist.all_gather(out, torch.zeros(nbytes, dtype=torch.uint8), group=self.group)


def open_blocks(path: str):
    """The file as a read-only uint8 memmap (nothing is read until touched)."""
    if os.path.getsize(path) == 0:
        return np.zeros(0, np.uint8)
    return np.memmap(path, dtype=np.uint8, mode="r")


def sliced_ingest(path: str, rank: int, world: int, comm, check_root: bytes = None, n_leaves: int = None,
                  frontier: bool = True) -> dict:
    """Returns {"blocks": the view for upload_rows (global fields + this rank's
    step slice), "row0", "nrows", "meta": all blocks' fields (no steps),
    "root": the recomputed manifest root, "seconds": {...}}. With check_root,
    the precheck verdict (root, then leaf count) raises on every rank alike."""
    t0 = time.perf_counter()
    data = open_blocks(path)
    L = int(data.size)
    with ThreadPoolExecutor(1) as ex:  # the decode releases the GIL
        fut = ex.submit(BlockSoA.from_jsonl_meta, data, L * rank // world, L * (rank + 1) // world, True)
        if hasattr(comm, "warm"):
            comm.warm(1 << 19)
        own, offs = fut.result()
    meta = own.meta_only()
    leaves = meta.leaf_hashes()
    t1 = time.perf_counter()
    parts = comm.allgather_object((meta, offs, leaves))
    t2 = time.perf_counter()
    allm = BlockSoA.concat_meta([p[0] for p in parts])
    all_offs = np.concatenate([p[1] for p in parts]).astype(np.uint64) if parts else np.zeros(0, np.uint64)
    taus = {p[0].tau for p in parts if p[0].n_blocks}
    if len(taus) > 1:
        raise ValueError("blocks disagree on tau (windows length) across the file")
    # precheck (verify_block_file_against_manifest, sezkp-merkle lib.rs:302-337)
    verdict = None
    root = None
    if rank == 0:
        root = merkle_root_of_leaves(b"".join(p[2] for p in parts), frontier)
        if check_root is not None:
            if root != check_root:
                verdict = (f"blocks/manifest mismatch: root mismatch: manifest={check_root.hex()}, "
                           f"recomputed={root.hex()}")
            elif n_leaves is not None and allm.n_blocks != n_leaves:
                verdict = (f"blocks/manifest mismatch: leaf count mismatch: manifest={n_leaves}, "
                           f"recomputed={allm.n_blocks}")
    verdict, root = comm.broadcast_object((verdict, root))
    if verdict:
        raise ValueError(verdict)
    t3 = time.perf_counter()
    # this rank's rows: whole blocks [a, b); the own decode holds blocks [oa, ob)
    row0, nrows = shard_rows(allm.step_start, rank, world)
    ss = allm.step_start
    a = int(np.searchsorted(ss, row0, side="right") - 1)
    b = int(np.searchsorted(ss, row0 + nrows, side="left"))
    oa = sum(int(p[0].n_blocks) for p in parts[:rank])
    ob = oa + int(own.n_blocks)
    tau = allm.tau

    def line_end(k):  # byte offset just past block k - 1's line
        return int(all_offs[k]) if k < all_offs.size else L

    pieces = []
    if a < min(b, oa):
        pieces.append(BlockSoA.from_jsonl_range(data, int(all_offs[a]), line_end(min(b, oa))))
    lo_k, hi_k = max(a, oa), min(b, ob)
    if lo_k < hi_k:
        r0, r1 = int(own.step_start[lo_k - oa]), int(own.step_start[hi_k - oa])
        pieces.append(_Steps(own.input_mv[r0:r1], own.mv[r0 * tau:r1 * tau], own.has_write[r0 * tau:r1 * tau],
                             own.wsym[r0 * tau:r1 * tau], own.step_start[lo_k - oa:hi_k - oa + 1] - r0))
    if max(a, ob) < b:
        pieces.append(BlockSoA.from_jsonl_range(data, int(all_offs[max(a, ob)]), line_end(b)))
    counts = np.concatenate([np.diff(x.step_start) for x in pieces]) if pieces else np.zeros(0, np.uint64)
    if counts.size != b - a or not np.array_equal(counts, np.diff(ss[a:b + 1])):
        raise ValueError("sliced decode disagrees with the metadata pass (file changed while reading?)")
    sl = _Steps(*(np.concatenate([getattr(x, f) for x in pieces]) if pieces else getattr(own, f)[:0]
                  for f in ("input_mv", "mv", "has_write", "wsym")), None)
    t4 = time.perf_counter()
    return {"blocks": allm.with_steps(sl), "row0": row0, "nrows": nrows, "meta": allm, "root": root,
            "lines": (a, b), "own_lines": (oa, ob),
            "seconds": {"decode_own": t1 - t0, "allgather": t2 - t1, "precheck": t3 - t2, "slice": t4 - t3,
                        "total": t4 - t0}}


class _Steps:
    """Step arrays of a run of whole blocks (what BlockSoA.with_steps takes)."""

    def __init__(self, input_mv, mv, has_write, wsym, step_start):
        self.input_mv, self.mv, self.has_write, self.wsym, self.step_start = input_mv, mv, has_write, wsym, step_start

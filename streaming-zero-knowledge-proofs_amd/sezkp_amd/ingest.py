"""Sliced ingest of a JSONL blocks file for a sharded prove (BASELINE config 5).

The reference streams `blocks.jsonl` line by line with bounded memory
(`stream_block_summaries_jsonl`, crates/sezkp-core/src/io_jsonl.rs:84) into
the O(log n) Frontier (crates/sezkp-merkle/src/lib.rs:173-207, 302-330). Here
each of the P ranks reads only its share of the file:

1. metadata pass: the lines that start in bytes [len g/P, len (g+1)/P) are
   decoded without their steps (fields + step count + byte offset per line);
2. the metadata and manifest leaf hashes are allgathered, so every rank knows
   every block's rows; rank 0 reduces the leaves to the Frontier / batch root
   and broadcasts the precheck verdict (main.rs:454-457);
3. each rank fully decodes only the lines of the blocks over its rows plus the
   halo (sezkp_shard_rows), and uploads that slice (sezkp_ctx_upload_rows).

`comm` provides allgather_object(obj) -> list and broadcast_object(obj) -> obj
(torch.distributed over gloo in the launcher; a stub in the CPU tests).
"""
from __future__ import annotations

import os
import time

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
    meta, offs = BlockSoA.from_jsonl_meta(data, L * rank // world, L * (rank + 1) // world)
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
    # this rank's rows: whole blocks [a, b), their lines decoded in full
    row0, nrows = shard_rows(allm.step_start, rank, world)
    ss = allm.step_start
    a = int(np.searchsorted(ss, row0, side="right") - 1)
    b = int(np.searchsorted(ss, row0 + nrows, side="left"))
    lo = int(all_offs[a])
    hi = int(all_offs[b]) if b < all_offs.size else L
    sl = BlockSoA.from_jsonl_range(data, lo, hi)
    if sl.n_blocks != b - a or not np.array_equal(np.diff(sl.step_start), np.diff(ss[a:b + 1])):
        raise ValueError("sliced decode disagrees with the metadata pass (file changed while reading?)")
    t4 = time.perf_counter()
    return {"blocks": allm.with_steps(sl), "row0": row0, "nrows": nrows, "meta": allm, "root": root,
            "lines": (a, b), "seconds": {"meta": t1 - t0, "allgather": t2 - t1, "precheck": t3 - t2,
                                         "slice_decode": t4 - t3, "total": t4 - t0}}

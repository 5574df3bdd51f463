"""Multi-GPU orchestration: one process per GPU over torch.distributed
(backend "nccl" = RCCL on ROCm; "gloo" for the CPU tests).

* `time_replicas`: weak-scaling driver for independent proofs — each rank
  times its own steps between barriers, the job time is the MAX over ranks.
* `HostCollectives`: the three exchanges of the sharded prover
  (`ShardedProverContext(comm="host")`: allgather, all-to-all, byte-sum
  allreduce) over a torch.distributed group on host buffers — gloo on CPU,
  so several ranks can share one GPU in tests. Production uses RCCL inside
  the library (comm="rccl").
* `sharded_merkle_root`: the BLAKE3 layer commitment of a power-of-two layer
  whose leaves are split into contiguous per-rank shards. Each rank reduces
  its shard to one subtree root (on the GPU in production), the P roots are
  gathered to rank 0 which builds the top log2(P) levels (the "cap"), and the
  root is broadcast. Bit-identical to the single-device root
  (merkle.rs:46-71: aligned power-of-two subtrees of a power-of-two tree).
"""
from __future__ import annotations

import ctypes as C
import time
from typing import Callable

import numpy as np
import torch
import torch.distributed as dist


def _world(group=None) -> tuple[int, int]:
    if not dist.is_available() or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def _device_for_collectives(group=None) -> torch.device:
    backend = dist.get_backend(group) if dist.is_initialized() else "gloo"
    return torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")


def time_replicas(step: Callable[[], object], steps: int, warmup: int, sync: Callable[[], None] = lambda: None,
                  group=None) -> float:
    """Run `warmup` untimed + `steps` timed calls of `step` on every rank;
    returns the max over ranks of the timed wall time (seconds)."""
    rank, world = _world(group)
    for _ in range(warmup):
        step()
    if world > 1:
        dist.barrier(group)
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if world > 1:
        dist.barrier(group)
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=_device_for_collectives(group))
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        dt = float(t.item())
    return dt


def blake3_parent(left: bytes, right: bytes, hash_fn: Callable[[bytes], bytes]) -> bytes:
    return hash_fn(left + right)


def sharded_merkle_root(shard_root: bytes, hash_fn: Callable[[bytes], bytes], group=None) -> bytes:
    """Combine per-rank subtree roots (rank order = leaf order) into the layer
    root on rank 0 and broadcast it. World size must be a power of two."""
    rank, world = _world(group)
    if world == 1:
        return shard_root
    if world & (world - 1):
        raise ValueError("world size must be a power of two for an aligned Merkle cap")
    dev = _device_for_collectives(group)
    mine = torch.frombuffer(bytearray(shard_root), dtype=torch.uint8).to(dev)
    gathered = [torch.empty(32, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(gathered, mine, group=group)
    out = torch.empty(32, dtype=torch.uint8, device=dev)
    if rank == 0:
        level = [bytes(t.cpu().numpy().tobytes()) for t in gathered]
        while len(level) > 1:  # cap: top log2(P) levels, rank 0 only
            level = [blake3_parent(level[i], level[i + 1], hash_fn) for i in range(0, len(level), 2)]
        out.copy_(torch.frombuffer(bytearray(level[0]), dtype=torch.uint8).to(dev))
    dist.broadcast(out, src=0, group=group)
    return bytes(out.cpu().numpy().tobytes())


def _host_u8(ptr: int, nbytes: int) -> torch.Tensor:
    """uint8 CPU tensor aliasing host memory at ptr (no copy)."""
    if nbytes == 0:
        return torch.empty(0, dtype=torch.uint8)
    arr = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(ptr))
    return torch.from_numpy(arr)


class HostCollectives:
    """sezkp_host_comm callbacks over a CPU (gloo) torch.distributed group."""

    def __init__(self, group=None):
        self.group = group
        self.calls = {"allgather": 0, "alltoall": 0, "allreduce": 0}

    def allgather(self, send: int, recv: int, nbytes: int) -> int:
        rank, world = _world(self.group)
        out = _host_u8(recv, nbytes * world)
        src = _host_u8(send, nbytes).clone()
        dist.all_gather(list(out.view(world, nbytes).unbind(0)) if nbytes else [out] * world, src, group=self.group)
        self.calls["allgather"] += 1
        return 0

    def alltoall(self, send: int, recv: int, nbytes: int) -> int:
        rank, world = _world(self.group)
        src = _host_u8(send, nbytes * world).clone()
        out = _host_u8(recv, nbytes * world)
        tmp = torch.empty_like(src)
        dist.all_to_all_single(tmp, src, group=self.group)
        out.copy_(tmp)
        self.calls["alltoall"] += 1
        return 0

    def allreduce_sum_u8(self, buf: int, nbytes: int) -> int:
        t = _host_u8(buf, nbytes)
        tmp = t.clone()
        dist.all_reduce(tmp, op=dist.ReduceOp.SUM, group=self.group)
        t.copy_(tmp)
        self.calls["allreduce"] += 1
        return 0

    def c_struct(self):
        from ._lib import ALLGATHER_FN, ALLREDUCE_FN, ALLTOALL_FN, HostComm

        def wrap(fn, n):
            def cb(user, *a):
                try:
                    return fn(*a)
                except Exception:  # never propagate into C
                    import traceback
                    traceback.print_exc()
                    return -1
            return cb
        # keep the CFUNCTYPE objects alive as long as this object
        self._cbs = (ALLGATHER_FN(wrap(self.allgather, 3)), ALLTOALL_FN(wrap(self.alltoall, 3)),
                     ALLREDUCE_FN(wrap(self.allreduce_sum_u8, 2)))
        return HostComm(None, *self._cbs)

"""Multi-GPU orchestration: one process per GPU over torch.distributed
(backend "nccl" = RCCL on ROCm; "gloo" for the CPU tests).

* `HostCollectives`: the three exchanges of the sharded prover
  (`ShardedProverContext(comm="host")`: allgather, all-to-all, byte-sum
  allreduce) over a torch.distributed group on host buffers — gloo on CPU,
  so several ranks can share one GPU in tests. Production uses RCCL inside
  the library (comm="rccl"). The replica headline's barrier and max-over-
  ranks timing live in bench.py; the sharded prover's caps are built inside
  the library (prover.cpp, allgathered run roots).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.distributed as dist


def _world(group=None) -> tuple[int, int]:
    if not dist.is_available() or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


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

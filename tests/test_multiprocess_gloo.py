"""World-size-2 (and 4) CPU tests of the multi-process path over gloo:
the replica timing driver and the sharded Merkle commitment (per-rank
subtrees + cap reduced on rank 0) must equal the single-device root.
The per-rank subtree is computed by the oracle here (CPU); on the GPU box the
same function receives the HIP subtree root (sezkp_merkle_root_u64).
"""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

from conftest import ORACLE, PKG


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, log_n, q):
    sys.path[:0] = [PKG, ORACLE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_ctypes as O
        from sezkp_amd.dist import sharded_merkle_root, time_replicas
        n = 1 << log_n
        vals = O.det_vec(n, 77)
        shard = n // world
        mine = vals[rank * shard:(rank + 1) * shard]
        leaves = b"".join(O.hash_leaf_u64(int(v)) for v in mine)
        root = sharded_merkle_root(O.merkle_root(leaves), lambda m: O.blake3(m), None)
        calls = []
        dt = time_replicas(lambda: calls.append(1), steps=3, warmup=2)
        q.put((rank, root, dt, len(calls)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,log_n", [(2, 6), (2, 11), (4, 8)])
def test_sharded_merkle_cap_equals_single_device_root(oracle, world, log_n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, log_n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    vals = oracle.det_vec(1 << log_n, 77)
    want = oracle.merkle_root(b"".join(oracle.hash_leaf_u64(int(v)) for v in vals))
    assert all(r[1] == want for r in res)
    assert all(r[3] == 5 for r in res)            # warmup + steps on every rank
    assert len({round(r[2], 9) for r in res}) == 1  # max-over-ranks time agreed

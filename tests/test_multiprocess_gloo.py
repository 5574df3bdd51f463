"""World-size-2 (and 4) CPU tests of the multi-process path over gloo: the
host collectives behind ShardedProverContext(comm="host") and models of the
sharded layouts and of the four-step distributed NTT."""
import os
import sys

import pytest
import torch.multiprocessing as mp

from conftest import ORACLE, PKG, free_port


def _free_port():
    return free_port()


# ------------------------------------------------- sharded prover (CPU side)
def _coll_worker(rank, world, port, q):
    sys.path[:0] = [PKG, ORACLE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import ctypes as C
    import numpy as np
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sezkp_amd.dist import HostCollectives
        hc = HostCollectives(None)
        nb = 24
        send = (C.c_uint8 * (nb * world))(*[(rank * 31 + i) % 251 for i in range(nb * world)])
        recv = (C.c_uint8 * (nb * world))()
        assert hc.allgather(C.addressof(send), C.addressof(recv), nb) == 0
        ag = bytes(recv)
        assert hc.alltoall(C.addressof(send), C.addressof(recv), nb) == 0
        a2a = bytes(recv)
        # byte-sum allreduce: disjoint writers reassemble the whole buffer
        body = (C.c_uint8 * (nb * world))()
        for i in range(nb):
            body[rank * nb + i] = (rank + 7 * i) % 256
        assert hc.allreduce_sum_u8(C.addressof(body), nb * world) == 0
        # the C-callable struct dispatches to the same methods
        s = hc.c_struct()
        assert s.allgather(None, C.addressof(send), C.addressof(recv), nb) == 0 and bytes(recv) == ag
        q.put((rank, ag, a2a, bytes(body), np.frombuffer(bytes(send), np.uint8).tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_host_collectives_gloo(world):
    """The three exchanges of sezkp_ctx_create_sharded_host over gloo."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_coll_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nb = 24
    sends = [bytes(r[4]) for r in res]
    for rank, ag, a2a, body, _ in res:
        assert ag == b"".join(s[:nb] for s in sends)
        assert a2a == b"".join(s[rank * nb:(rank + 1) * nb] for s in sends)
        assert body == bytes((r + 7 * i) % 256 for r in range(world) for i in range(nb))


def _layout_worker(rank, world, port, log_n, q):
    """numpy model of the sharded LDE/FRI layout (same index maps as
    k_cyc_pack / k_cyc_unpack / k_runroots_scatter / the path ownership)."""
    sys.path[:0] = [PKG, ORACLE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_ctypes as O
        S, P = 4096, world
        logP = P.bit_length() - 1
        n = 1 << log_n
        base = O.det_vec(n, 5)
        z = 0x1234567 % O.P if hasattr(O, "P") else 0x1234567
        full = O.lde_deep(base, 3, z)          # natural-order layer 0 (oracle)
        N = full.size
        M = N // P
        cyc = full[rank::P]                    # rank's coset values f(3 w^(rank + P j))
        lsp = 12 - logP
        o = np.arange(M, dtype=np.int64)
        d, r = o // (M // P), o % (M // P)
        send = cyc[((r >> lsp) << 12) + (d << lsp) + (r & ((1 << lsp) - 1))]
        recv = torch.empty(M, dtype=torch.int64)
        dist.all_to_all_single(recv, torch.from_numpy(send.view(np.int64).copy()))
        recv = recv.numpy().view(np.uint64)
        g, r = o // (M // P), o % (M // P)
        local = np.empty(M, np.uint64)
        local[((r >> lsp) << 12) + ((r & ((1 << lsp) - 1)) << logP) + g] = recv
        # expected: runs k1 of [k1*P*S + rank*S, +S)
        runs = full.reshape(-1, P, S)[:, rank, :].reshape(-1)
        ok_layout = bool(np.array_equal(local, runs))
        # local fold == global fold restricted (i and i+len/2 share i mod P*S)
        beta = 0xABCDEF
        pp = O.P if hasattr(O, "P") else 0xFFFFFFFF00000001
        gf = np.array([(int(full[i]) + beta * int(full[i + N // 2])) % pp for i in range(N // 2)], np.uint64)
        lf = np.array([(int(local[i]) + beta * int(local[i + M // 2])) % pp for i in range(M // 2)], np.uint64)
        ok_fold = bool(np.array_equal(lf, gf.reshape(-1, P, S)[:, rank, :].reshape(-1)))
        # run subtree roots -> allgather -> cap in global run order (k1 * P + d)
        rr = [O.merkle_root(b"".join(O.hash_leaf_u64(int(v)) for v in local[j * S:(j + 1) * S]))
              for j in range(M // S)]
        gath = [None] * P
        dist.all_gather_object(gath, rr)
        level = [gath[dd][k1] for k1 in range(M // S) for dd in range(P)]
        while len(level) > 1:
            level = [O.blake3(level[i] + level[i + 1]) for i in range(0, len(level), 2)]
        q.put((rank, ok_layout, ok_fold, level[0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,log_n", [(2, 12), (4, 12)])
def test_sharded_layout_model_gloo(oracle, world, log_n):
    """Coset split + all-to-all + run subtrees + cap == the single-device
    layer-0 commitment; rank-local folds == the global fold."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_layout_worker, args=(r, world, port, log_n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    base = oracle.det_vec(1 << log_n, 5)
    full = oracle.lde_deep(base, 3, 0x1234567)
    want = oracle.merkle_root(b"".join(oracle.hash_leaf_u64(int(v)) for v in full))
    for rank, ok_layout, ok_fold, root in res:
        assert ok_layout and ok_fold
        assert root == want


GL = 0xFFFFFFFF00000001


def _dntt_worker(rank, world, port, log_n, q):
    """The four-step distributed NTT of sezkp_ctx_dist_ntt restated on the
    CPU: local M-point NTT (oracle), twiddle w_N^(g k2), one gloo all-to-all,
    P-point DFTs. Checks the algorithm and the documented layouts."""
    sys.path[:0] = [PKG, ORACLE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_ctypes as O
        n = 1 << log_n
        M, Q = n // world, n // world // world
        x = O.det_vec(n, 5)
        Y = O.ntt_forward(np.ascontiguousarray(x[rank::world]))
        wN = pow(7, (GL - 1) >> log_n, GL)
        s = np.array([int(Y[k]) * pow(wN, rank * k, GL) % GL for k in range(M)], dtype=np.uint64)
        recv = torch.empty(M, dtype=torch.int64)
        dist.all_to_all_single(recv, torch.from_numpy(s.view(np.int64)))
        r = recv.numpy().view(np.uint64)
        wP = pow(7, (GL - 1) // world, GL)
        out = np.zeros(M, dtype=np.uint64)
        for qq in range(Q):
            v = [int(r[g * Q + qq]) for g in range(world)]
            for k1 in range(world):
                out[k1 * Q + qq] = sum(v[g] * pow(wP, g * k1, GL) for g in range(world)) % GL
        X = O.ntt_forward(x)
        want = X.reshape(world, M)[:, rank * Q:(rank + 1) * Q].reshape(-1)
        q.put((rank, bool(np.array_equal(out, want))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,log_n", [(2, 10), (4, 10)])
def test_four_step_dist_ntt_model_gloo(oracle, world, log_n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dntt_worker, args=(r, world, port, log_n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res)

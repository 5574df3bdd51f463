"""GPU parity of the distributed four-step NTT (sezkp_ctx_dist_ntt; SURVEY
8(e), BASELINE config 4) against the oracle's single-domain NTT (ntt.rs:79-155).

P ranks share the box's one GPU and exchange through HostCollectives (gloo);
the kernels and layouts are the production ones, only the all-to-all
transport differs from RCCL. Layouts (sezkp_stark.h): rank g's input is
x[g + P j]; its output is X[g Q + q + M k1] at k1 Q + q (M = n/P, Q = M/P).
"""
import os
import sys

import numpy as np
import pytest

from conftest import ORACLE, PKG, free_port

pytestmark = pytest.mark.gpu


def _port():
    return free_port()


def expected_local(X: np.ndarray, rank: int, world: int) -> np.ndarray:
    M = X.size // world
    Q = M // world
    return X.reshape(world, M)[:, rank * Q:(rank + 1) * Q].reshape(-1)


def _worker(rank, world, port, log_n, seed, q):
    sys.path[:0] = [PKG, ORACLE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_ctypes as orc
        import sezkp_amd
        x = orc.det_vec(1 << log_n, seed)
        X = orc.ntt_forward(x)
        ctx = sezkp_amd.ShardedProverContext(rank, world, device=0, comm="host")
        loc = torch.from_numpy(np.ascontiguousarray(x[rank::world]).view(np.int64)).cuda()
        ctx.dist_ntt(loc)
        fwd_ok = np.array_equal(loc.cpu().numpy().view(np.uint64), expected_local(X, rank, world))
        ctx.dist_ntt(loc, inverse=True)
        inv_ok = np.array_equal(loc.cpu().numpy().view(np.uint64), x[rank::world])
        calls = dict(ctx._coll.calls)
        ctx.close()
        q.put((rank, fwd_ok, inv_ok, calls))
    except Exception as e:
        q.put((rank, f"ERR {type(e).__name__}: {e}", False, {}))
    finally:
        dist.destroy_process_group()


def sampled_spectrum(x: np.ndarray, w_R: int, R: int = 256) -> dict:
    """X[m n/R] for m < R, exactly, in O(n): X[m n/R] = sum_r w_R^(r m) S_r with
    S_r = sum of x_j over j = r (mod R) (summed as 32-bit halves, no overflow)."""
    P = 0xFFFFFFFF00000001
    n = x.size
    xr = x.reshape(n // R, R)
    lo = (xr & np.uint64(0xFFFFFFFF)).sum(axis=0, dtype=np.uint64)
    hi = (xr >> np.uint64(32)).sum(axis=0, dtype=np.uint64)
    S = [((int(h) << 32) + int(lo_)) % P for h, lo_ in zip(hi, lo)]
    wp = [pow(w_R, k, P) for k in range(R)]
    return {m * (n // R): sum(S[r] * wp[(r * m) % R] for r in range(R)) % P for m in range(R)}


def _worker_full(rank, world, port, log_n, seed, want_path, q):
    """Config 4 size: every one of the 2^26 outputs against the OpenMP
    oracle's NTT (ntt.rs:79-111 restated, computed once by the parent and
    memory-mapped here), plus an independent O(n) check of the n/256-spaced
    frequencies (residue-class sums, no NTT) and the round trip."""
    sys.path[:0] = [PKG, ORACLE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_ctypes as orc
        import sezkp_amd
        n = 1 << log_n
        x = orc.det_vec(n, seed)
        e = np.zeros(256, dtype=np.uint64)
        e[1] = 1
        sampled = sampled_spectrum(x, int(orc.ntt_forward(e)[1]))
        X = np.load(want_path, mmap_mode="r")
        ctx = sezkp_amd.ShardedProverContext(rank, world, device=0, comm="host")
        loc = torch.from_numpy(np.ascontiguousarray(x[rank::world]).view(np.int64)).cuda()
        ctx.dist_ntt(loc)
        out = loc.cpu().numpy().view(np.uint64)
        full_ok = np.array_equal(out, expected_local(X, rank, world))
        M = n // world
        Q = M // world
        seen, samp_ok = 0, True
        for i, v in sampled.items():  # X[i] with i = g Q + q + M k1 sits at k1 Q + q on rank g
            k1, rem = divmod(i, M)
            g, qq = divmod(rem, Q)
            if g == rank:
                seen += 1
                samp_ok = samp_ok and int(out[k1 * Q + qq]) == v
        ctx.dist_ntt(loc, inverse=True)
        inv_ok = np.array_equal(loc.cpu().numpy().view(np.uint64), x[rank::world])
        ctx.close()
        q.put((rank, full_ok, samp_ok, inv_ok, seen))
    except Exception as e:
        q.put((rank, f"ERR {type(e).__name__}: {e}", False, False, 0))
    finally:
        dist.destroy_process_group()


def test_dist_ntt_config4_size_p8(gpu_ok, oracle, tmp_path):
    """BASELINE config 4's shape: 2^26 points over P = 8 ranks, every output
    compared with the oracle (OpenMP build, same restated ntt.rs:79-111)."""
    import torch.multiprocessing as mp
    log_n, seed = 26, 2024
    x = oracle.det_vec(1 << log_n, seed)
    oracle.use_mt(int(os.environ.get("OMP_NUM_THREADS", "8")))
    want_path = str(tmp_path / "ntt_2e26.npy")
    np.save(want_path, oracle.ntt_forward(x))
    del x
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_full, args=(r, 8, port, log_n, seed, want_path, q)) for r in range(8)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=600) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert sum(r[4] for r in res) == 256  # every sampled frequency was owned by exactly one rank
    for rank, full_ok, samp_ok, inv_ok, _ in res:
        assert full_ok is True, f"rank {rank}: {full_ok}"
        assert samp_ok, f"rank {rank}: sampled frequencies differ"
        assert inv_ok, f"rank {rank}: inverse did not round-trip"


@pytest.mark.parametrize("world,log_n,seed", [(2, 9, 1), (2, 16, 2), (4, 10, 3), (4, 20, 4), (8, 14, 5)])
def test_dist_ntt_matches_oracle(gpu_ok, world, log_n, seed):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, log_n, seed, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=600) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for rank, fwd_ok, inv_ok, calls in res:
        assert fwd_ok is True, f"rank {rank}: {fwd_ok}"
        assert inv_ok, f"rank {rank}: inverse did not round-trip"
        assert calls["alltoall"] == 2  # one transpose per direction


@pytest.mark.parametrize("log_n", [8, 12, 18, 20, 22, 25])
def test_dist_ntt_one_rank_is_plain_ntt(gpu_ok, product, oracle, log_n):
    """One rank: DIF forward + in-place bit reversal, and the inverse through
    the DIT passes (12, 18, 20 and 25 take the in-tile radix-16 pass)."""
    torch = gpu_ok
    if log_n >= 24:
        oracle.use_mt(int(os.environ.get("OMP_NUM_THREADS", "8")))
    x = oracle.det_vec(1 << log_n, 40 + log_n)
    ctx = product.ProverContext(0)
    d = torch.from_numpy(x.view(np.int64).copy()).cuda()
    ctx.dist_ntt(d)
    np.testing.assert_array_equal(d.cpu().numpy().view(np.uint64), oracle.ntt_forward(x))
    ctx.dist_ntt(d, inverse=True)
    np.testing.assert_array_equal(d.cpu().numpy().view(np.uint64), x)
    ctx.close()


def test_dist_ntt_rejects_bad_sizes(gpu_ok, product):
    import ctypes as C
    import sezkp_amd._lib as L
    torch = gpu_ok
    ctx = product.ProverContext(0)
    d = torch.zeros(128, dtype=torch.int64, device="cuda")
    err = C.create_string_buffer(256)
    assert L.lib.sezkp_ctx_dist_ntt(ctx._h, d.data_ptr(), d.data_ptr(), 7, 1, err, 256) == L.SEZKP_E_INVALID
    assert b"2^(8 + log P)" in err.value
    assert L.lib.sezkp_ctx_dist_ntt(ctx._h, d.data_ptr(), d.data_ptr(), 8, 0, err, 256) == L.SEZKP_E_INVALID
    ctx.close()

"""GPU parity of the sharded (one proof over P GPUs) prover, SURVEY 8(e).

The box has one GPU, so P ranks share it and exchange through
`HostCollectives` (gloo, host-staged) instead of RCCL; the data path,
layouts and kernels are the production ones. Every rank must return the
oracle's proof bytes.
"""
import hashlib
import os
import sys

import pytest

from conftest import ORACLE, PKG, free_port, insert_zero_step_blocks

pytestmark = pytest.mark.gpu


def _port():
    return free_port()


def _worker(rank, world, port, T, b, tau, seed, q, zero_at=None):
    sys.path[:0] = [PKG, ORACLE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sezkp_amd
        blocks = sezkp_amd.synthetic_blocks(T, b, tau, seed)
        if zero_at:
            blocks = insert_zero_step_blocks(blocks, zero_at)
        ctx = sezkp_amd.ShardedProverContext(rank, world, device=0, comm="host")
        ctx.upload(blocks)
        root = blocks.manifest_root()
        p1 = ctx.prove(root).proof_bytes
        p2 = ctx.prove(root).proof_bytes
        calls = dict(ctx._coll.calls)
        calls["stats"] = ctx.comm_stats()
        ctx.close()
        q.put((rank, hashlib.sha256(p1).hexdigest(), p1 == p2, calls))
    except Exception as e:
        q.put((rank, f"ERR {type(e).__name__}: {e}", False, {}))
    finally:
        dist.destroy_process_group()


def _run(world, T, b, tau, seed, zero_at=None):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, T, b, tau, seed, q, zero_at)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=600) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("world,T,b,tau,seed", [
    (2, 1 << 13, 512, 2, 42),   # smallest legal shard (n = 4096 P)
    (4, 1 << 14, 512, 3, 7),
    (2, 1 << 15, 100, 8, 9),    # ragged blocks crossing rank boundaries, tau = 8
])
def test_sharded_proof_matches_oracle(gpu_ok, product, oracle, world, T, b, tau, seed):
    blocks = product.synthetic_blocks(T, b, tau, seed)
    want = hashlib.sha256(oracle.prove_v1(blocks, blocks.manifest_root())).hexdigest()
    res = _run(world, T, b, tau, seed)
    for rank, digest, repeat_ok, calls in res:
        assert digest == want, f"rank {rank}: {digest}"
        assert repeat_ok
        # per prove: one all-to-all (the LDE's; none at P = 2, where every
        # rank computes the whole LDE), one byte-sum (proof body), allgathers
        # (the replicated INTT's values ride in one of them)
        a2a = 0 if world == 2 else 1
        assert calls["alltoall"] == 2 * a2a and calls["allreduce"] == 2 and calls["allgather"] > 0
        # sezkp_ctx_comm_stats: one entry per collective of the last prove
        st = {c["name"]: c for c in calls["stats"]}
        assert {"col_chunk_roots", "d_values", "layer0_run_roots", "fri_rep_values", "fri_run_roots",
                "proof_allreduce"} | ({"lde_alltoall"} if a2a else set()) == set(st), sorted(st)
        assert all(c["bytes"] > 0 and c["ms"] >= 0 for c in calls["stats"])


def test_sharded_zero_step_blocks_match_oracle(gpu_ok, product, oracle):
    """Zero-step blocks at rank boundaries of a P = 4 sharded proof (the
    blocks a rank reads are found from step_start, where they repeat a
    boundary): every rank returns the oracle's bytes."""
    T, b, tau, seed = 1 << 14, 512, 3, 7
    at = [0, 8, 8, 16, 24, 32]  # 4096-row shards start at blocks 8, 16, 24
    blocks = insert_zero_step_blocks(product.synthetic_blocks(T, b, tau, seed), at)
    want = hashlib.sha256(oracle.prove_v1(blocks, blocks.manifest_root())).hexdigest()
    for rank, digest, repeat_ok, _ in _run(4, T, b, tau, seed, at):
        assert digest == want and repeat_ok, f"rank {rank}: {digest}"


@pytest.mark.parametrize("T,tau,seed", [(1 << 22, 8, 5), (1 << 21, 2, 6)])
def test_sharded_config5_size_p8_matches_openmp_oracle(gpu_ok, product, T, tau, seed):
    """BASELINE config 5's shape: T = 2^22 (N = 2^25), tau = 8, over P = 8
    ranks (here sharing one GPU through host collectives); and the headline's
    N = 2^24 over P = 8 (M = 2^21 LDE points per rank: the 2048-leaf tree
    workgroups). Every rank returns the bytes of the OpenMP oracle, run in a
    child process on 16 threads."""
    import subprocess
    from conftest import ROOT
    b = 512
    code = ("import sys; sys.path[:0]=[%r,%r]\n"
            "import hashlib, oracle_ctypes as O, sezkp_amd as S\n"
            "O.use_mt(16)\n"
            "bl=S.synthetic_blocks(%d,%d,%d,%d); print(hashlib.sha256(O.prove_v1(bl, bl.manifest_root())).hexdigest())\n"
            % (PKG, os.path.join(ROOT, "oracle"), T, b, tau, seed))
    child = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    res = _run(8, T, b, tau, seed)
    out, err = child.communicate(timeout=300)
    assert child.returncode == 0, err[-1500:]
    for rank, digest, repeat_ok, calls in res:
        assert digest == out.strip(), f"rank {rank}: {digest}"
        assert repeat_ok


def test_sharded_per_point_deep_matches_oracle(gpu_ok, product, oracle, monkeypatch):
    """SEZKP_NO_DEEP_POLY=1: the sharded ranks divide every coset point by
    (x_i - z) in the last LDE pass instead of folding the DEEP polynomial
    (the default); same bytes either way."""
    monkeypatch.setenv("SEZKP_NO_DEEP_POLY", "1")
    T, b, tau, seed = 1 << 13, 512, 2, 5
    blocks = product.synthetic_blocks(T, b, tau, seed)
    want = hashlib.sha256(oracle.prove_v1(blocks, blocks.manifest_root())).hexdigest()
    for rank, digest, repeat_ok, _ in _run(2, T, b, tau, seed):
        assert digest == want, f"rank {rank}: {digest}"
        assert repeat_ok


@pytest.mark.parametrize("no_deep_poly", [False, True])
@pytest.mark.parametrize("world,T,b,tau,seed", [(4, 1 << 14, 512, 3, 11), (2, 1 << 15, 100, 8, 9),
                                                (8, 1 << 16, 333, 2, 13)])
def test_sharded_distributed_intt_matches_oracle(gpu_ok, product, oracle, monkeypatch, no_deep_poly, world, T, b,
                                                 tau, seed):
    """SEZKP_DIST_INTT=1: the distributed INTT (two all-to-alls, P-point DFTs,
    a local n/P-point INTT, the coefficient allgather) instead of the default
    replicated n-point INTT on every rank; same bytes, three all-to-alls per
    prove (two of them the INTT's)."""
    monkeypatch.setenv("SEZKP_DIST_INTT", "1")
    if no_deep_poly:
        monkeypatch.setenv("SEZKP_NO_DEEP_POLY", "1")
    blocks = product.synthetic_blocks(T, b, tau, seed)
    want = hashlib.sha256(oracle.prove_v1(blocks, blocks.manifest_root())).hexdigest()
    for rank, digest, repeat_ok, calls in _run(world, T, b, tau, seed):
        assert digest == want, f"rank {rank}: {digest}"
        assert repeat_ok
        assert calls["alltoall"] == (4 if world == 2 else 6)
        st = {c["name"] for c in calls["stats"]}
        assert {"intt_alltoall1", "intt_alltoall2", "intt_coeffs"} <= st, sorted(st)


def test_sharded_context_world1_is_single_gpu(gpu_ok, product, oracle):
    blocks = product.synthetic_blocks(1 << 12, 512, 2, 3)
    root = blocks.manifest_root()
    ctx = product.ShardedProverContext(0, 1, device=0, comm="rccl")
    ctx.upload(blocks)
    assert ctx.prove(root).proof_bytes == oracle.prove_v1(blocks, root)
    ctx.close()


def test_sharded_rejects_small_trace(gpu_ok, product):
    from sezkp_amd.dist import HostCollectives
    import sezkp_amd._lib as L
    import ctypes as C
    hc = HostCollectives(None).c_struct()  # never called: upload fails first
    err = C.create_string_buffer(1024)
    h = L.lib.sezkp_ctx_create_sharded_host(0, 0, 2, C.byref(hc), err, 1024)
    assert h
    blocks = product.synthetic_blocks(1 << 12, 512, 2, 3)  # n = 4096 < 4096 * 2
    rc = L.lib.sezkp_ctx_upload(h, C.byref(blocks.view()), err, 1024)
    L.lib.sezkp_ctx_destroy(h)
    assert rc == L.SEZKP_E_INVALID and b"n >= 4096 * P" in err.value
    assert not L.lib.sezkp_ctx_create_sharded_host(0, 0, 3, C.byref(hc), err, 1024)  # world not a power of two


@pytest.mark.parametrize("T,b,tau", [(1 << 12, 512, 2), (1 << 15, 200, 8)])
def test_sharded_algorithm_over_rccl_one_rank(gpu_ok, product, oracle, monkeypatch, T, b, tau):
    """SEZKP_FORCE_SHARDED runs the sharded algorithm with a one-rank RCCL
    communicator: every RCCL call (allgather, all-to-all, allreduce) and the
    run/cap layouts execute on the device, bit-exact with the oracle."""
    monkeypatch.setenv("SEZKP_FORCE_SHARDED", "1")
    blocks = product.synthetic_blocks(T, b, tau, 11)
    root = blocks.manifest_root()
    ctx = product.ShardedProverContext(0, 1, device=0, comm="rccl")
    ctx.upload(blocks)
    assert ctx.prove(root).proof_bytes == oracle.prove_v1(blocks, root)
    ctx.close()


@pytest.mark.parametrize("gpus,stream", [(2, False), (1, True)])
def test_launcher_jsonl_artifact_matches_oracle(gpu_ok, product, oracle, tmp_path, gpus, stream):
    """Config 5 path: blocks.jsonl -> `python -m sezkp_amd.launch prove` (manifest
    precheck, one proof over `gpus` ranks) -> CBOR artifact == the oracle's."""
    import subprocess
    import cbor_min
    T, tau = 1 << 13, 2
    blocks = product.synthetic_blocks(T, 512, tau, 21)
    root = blocks.manifest_root()
    (tmp_path / "b.jsonl").write_bytes(blocks.to_jsonl())
    (tmp_path / "m.cbor").write_bytes(cbor_min.dumps({"root": list(root), "n_leaves": int(blocks.block_id.size)}))
    cmd = [sys.executable, "-m", "sezkp_amd.launch", "prove", "--blocks", str(tmp_path / "b.jsonl"),
           "--manifest", str(tmp_path / "m.cbor"), "--out", str(tmp_path / "p.cbor"), "--gpus", str(gpus),
           "--comm", "host" if gpus > 1 else "rccl"] + (["--stream"] if stream else [])
    r = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    meta = {"proto": "stark-v1", "domain_n": 8 * T, "tau": tau}
    if stream:
        meta["mode"] = "streaming"
    want = cbor_min.proof_artifact_cbor("stark", root, oracle.prove_v1(blocks, root), meta)
    assert (tmp_path / "p.cbor").read_bytes() == want
    # a manifest that does not match the blocks is refused before proving
    (tmp_path / "bad.cbor").write_bytes(cbor_min.dumps({"root": [0] * 32, "n_leaves": 1}))
    bad = cmd[:]
    bad[bad.index(str(tmp_path / "m.cbor"))] = str(tmp_path / "bad.cbor")
    r = subprocess.run(bad, cwd=PKG, capture_output=True, text=True, timeout=600)
    assert r.returncode == 1 and "root mismatch" in r.stderr


def _trip_worker(rank, world, port, q):
    sys.path[:0] = [PKG, ORACLE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SEZKP_DEBUG_TRIP_GUARD="1")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sezkp_amd
        blocks = sezkp_amd.synthetic_blocks(1 << 13, 512, 2, 42)
        ctx = sezkp_amd.ShardedProverContext(rank, world, device=0, comm="host")
        ctx.upload(blocks)
        try:
            ctx.prove(blocks.manifest_root())
            q.put((rank, "no error"))
        except Exception as e:
            q.put((rank, str(e)))
        ctx.close()
    finally:
        dist.destroy_process_group()


def test_sharded_guard_trip_fails_every_rank(gpu_ok):
    """A guard trip on ONE rank (test hook) must fail every rank at the same
    point, so no rank blocks in a collective its peers never reach."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_trip_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for rank, msg in res:
        assert "guard tripped on rank 1" in msg, (rank, msg)


def _fail_worker(rank, world, port, point, q):
    """Rank 1 fails right before collective `point` (test hook); gloo's own
    timeout (20 s) bounds the wait of the rank left inside the collective."""
    import datetime
    import time
    sys.path[:0] = [PKG, ORACLE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SEZKP_DEBUG_FAIL_AT=f"1:{point}")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=20))
    res = [rank]
    try:
        import sezkp_amd
        blocks = sezkp_amd.synthetic_blocks(1 << 13, 512, 2, 42)
        ctx = sezkp_amd.ShardedProverContext(rank, world, device=0, comm="host")
        ctx.upload(blocks)
        t0 = time.monotonic()
        try:
            ctx.prove(blocks.manifest_root())
            res += ["no error", 0.0]
        except Exception as e:
            res += [str(e), time.monotonic() - t0]
        try:  # the context is unusable afterwards
            ctx.prove(blocks.manifest_root())
            res.append("no error")
        except Exception as e:
            res.append(str(e))
        ctx.close()
    except Exception as e:
        res += [f"setup: {e}", 0.0, ""]
    q.put(tuple(res))
    q.close()
    q.join_thread()  # the result must reach the parent before the hard exit below
    os._exit(0)  # gloo may hold a timed-out collective: leave without a teardown handshake


@pytest.mark.parametrize("point", ["d_values", "fri_run_roots", "proof_allreduce"])
def test_sharded_failure_on_one_rank_fails_every_rank(gpu_ok, point):
    """A rank that fails after the first collective of a prove (injected right
    before a later collective) must not leave its peers blocked: every rank
    returns an error within the collective deadline, and both contexts refuse
    further proofs (the communicator is aborted)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_fail_worker, args=(r, 2, port, point, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=150) for _ in ps)
    for p in ps:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert f"injected failure before collective {point} on rank 1" in res[1][1], res[1]
    assert res[0][1] != "no error" and res[0][2] < 60, res[0]
    for r in res:
        assert "context unusable" in r[3], r


def test_sharded_rccl_abort_after_failure(gpu_ok, product):
    """One-rank RCCL communicator (SEZKP_FORCE_SHARDED): a failure injected
    before the LDE all-to-all aborts the communicator (ncclCommAbort); the
    error comes back, later proofs are refused, and destroy does not hang. In
    a child process (the switches are read once per process)."""
    import subprocess
    code = ("import sys; sys.path[:0]=[%r]\n"
            "import sezkp_amd as S\n"
            "bl=S.synthetic_blocks(1<<12,512,2,3); c=S.ShardedProverContext(0,1,device=0,comm='rccl'); c.upload(bl)\n"
            "for i in range(2):\n"
            "    try:\n"
            "        c.prove(bl.manifest_root()); print('no error')\n"
            "    except Exception as e:\n"
            "        print('ERR', e)\n"
            "c.close(); print('closed')\n" % PKG)
    env = dict(os.environ, SEZKP_FORCE_SHARDED="1", SEZKP_DEBUG_FAIL_AT="0:lde_alltoall")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-1500:]
    # RCCL prints a banner on stdout: keep the script's own lines
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.startswith(("ERR", "no error", "closed"))]
    assert "injected failure before collective lde_alltoall on rank 0" in lines[0], lines
    assert "context unusable" in lines[1], lines
    assert lines[2] == "closed"


def _stall_worker(rank, world, port, q):
    """Rank 1's stream is held after the proof's last collective (test hook):
    its wait must give up at SEZKP_COLL_TIMEOUT_S through the transport-
    agnostic deadline of Comm::wait, and destroy must not hang."""
    import datetime
    import time
    sys.path[:0] = [PKG, ORACLE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      SEZKP_DEBUG_STALL_AFTER="1:proof_allreduce", SEZKP_COLL_TIMEOUT_S="3")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=20))
    res = [rank]
    try:
        import sezkp_amd
        blocks = sezkp_amd.synthetic_blocks(1 << 13, 512, 2, 42)
        ctx = sezkp_amd.ShardedProverContext(rank, world, device=0, comm="host")
        ctx.upload(blocks)
        t0 = time.monotonic()
        try:
            ctx.prove(blocks.manifest_root())
            res += ["no error", time.monotonic() - t0]
        except Exception as e:
            res += [str(e), time.monotonic() - t0]
        if rank == 1:
            try:
                ctx.prove(blocks.manifest_root())
                res.append("no error")
            except Exception as e:
                res.append(str(e))
        else:
            res.append("")
        t1 = time.monotonic()
        ctx.close()
        res.append(time.monotonic() - t1)
    except Exception as e:
        res += [f"setup: {e}", 0.0, "", 0.0]
    q.put(tuple(res))
    q.close()
    q.join_thread()
    os._exit(0)


def test_sharded_stalled_stream_hits_the_deadline(gpu_ok):
    """the collective deadline (poll + timeout + abort) used to
    live in the RCCL transport only and never ran with a stuck peer. Rank 1's
    stream now stalls after its last collective: rank 1 returns the timeout
    error within the 3 s deadline (+ margin), refuses later proofs, and its
    context is destroyed without hanging; rank 0 is unaffected."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_stall_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=150) for _ in ps)
    for p in ps:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert res[0][1] == "no error", res[0]
    assert "collective timeout" in res[1][1] and 2.5 < res[1][2] < 20, res[1]
    assert "context unusable" in res[1][3], res[1]
    assert res[1][4] < 20, res[1]


def test_sharded_rccl_stalled_stream_aborts(gpu_ok):
    """The same deadline on a one-rank RCCL communicator: the wait times out,
    the communicator is aborted (ncclCommAbort), the stalled stream is released
    at destroy, and destroy returns (in a child: the switches are read once)."""
    import subprocess
    code = ("import sys, time; sys.path[:0]=[%r]\n"
            "import sezkp_amd as S\n"
            "bl=S.synthetic_blocks(1<<12,512,2,3); c=S.ShardedProverContext(0,1,device=0,comm='rccl'); c.upload(bl)\n"
            "t0=time.monotonic()\n"
            "try:\n"
            "    c.prove(bl.manifest_root()); print('no error')\n"
            "except Exception as e:\n"
            "    print('ERR', e)\n"
            "print('T %%.2f' %% (time.monotonic()-t0))\n"
            "c.close(); print('closed')\n" % PKG)
    env = dict(os.environ, SEZKP_FORCE_SHARDED="1", SEZKP_DEBUG_STALL_AFTER="0:proof_allreduce",
               SEZKP_COLL_TIMEOUT_S="3")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-1500:]
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.startswith(("ERR", "no error", "closed", "T "))]
    assert "collective timeout" in lines[0], lines
    assert 2.5 < float(lines[1].split()[1]) < 20, lines
    assert lines[2] == "closed", lines


def _sliced_worker(rank, world, port, path, q):
    sys.path[:0] = [PKG, ORACLE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sezkp_amd
        from sezkp_amd.ingest import TorchComm, sliced_ingest
        ing = sliced_ingest(path, rank, world, TorchComm(), None)
        ctx = sezkp_amd.ShardedProverContext(rank, world, device=0, comm="host")
        ctx.upload_rows(ing["blocks"], ing["row0"], ing["nrows"])
        p = ctx.prove(ing["root"]).proof_bytes
        ctx.close()
        q.put((rank, hashlib.sha256(p).hexdigest(), ing["row0"], ing["nrows"]))
    except Exception as e:
        q.put((rank, f"ERR {type(e).__name__}: {e}", 0, 0))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,tau,zero", [(2, 3, False), (4, 3, False), (8, 3, False), (2, 8, False), (8, 8, False),
                                            (4, 3, True)])
def test_sharded_sliced_upload_matches_full(gpu_ok, product, oracle, tmp_path, world, tau, zero):
    """each rank ingests only its slice of a JSONL file (the
    metadata of 1/P of the lines, then the lines over its own rows plus the
    halo) and uploads it with sezkp_ctx_upload_rows. Ragged 333-step blocks
    cross every rank boundary. Every rank's proof equals the oracle's proof of
    the whole trace (bound to the file's Frontier root), and no rank holds
    the whole trace (row slices of about n / P). tau = 8 takes the 8-tape
    transposition kernel with slice starts that are not multiples of 8
    (ADVICE r04). zero: zero-step blocks (step_hi = step_lo - 1) in the
    file, some where the ranks' byte slices and row slices begin."""
    T, b, seed = 1 << 15, 333, 17
    blocks = product.synthetic_blocks(T, b, tau, seed)
    if zero:
        blocks = insert_zero_step_blocks(blocks, [0, 25, 25, 49, 50, 74, blocks.n_blocks])
    path = tmp_path / "b.jsonl"
    path.write_bytes(blocks.to_jsonl())
    root = blocks.manifest_frontier_root()
    want = hashlib.sha256(oracle.prove_v1(blocks, root)).hexdigest()
    port = free_port()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_sliced_worker, args=(r, world, port, str(path), q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=600) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for rank, digest, row0, nrows in res:
        assert digest == want, f"rank {rank}: {digest}"
        assert nrows < T // world + 2 * b + 2, (rank, row0, nrows)
    # a slice that misses rows the context reads is refused
    full = product.BlockSoA.from_jsonl(path.read_bytes())
    c = product.ProverContext(0)
    with pytest.raises(product.SezkpError, match="needs rows"):
        c.upload_rows(full.with_steps(product.BlockSoA.from_jsonl_range(path.read_bytes(), 0, 0)), 0, 0)
    c.close()


def test_config5_cli_jsonl_launcher_p8_matches_openmp_oracle(gpu_ok, product, tmp_path):
    """BASELINE config 5 end to end at full size: the
    CLI writes T = 2^22, tau = 8 blocks (`simulate`, the reference generator),
    `export-jsonl` turns them into blocks.jsonl (829 MB), `commit` writes the
    manifest (Frontier root), and `python -m sezkp_amd.launch prove --gpus 8
    --comm host` proves from the JSONL file in per-rank slices (8 ranks sharing
    this GPU through host collectives). The artifact equals the one built from
    the OpenMP oracle's proof of the same blocks, and the JSONL decodes back to
    CBOR blocks byte-identical to the CLI's blocks.cbor."""
    import subprocess
    import cbor_min
    from conftest import ROOT
    cli = os.path.join(PKG, "bin", "sezkp-cli")
    T, b, tau = 1 << 22, 512, 8
    cb, jl, man, out = (tmp_path / n for n in ("blocks.cbor", "blocks.jsonl", "manifest.cbor", "proof.cbor"))
    for args in (["simulate", "--t", str(T), "--b", str(b), "--tau", str(tau), "--out-blocks", str(cb)],
                 ["export-jsonl", "--input", str(cb), "--output", str(jl)],
                 ["commit", "--blocks", str(jl), "--out", str(man)]):
        r = subprocess.run([cli] + args, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, (args[0], r.stderr[-1500:])
    assert product.BlockSoA.from_jsonl(jl.read_bytes()).to_cbor() == cb.read_bytes()
    code = ("import sys, hashlib; sys.path[:0]=[%r,%r]\n"
            "import oracle_ctypes as O, sezkp_amd as S\n"
            "O.use_mt(16)\n"
            "bl=S.BlockSoA.from_cbor(open(%r,'rb').read()); r=bl.manifest_frontier_root()\n"
            "sys.stdout.write(r.hex()+' '+O.prove_v1(bl, r).hex())\n" % (PKG, os.path.join(ROOT, "oracle"), str(cb)))
    child = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    cmd = [sys.executable, "-u", "-m", "sezkp_amd.launch", "prove", "--blocks", str(jl), "--manifest", str(man),
           "--out", str(out), "--gpus", "8", "--comm", "host"]
    r = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    o_out, o_err = child.communicate(timeout=600)
    assert child.returncode == 0, o_err[-1500:]
    root_hex, proof_hex = o_out.split()
    root = bytes.fromhex(root_hex)
    want = cbor_min.proof_artifact_cbor("stark", root, bytes.fromhex(proof_hex),
                                        {"proto": "stark-v1", "domain_n": 8 * T, "tau": tau})
    assert out.read_bytes() == want

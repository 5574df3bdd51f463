"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle.

Bit-exact equality is required everywhere (Goldilocks integer arithmetic and
BLAKE3 bytes; there is no floating point on this path). Sizes are chosen so
the single-threaded oracle finishes in seconds, plus one T=2^18 full prove
(BASELINE config 3's size) and the 2^20 NTT round trip (config 2).
"""
import ctypes as C
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PKG, ROOT

pytestmark = pytest.mark.gpu
P = 0xFFFFFFFF00000001
FIXTURES = {
    "root_blocks": ("tests/golden/ref_blocks.cbor", "tests/golden/ref_manifest.cbor"),
    "minimal_riscv": ("tests/golden/riscv_blocks.cbor", "tests/golden/riscv_manifest.cbor"),
}


def _dev(torch, arr: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(arr).view(np.int64)).cuda()


def _host(t) -> np.ndarray:
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("log_n", list(range(1, 21)))
def test_ntt_roundtrip_matches_oracle(gpu_ok, product, oracle, log_n):
    """ntt_roundtrip.rs:29-81 + exact forward values vs sezkp-ffts (config 2 at
    2^20). 2^10..2^12 and 2^17..2^20 run the in-tile radix-16 (X16) pass."""
    torch = gpu_ok
    n = 1 << log_n
    x = oracle.det_vec(n, 2024)
    d = _dev(torch, x)
    scratch = torch.empty_like(d)
    assert product.lib.sezkp_gl_ntt(d.data_ptr(), scratch.data_ptr(), log_n, 1, None) == 0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(d), oracle.ntt_forward(x))
    assert product.lib.sezkp_gl_ntt(d.data_ptr(), scratch.data_ptr(), log_n, -1, None) == 0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(d), x)


@pytest.mark.parametrize("log_n", [21, 22, 23, 24, 25, 26])
def test_ntt_large_matches_openmp_oracle(gpu_ok, product, oracle, log_n):
    """The headline LDE size (2^24) and config 4's 2^26 on one device: every
    output of sezkp_gl_ntt against the OpenMP oracle (ntt.rs:79-155), and the
    inverse round trip."""
    torch = gpu_ok
    oracle.use_mt(int(os.environ.get("OMP_NUM_THREADS", "8")))
    x = oracle.det_vec(1 << log_n, 2024 + log_n)
    d = _dev(torch, x)
    scratch = torch.empty_like(d)
    assert product.lib.sezkp_gl_ntt(d.data_ptr(), scratch.data_ptr(), log_n, 1, None) == 0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(d), oracle.ntt_forward(x))
    assert product.lib.sezkp_gl_ntt(d.data_ptr(), scratch.data_ptr(), log_n, -1, None) == 0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(d), x)


@pytest.mark.parametrize("log_n", [4, 11, 12, 16, 20, 21, 24])
def test_ntt_edge_values_match_oracle(gpu_ok, product, oracle, log_n):
    """Canonical values at the carry / borrow boundaries of the 32-bit-lane
    Goldilocks arithmetic (0, 1, p - 1, p - 2, eps = 2^32 - 1, 2^32, 2^63,
    p - eps, ...), drawn at random and as constant runs of p - 1, through
    every pass form (plain, X16, the 2^20 radix-8 passes, the natural-order
    DIT, the headline 2^24): forward values against the oracle, then the
    inverse round trip."""
    torch = gpu_ok
    if log_n > 20:
        oracle.use_mt(int(os.environ.get("OMP_NUM_THREADS", "8")))
    n = 1 << log_n
    eps = (1 << 32) - 1
    edge = np.array([0, 1, 2, P - 1, P - 2, eps, eps + 1, eps - 1, 1 << 32, (1 << 32) + 1, 1 << 63, (1 << 63) - 1,
                     P - eps, P - eps - 1, P - (1 << 32), (1 << 64) - (1 << 33), P >> 1, (P >> 1) + 1], dtype=np.uint64)
    rng = np.random.default_rng(log_n)
    x = edge[rng.integers(0, len(edge), n)]
    x[: n // 4] = P - 1
    d = _dev(torch, x)
    scratch = torch.empty_like(d)
    assert product.lib.sezkp_gl_ntt(d.data_ptr(), scratch.data_ptr(), log_n, 1, None) == 0
    torch.cuda.synchronize()
    got = _host(d)
    assert (got < P).all()
    np.testing.assert_array_equal(got, oracle.ntt_forward(x))
    assert product.lib.sezkp_gl_ntt(d.data_ptr(), scratch.data_ptr(), log_n, -1, None) == 0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(d), x)


@pytest.mark.parametrize("vec", ["zeros", "delta", "ap"])
def test_ntt_special_vectors(gpu_ok, product, oracle, vec):
    torch = gpu_ok
    for log_n in (1, 5, 10):
        n = 1 << log_n
        x = {"zeros": np.zeros(n, np.uint64), "delta": np.eye(1, n, dtype=np.uint64)[0],
             "ap": np.arange(n, dtype=np.uint64)}[vec]
        d = _dev(torch, x)
        s = torch.empty_like(d)
        product.lib.sezkp_gl_ntt(d.data_ptr(), s.data_ptr(), log_n, 1, None)
        product.lib.sezkp_gl_ntt(d.data_ptr(), s.data_ptr(), log_n, -1, None)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_host(d), x)


@pytest.mark.parametrize("log_n", [0, 1, 2, 3, 5, 8, 11, 13])
def test_coset_lde_deep_matches_oracle(gpu_ok, product, oracle, log_n):
    """lde.rs:42-97: INTT -> coset(3) NTT x8 -> DEEP divide."""
    torch = gpu_ok
    n = 1 << log_n
    base = oracle.det_vec(n, 7 + log_n)
    z = 0x1234567890ABCDEF % P
    want = oracle.lde_deep(base, 3, z)
    d_in = _dev(torch, base)
    d_out = torch.empty(8 * n, dtype=torch.int64, device="cuda")
    assert product.lib.sezkp_gl_coset_lde_deep(d_in.data_ptr(), log_n, 3, 3, z, d_out.data_ptr(), None, None) == 0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(d_out), want)


@pytest.mark.parametrize("log_n", [5, 13, 18])
def test_coset_lde_deep_edge_values(gpu_ok, product, oracle, log_n):
    """The LDE + DEEP path on trace values at the carry / borrow boundaries
    (p - 1 runs, eps, 2^63, ...) and z = p - 1: every output against the oracle."""
    torch = gpu_ok
    n = 1 << log_n
    eps = (1 << 32) - 1
    edge = np.array([0, 1, P - 1, P - 2, eps, 1 << 32, 1 << 63, P - eps, (1 << 64) - (1 << 33)], dtype=np.uint64)
    base = edge[np.random.default_rng(log_n).integers(0, len(edge), n)]
    base[: n // 2] = P - 1
    z = P - 1
    want = oracle.lde_deep(base, 3, z)
    d_in = _dev(torch, base)
    d_out = torch.empty(8 * n, dtype=torch.int64, device="cuda")
    assert product.lib.sezkp_gl_coset_lde_deep(d_in.data_ptr(), log_n, 3, 3, z, d_out.data_ptr(), None, None) == 0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(d_out), want)


@pytest.mark.parametrize("log_n", [0, 1, 2, 3, 6, 7, 10, 11, 15])
def test_merkle_root_matches_oracle(gpu_ok, product, oracle, log_n):
    """hash_field_leaves + MerkleTree::from_leaves (merkle.rs:46-71,150-160)."""
    torch = gpu_ok
    n = 1 << log_n
    vals = oracle.det_vec(n, 99)
    leaves = b"".join(oracle.hash_leaf_u64(int(v)) for v in vals)
    d = _dev(torch, vals)
    root = C.create_string_buffer(32)
    assert product.lib.sezkp_merkle_root_u64(d.data_ptr(), n, root, None) == 0
    assert root.raw == oracle.merkle_root(leaves)


@pytest.mark.parametrize("log_out", [0, 1, 4, 10, 12])
def test_fri_fold_commit_matches_oracle(gpu_ok, product, oracle, log_out):
    """fold y'_i = y_i + beta*y_{i+h} (prover.rs:208-230) + its layer root."""
    torch = gpu_ok
    n = 1 << log_out
    vals = oracle.det_vec(2 * n, 5)
    beta = 0xDEADBEEFCAFEF00D % P
    want = np.array([(int(vals[i]) + beta * int(vals[i + n])) % P for i in range(n)], dtype=np.uint64)
    d_in = _dev(torch, vals)
    d_out = torch.empty(n, dtype=torch.int64, device="cuda")
    root = C.create_string_buffer(32)
    assert product.lib.sezkp_fri_fold_commit(d_in.data_ptr(), n, beta, d_out.data_ptr(), root, None) == 0
    np.testing.assert_array_equal(_host(d_out), want)
    assert root.raw == oracle.merkle_root(b"".join(oracle.hash_leaf_u64(int(v)) for v in want))


# ------------------------------------------------------------- full prove
def _fixture(name):
    import cbor_min
    b, m = FIXTURES[name]
    raw = open(os.path.join(ROOT, b), "rb").read()
    man = cbor_min.loads(open(os.path.join(ROOT, m), "rb").read())
    return raw, bytes(man["root"])


@pytest.mark.parametrize("name", sorted(FIXTURES))
def test_prove_reference_fixtures_bit_exact(gpu_ok, product, oracle, name):
    """The reference's own committed block files: GPU proof == oracle proof ==
    committed golden digest (tests/golden/v1_proofs.json)."""
    raw, mroot = _fixture(name)
    blocks = product.BlockSoA.from_cbor(raw)
    art = product.StarkV1.prove(blocks, mroot)
    want = oracle.prove_v1(blocks, mroot)
    assert art.proof_bytes == want
    gold = json.load(open(os.path.join(GOLDEN, "v1_proofs.json")))[name]
    assert hashlib.sha256(art.proof_bytes).hexdigest() == gold["proof_sha256"]
    assert art.meta == {"proto": "stark-v1", "domain_n": 8 * blocks.n_rows, "tau": blocks.tau}


CASES = [  # (T, b, tau, seed)
    (4096, 512, 8, 42),     # config 1 shape (CLI plumbing case)
    (1024, 64, 2, 1),
    (2048, 100, 3, 2),      # ragged last block
    (256, 1, 1, 3),         # one-row blocks (first == last)
    (8, 8, 2, 4),           # n < 1024: single short column chunk
    (2, 2, 1, 5),
    (1, 1, 1, 6),           # n = 1 -> N = 8
    (512, 512, 0, 7),       # tau = 0: only the 3 scalar columns
    (1 << 13, 8192, 4, 8),  # one block spanning many column chunks
    (1 << 14, 333, 4, 9),   # block starts inside 4-row head groups (delta-plan fallback)
]


@pytest.mark.parametrize("T,b,tau,seed", CASES)
def test_prove_synthetic_bit_exact(gpu_ok, product, oracle, T, b, tau, seed):
    blocks = product.synthetic_blocks(T, b, tau, seed)
    mroot = blocks.manifest_root()
    assert mroot == oracle.manifest_root(blocks)
    art = product.StarkV1.prove(blocks, mroot)
    assert art.proof_bytes == oracle.prove_v1(blocks, mroot)


def test_prove_wide_values_bit_exact(gpu_ok, product, oracle):
    """Edge values the domain allows: i8 moves outside {-1,0,1}, u16 symbols,
    large/negative windows and offsets (AIR C2 and range terms non-zero)."""
    rng = np.random.default_rng(11)
    T, tau = 1024, 3
    imv = rng.integers(-128, 128, T, dtype=np.int8)
    mv = rng.integers(-128, 128, (T, tau), dtype=np.int8)
    hw = (rng.random((T, tau)) < 0.7).astype(np.uint8)
    ws = (rng.integers(0, 65536, (T, tau)) * hw).astype(np.uint16)
    blocks = product.partition(imv, mv, hw, ws, 128)
    blocks.win_left[:] = rng.integers(-(1 << 40), 1 << 40, blocks.win_left.size)
    blocks.off_out[:] = 0xFFFFFFFF
    mroot = bytes(range(32))
    art = product.StarkV1.prove(blocks, mroot)
    assert art.proof_bytes == oracle.prove_v1(blocks, mroot)


@pytest.mark.parametrize("bad", [0, 5, 65537])
def test_prove_invalid_moves_bit_exact(gpu_ok, product, oracle, bad):
    """`bad` rows move by +-2 (AIR C2: mv^3 - mv != 0 on exactly those rows,
    the rest of the trace valid): the proof still equals the reference's."""
    T, tau = 1 << 17, 1
    imv = np.zeros(T, np.int8)
    mv = np.zeros((T, tau), np.int8)
    mv[:bad, 0] = np.where(np.arange(bad) % 2 == 0, 2, -2)
    hw = np.zeros((T, tau), np.uint8)
    ws = np.zeros((T, tau), np.uint16)
    blocks = product.partition(imv, mv, hw, ws, 4096)
    mroot = blocks.manifest_root()
    assert product.StarkV1.prove(blocks, mroot).proof_bytes == oracle.prove_v1(blocks, mroot)


def test_prove_dictionary_branches_bit_exact(gpu_ok, product, oracle, monkeypatch):
    """Dense columns are committed through range dictionaries whose table level K
    is chosen per column on the device; force every branch at T = 2^17 in one
    block: head of tape 0 drifts by +1 per row (range 2^17 -> K = -1, computed
    leaves), full u16 symbols on tape 0 (R = 65536 -> K = 0), 16 symbols on
    tape 1 (K = 2), {-1,0,1} moves (K = 3), all-zero tape 2 (R = 1 -> K = 4).
    The same bytes must come out with the dictionary path disabled."""
    rng = np.random.default_rng(17)
    T, tau = 1 << 17, 3
    imv = rng.integers(-1, 2, T, dtype=np.int8)
    mv = np.zeros((T, tau), np.int8)
    mv[:, 0] = 1
    mv[:, 1] = rng.integers(-1, 2, T, dtype=np.int8)
    hw = np.zeros((T, tau), np.uint8)
    hw[:, :2] = 1
    ws = np.zeros((T, tau), np.uint16)
    ws[:, 0] = rng.integers(0, 65536, T)
    ws[:, 1] = rng.integers(0, 16, T)
    blocks = product.partition(imv, mv, hw, ws, T)
    mroot = blocks.manifest_root()
    want = oracle.prove_v1(blocks, mroot)
    assert product.StarkV1.prove(blocks, mroot).proof_bytes == want
    # smaller tables above level 0 (lower K per column; the A/B switch)
    for cap in ("16", "4096"):
        monkeypatch.setenv("SEZKP_DICT_TAB_CAP", cap)
        assert product.StarkV1.prove(blocks, mroot).proof_bytes == want
    monkeypatch.delenv("SEZKP_DICT_TAB_CAP")
    monkeypatch.setenv("SEZKP_NO_DICT", "1")
    assert product.StarkV1.prove(blocks, mroot).proof_bytes == want


def test_prove_random_shapes_one_context(gpu_ok, product, oracle):
    """64 seeded random traces through ONE resident context (each upload reuses
    or replaces the previous workspace): T = 2^0..2^14, block length 1..1000,
    tau 0..8, move ranges from {-1,0,1} up to the whole i8 range, write
    probability 0..1, symbols from 1 to 16 bits. Every proof equals the oracle's."""
    rng = np.random.default_rng(2026)
    ctx = product.ProverContext(0)
    for case in range(64):
        T = 1 << int(rng.integers(0, 15))
        tau = int(rng.integers(0, 9))
        b = int(rng.integers(1, 1001))
        mr = int(rng.choice([1, 1, 2, 127]))
        imv = rng.integers(-mr, mr + 1, T, dtype=np.int8)
        mv = rng.integers(-mr, mr + 1, (T, tau), dtype=np.int8)
        hw = (rng.random((T, tau)) < rng.random()).astype(np.uint8)
        ws = (rng.integers(0, 1 << int(rng.integers(1, 17)), (T, tau)) * hw).astype(np.uint16)
        blocks = product.partition(imv, mv, hw, ws, b)
        mroot = rng.bytes(32)
        ctx.upload(blocks)
        got = ctx.prove(mroot).proof_bytes
        assert got == oracle.prove_v1(blocks, mroot), (case, T, b, tau, mr)
    ctx.close()


@pytest.mark.parametrize("rows", ["1", "2"])
def test_compose_rows_per_lane_bit_exact(gpu_ok, product, oracle, monkeypatch, rows):
    """The composition kernel with 1 and 2 (default) rows per lane, on a
    trace with ragged blocks (first/last rows inside a lane's group)."""
    monkeypatch.setenv("SEZKP_COMPOSE_ROWS", rows)
    blocks = product.synthetic_blocks(1 << 13, 333, 5, 31)
    mroot = blocks.manifest_root()
    assert product.StarkV1.prove(blocks, mroot).proof_bytes == oracle.prove_v1(blocks, mroot)


@pytest.mark.parametrize("T", [16, 1 << 12, 1 << 16])
def test_prove_deep_paths_bit_exact(gpu_ok, product, oracle, monkeypatch, T):
    """Single device: DEEP as the LDE of q + c*S (DeepPoly, the default) and the
    per-point division fused into the last LDE pass (SEZKP_NO_DEEP_POLY=1)
    give the reference's bytes; T = 16 is the smallest size on the polynomial path."""
    blocks = product.synthetic_blocks(T, min(T, 512), 3, 7)
    mroot = blocks.manifest_root()
    want = oracle.prove_v1(blocks, mroot)
    assert product.StarkV1.prove(blocks, mroot).proof_bytes == want
    monkeypatch.setenv("SEZKP_NO_DEEP_POLY", "1")
    assert product.StarkV1.prove(blocks, mroot).proof_bytes == want


def test_prove_rejects_bad_shapes(gpu_ok, product):
    blocks = product.synthetic_blocks(96, 32, 2)  # n = 96, not a power of two
    with pytest.raises(product.SezkpError, match="power of two"):
        product.StarkV1.prove(blocks, bytes(32))
    blocks = product.synthetic_blocks(64, 32, 2)
    blocks.step_hi[0] += 1  # step count disagrees with step_lo/step_hi
    with pytest.raises(product.SezkpError):
        product.StarkV1.prove(blocks, bytes(32))
    # step offsets that would index past the step arrays are refused on the host
    blocks = product.synthetic_blocks(64, 32, 2)
    blocks.step_start[:] += 32
    with pytest.raises(product.SezkpError, match="step_start"):
        product.StarkV1.prove(blocks, bytes(32))
    # a zero-step range over a block that still holds steps is refused
    blocks = product.synthetic_blocks(64, 32, 2)
    blocks.step_hi[1] = blocks.step_lo[1] - 1
    with pytest.raises(product.SezkpError, match="zero-step"):
        product.StarkV1.prove(blocks, bytes(32))


@pytest.mark.parametrize("T,b,tau,seed,at", [
    (1 << 12, 512, 8, 42, [0, 3, 3, 8]),          # first, two in a row, last
    (1 << 16, 100, 3, 7, [1, 17, 17, 17, 200, 656]),
    (1 << 12, 4096, 2, 3, [0, 1]),                # one real block
])
def test_prove_zero_step_blocks_bit_exact(gpu_ok, product, oracle, T, b, tau, seed, at):
    """Blocks of zero steps (step_hi = step_lo - 1) count 0 rows and are
    skipped, as in the reference (columns.rs:254-257,281-284; RowIter
    openings.rs:209-238) and the oracle: the proof equals oracle.prove_v1 on
    the same blocks, and the proof of the blocks without them under the same
    manifest root. Also through a staged upload of the same shape."""
    from conftest import insert_zero_step_blocks
    base = product.synthetic_blocks(T, b, tau, seed)
    blocks = insert_zero_step_blocks(base, at)
    mroot = blocks.manifest_root()
    want = oracle.prove_v1(blocks, mroot)
    assert want == oracle.prove_v1(base, mroot)
    assert product.StarkV1.prove(blocks, mroot).proof_bytes == want
    ctx = product.ProverContext(0)
    ctx.upload(insert_zero_step_blocks(product.synthetic_blocks(T, b, tau, seed + 1), at))
    ctx.stage(blocks)
    assert ctx.prove(mroot).proof_bytes == want
    ctx.close()


def test_prove_rejects_head_outside_i32(gpu_ok, product):
    """The head columns are stored as i32 on the device (the reference keeps
    i64 heads, air.rs:54). One block of 2^25 rows moving +127 per row reaches
    head 2^25 * 127 > 2^31: k_expand's guard must refuse the trace instead
    of committing wrapped heads."""
    T = 1 << 25
    imv = np.zeros(T, np.int8)
    mv = np.full((T, 1), 127, np.int8)
    hw = np.zeros((T, 1), np.uint8)
    ws = np.zeros((T, 1), np.uint16)
    blocks = product.partition(imv, mv, hw, ws, T)
    with pytest.raises(product.SezkpError, match="i32 range"):
        product.StarkV1.prove(blocks, bytes(32))
    # the guard is data-dependent, so a refused trace must not
    # poison the context: a good trace of the same shape staged next proves
    ctx = product.ProverContext(0)
    ctx.upload(blocks)
    with pytest.raises(product.SezkpError, match="i32 range"):
        ctx.prove(bytes(32))
    good = product.partition(imv, np.ones((T, 1), np.int8), hw, ws, T)
    ctx.stage(good)
    assert len(ctx.prove(bytes(32)).proof_bytes) > 0
    ctx.close()
    # the same trace in blocks of 2^24 rows (head <= 2^24 * 127 < 2^31) is accepted
    blocks = product.partition(imv, mv, hw, ws, 1 << 24)
    ctx = product.ProverContext(0)
    ctx.upload(blocks)
    assert len(ctx.prove(bytes(32)).proof_bytes) > 0
    ctx.close()


def test_prove_full_size_config3(gpu_ok, product, oracle):
    """T = 2^18 (BASELINE config 3 size, N = 2^21): bytes identical to the oracle."""
    blocks = product.synthetic_blocks(1 << 18, 512, 8, 42)
    mroot = blocks.manifest_root()
    ctx = product.ProverContext(0)
    ctx.upload(blocks)
    art = ctx.prove(mroot)
    assert art.proof_bytes == oracle.prove_v1(blocks, mroot)
    again = ctx.prove(mroot)  # resident inputs: repeated proofs are deterministic
    assert again.proof_bytes == art.proof_bytes
    view = ctx.prove_view(mroot)  # borrowed pinned buffer, same bytes
    assert view.readonly and bytes(view) == art.proof_bytes


def test_stage_events_opt_in_same_bytes(gpu_ok, product, oracle, monkeypatch):
    """Per-stage timed events are recorded only on request
    (SEZKP_STAGE_EVENTS=1): without them the device stage times read 0 and the
    host times are still measured; the proof bytes are the same either way."""
    blocks = product.synthetic_blocks(1 << 12, 100, 3, 21)
    mroot = blocks.manifest_root()
    want = oracle.prove_v1(blocks, mroot)
    ctx = product.ProverContext(0)
    ctx.upload(blocks)
    monkeypatch.delenv("SEZKP_STAGE_EVENTS", raising=False)
    monkeypatch.delenv("SEZKP_KERNEL_EVENTS", raising=False)
    assert ctx.prove(mroot).proof_bytes == want
    st = ctx.stage_times_ms()
    assert st["total"] == 0 and st["lde_ntt"] == 0 and st["host_wall"] > 0
    monkeypatch.setenv("SEZKP_STAGE_EVENTS", "1")
    assert ctx.prove(mroot).proof_bytes == want
    st = ctx.stage_times_ms()
    assert st["total"] > 0 and st["lde_ntt"] > 0 and st["total"] >= st["lde_ntt"]
    ctx.close()


def test_prove_headline_size_matches_openmp_oracle(gpu_ok, product, monkeypatch):
    """The bench workload itself: `sezkp-cli simulate --t 2097152 --b 512
    --tau 8` blocks (T = 2^21, N = 2^24). The GPU proof equals the OpenMP build
    of the C oracle byte for byte (twice on one context: a re-proof of a
    resident trace); the oracle runs in a child process on 16 threads
    (~10 s), so the other tests keep the single-thread build."""
    import sys
    T = 1 << 21
    code = ("import sys; sys.path[:0]=[%r,%r]\n"
            "import hashlib, oracle_ctypes as O, sezkp_amd as S\n"
            "O.use_mt(16)\n"
            "bl=S.reference_blocks(%d,512,8,42); print(hashlib.sha256(O.prove_v1(bl, bl.manifest_root())).hexdigest())\n"
            % (PKG, os.path.join(ROOT, "oracle"), T))
    child = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    blocks = product.reference_blocks(T, 512, 8, 42)
    ctx = product.ProverContext(0)
    ctx.upload(blocks)
    got = hashlib.sha256(ctx.prove(blocks.manifest_root()).proof_bytes).hexdigest()
    got_repeat = hashlib.sha256(ctx.prove(blocks.manifest_root()).proof_bytes).hexdigest()
    ctx.close()
    out, err = child.communicate(timeout=150)
    assert child.returncode == 0, err[-1500:]
    assert got == out.strip() and got_repeat == got


def test_prove_config5_size_one_gpu_matches_openmp_oracle(gpu_ok, product):
    """Config 5's trace (T = 2^22, N = 2^25) proven on ONE device: the LDE's
    first pass is an X16 tile (12 stages, DEEP-polynomial load), so the 2^25
    transform takes 3 passes. Equal to the OpenMP oracle byte for byte."""
    import sys
    T, b, tau, seed = 1 << 22, 512, 8, 5
    code = ("import sys; sys.path[:0]=[%r,%r]\n"
            "import hashlib, oracle_ctypes as O, sezkp_amd as S\n"
            "O.use_mt(16)\n"
            "bl=S.synthetic_blocks(%d,%d,%d,%d); print(hashlib.sha256(O.prove_v1(bl, bl.manifest_root())).hexdigest())\n"
            % (PKG, os.path.join(ROOT, "oracle"), T, b, tau, seed))
    child = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    blocks = product.synthetic_blocks(T, b, tau, seed)
    ctx = product.ProverContext(0)
    ctx.upload(blocks)
    got = hashlib.sha256(ctx.prove(blocks.manifest_root()).proof_bytes).hexdigest()
    ctx.close()
    out, err = child.communicate(timeout=300)
    assert child.returncode == 0, err[-1500:]
    assert got == out.strip()


def test_reupload_reuses_workspace_bit_exact(gpu_ok, product, oracle):
    """upload() keeps the previous workspace for a trace of the same shape, so
    every buffer holds the old trace's data when the new proof starts: each
    proof still equals the oracle's. Shapes alternate so that some blocks are
    reused and some freshly allocated."""
    from sezkp_amd._lib import VIEW_FIELDS
    ctx = product.ProverContext(0)
    for T, b, tau, seed in [(1 << 14, 512, 4, 1), (1 << 14, 512, 4, 2), (1 << 12, 256, 2, 3),
                            (1 << 14, 512, 4, 4), (1 << 14, 256, 4, 5)]:
        blocks = product.synthetic_blocks(T, b, tau, seed)
        mroot = blocks.manifest_root()
        want = oracle.prove_v1(blocks, mroot)
        ctx.upload(blocks)
        assert ctx.prove(mroot).proof_bytes == want, (T, b, tau, seed)
    # the device transposition reads has_write as a boolean and ignores wsym
    # where it is clear (Option<u8> in the reference: columns.rs:71-72)
    arrays = {f: getattr(blocks, f).copy() for f, _ in VIEW_FIELDS}
    hw = arrays["has_write"]
    arrays["has_write"] = np.where(hw != 0, np.uint8(7), np.uint8(0))
    arrays["wsym"] = np.where(hw != 0, arrays["wsym"], np.uint16(0xBEEF))
    ctx.upload(product.BlockSoA(blocks.tau, **arrays))
    assert ctx.prove(mroot).proof_bytes == want


def test_streaming_meta_and_verify(gpu_ok, product, oracle):
    """prove_streaming: same bytes, meta gains mode; the host verifier accepts
    proofs of a trace whose AIR holds (non-negative heads) and rejects tampering."""
    rng = np.random.default_rng(3)
    T, tau = 4096, 4
    mv = rng.integers(0, 2, (T, tau), dtype=np.int8)  # heads never go left of 0
    hw = (rng.random((T, tau)) < 0.4).astype(np.uint8)
    ws = (rng.integers(0, 16, (T, tau)) * hw).astype(np.uint16)
    blocks = product.partition(rng.integers(-1, 2, T, dtype=np.int8), mv, hw, ws, 512)
    mroot = blocks.manifest_root()
    a = product.StarkV1.prove(blocks, mroot)
    s = product.StarkV1.prove_streaming(blocks, mroot)
    assert s.proof_bytes == a.proof_bytes and s.meta["mode"] == "streaming"
    product.StarkV1.verify(a, blocks, mroot)
    bad = bytearray(a.proof_bytes)
    bad[len(bad) // 2] ^= 1
    with pytest.raises(product.SezkpError):
        product.StarkV1.verify(product.ProofArtifact("stark", mroot, bytes(bad), a.meta), blocks, mroot)


def test_cli_prove_verify_matches_oracle_artifact(gpu_ok, product, oracle, tmp_path):
    """`sezkp-cli prove --backend stark` drop-in: CBOR artifact byte-identical
    to the reference layout built from the oracle's proof bytes."""
    import cbor_min
    raw, mroot = _fixture("minimal_riscv")
    bpath, mpath = tmp_path / "blocks.cbor", tmp_path / "manifest.cbor"
    bpath.write_bytes(raw)
    cli = os.path.join(PKG, "bin", "sezkp-cli")
    subprocess.run([cli, "commit", "--blocks", str(bpath), "--out", str(mpath)], check=True)
    assert bytes(cbor_min.loads(mpath.read_bytes())["root"]) == mroot
    out = tmp_path / "proof.cbor"
    r = subprocess.run([cli, "prove", "--backend", "stark", "--blocks", str(bpath), "--manifest", str(mpath),
                        "--out", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    blocks = product.BlockSoA.from_cbor(raw)
    want = cbor_min.proof_artifact_cbor("stark", mroot, oracle.prove_v1(blocks, mroot),
                                        {"proto": "stark-v1", "domain_n": 8 * blocks.n_rows, "tau": blocks.tau})
    assert out.read_bytes() == want
    # the same blocks as a real .jsonl file: the precheck passes (8 blocks: the
    # Frontier root equals the batch root) and the stark path refuses the
    # extension (io.rs:78-88), writing nothing
    jl = tmp_path / "b.jsonl"
    jl.write_bytes(blocks.to_jsonl())
    out2 = tmp_path / "proof2.cbor"
    r = subprocess.run([cli, "prove", "--backend", "stark", "--blocks", str(jl), "--manifest", str(mpath),
                        "--out", str(out2)], capture_output=True, text=True)
    assert r.returncode != 0 and "unsupported blocks extension: jsonl" in r.stderr, r.stderr
    assert not out2.exists()


def test_cli_config1_simulate_commit_prove_verify(gpu_ok, product, oracle, tmp_path):
    """BASELINE config 1 end to end, as scripts/test_all.zsh:17-30 runs it:
    `sezkp-cli simulate --t 4096 --b 512 --tau 8` (the reference's generator,
    seed 42) -> `commit` -> `prove --backend stark` -> `verify`. The blocks are
    reference_blocks(4096, 512, 8, 42); the artifact equals the one built from
    the oracle's proof of those blocks byte for byte."""
    import cbor_min
    cli = os.path.join(PKG, "bin", "sezkp-cli")
    bpath, mpath, ppath = tmp_path / "blocks.cbor", tmp_path / "manifest.cbor", tmp_path / "proof.cbor"
    for cmd in (["simulate", "--t", "4096", "--b", "512", "--tau", "8", "--out-blocks", str(bpath)],
                ["commit", "--blocks", str(bpath), "--out", str(mpath)],
                ["prove", "--backend", "stark", "--blocks", str(bpath), "--manifest", str(mpath), "--out", str(ppath)]):
        r = subprocess.run([cli] + cmd, capture_output=True, text=True)
        assert r.returncode == 0, (cmd[0], r.stderr)
    blocks = product.reference_blocks(4096, 512, 8, 42)
    assert bpath.read_bytes() == blocks.to_cbor()
    mroot = blocks.manifest_root()
    assert bytes(cbor_min.loads(mpath.read_bytes())["root"]) == mroot
    want = cbor_min.proof_artifact_cbor("stark", mroot, oracle.prove_v1(blocks, mroot),
                                        {"proto": "stark-v1", "domain_n": 8 * 4096, "tau": 8})
    assert ppath.read_bytes() == want
    # the reference's verifier may reject simulate traces (AIR boundary terms,
    # SURVEY 3C): the CLI's verdict must be the oracle verifier's verdict
    # (oracle/sezkp_oracle_py.py verify_v1, verify.rs:60-196) on the same bytes
    import sezkp_oracle_py as V
    want_v = V.verify_v1(oracle.prove_v1(blocks, mroot), 8)
    r = subprocess.run([cli, "verify", "--backend", "stark", "--blocks", str(bpath), "--manifest", str(mpath),
                        "--proof", str(ppath)], capture_output=True, text=True)
    if want_v is None:
        assert r.returncode == 0 and "OK: proof verified" in r.stdout, r.stderr
    else:
        assert r.returncode != 0 and want_v in r.stderr, (r.stderr, want_v)


def test_launcher_jsonl_frontier_manifest(gpu_ok, product, oracle, tmp_path):
    """Config 5's path on a 7-block JSONL file (T = 2^12, 600 steps per block):
    `sezkp-cli commit --blocks b.jsonl` writes the Frontier root (lib.rs:265-278,
    which differs from the batch root at 7 blocks), the launcher's precheck
    accepts it (lib.rs:309-331), and the artifact equals the oracle's proof
    bound to that root."""
    import sys
    import cbor_min
    blocks = product.synthetic_blocks(1 << 12, 600, 8, 11)
    assert blocks.n_blocks == 7
    jl, mpath, out = tmp_path / "b.jsonl", tmp_path / "m.cbor", tmp_path / "p.cbor"
    jl.write_bytes(blocks.to_jsonl())
    cli = os.path.join(PKG, "bin", "sezkp-cli")
    subprocess.run([cli, "commit", "--blocks", str(jl), "--out", str(mpath)], check=True, capture_output=True)
    froot = bytes(cbor_min.loads(mpath.read_bytes())["root"])
    assert froot == blocks.manifest_frontier_root() != blocks.manifest_root()
    r = subprocess.run([sys.executable, "-m", "sezkp_amd.launch", "prove", "--blocks", str(jl), "--manifest",
                        str(mpath), "--out", str(out)], cwd=PKG, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    want = cbor_min.proof_artifact_cbor("stark", froot, oracle.prove_v1(blocks, froot),
                                        {"proto": "stark-v1", "domain_n": 8 * 4096, "tau": 8})
    assert out.read_bytes() == want
    # the batch-root manifest (commit of the same blocks as .cbor) is refused
    # for the JSONL file by the precheck
    cb, bad = tmp_path / "b.cbor", tmp_path / "mb.cbor"
    cb.write_bytes(blocks.to_cbor())
    subprocess.run([cli, "commit", "--blocks", str(cb), "--out", str(bad)], check=True, capture_output=True)
    r = subprocess.run([sys.executable, "-m", "sezkp_amd.launch", "prove", "--blocks", str(jl), "--manifest",
                        str(bad), "--out", str(tmp_path / "p2.cbor")], cwd=PKG, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 1 and "root mismatch" in r.stderr, r.stderr[-2000:]


def test_async_proofs_in_flight_bit_exact(gpu_ok, product, oracle):
    """sezkp_ctx_prove_async / sezkp_ctx_wait: three contexts (distinct
    traces) in flight on one GPU, resubmitted round-robin; every proof equals
    the oracle's, and misuse is refused without disturbing the context."""
    traces = [product.synthetic_blocks(1 << 12, 512, 4, s) for s in (1, 2, 3)]
    roots = [b.manifest_root() for b in traces]
    want = [oracle.prove_v1(b, r) for b, r in zip(traces, roots)]
    ctxs = []
    for b in traces:
        c = product.ProverContext(0)
        c.upload(b)
        ctxs.append(c)
    for c, r in zip(ctxs, roots):
        c.prove_async(r)
    for rnd in range(3):
        for i, c in enumerate(ctxs):
            assert bytes(c.wait_view()) == want[i]
            if rnd < 2:
                c.prove_async(roots[i])
    c = ctxs[0]
    with pytest.raises(product.SezkpError, match="no proof in flight"):
        c.wait_view()
    c.prove_async(roots[0])
    with pytest.raises(product.SezkpError, match="in flight"):
        c.prove_async(roots[0])
    with pytest.raises(product.SezkpError, match="in flight"):
        c.prove(roots[0])
    assert bytes(c.wait_view()) == want[0]
    assert c.prove(roots[0]).proof_bytes == want[0]
    ctxs[1].prove_async(roots[1])  # destroy with a proof in flight waits for it
    for c in ctxs:
        c.close()


def test_staged_uploads_pipeline_bit_exact(gpu_ok, product, oracle):
    """sezkp_ctx_stage: the next trace (same shape, other values) goes over
    PCIe into the spare trace image while a proof is in flight; every proof
    equals the oracle's for ITS trace, whether staged from pinned or pageable
    memory, staged twice before a prove, or not staged at all."""
    T, b, tau = 1 << 13, 512, 4
    traces = [product.synthetic_blocks(T, b, tau, s) for s in range(5)]
    traces[1].pin()
    traces[3].pin()
    roots = [t.manifest_root() for t in traces]
    want = [oracle.prove_v1(t, r) for t, r in zip(traces, roots)]
    c = product.ProverContext(0)
    c.upload(traces[0])
    c.prove_async(roots[0])
    c.stage(traces[1])                     # overlaps proof 0
    assert bytes(c.wait_view()) == want[0]
    c.prove_async(roots[1])
    c.stage(traces[2])                     # pageable source
    assert bytes(c.wait_view()) == want[1]
    c.stage(traces[3])                     # replaces the staged trace 2
    assert bytes(c.prove_view(roots[3])) == want[3]
    assert bytes(c.prove_view(roots[3])) == want[3]  # nothing staged: same trace again
    c.stage(traces[4])
    assert c.prove(roots[4]).proof_bytes == want[4]
    other = product.synthetic_blocks(T, 520, tau, 9)  # 16 blocks again, other boundaries
    with pytest.raises(product.SezkpError, match="block boundaries"):
        c.stage(other)
    with pytest.raises(product.SezkpError, match="another shape"):
        c.stage(product.synthetic_blocks(T, 256, tau, 9))  # other block count
    with pytest.raises(product.SezkpError, match="another shape"):
        c.stage(product.synthetic_blocks(T, b, tau + 1, 9))
    c.upload(other)                        # a new shape goes through upload
    assert c.prove(other.manifest_root()).proof_bytes == oracle.prove_v1(other, other.manifest_root())
    c.close()
    for t in traces:
        t.unpin()


def test_stage_then_prove_at_once_bit_exact(gpu_ok, product, oracle):
    """The prove call right after a pinned stage() finds the copies still in
    flight: it waits for them on the host (the copy stream holds only copies)
    and transposes the step arrays on its own stream. A stage() that replaces
    a staged trace whose copies are still running waits for them too."""
    T, b, tau = 1 << 18, 512, 8
    tr = [product.synthetic_blocks(T, b, tau, s) for s in (61, 62)]
    for t in tr:
        t.pin()
    roots = [t.manifest_root() for t in tr]
    want = [oracle.prove_v1(t, r) for t, r in zip(tr, roots)]
    c = product.ProverContext(0)
    c.upload(tr[0])
    assert bytes(c.prove_view(roots[0])) == want[0]
    for i in (1, 0, 1):
        c.stage(tr[i])
        assert bytes(c.prove_view(roots[i])) == want[i]
    c.stage(tr[0])
    c.stage(tr[1])  # replaces the staged trace 0 while its copies may still run
    assert bytes(c.prove_view(roots[1])) == want[1]
    c.close()
    for t in tr:
        t.unpin()


def test_stage_after_prove_async_feeds_the_next_proof(gpu_ok, product, oracle):
    """prove_async(i) then stage(i + 1) at once: proof i must read trace i even
    when its worker starts late. SEZKP_TEST_WORKER_DELAY_US holds the worker
    back 50 ms (read once per process, so in a child), so the stage always
    lands before the proof starts; every proof is checked against its own
    trace's oracle bytes."""
    import sys
    T, b, tau = 1 << 12, 512, 4
    seeds = (21, 22, 23)
    code = ("import sys, hashlib; sys.path[:0]=[%r]\n"
            "import sezkp_amd as S\n"
            "tr=[S.synthetic_blocks(%d,%d,%d,s) for s in %r]; rt=[t.manifest_root() for t in tr]\n"
            "c=S.ProverContext(0); c.upload(tr[0]); out=[]\n"
            "c.prove_async(rt[0]); c.stage(tr[1]); out.append(bytes(c.wait_view()))\n"
            "c.prove_async(rt[1]); c.stage(tr[2]); out.append(bytes(c.wait_view()))\n"
            "c.prove_async(rt[2]); out.append(bytes(c.wait_view()))\n"
            "c.prove_async(rt[2]); out.append(bytes(c.wait_view()))\n"
            "c.close(); print(' '.join(hashlib.sha256(x).hexdigest() for x in out))\n"
            % (PKG, T, b, tau, seeds))
    env = dict(os.environ, SEZKP_TEST_WORKER_DELAY_US="50000")
    child = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert child.returncode == 0, child.stderr[-1500:]
    traces = [product.synthetic_blocks(T, b, tau, s) for s in seeds]
    want = [hashlib.sha256(oracle.prove_v1(t, t.manifest_root())).hexdigest() for t in traces]
    assert child.stdout.split() == want + [want[2]]


def test_upload_right_after_stage_bit_exact(gpu_ok, product, oracle):
    """upload() while a stage() may still be copying into the spare image (from
    pinned memory, so the copy is real DMA on the copy stream): upload waits
    for the copy stream before reusing those buffers, for a new shape and for
    the same shape."""
    T, b, tau = 1 << 13, 512, 4
    t0, t1, t3 = (product.synthetic_blocks(T, b, tau, s) for s in (31, 32, 33))
    t2 = product.synthetic_blocks(1 << 12, 256, 2, 34)
    t1.pin()
    c = product.ProverContext(0)
    c.upload(t0)
    c.stage(t1)
    c.upload(t2)  # other shape
    assert c.prove(t2.manifest_root()).proof_bytes == oracle.prove_v1(t2, t2.manifest_root())
    c.upload(t0)
    c.stage(t1)
    c.upload(t3)  # same shape as the staged trace
    assert c.prove(t3.manifest_root()).proof_bytes == oracle.prove_v1(t3, t3.manifest_root())
    c.close()
    t1.unpin()

"""GPU parity of the kernel-level C ABI against the oracle:
leaf hashing (merkle.rs:132-160), MerkleTree::from_leaves / open with odd
promotion (merkle.rs:46-108), the plain FRI fold (prover.rs:208-230) and the
coset LDE + DEEP with a caller-chosen shift and fused leaf digests
(lde.rs:42-97, coset.rs:85-102). Bit-exact everywhere."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
import sezkp_amd._lib as L  # noqa: E402  (conftest puts the package on sys.path)
P = 0xFFFFFFFF00000001


def _dev(torch, arr: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(arr).view(np.int64)).cuda()


def _host(t) -> np.ndarray:
    return t.cpu().numpy().view(np.uint64)


def _digests(torch, count: int):
    return torch.zeros(max(count, 1) * 4, dtype=torch.int64, device="cuda")  # 32 B each


def _bytes(t, count: int) -> bytes:
    return t.cpu().numpy().tobytes()[:32 * count]


@pytest.mark.parametrize("n", [1, 2, 3, 255, 4096, 70000])
def test_leaves_u64_match_oracle(gpu_ok, product, oracle, n):
    torch = gpu_ok
    vals = oracle.det_vec(n, 11)
    vals[0] = np.uint64(0xFFFFFFFFFFFFFFFF)  # raw 8 LE bytes, not reduced (hash_field_leaves takes [u8; 8])
    d = _dev(torch, vals)
    out = _digests(torch, n)
    assert product.lib.sezkp_blake3_leaves_u64(d.data_ptr(), n, out.data_ptr(), None) == 0
    want = b"".join(oracle.hash_leaf_u64(int(v)) for v in vals)
    assert _bytes(out, n) == want


@pytest.mark.parametrize("label", ["input_mv", "mv_0", "head_bits_b15_t7", "x", "a" * 44])
def test_leaves_labeled_match_oracle(gpu_ok, product, oracle, label):
    torch = gpu_ok
    n = 1000
    vals = oracle.det_vec(n, len(label))
    d = _dev(torch, vals)
    out = _digests(torch, n)
    lab = label.encode()
    assert product.lib.sezkp_blake3_leaves_labeled(d.data_ptr(), n, lab, len(lab), out.data_ptr(), None) == 0
    want = b"".join(oracle.hash_leaf_labeled(int(v), label) for v in vals)
    assert _bytes(out, n) == want


def test_leaves_labeled_rejects_long_label(gpu_ok, product):
    torch = gpu_ok
    d = torch.zeros(4, dtype=torch.int64, device="cuda")
    out = _digests(torch, 4)
    lab = b"b" * 45
    assert product.lib.sezkp_blake3_leaves_labeled(d.data_ptr(), 4, lab, 45, out.data_ptr(), None) == L.SEZKP_E_INVALID


@pytest.mark.parametrize("n", [0, 1, 2, 3, 5, 7, 11, 13, 64, 1000, 4097, 1 << 16])
def test_merkle_build_and_paths_match_oracle(gpu_ok, product, oracle, n):
    """Every level (odd promotion at 3, 5, 7, 11, 13, 1000, 4097) and the
    paths of MerkleTree::open, including indices >= n (idx %= n)."""
    torch = gpu_ok
    vals = oracle.det_vec(max(n, 1), 3 + n)[:n]
    leaves = b"".join(oracle.hash_leaf_u64(int(v)) for v in vals)
    cnt = product.lib.sezkp_merkle_node_count(n)
    want_nodes = oracle.merkle_nodes(leaves)
    assert cnt == len(want_nodes) // 32
    d_leaves = torch.from_numpy(np.frombuffer(leaves or b"\0" * 32, dtype=np.int64).copy()).cuda()
    nodes = _digests(torch, cnt)
    assert product.lib.sezkp_merkle_build(d_leaves.data_ptr(), n, nodes.data_ptr(), None) == 0
    assert _bytes(nodes, cnt) == want_nodes
    rng = np.random.default_rng(n)
    idx = np.concatenate([np.arange(min(n, 8)), rng.integers(0, 1 << 40, 30)]).astype(np.uint64)
    d_idx = _dev(torch, idx)
    want = oracle.merkle_open(leaves, idx)
    depth = len(want[0])
    out = _digests(torch, len(idx) * depth)
    assert product.lib.sezkp_merkle_paths(nodes.data_ptr(), n, d_idx.data_ptr(), len(idx), out.data_ptr(), None) == 0
    got = _bytes(out, len(idx) * depth)
    for i, sibs in enumerate(want):
        assert got[32 * depth * i:32 * depth * (i + 1)] == b"".join(sibs), f"path of index {int(idx[i])}"


def test_merkle_build_in_place(gpu_ok, product, oracle):
    """nodes32 == leaves32: the buffer holds the leaves and room for the upper levels."""
    torch = gpu_ok
    n = 777
    vals = oracle.det_vec(n, 1)
    leaves = b"".join(oracle.hash_leaf_u64(int(v)) for v in vals)
    cnt = product.lib.sezkp_merkle_node_count(n)
    buf = _digests(torch, cnt)
    assert product.lib.sezkp_blake3_leaves_u64(_dev(torch, vals).data_ptr(), n, buf.data_ptr(), None) == 0
    assert product.lib.sezkp_merkle_build(buf.data_ptr(), n, buf.data_ptr(), None) == 0
    assert _bytes(buf, cnt) == oracle.merkle_nodes(leaves)


@pytest.mark.parametrize("log_out", [0, 1, 2, 3, 9, 16])
def test_fri_fold_matches_oracle(gpu_ok, product, oracle, log_out):
    torch = gpu_ok
    n = 1 << log_out
    vals = oracle.det_vec(2 * n, 17)
    beta = 0x0123456789ABCDEF % P
    want = np.array([(int(vals[i]) + beta * int(vals[i + n])) % P for i in range(n)], dtype=np.uint64)
    d_in = _dev(torch, vals)
    d_out = torch.empty(n, dtype=torch.int64, device="cuda")
    assert product.lib.sezkp_fri_fold(d_in.data_ptr(), n, beta, d_out.data_ptr(), None) == 0
    np.testing.assert_array_equal(_host(d_out), want)


@pytest.mark.parametrize("beta", [0, 1, P - 1, (1 << 32) - 1, 1 << 63, P - (1 << 32)])
def test_fri_fold_edge_values(gpu_ok, product, beta):
    """fri.rs fold (lo + beta * hi) on values at the carry / borrow boundaries
    of the 32-bit-lane arithmetic, with boundary betas: exact against Python
    integers."""
    torch = gpu_ok
    n = 1 << 12
    eps = (1 << 32) - 1
    edge = np.array([0, 1, P - 1, P - 2, eps, eps + 1, 1 << 63, P - eps, (1 << 64) - (1 << 33)], dtype=np.uint64)
    vals = edge[np.random.default_rng(beta % 1000).integers(0, len(edge), 2 * n)]
    vals[: n // 2] = P - 1
    vals[n: n + n // 2] = P - 1
    want = np.array([(int(vals[i]) + beta * int(vals[i + n])) % P for i in range(n)], dtype=np.uint64)
    d_in = _dev(torch, vals)
    d_out = torch.empty(n, dtype=torch.int64, device="cuda")
    assert product.lib.sezkp_fri_fold(d_in.data_ptr(), n, beta, d_out.data_ptr(), None) == 0
    np.testing.assert_array_equal(_host(d_out), want)


@pytest.mark.parametrize("log_n,log_blowup,shift", [(0, 3, 3), (4, 3, 7), (5, 0, 5), (6, 1, 3), (8, 2, 11),
                                                    (10, 3, 2 ** 40 + 1), (13, 3, P - 1), (16, 3, 7)])
def test_coset_lde_deep_shift_and_leaves(gpu_ok, product, oracle, log_n, log_blowup, shift):
    """lde.rs:42-97 with the coset shift of coset.rs:85-102 as a parameter and
    the layer-0 leaf digests fused (fri_stream.rs:37-41)."""
    torch = gpu_ok
    n = 1 << log_n
    N = n << log_blowup
    base = oracle.det_vec(n, 40 + log_n)
    z = 0x0FEDCBA987654321 % P
    want = oracle.lde_deep_shift(base, log_blowup, shift, z)
    d_in = _dev(torch, base)
    d_out = torch.empty(N, dtype=torch.int64, device="cuda")
    leaves = _digests(torch, N)
    assert product.lib.sezkp_gl_coset_lde_deep(d_in.data_ptr(), log_n, log_blowup, shift, z, d_out.data_ptr(),
                                               leaves.data_ptr(), None) == 0
    got = _host(d_out)
    np.testing.assert_array_equal(got, want)
    if N <= 4096:
        assert _bytes(leaves, N) == b"".join(oracle.hash_leaf_u64(int(v)) for v in want)
    else:  # spot-check: one digest in 64
        raw = _bytes(leaves, N)
        for i in range(0, N, 64):
            assert raw[32 * i:32 * i + 32] == oracle.hash_leaf_u64(int(want[i]))


def test_coset_lde_deep_rejects_vanishing_denominator(gpu_ok, product, oracle):
    """z on the coset (z = shift * w^i): some shift w^i - z is 0."""
    torch = gpu_ok
    log_n, shift = 4, 5
    w = int(oracle.ntt_forward(np.eye(1, 1 << (log_n + 3), 1, dtype=np.uint64)[0])[1])  # w_N
    z = shift * pow(w, 9, P) % P
    d_in = _dev(torch, oracle.det_vec(16, 1))
    d_out = torch.empty(128, dtype=torch.int64, device="cuda")
    assert product.lib.sezkp_gl_coset_lde_deep(d_in.data_ptr(), log_n, 3, shift, z, d_out.data_ptr(), None,
                                               None) == L.SEZKP_E_INVALID
    assert product.lib.sezkp_gl_coset_lde_deep(d_in.data_ptr(), log_n, 3, 0, 1, d_out.data_ptr(), None,
                                               None) == L.SEZKP_E_INVALID
    # N = 1 (log_n = log_blowup = 0) is rejected before anything is launched;
    # N = 2 from one point (log_blowup = 1) still works
    assert product.lib.sezkp_gl_coset_lde_deep(d_in.data_ptr(), 0, 0, 3, 5, d_out.data_ptr(), None,
                                               None) == L.SEZKP_E_INVALID
    one = oracle.det_vec(1, 3)
    d1 = _dev(torch, one)
    d2 = torch.empty(2, dtype=torch.int64, device="cuda")
    assert product.lib.sezkp_gl_coset_lde_deep(d1.data_ptr(), 0, 1, 3, 5, d2.data_ptr(), None, None) == 0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(d2), oracle.lde_deep_shift(one, 1, 3, 5))

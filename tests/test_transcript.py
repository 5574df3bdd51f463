"""The prover's Fiat-Shamir transcript (host, csrc/host_crypto.cpp), CPU.

Known answers through the C ABI `sezkp_fs_xof` (BLAKE3 XOF of stream prefix ||
suffix, the core of Blake3Transcript::challenge_bytes,
crates/sezkp-crypto/src/lib.rs:102-123) against the C oracle's BLAKE3 and the
reference's committed v0 proofs, and the reference's transcript input vector
(specs/stark-v1/transcript_inputs.json, crates/sezkp-stark/tests/param_vectors.rs).
(Round 4's device transcript was removed in round 5: it measured slower than
the host round trips it replaced.)
"""
import ctypes as C
import json
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN

def fs_xof(product, stream: bytes, chals):
    """chals: [(pos, suffix bytes, out_len)] -> [bytes] via sezkp_fs_xof."""
    n = len(chals)
    pos = (C.c_uint32 * n)(*[c[0] for c in chals])
    sl = (C.c_uint32 * n)(*[len(c[1]) for c in chals])
    ol = (C.c_uint32 * n)(*[c[2] for c in chals])
    sfx = b"".join(c[1] for c in chals)
    out = C.create_string_buffer(sum(c[2] for c in chals))
    rc = product.lib.sezkp_fs_xof(stream, len(stream), pos, sfx, sl, ol, n, out, None)
    assert rc == 0, rc
    res, o = [], 0
    for c in chals:
        res.append(out.raw[o:o + c[2]])
        o += c[2]
    return res


def sfx(label: str) -> bytes:
    lb = label.encode()
    return b"challenge" + struct.pack("<I", len(lb)) + lb


@pytest.mark.parametrize("seed", range(6))
def test_fs_xof_random_streams_match_blake3(product, oracle, seed):
    """Prefixes at random and at chunk / block edges (0, 63, 64, 1023, 1024,
    2048 + 1, a suffix that completes or crosses a chunk), suffixes of 1-60
    bytes, outputs of 8-512 bytes (1-8 XOF blocks), 16 challenges a batch."""
    rng = np.random.default_rng(100 + seed)
    L = int(rng.integers(3000, 12000))
    stream = rng.bytes(L)
    edges = [0, 63, 64, 1023, 1024, 1024 - 10, 2049, 4096, L]
    chals = []
    for i in range(16):
        p = edges[i] if i < len(edges) else int(rng.integers(0, L + 1))
        p = min(p, L)
        s = rng.bytes(int(rng.integers(1, 61)))
        ol = 8 * int(rng.integers(1, 65))
        chals.append((p, s, ol))
    got = fs_xof(product, stream, chals)
    for (p, s, ol), g in zip(chals, got):
        assert g == oracle.blake3(stream[:p] + s, ol), (p, len(s), ol)


def test_fs_xof_host_blake3_size_sweep(product, oracle):
    """A size sweep of the host BLAKE3-XOF behind the transcript: stream
    prefixes of 0..40 KB (single-chunk, exactly one chunk, 2..39 chunks: each
    stack shape of the chunk-CV merges) against the oracle's BLAKE3."""
    rng = np.random.default_rng(7)
    stream = rng.bytes(40000)
    for base in range(0, 40000, 16 * 1024):
        chals = []
        for j in range(16):
            p = min(base + 1024 * j + int(rng.integers(0, 1024)), len(stream))
            chals.append((p, sfx("x" * int(rng.integers(1, 20))), 64))
        for (p, s, ol), g in zip(chals, fs_xof(product, stream, chals)):
            assert g == oracle.blake3(stream[:p] + s, ol), p


def _v0_streams(blocks, mroot):
    """The two v0 transcripts of the committed proof_stark.cbor files
    (sezkp-stark/src/lib.rs:66-95, commit.rs:47-90: rows in 4096-row chunks)."""
    import sezkp_oracle_py as V
    tau = blocks.tau
    t = V.Transcript("sezkp-stark/v0/row-stream")
    t.absorb_u64("tau", tau)
    nrow = int(blocks.step_start[-1])
    mv = blocks.mv.reshape(nrow, tau).astype(np.int16) + 1
    hw = blocks.has_write.reshape(nrow, tau) != 0
    rows = np.zeros((nrow, 1 + 2 * tau), np.uint8)
    rows[:, 0] = blocks.input_mv.view(np.uint8)
    rows[:, 1::2] = mv.astype(np.uint8)
    rows[:, 2::2] = hw
    for s in range(0, nrow, 4096):
        t.absorb("rows", rows[s:s + 4096].tobytes())
    return t, nrow


@pytest.mark.parametrize("name", ["ref", "riscv"])
def test_fs_xof_reproduces_v0_fixture_proofs(product, name):
    """The reference's own committed v0 proofs pin the transcript framing, the
    challenge / after_challenge ratchet and the XOF: the device computes both
    of their transcripts' challenges and returns the committed 64 bytes."""
    import cbor_min
    import sezkp_oracle_py as V
    blocks = product.BlockSoA.from_cbor(open(os.path.join(GOLDEN, f"{name}_blocks.cbor"), "rb").read())
    man = cbor_min.loads(open(os.path.join(GOLDEN, f"{name}_manifest.cbor"), "rb").read())
    art = cbor_min.loads(open(os.path.join(GOLDEN, f"{name}_proof_stark_v0.cbor"), "rb").read())
    want = bytes(art["proof_bytes"])
    t, nrow = _v0_streams(blocks, bytes(man["root"]))
    (root,) = fs_xof(product, t.stream, [(len(t.stream), sfx("root"), 32)])
    t2 = V.Transcript("sezkp-stark-v0")
    t2.absorb("manifest_root", bytes(man["root"]))
    t2.absorb("commit_root", root)
    t2.absorb_u64("n_rows", nrow)
    t2.absorb_u64("tau", blocks.tau)
    p_alpha = len(t2.stream)
    t2.challenge("alpha", 32)  # appends the after_challenge ratchet
    a, b = fs_xof(product, t2.stream, [(p_alpha, sfx("alpha"), 32), (len(t2.stream), sfx("beta"), 32)])
    assert a + b == want


def test_transcript_input_vector(product):
    """specs/stark-v1/transcript_inputs.json (param_vectors.rs:40-90): bind the
    vector's public inputs as the protocol does, derive alphas and the row
    queries on the device; they equal the host restatement's, the alphas are
    non-degenerate and every query row is in [0, n)."""
    import sezkp_oracle_py as V
    v = json.load(open(os.path.join(GOLDEN, "transcript_inputs.json")))
    t = V.Transcript("sezkp-stark/v1")
    t.absorb("manifest_root", bytes.fromhex(v["manifest_root_hex"]))
    t.absorb_u64("n", v["n"])
    t.absorb_u64("tau", v["tau"])
    t.absorb_u64("n_cols", len(v["col_roots_hex"]))
    for h in v["col_roots_hex"]:
        t.absorb("col_root", bytes.fromhex(h))
    p0 = len(t.stream)
    want_a = t.challenge("alphas", 64)
    p1 = len(t.stream)
    want_q = t.challenge("row_queries", 240)
    a, q = fs_xof(product, t.stream, [(p0, sfx("alphas"), 64), (p1, sfx("row_queries"), 240)])
    assert a == want_a and q == want_q
    P = 0xFFFFFFFF00000001
    alphas = [int.from_bytes(a[8 * i:8 * i + 8], "little") % P for i in range(8)]
    rows = [int.from_bytes(q[8 * i:8 * i + 8], "little") % v["n"] for i in range(30)]
    assert any(alphas) and len(rows) == 30 and all(0 <= r < v["n"] for r in rows)

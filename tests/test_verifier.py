"""The product verifier (csrc/verify.cpp, host CPU) against an independent
restatement of the reference's verify_v1 (oracle/sezkp_oracle_py.py,
crates/sezkp-stark/src/v1/verify.rs:60-196, fri.rs:130-222, merkle.rs:243-280):
same verdict and same reason on honest proofs (accepted, or rejected by the
AIR boundary terms SURVEY 3C describes) and on tampered ones. CPU only: the
proofs come from the C oracle."""
import os

import pytest

from conftest import GOLDEN


def _product_verdict(product, blocks, root, proof):
    art = product.ProofArtifact("stark", root, proof, {})
    try:
        product.StarkV1.verify(art, blocks, root)
        return None
    except product.SezkpError as e:
        return str(e)


def _cases(product):
    out = []
    for f in ("ref_blocks.cbor", "riscv_blocks.cbor"):
        b = product.BlockSoA.from_cbor(open(os.path.join(GOLDEN, f), "rb").read())
        out.append((f, b))
    out.append(("synthetic_256", product.synthetic_blocks(256, 64, 2, 5)))
    # a trace whose blocks have zero-width boundary terms everywhere (no moves):
    # the AIR check holds on every row, so verify must accept
    import numpy as np
    T, tau = 128, 2
    z = np.zeros((T, tau), np.int8)
    out.append(("still_128", product.partition(np.zeros(T, np.int8), z, z.astype(np.uint8),
                                               z.astype(np.uint16), 32)))
    return out


def test_verifiers_agree_on_honest_proofs(product, oracle):
    import sezkp_oracle_py as V
    seen_accept = False
    for name, blocks in _cases(product):
        root = blocks.manifest_root()
        proof = oracle.prove_v1(blocks, root)
        want = V.verify_v1(proof, blocks.tau)
        got = _product_verdict(product, blocks, root, proof)
        assert (got is None) == (want is None), (name, got, want)
        if want is not None:
            assert want in got, (name, got, want)
        seen_accept |= want is None
    assert seen_accept


@pytest.mark.parametrize("what", ["col_path", "fri_path", "final", "row", "fri_root"])
def test_verifiers_agree_on_tampered_proofs(product, oracle, what):
    import sezkp_oracle_py as V
    T, tau = 128, 2
    import numpy as np
    z = np.zeros((T, tau), np.int8)
    blocks = product.partition(np.zeros(T, np.int8), z, z.astype(np.uint8), z.astype(np.uint16), 32)
    root = blocks.manifest_root()
    proof = bytearray(oracle.prove_v1(blocks, root))
    assert V.verify_v1(bytes(proof), tau) is None
    pf = V.parse_proof_v1(bytes(proof))
    # byte offsets from the layout (bincode, proof.rs:80-98)
    hdr = 24 + sum(8 + len(l) + 32 for l, _ in pf["col_roots"])
    logn = 7
    ob = 80 + 32 * logn                       # one opening
    qb = 16 + (9 * tau + 3) * ob              # one row query
    fr_off = hdr + 8 + 30 * qb                # FRI roots vector
    k = len(pf["fri_roots"]) - 1
    if what == "col_path":
        proof[hdr + 8 + 16 + 8 * 4 + 32 + 8] ^= 1      # first sibling of query 0's first opening
        want_kind = "chunked merkle path failed"
    elif what == "row":
        proof[hdr + 8] ^= 1                              # query 0's row
        want_kind = "AIR query row mismatch"
    elif what == "fri_root":
        proof[fr_off + 8 + 32 * 3] ^= 1                 # FRI root of layer 3 (changes the transcript)
        want_kind = "AIR query row mismatch"
    elif what == "final":
        proof[len(proof) - 40] ^= 1                      # final value
        want_kind = "final FRI value mismatch"
    else:
        fq0 = fr_off + 8 + 32 * (k + 1) + 8             # first FRI query record
        first_path = fq0 + 8 + 8 * (k + 1) + 8 + 8 + 8  # after positions, count k, value, path length
        proof[first_path] ^= 1
        want_kind = "FRI Merkle path failed at layer 0"
    want = V.verify_v1(bytes(proof), tau)
    got = _product_verdict(product, blocks, root, bytes(proof))
    assert want is not None and want_kind in want, want
    assert got is not None and want_kind in got, (got, want)

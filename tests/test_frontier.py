"""The streaming Frontier manifest root of the reference's .jsonl commit path
(crates/sezkp-merkle/src/lib.rs:167-208 Frontier, 259-295 commit_block_file,
302-337 verify_block_file_against_manifest), in the product: the C ABI, the
CLI's `commit` and prove/verify precheck, and the launcher's precheck (CPU).

The Frontier differs from the batch merkle_root at 7, 11, 13, 14, 15, 19, ...
leaves (the reference's own frontier/batch mismatch); the product
reproduces the reference's value, so `commit` on a .jsonl and on a .cbor file
with the same blocks gives different manifests, exactly as the reference does.
"""
import os
import subprocess

import pytest

from conftest import GOLDEN, PKG

CLI = os.path.join(PKG, "bin", "sezkp-cli")
# (T, steps per block) -> 7, 11 and 13 blocks (the ragged last block included)
SHAPES = [(4096, 600, 7), (4096, 373, 11), (4096, 316, 13)]


def _leaves(oracle, blocks) -> bytes:
    return b"".join(oracle.manifest_leaf_hash(blocks, k) for k in range(blocks.n_blocks))


def test_c_and_python_oracles_agree_on_frontier(oracle):
    """The two oracle restatements of Frontier agree for 0..40 leaves, equal the
    batch root at powers of two and differ from it at 7, 11, 13."""
    import hashlib
    import sezkp_oracle_py as PY
    leaves = [hashlib.sha256(bytes([i])).digest() for i in range(40)]
    for n in range(41):
        f = oracle.manifest_frontier_root(b"".join(leaves[:n]))
        assert f == PY.frontier_root(leaves[:n]), n
        batch = PY.tree_levels(leaves[:n])[-1][0] if n else b"\0" * 32
        if n & (n - 1) == 0:
            assert f == batch, n
        if n in (7, 11, 13, 14, 15, 19):
            assert f != batch, n


@pytest.mark.parametrize("T,b,nb", SHAPES)
def test_product_frontier_matches_oracle(product, oracle, T, b, nb):
    blocks = product.synthetic_blocks(T, b, 2, nb)
    assert blocks.n_blocks == nb
    leaves = _leaves(oracle, blocks)
    assert blocks.manifest_frontier_root() == oracle.manifest_frontier_root(leaves)
    assert blocks.manifest_root() == oracle.merkle_root(leaves) == oracle.manifest_root(blocks)
    assert blocks.manifest_frontier_root() != blocks.manifest_root()
    assert blocks.file_root("x.jsonl") == blocks.file_root("x.NDJSON") == blocks.manifest_frontier_root()
    assert blocks.file_root("x.cbor") == blocks.file_root("x.json") == blocks.manifest_root()
    # powers of two and the reference fixtures (8 blocks): the two roots agree
    for raw in ("ref_blocks.cbor", "riscv_blocks.cbor"):
        fb = product.BlockSoA.from_cbor(open(os.path.join(GOLDEN, raw), "rb").read())
        assert fb.manifest_frontier_root() == fb.manifest_root()


def _commit(path, out):
    r = subprocess.run([CLI, "commit", "--blocks", str(path), "--out", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return r.stdout


@pytest.mark.parametrize("T,b,nb", SHAPES)
def test_cli_commit_jsonl_writes_frontier_root(product, oracle, tmp_path, T, b, nb):
    """`sezkp-cli commit --blocks x.jsonl` writes the Frontier root (lib.rs:265-278);
    the same blocks as .cbor give the batch root (lib.rs:279-284)."""
    import cbor_min
    blocks = product.synthetic_blocks(T, b, 3, 100 + nb)
    leaves = _leaves(oracle, blocks)
    jl, cb = tmp_path / "b.jsonl", tmp_path / "b.cbor"
    jl.write_bytes(blocks.to_jsonl())
    cb.write_bytes(blocks.to_cbor())
    out = _commit(jl, tmp_path / "mj.cbor")
    man_j = cbor_min.loads((tmp_path / "mj.cbor").read_bytes())
    assert bytes(man_j["root"]) == oracle.manifest_frontier_root(leaves)
    assert man_j["n_leaves"] == nb and man_j["version"] == 1
    assert f"Committed {nb} leaves, root={bytes(man_j['root']).hex()}" in out
    _commit(cb, tmp_path / "mc.cbor")
    man_c = cbor_min.loads((tmp_path / "mc.cbor").read_bytes())
    assert bytes(man_c["root"]) == oracle.merkle_root(leaves)
    assert man_c["root"] != man_j["root"]
    # .ndjson is the same path; a JSON manifest carries the same root
    nd = tmp_path / "b.ndjson"
    nd.write_bytes(blocks.to_jsonl())
    _commit(nd, tmp_path / "mn.json")
    import json
    assert bytes(json.loads((tmp_path / "mn.json").read_text())["root"]) == bytes(man_j["root"])


def _prove(blocks, manifest, out, *extra):
    return subprocess.run([CLI, "prove", "--backend", "stark", "--blocks", str(blocks), "--manifest", str(manifest),
                           "--out", str(out), *extra], capture_output=True, text=True)


def test_cli_precheck_uses_frontier_for_jsonl(product, tmp_path):
    """prove on a real .jsonl file: the precheck runs first with the Frontier
    root (main.rs:454-457 -> lib.rs:309-331). A Frontier manifest passes it and
    the stark path then refuses the extension (io.rs:78-88, main.rs:509-512); a
    batch-root manifest fails the precheck. A .cbor file is checked against the
    batch root, so the Frontier manifest of 7 blocks does not match it."""
    blocks = product.synthetic_blocks(4096, 600, 2, 7)
    jl, cb = tmp_path / "b.jsonl", tmp_path / "b.cbor"
    jl.write_bytes(blocks.to_jsonl())
    cb.write_bytes(blocks.to_cbor())
    _commit(jl, tmp_path / "mj.cbor")
    _commit(cb, tmp_path / "mc.cbor")
    r = _prove(jl, tmp_path / "mj.cbor", tmp_path / "p.cbor")
    assert r.returncode != 0 and "unsupported blocks extension: jsonl" in r.stderr, r.stderr
    r = _prove(jl, tmp_path / "mc.cbor", tmp_path / "p.cbor")
    assert r.returncode != 0 and "blocks/manifest mismatch: root mismatch" in r.stderr, r.stderr
    r = _prove(cb, tmp_path / "mj.cbor", tmp_path / "p.cbor")
    assert r.returncode != 0 and "blocks/manifest mismatch: root mismatch" in r.stderr, r.stderr
    # --assume-committed skips the precheck: the extension rule still holds
    r = _prove(jl, tmp_path / "mj.cbor", tmp_path / "p.cbor", "--assume-committed")
    assert r.returncode != 0 and "unsupported blocks extension: jsonl" in r.stderr, r.stderr
    # a manifest with the right root but another leaf count
    import cbor_min  # noqa: F401
    from sezkp_amd.launch import _read_manifest
    root, n = _read_manifest(str(tmp_path / "mj.cbor"))
    assert n == 7 and root == blocks.manifest_frontier_root()


def test_launcher_precheck_frontier(product, tmp_path):
    """The launcher's precheck (launch._precheck) follows the same rule."""
    from sezkp_amd.launch import _precheck, _read_manifest
    blocks = product.synthetic_blocks(4096, 600, 2, 7)
    jl = tmp_path / "b.jsonl"
    jl.write_bytes(blocks.to_jsonl())
    _commit(jl, tmp_path / "mj.cbor")
    root, n = _read_manifest(str(tmp_path / "mj.cbor"))
    loaded = product.BlockSoA.from_file(str(jl))
    _precheck(loaded, str(jl), root, n)                       # accepted
    with pytest.raises(RuntimeError, match="root mismatch"):
        _precheck(loaded, str(tmp_path / "b.cbor"), root, n)  # batch rule for .cbor
    with pytest.raises(RuntimeError, match="leaf count mismatch"):
        _precheck(loaded, str(jl), root, n + 1)

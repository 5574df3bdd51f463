"""Regenerate tests/golden/v1_proofs.json (committed; run from the repo root).

The reference publishes no v1 proof, so the v1 golden digests
are produced by the two independent CPU restatements (oracle/sezkp_oracle.c
and oracle/sezkp_oracle_py.py), which must agree byte for byte before a
digest is recorded. Inputs are the reference's committed block files (copied
here unchanged) and one synthetic trace.
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "streaming-zero-knowledge-proofs_amd")]
import cbor_min  # noqa: E402
import oracle_ctypes as O  # noqa: E402
import sezkp_oracle_py as PY  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
out = {}
for name, (b, m) in {"root_blocks": ("ref_blocks.cbor", "ref_manifest.cbor"),
                     "minimal_riscv": ("riscv_blocks.cbor", "riscv_manifest.cbor")}.items():
    dicts = cbor_min.loads(open(os.path.join(G, b), "rb").read())
    mroot = bytes(cbor_min.loads(open(os.path.join(G, m), "rb").read())["root"])
    c = O.prove_v1(O.Blocks(dicts), mroot)
    p = PY.prove_v1(dicts, mroot)
    assert c == p, f"oracles disagree on {name}"
    out[name] = {"blocks": b, "manifest_root": mroot.hex(), "proof_len": len(c),
                 "proof_sha256": hashlib.sha256(c).hexdigest(), "head_hex": c[:96].hex()}
json.dump(out, open(os.path.join(G, "v1_proofs.json"), "w"), indent=2, sort_keys=True)
print(json.dumps(out, indent=2))

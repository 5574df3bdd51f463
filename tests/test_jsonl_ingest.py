"""Block ingest formats: JSON Lines reader/writer of the
reference's io_jsonl.rs and the manifest decoder, against the reference's
own committed block files (CPU only)."""
import json
import os

import numpy as np
import pytest

from conftest import ROOT

FIX = [("tests/golden/ref_blocks.cbor", "tests/golden/ref_manifest.cbor"),
       ("tests/golden/riscv_blocks.cbor", "tests/golden/riscv_manifest.cbor")]


def _fields(product):
    from sezkp_amd._lib import VIEW_FIELDS
    return [f for f, _ in VIEW_FIELDS]


@pytest.mark.parametrize("blocks_path,manifest_path", FIX)
def test_jsonl_matches_cbor_and_serde_layout(product, blocks_path, manifest_path):
    import cbor_min
    raw = open(os.path.join(ROOT, blocks_path), "rb").read()
    b_cbor = product.BlockSoA.from_cbor(raw)
    # serde_json compact layout of the same Vec<BlockSummary>, one object per line
    want = b"".join(json.dumps(x, separators=(",", ":")).encode() + b"\n" for x in cbor_min.loads(raw))
    assert b_cbor.to_jsonl() == want  # write_block_summaries_jsonl byte-for-byte
    for data in (want, want.replace(b"\n", b"\r\n"), want.rstrip(b"\n")):
        b = product.BlockSoA.from_jsonl(data)
        for f in _fields(product):
            np.testing.assert_array_equal(getattr(b, f), getattr(b_cbor, f))
        assert b.tau == b_cbor.tau
    from sezkp_amd.launch import _read_manifest
    assert _read_manifest(os.path.join(ROOT, manifest_path)) == (b_cbor.manifest_root(), b_cbor.n_blocks)


def test_jsonl_errors_name_the_line(product):
    good = product.synthetic_blocks(64, 16, 2, 1).to_jsonl().split(b"\n")
    with pytest.raises(product.SezkpError, match="line 3: empty line"):
        product.BlockSoA.from_jsonl(b"\n".join(good[:2] + [b""] + good[2:]))
    with pytest.raises(product.SezkpError, match="line 2"):
        product.BlockSoA.from_jsonl(good[0] + b"\n{\"version\": 1\n")


def test_jsonl_synthetic_roundtrip(product):
    b = product.synthetic_blocks(1 << 12, 100, 3, 5)
    r = product.BlockSoA.from_jsonl(b.to_jsonl())
    assert r.manifest_root() == b.manifest_root()
    for f in _fields(product):
        np.testing.assert_array_equal(getattr(r, f), getattr(b, f))


def test_jsonl_parallel_ranges_match_sequential(product, monkeypatch):
    """The reader cuts the file at line ends into one range per host thread
    (>= 4 MB each) and concatenates the ranges in order: the same blocks as
    one thread, and an error still names the first failing line of the file."""
    b = product.synthetic_blocks(1 << 18, 100, 4, 7)  # ~30 MB of JSONL, ragged last block
    data = b.to_jsonl()
    assert len(data) > 6 * (4 << 20)
    outs = []
    for threads in ("1", "3", "6", "64"):
        monkeypatch.setenv("SEZKP_HOST_THREADS", threads)
        outs.append(product.BlockSoA.from_jsonl(data))
    for r in outs:
        assert r.tau == b.tau
        for f in _fields(product):
            np.testing.assert_array_equal(getattr(r, f), getattr(b, f))
    lines = data.split(b"\n")
    n = len(lines) - 1  # trailing newline
    bad = list(lines)
    bad[n - 2] = b"{\"version\": x}"   # in the last range
    bad[n // 3] = b""                   # in an earlier range: reported first
    monkeypatch.setenv("SEZKP_HOST_THREADS", "6")
    with pytest.raises(product.SezkpError, match=f"line {n // 3 + 1}: empty line"):
        product.BlockSoA.from_jsonl(b"\n".join(bad))

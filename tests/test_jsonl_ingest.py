"""Block ingest formats: JSON Lines reader/writer of the
reference's io_jsonl.rs and the manifest decoder, against the reference's
own committed block files (CPU only)."""
import json
import os

import numpy as np
import pytest

from conftest import ROOT, free_port

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


# ------------------------------------------------ sliced ingest (config 5)
def _sliced_worker(rank, world, port, path, q):
    import hashlib
    import os
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sezkp_amd.ingest import TorchComm, sliced_ingest
        r = sliced_ingest(path, rank, world, TorchComm(), None)
        b = r["blocks"]
        dig = hashlib.sha256(b.input_mv.tobytes() + b.mv.tobytes() + b.has_write.tobytes() + b.wsym.tobytes())
        q.put((rank, r["row0"], r["nrows"], dig.hexdigest(), r["root"], int(b.n_blocks), r["seconds"]["total"]))
    except Exception as e:
        q.put((rank, f"ERR {type(e).__name__}: {e}", 0, "", b"", 0, 0.0))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,log_t", [(2, 14), (4, 14), (8, 15)])
def test_sliced_ingest_matches_full_decode(product, tmp_path, world, log_t):
    """Each rank reads 1/P of the JSONL lines' metadata, the metadata and the
    leaf hashes are allgathered (gloo), rank 0 reduces the Frontier root, and
    each rank decodes only the lines over its rows: ragged blocks (333 steps)
    cross every rank boundary, and a rank's rows reach into its neighbours'
    byte ranges (those lines are decoded again). Every rank's
    step slice equals the full decode's rows [row0, row0 + nrows), and the
    root is the file's Frontier root."""
    import hashlib
    import torch.multiprocessing as mp
    import numpy as np
    from sezkp_amd.blocks import shard_rows
    blocks = product.synthetic_blocks(1 << log_t, 333, 3, 11)
    path = tmp_path / "b.jsonl"
    path.write_bytes(blocks.to_jsonl())
    full = product.BlockSoA.from_file(str(path))
    port = free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_sliced_worker, args=(r, world, port, str(path), q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    tau = full.tau
    for rank, row0, nrows, dig, root, nb, _ in res:
        assert not str(row0).startswith("ERR"), row0
        assert (row0, nrows) == shard_rows(full.step_start, rank, world)
        want = hashlib.sha256(full.input_mv[row0:row0 + nrows].tobytes() +
                              full.mv[row0 * tau:(row0 + nrows) * tau].tobytes() +
                              full.has_write[row0 * tau:(row0 + nrows) * tau].tobytes() +
                              full.wsym[row0 * tau:(row0 + nrows) * tau].tobytes()).hexdigest()
        assert dig == want and nb == full.n_blocks and root == full.manifest_frontier_root(), rank
    # the row slices cover the trace, overlapping only in boundary blocks
    assert res[0][1] == 0 and res[-1][1] + res[-1][2] == full.n_rows
    assert all(res[i][1] <= res[i + 1][1] <= res[i][1] + res[i][2] for i in range(world - 1))


def test_jsonl_meta_ranges_cover_every_line_once(product):
    """The metadata pass's byte ranges [len g/P, len (g+1)/P) cut at line ends
    cover each line once for any P (including ranges with no line start), and
    the leaf hashes give both manifest roots."""
    import numpy as np
    from sezkp_amd.blocks import BlockSoA, merkle_root_of_leaves
    blocks = product.synthetic_blocks(3000, 97, 2, 3)
    jl = blocks.to_jsonl()
    full = BlockSoA.from_jsonl(jl)
    for P in (1, 2, 3, 7, 16, 64):
        parts = [BlockSoA.from_jsonl_meta(jl, len(jl) * g // P, len(jl) * (g + 1) // P) for g in range(P)]
        allm = BlockSoA.concat_meta([p[0] for p in parts])
        offs = np.concatenate([p[1] for p in parts])
        assert allm.n_blocks == full.n_blocks and np.array_equal(allm.step_start, full.step_start), P
        assert np.array_equal(offs, np.sort(offs)) and len(set(offs.tolist())) == full.n_blocks
        leaves = b"".join(p[0].leaf_hashes() for p in parts)
        assert merkle_root_of_leaves(leaves, False) == full.manifest_root()
        assert merkle_root_of_leaves(leaves, True) == full.manifest_frontier_root()
        # the full decode of a run of lines from the offsets
        a, b = 3, 9
        sl = BlockSoA.from_jsonl_range(jl, int(offs[a]), int(offs[b]))
        assert np.array_equal(sl.block_id, full.block_id[a:b])


def test_jsonl_noncanonical_forms_decode_alike(product):
    """The decoder's fast paths read only the canonical step encoding
    (serde's field order, no white space); spaced, reordered and extended
    forms take the general parser and give the same blocks, in the full and
    the metadata decode; out-of-range values are errors on both paths."""
    import json as js
    from sezkp_amd.blocks import BlockSoA
    b = product.synthetic_blocks(2000, 61, 3, 9)
    canon = b.to_jsonl()
    objs = [js.loads(x) for x in canon.split(b"\n") if x]

    def dump(os_, **kw):
        return b"".join(js.dumps(o, **kw).encode() + b"\n" for o in os_)

    def remap(fn):
        out = []
        for o in objs:
            o = js.loads(js.dumps(o))
            o["movement_log"]["steps"] = [fn(s) for s in o["movement_log"]["steps"]]
            out.append(o)
        return out

    variants = [
        dump(objs),  # ", " and ": " separators
        dump(remap(lambda s: {"input_mv": s["input_mv"],
                              "tapes": [{"mv": t["mv"], "write": t["write"]} for t in s["tapes"]]}),
             separators=(",", ":")),
        dump(remap(lambda s: {"tapes": s["tapes"], "input_mv": s["input_mv"]}), separators=(",", ":")),
        dump(remap(lambda s: {"input_mv": s["input_mv"], "tapes": [dict(t, x=[1, {"y": "]"}]) for t in s["tapes"]],
                              "z": "}"}), separators=(",", ":")),
        # escaped quotes and brackets inside strings: the step counter's SIMD
        # scan falls back to the exact byte scan
        dump(remap(lambda s: {"input_mv": s["input_mv"], "tapes": s["tapes"], "z": 'a\\"],{"\\\\'}),
             separators=(",", ":")),
    ]
    for v in variants:
        assert v != canon
        r = BlockSoA.from_jsonl(v)
        for f in _fields(product):
            np.testing.assert_array_equal(getattr(r, f), getattr(b, f))
        m, _ = BlockSoA.from_jsonl_meta(v, 0, len(v))
        assert np.array_equal(m.step_start, b.step_start)
    bad_mv = canon.replace(b'"mv":-1}', b'"mv":200}', 1)
    bad_w = canon.replace(b'{"write":', b'{"write":70000', 1)
    with pytest.raises(product.SezkpError, match="mv out of i8 range"):
        BlockSoA.from_jsonl(bad_mv)
    with pytest.raises(product.SezkpError):
        BlockSoA.from_jsonl(bad_w)


def test_jsonl_meta_threads_match_one_thread(product, monkeypatch):
    """The metadata pass cuts its byte range at line ends into one range per
    host thread: the same blocks and offsets as one thread, and an error
    names its line."""
    from sezkp_amd.blocks import BlockSoA
    b = product.synthetic_blocks(1 << 18, 100, 4, 7)
    data = b.to_jsonl()
    outs = []
    for threads in ("1", "5"):
        monkeypatch.setenv("SEZKP_HOST_THREADS", threads)
        outs.append(BlockSoA.from_jsonl_meta(data, len(data) // 7, len(data)))
    (m1, o1), (m5, o5) = outs
    assert np.array_equal(o1, o5) and np.array_equal(m1.step_start, m5.step_start)
    assert np.array_equal(m1.block_id, m5.block_id) and m1.tau == m5.tau == b.tau
    lines = data.split(b"\n")
    lines[len(lines) * 3 // 4] = b""
    with pytest.raises(product.SezkpError, match="empty line"):
        BlockSoA.from_jsonl_meta(b"\n".join(lines), 0, len(data))

"""Minimal CBOR codec — ORACLE-SIDE test infrastructure.

Decodes the reference's committed fixtures (serde/ciborium 0.2.2 encoding of
`Vec<BlockSummary>`, `CommitManifest`, `ProofArtifact`;
crates/sezkp-core/src/io.rs:57-75,176-183) and encodes `ProofArtifact`
envelopes the way ciborium does (struct -> map with text keys in declaration
order, `[u8; N]`/`Vec<u8>` -> arrays of uints, minimal-length heads).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline use this.
"""
from __future__ import annotations

import struct


class CborError(ValueError):
    pass


def _head(buf: bytes, i: int):
    if i >= len(buf):
        raise CborError("truncated CBOR")
    ib = buf[i]
    major, info = ib >> 5, ib & 31
    i += 1
    if info < 24:
        return major, info, i
    if info == 24:
        return major, buf[i], i + 1
    if info == 25:
        return major, struct.unpack(">H", buf[i:i + 2])[0], i + 2
    if info == 26:
        return major, struct.unpack(">I", buf[i:i + 4])[0], i + 4
    if info == 27:
        return major, struct.unpack(">Q", buf[i:i + 8])[0], i + 8
    if info == 31:
        return major, None, i
    raise CborError(f"bad additional info {info}")


def _dec(buf: bytes, i: int):
    major, val, i = _head(buf, i)
    if major == 0:
        return val, i
    if major == 1:
        return -1 - val, i
    if major == 2:
        return bytes(buf[i:i + val]), i + val
    if major == 3:
        return buf[i:i + val].decode("utf-8"), i + val
    if major == 4:
        out = []
        if val is None:
            while buf[i] != 0xFF:
                v, i = _dec(buf, i)
                out.append(v)
            return out, i + 1
        for _ in range(val):
            v, i = _dec(buf, i)
            out.append(v)
        return out, i
    if major == 5:
        out = {}
        n = val
        while (n is None and buf[i] != 0xFF) or (n is not None and len(out) < n):
            k, i = _dec(buf, i)
            v, i = _dec(buf, i)
            out[k] = v
        if n is None:
            i += 1
        return out, i
    if major == 6:
        return _dec(buf, i)
    if major == 7:
        if val == 20:
            return False, i
        if val == 21:
            return True, i
        if val == 22 or val == 23:
            return None, i
        raise CborError(f"unsupported simple/float {val}")
    raise CborError("unreachable")


def loads(buf: bytes):
    v, i = _dec(bytes(buf), 0)
    if i != len(buf):
        raise CborError(f"trailing bytes at {i}/{len(buf)}")
    return v


def _enc_head(major: int, val: int) -> bytes:
    if val < 24:
        return bytes([(major << 5) | val])
    if val < 1 << 8:
        return bytes([(major << 5) | 24, val])
    if val < 1 << 16:
        return bytes([(major << 5) | 25]) + struct.pack(">H", val)
    if val < 1 << 32:
        return bytes([(major << 5) | 26]) + struct.pack(">I", val)
    return bytes([(major << 5) | 27]) + struct.pack(">Q", val)


def dumps(v) -> bytes:
    """Encode with ciborium's conventions. bytes/bytearray encode as ARRAYS of
    uints (serde's default for Vec<u8>/[u8;N]); dict keys keep insertion order."""
    if v is None:
        return b"\xf6"
    if v is True:
        return b"\xf5"
    if v is False:
        return b"\xf4"
    if isinstance(v, int):
        return _enc_head(0, v) if v >= 0 else _enc_head(1, -1 - v)
    if isinstance(v, str):
        b = v.encode("utf-8")
        return _enc_head(3, len(b)) + b
    if isinstance(v, (bytes, bytearray)):
        out = bytearray(_enc_head(4, len(v)))
        for x in v:
            out += _enc_head(0, x)
        return bytes(out)
    if isinstance(v, (list, tuple)):
        return _enc_head(4, len(v)) + b"".join(dumps(x) for x in v)
    if isinstance(v, dict):
        return _enc_head(5, len(v)) + b"".join(dumps(k) + dumps(x) for k, x in v.items())
    raise TypeError(type(v))


def proof_artifact_cbor(backend: str, manifest_root: bytes, proof_bytes: bytes, meta: dict) -> bytes:
    """ProofArtifact (crates/sezkp-core/src/artifact.rs:55-68) as ciborium
    writes it: map{backend, manifest_root, proof_bytes, meta}; meta keys sorted
    (serde_json Map = BTreeMap, no preserve_order)."""
    return dumps({
        "backend": backend,
        "manifest_root": bytes(manifest_root),
        "proof_bytes": bytes(proof_bytes),
        "meta": {k: meta[k] for k in sorted(meta)},
    })

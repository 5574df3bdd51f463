"""ctypes binding of the C oracle — TEST INFRASTRUCTURE ONLY.

Loads oracle/_build/libsezkp_oracle.so (built by oracle/Makefile). Used by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker / CPU baseline; the product path never imports this module.

`Blocks` is the oracle-side struct-of-arrays view of `Vec<BlockSummary>`
(crates/sezkp-core/src/types.rs:116-151). Any object exposing the same numpy
attributes (e.g. the product's `sezkp_amd.blocks.BlockSoA`) is accepted.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libsezkp_oracle.so")

_FIELDS = [
    ("version", np.uint16), ("block_id", np.uint32), ("step_lo", np.uint64), ("step_hi", np.uint64),
    ("ctrl_in", np.uint16), ("ctrl_out", np.uint16), ("in_head_in", np.int64), ("in_head_out", np.int64),
    ("win_left", np.int64), ("win_right", np.int64), ("off_in", np.uint32), ("off_out", np.uint32),
    ("step_start", np.uint64), ("input_mv", np.int8), ("mv", np.int8), ("has_write", np.uint8),
    ("wsym", np.uint16),
]


class _OrcBlocks(C.Structure):
    _fields_ = [("n_blocks", C.c_uint32), ("tau", C.c_uint32)] + [(f, C.c_void_p) for f, _ in _FIELDS]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    global _lib
    _lib = None


def use_mt(threads: int) -> int:
    """Switch to the OpenMP build of the same source (multi-core compute-once
    CPU baseline); returns the thread count in use."""
    global LIB_PATH, _lib
    LIB_PATH = os.path.join(HERE, "_build", "libsezkp_oracle_mt.so")
    _lib = None
    L = lib()
    L.orc_set_threads.restype = C.c_int
    L.orc_set_threads.argtypes = [C.c_int]
    return L.orc_set_threads(threads)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_gl_mul.restype = C.c_uint64
        L.orc_gl_mul.argtypes = [C.c_uint64, C.c_uint64]
        L.orc_gl_inv.restype = C.c_uint64
        L.orc_gl_inv.argtypes = [C.c_uint64]
        L.orc_gl_root_2exp.restype = C.c_uint64
        L.orc_gl_root_2exp.argtypes = [C.c_uint32]
        L.orc_ntt_forward.argtypes = [C.c_void_p, C.c_size_t]
        L.orc_ntt_inverse.argtypes = [C.c_void_p, C.c_size_t]
        L.orc_coset_lde.argtypes = [C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint64, C.c_void_p]
        L.orc_det_vec.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        L.orc_lde_deep.argtypes = [C.c_void_p, C.c_size_t, C.c_uint, C.c_uint64, C.c_void_p]
        L.orc_blake3.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.orc_tr_new.restype = C.c_void_p
        L.orc_tr_new.argtypes = [C.c_char_p]
        L.orc_tr_free.argtypes = [C.c_void_p]
        L.orc_tr_absorb.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_size_t]
        L.orc_tr_absorb_u64.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64]
        L.orc_tr_challenge.argtypes = [C.c_void_p, C.c_char_p, C.c_void_p, C.c_size_t]
        L.orc_merkle_root.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p]
        L.orc_merkle_nodes.restype = C.c_size_t
        L.orc_merkle_nodes.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p]
        L.orc_merkle_open.restype = C.c_size_t
        L.orc_merkle_open.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p]
        L.orc_lde_deep_shift.argtypes = [C.c_void_p, C.c_size_t, C.c_uint, C.c_uint64, C.c_uint64, C.c_void_p]
        L.orc_manifest_leaf_hash.argtypes = [C.POINTER(_OrcBlocks), C.c_uint32, C.c_void_p]
        L.orc_manifest_root.argtypes = [C.POINTER(_OrcBlocks), C.c_void_p]
        L.orc_manifest_frontier_root.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p]
        L.orc_hash_leaf_u64.argtypes = [C.c_uint64, C.c_void_p]
        L.orc_hash_leaf_labeled.argtypes = [C.c_uint64, C.c_char_p, C.c_void_p]
        L.orc_v0_proof.argtypes = [C.POINTER(_OrcBlocks), C.c_char_p, C.c_void_p, C.POINTER(C.c_uint64)]
        L.orc_prove_v1.argtypes = [C.POINTER(_OrcBlocks), C.c_char_p, C.c_int, C.POINTER(C.c_void_p),
                                   C.POINTER(C.c_size_t), C.c_char_p, C.c_size_t]
        L.orc_prove_v1_debug.argtypes = [C.POINTER(_OrcBlocks), C.c_char_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_char_p, C.c_size_t]
        L.orc_free.argtypes = [C.c_void_p]
        L.orc_time_lde_pass.restype = C.c_double
        L.orc_time_lde_pass.argtypes = [C.POINTER(_OrcBlocks), C.c_char_p]
        _lib = L
    return _lib


# ----------------------------------------------------------------- blocks
class Blocks:
    """SoA view of Vec<BlockSummary> built from decoded CBOR/JSON dicts."""

    def __init__(self, dicts: list[dict]):
        tau = len(dicts[0]["windows"]) if dicts else 0
        self.tau = tau
        self.n_blocks = len(dicts)
        g = lambda k, dt: np.array([d[k] for d in dicts], dtype=dt)
        self.version = g("version", np.uint16)
        self.block_id = g("block_id", np.uint32)
        self.step_lo = g("step_lo", np.uint64)
        self.step_hi = g("step_hi", np.uint64)
        self.ctrl_in = g("ctrl_in", np.uint16)
        self.ctrl_out = g("ctrl_out", np.uint16)
        self.in_head_in = g("in_head_in", np.int64)
        self.in_head_out = g("in_head_out", np.int64)
        self.win_left = np.array([w["left"] for d in dicts for w in d["windows"]], dtype=np.int64)
        self.win_right = np.array([w["right"] for d in dicts for w in d["windows"]], dtype=np.int64)
        self.off_in = np.array([x for d in dicts for x in d["head_in_offsets"]], dtype=np.uint32)
        self.off_out = np.array([x for d in dicts for x in d["head_out_offsets"]], dtype=np.uint32)
        counts = [len(d["movement_log"]["steps"]) for d in dicts]
        self.step_start = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
        steps = [s for d in dicts for s in d["movement_log"]["steps"]]
        self.input_mv = np.array([s["input_mv"] for s in steps], dtype=np.int8)
        ops = [op for s in steps for op in s["tapes"]]
        self.mv = np.array([op["mv"] for op in ops], dtype=np.int8)
        self.has_write = np.array([op["write"] is not None for op in ops], dtype=np.uint8)
        self.wsym = np.array([op["write"] or 0 for op in ops], dtype=np.uint16)
        for d in dicts:
            for k in ("windows", "head_in_offsets", "head_out_offsets"):
                if len(d[k]) != tau:
                    raise ValueError(f"block {d['block_id']}: {k} has {len(d[k])} entries, tau={tau}")
            for s in d["movement_log"]["steps"]:
                if len(s["tapes"]) != tau:
                    raise ValueError("step with tapes.len() != tau")


def _struct(b) -> tuple[_OrcBlocks, list]:
    keep = []
    s = _OrcBlocks()
    s.n_blocks = int(b.n_blocks)
    s.tau = int(b.tau)
    for f, dt in _FIELDS:
        a = np.ascontiguousarray(getattr(b, f), dtype=dt)
        if a.size == 0:
            a = np.zeros(1, dtype=dt)
        keep.append(a)
        setattr(s, f, a.ctypes.data)
    return s, keep


# ---------------------------------------------------------------- wrappers
def blake3(data: bytes, out_len: int = 32) -> bytes:
    out = C.create_string_buffer(out_len)
    lib().orc_blake3(data, len(data), out, out_len)
    return out.raw


def ntt_forward(a: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(a, dtype=np.uint64).copy()
    lib().orc_ntt_forward(x.ctypes.data, x.size)
    return x


def ntt_inverse(a: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(a, dtype=np.uint64).copy()
    lib().orc_ntt_inverse(x.ctypes.data, x.size)
    return x


def coset_lde(coeffs: np.ndarray, k_log2: int, shift: int) -> np.ndarray:
    c = np.ascontiguousarray(coeffs, dtype=np.uint64)
    out = np.zeros(1 << k_log2, dtype=np.uint64)
    lib().orc_coset_lde(c.ctypes.data, c.size, k_log2, shift, out.ctypes.data)
    return out


def det_vec(n: int, seed: int) -> np.ndarray:
    out = np.zeros(n, dtype=np.uint64)
    lib().orc_det_vec(out.ctypes.data, n, seed)
    return out


def lde_deep(base: np.ndarray, blow_log2: int, z: int) -> np.ndarray:
    b = np.ascontiguousarray(base, dtype=np.uint64)
    out = np.zeros(b.size << blow_log2, dtype=np.uint64)
    lib().orc_lde_deep(b.ctypes.data, b.size, blow_log2, z, out.ctypes.data)
    return out


def lde_deep_shift(base: np.ndarray, blow_log2: int, shift: int, z: int) -> np.ndarray:
    """lde.rs:42-97 with the coset shift as a parameter."""
    b = np.ascontiguousarray(base, dtype=np.uint64)
    out = np.zeros(b.size << blow_log2, dtype=np.uint64)
    lib().orc_lde_deep_shift(b.ctypes.data, b.size, blow_log2, shift, z, out.ctypes.data)
    return out


def merkle_nodes(leaves: bytes) -> bytes:
    """MerkleTree::from_leaves (merkle.rs:46-71): every level, bottom -> top."""
    n = len(leaves) // 32
    cnt = lib().orc_merkle_nodes(leaves, n, None)
    out = C.create_string_buffer(32 * cnt)
    lib().orc_merkle_nodes(leaves, n, out)
    return out.raw


def merkle_open(leaves: bytes, idx) -> list:
    """MerkleTree::open (merkle.rs:80-108) per index: the sibling digests."""
    n = len(leaves) // 32
    ix = np.ascontiguousarray(idx, dtype=np.uint64)
    depth = 0
    m = max(n, 1)
    while m > 1:
        m = (m + 1) // 2
        depth += 1
    out = C.create_string_buffer(32 * depth * max(ix.size, 1))
    lib().orc_merkle_open(leaves, n, ix.ctypes.data, ix.size, out)
    raw = out.raw
    return [[raw[32 * (depth * i + l):32 * (depth * i + l + 1)] for l in range(depth)] for i in range(ix.size)]


def merkle_root(leaves: bytes) -> bytes:
    out = C.create_string_buffer(32)
    lib().orc_merkle_root(leaves, len(leaves) // 32, out)
    return out.raw


def hash_leaf_u64(v: int) -> bytes:
    out = C.create_string_buffer(32)
    lib().orc_hash_leaf_u64(v, out)
    return out.raw


def hash_leaf_labeled(v: int, label: str) -> bytes:
    out = C.create_string_buffer(32)
    lib().orc_hash_leaf_labeled(v, label.encode(), out)
    return out.raw


def manifest_leaf_hash(b, k: int) -> bytes:
    s, keep = _struct(b)
    out = C.create_string_buffer(32)
    lib().orc_manifest_leaf_hash(C.byref(s), k, out)
    return out.raw


def manifest_root(b) -> bytes:
    s, keep = _struct(b)
    out = C.create_string_buffer(32)
    lib().orc_manifest_root(C.byref(s), out)
    return out.raw


def manifest_frontier_root(leaves: bytes) -> bytes:
    out = C.create_string_buffer(32)
    lib().orc_manifest_frontier_root(leaves, len(leaves) // 32, out)
    return out.raw


def v0_proof(b, manifest_root_: bytes) -> tuple[bytes, int]:
    s, keep = _struct(b)
    out = C.create_string_buffer(64)
    nr = C.c_uint64(0)
    lib().orc_v0_proof(C.byref(s), manifest_root_, out, C.byref(nr))
    return out.raw, nr.value


class OracleError(RuntimeError):
    pass


def prove_v1(b, manifest_root_: bytes, mode: int = 0) -> bytes:
    s, keep = _struct(b)
    p = C.c_void_p()
    n = C.c_size_t()
    err = C.create_string_buffer(512)
    rc = lib().orc_prove_v1(C.byref(s), manifest_root_, mode, C.byref(p), C.byref(n), err, 512)
    if rc != 0:
        raise OracleError(err.value.decode())
    out = C.string_at(p, n.value)
    lib().orc_free(p)
    return out


def prove_v1_debug(b, manifest_root_: bytes):
    s, keep = _struct(b)
    n = int(b.step_start[-1]) if b.n_blocks else 0
    N = 8 * n
    ncols = 3 + 7 * int(b.tau)
    col_roots = C.create_string_buffer(32 * ncols)
    base = np.zeros(max(n, 1), dtype=np.uint64)
    lde = np.zeros(max(N, 1), dtype=np.uint64)
    root0 = C.create_string_buffer(32)
    err = C.create_string_buffer(512)
    rc = lib().orc_prove_v1_debug(C.byref(s), manifest_root_, col_roots, base.ctypes.data, lde.ctypes.data,
                                  root0, err, 512)
    if rc != 0:
        raise OracleError(err.value.decode())
    return {"col_roots": [col_roots.raw[32 * i:32 * i + 32] for i in range(ncols)],
            "base_evals": base[:n], "lde": lde[:N], "root0": root0.raw}


def time_lde_pass(b, manifest_root_: bytes) -> float:
    s, keep = _struct(b)
    return lib().orc_time_lde_pass(C.byref(s), manifest_root_)

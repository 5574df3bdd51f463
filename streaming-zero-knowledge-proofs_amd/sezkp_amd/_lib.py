"""ctypes loader for the MI355X C ABI (include/sezkp_stark.h).

The product path has no CPU fallback: if lib/libsezkp_stark.so is missing or
fails to load, importing this module raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_ROOT, "lib", "libsezkp_stark.so")

SEZKP_OK = 0
SEZKP_E_INVALID = -1
SEZKP_E_DEVICE = -2
SEZKP_E_NOMEM = -3
SEZKP_E_DECODE = -4
SEZKP_E_VERIFY = -5
SEZKP_FLAG_STREAMING = 1
ABI_VERSION = 4  # include/sezkp_stark.h SEZKP_ABI_VERSION: the layouts this module binds

# every symbol include/sezkp_stark.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "sezkp_abi_version", "sezkp_version", "sezkp_buf_free", "sezkp_stark_v1_prove",
    "sezkp_stark_v1_prove_artifact_cbor", "sezkp_stark_v1_verify", "sezkp_ctx_create", "sezkp_ctx_destroy",
    "sezkp_ctx_upload", "sezkp_ctx_prove", "sezkp_ctx_stage_times", "sezkp_ctx_stream", "sezkp_gl_ntt",
    "sezkp_gl_coset_lde_deep", "sezkp_fri_fold_commit", "sezkp_merkle_root_u64", "sezkp_manifest_root",
    "sezkp_blocks_decode_cbor", "sezkp_blocks_view", "sezkp_blocks_free", "sezkp_blake3",
    "sezkp_comm_unique_id", "sezkp_ctx_create_sharded", "sezkp_ctx_create_sharded_host", "sezkp_ctx_prove_borrow",
    "sezkp_blocks_decode_jsonl", "sezkp_blocks_encode_jsonl", "sezkp_manifest_decode", "sezkp_ctx_dist_ntt",
    "sezkp_blocks_encode_cbor", "sezkp_simulate_trace", "sezkp_simulate_blocks",
    "sezkp_ctx_prove_async", "sezkp_ctx_wait", "sezkp_ctx_stage", "sezkp_host_register", "sezkp_host_unregister",
    "sezkp_fri_fold", "sezkp_blake3_leaves_u64", "sezkp_blake3_leaves_labeled", "sezkp_merkle_node_count",
    "sezkp_merkle_build", "sezkp_merkle_paths", "sezkp_manifest_frontier_root", "sezkp_ctx_comm_stats",
    "sezkp_fs_xof", "sezkp_ctx_upload_rows", "sezkp_shard_rows", "sezkp_blocks_decode_jsonl_meta",
    "sezkp_blocks_line_offsets", "sezkp_manifest_leaf_hashes", "sezkp_merkle_root_of_leaves",
    "sezkp_ctx_create_sharded_solo", "sezkp_blocks_decode_jsonl_lines",
]


class CommStat(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("bytes", C.c_uint64), ("ms", C.c_double)]


class SezkpError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class Buf(C.Structure):
    _fields_ = [("data", C.POINTER(C.c_uint8)), ("len", C.c_size_t)]


VIEW_FIELDS = [
    ("version", C.c_uint16), ("block_id", C.c_uint32), ("step_lo", C.c_uint64), ("step_hi", C.c_uint64),
    ("ctrl_in", C.c_uint16), ("ctrl_out", C.c_uint16), ("in_head_in", C.c_int64), ("in_head_out", C.c_int64),
    ("win_left", C.c_int64), ("win_right", C.c_int64), ("off_in", C.c_uint32), ("off_out", C.c_uint32),
    ("step_start", C.c_uint64), ("input_mv", C.c_int8), ("mv", C.c_int8), ("has_write", C.c_uint8),
    ("wsym", C.c_uint16),
]


# host collectives for sezkp_ctx_create_sharded_host (buffers are host memory)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t)
ALLTOALL_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_void_p, C.c_size_t)


class HostComm(C.Structure):
    _fields_ = [("user", C.c_void_p), ("allgather", ALLGATHER_FN), ("alltoall", ALLTOALL_FN),
                ("allreduce_sum_u8", ALLREDUCE_FN)]


class BlockView(C.Structure):
    _fields_ = [("n_blocks", C.c_uint32), ("tau", C.c_uint32)] + [(f, C.POINTER(t)) for f, t in VIEW_FIELDS]


def _one_hip_runtime() -> None:
    """PyTorch-ROCm wheels bundle their own libamdhip64 / libhsa-runtime64
    (same SONAMEs as /opt/rocm's). If this library is loaded first, torch later
    maps a second copy of the runtime by path, and whichever copy initialises
    second finds no device. Importing torch first makes the dynamic linker
    resolve this library's libamdhip64.so.7 to the copy torch already mapped,
    so the process has one HIP runtime and torch tensors share its context.
    Without torch installed there is only /opt/rocm's runtime."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def _load():
    _one_hip_runtime()
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `make -C {PKG_ROOT}` (or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    L.sezkp_abi_version.restype = C.c_uint32
    if L.sezkp_abi_version() != ABI_VERSION:
        raise ImportError(f"{LIB_PATH} has C ABI {L.sezkp_abi_version()}, this module binds ABI {ABI_VERSION}: "
                          f"rebuild it (make -C {PKG_ROOT})")
    L.sezkp_version.restype = C.c_char_p
    L.sezkp_buf_free.argtypes = [C.POINTER(Buf)]
    E = [C.c_char_p, C.c_size_t]
    L.sezkp_stark_v1_prove.argtypes = [C.POINTER(BlockView), C.c_char_p, C.c_uint32, C.POINTER(Buf), C.POINTER(Buf)] + E
    L.sezkp_stark_v1_prove_artifact_cbor.argtypes = [C.POINTER(BlockView), C.c_char_p, C.c_uint32, C.POINTER(Buf)] + E
    L.sezkp_stark_v1_verify.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(BlockView), C.c_char_p] + E
    L.sezkp_ctx_create.restype = C.c_void_p
    L.sezkp_ctx_create.argtypes = [C.c_int32] + E
    L.sezkp_ctx_destroy.argtypes = [C.c_void_p]
    L.sezkp_ctx_upload.argtypes = [C.c_void_p, C.POINTER(BlockView)] + E
    L.sezkp_ctx_prove.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.POINTER(Buf)] + E
    L.sezkp_ctx_prove_borrow.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32, C.POINTER(C.POINTER(C.c_uint8)),
                                         C.POINTER(C.c_size_t)] + E
    L.sezkp_ctx_stage_times.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_int32]
    L.sezkp_ctx_stream.restype = C.c_void_p
    L.sezkp_ctx_comm_stats.argtypes = [C.c_void_p, C.POINTER(CommStat), C.c_int32]
    L.sezkp_ctx_stream.argtypes = [C.c_void_p]
    L.sezkp_gl_ntt.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int32, C.c_void_p]
    L.sezkp_gl_coset_lde_deep.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint64, C.c_void_p,
                                          C.c_void_p, C.c_void_p]
    L.sezkp_fri_fold.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p]
    L.sezkp_blake3_leaves_u64.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
    L.sezkp_blake3_leaves_labeled.argtypes = [C.c_void_p, C.c_uint64, C.c_char_p, C.c_uint32, C.c_void_p, C.c_void_p]
    L.sezkp_merkle_node_count.restype = C.c_uint64
    L.sezkp_merkle_node_count.argtypes = [C.c_uint64]
    L.sezkp_merkle_build.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
    L.sezkp_merkle_paths.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
    L.sezkp_fri_fold_commit.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_char_p, C.c_void_p]
    L.sezkp_merkle_root_u64.argtypes = [C.c_void_p, C.c_uint64, C.c_char_p, C.c_void_p]
    L.sezkp_manifest_root.argtypes = [C.POINTER(BlockView), C.c_char_p]
    L.sezkp_manifest_frontier_root.argtypes = [C.POINTER(BlockView), C.c_char_p]
    L.sezkp_blocks_decode_cbor.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_void_p)] + E
    L.sezkp_blocks_decode_jsonl.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_void_p)] + E
    L.sezkp_blocks_encode_jsonl.argtypes = [C.POINTER(BlockView), C.POINTER(Buf)]
    L.sezkp_manifest_decode.argtypes = [C.c_char_p, C.c_size_t, C.c_int32, C.c_char_p, C.POINTER(C.c_uint32)] + E
    L.sezkp_blocks_view.restype = C.POINTER(BlockView)
    L.sezkp_blocks_view.argtypes = [C.c_void_p]
    L.sezkp_blocks_free.argtypes = [C.c_void_p]
    L.sezkp_blake3.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]
    L.sezkp_comm_unique_id.argtypes = [C.c_char_p] + E
    L.sezkp_ctx_create_sharded.restype = C.c_void_p
    L.sezkp_ctx_create_sharded.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_char_p] + E
    L.sezkp_ctx_create_sharded_host.restype = C.c_void_p
    L.sezkp_ctx_create_sharded_host.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.POINTER(HostComm)] + E
    L.sezkp_blocks_encode_cbor.argtypes = [C.POINTER(BlockView), C.POINTER(Buf)]
    L.sezkp_simulate_trace.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64] + [C.c_void_p] * 4
    L.sezkp_simulate_blocks.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint64, C.POINTER(C.c_void_p)] + E
    L.sezkp_ctx_prove_async.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32] + E
    L.sezkp_ctx_wait.argtypes = [C.c_void_p, C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_size_t)] + E
    L.sezkp_ctx_stage.argtypes = [C.c_void_p, C.POINTER(BlockView)] + E
    L.sezkp_host_register.argtypes = [C.c_void_p, C.c_size_t]
    L.sezkp_host_unregister.argtypes = [C.c_void_p]
    L.sezkp_ctx_dist_ntt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int32] + E
    L.sezkp_fs_xof.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_uint32), C.c_char_p, C.POINTER(C.c_uint32),
                               C.POINTER(C.c_uint32), C.c_uint32, C.c_char_p, C.c_void_p]
    L.sezkp_ctx_upload_rows.argtypes = [C.c_void_p, C.POINTER(BlockView), C.c_uint64, C.c_uint64] + E
    L.sezkp_shard_rows.argtypes = [C.c_void_p, C.c_uint32, C.c_int32, C.c_int32, C.POINTER(C.c_uint64),
                                   C.POINTER(C.c_uint64)]
    L.sezkp_blocks_decode_jsonl_meta.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64, C.c_uint64,
                                                 C.POINTER(C.c_void_p)] + E
    L.sezkp_blocks_decode_jsonl_lines.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64, C.c_uint64, C.c_int32,
                                                  C.POINTER(C.c_void_p)] + E
    L.sezkp_blocks_line_offsets.argtypes = [C.c_void_p, C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.c_size_t)]
    L.sezkp_manifest_leaf_hashes.argtypes = [C.POINTER(BlockView), C.c_void_p]
    L.sezkp_merkle_root_of_leaves.argtypes = [C.c_char_p, C.c_size_t, C.c_int32, C.c_char_p]
    L.sezkp_ctx_create_sharded_solo.restype = C.c_void_p
    L.sezkp_ctx_create_sharded_solo.argtypes = [C.c_int32, C.c_int32, C.c_int32] + E
    return L


lib = _load()


def take_buf(b: Buf) -> bytes:
    out = C.string_at(b.data, b.len) if b.len else b""
    lib.sezkp_buf_free(C.byref(b))
    return out


def check(rc: int, err) -> None:
    if rc != SEZKP_OK:
        raise SezkpError(rc, err.value.decode(errors="replace"))

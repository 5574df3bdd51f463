"""Host-side mirror of the reference's `ProvingBackend` for `StarkV1`
(crates/sezkp-core/src/backend.rs:41-61, crates/sezkp-stark/src/lib.rs:126-190)
over the MI355X C ABI. Same names, same argument meaning, same artifact
(`ProofArtifact`, crates/sezkp-core/src/artifact.rs:55-68); errors raise
`SezkpError` where the reference returns `anyhow::Error`.
"""
from __future__ import annotations

import ctypes as C
import json
import struct
from dataclasses import dataclass, field

from ._lib import SEZKP_FLAG_STREAMING, Buf, SezkpError, check, lib, take_buf
from .blocks import BlockSoA

STAGES = ["expand", "col_commit", "col_outer", "compose", "intt", "lde_ntt", "deep", "layer0_tree",
          "layer0_upper", "fri_fold_trees", "col_openings", "fri_paths", "total",
          # host-side split of the same prove() call (wall clock)
          "host_wall", "host_sync_wait", "host_final_wait", "host_serialize",
          # the FRI forest launch (SEZKP_KERNEL_EVENTS=1; 0 when not recorded)
          "k_forest16"]


@dataclass
class ProofArtifact:
    backend: str
    manifest_root: bytes
    proof_bytes: bytes
    meta: dict = field(default_factory=dict)

    def to_cbor(self) -> bytes:
        """ciborium encoding (io.rs:176-183): map{backend, manifest_root, proof_bytes, meta},
        byte vectors as arrays of uints, meta keys sorted."""
        out = bytearray(b"\xa4")
        def text(s: str):
            b = s.encode()
            return _head(3, len(b)) + b
        def barr(bs: bytes):
            return _head(4, len(bs)) + b"".join(bytes([x]) if x < 24 else bytes([0x18, x]) for x in bs)
        out += text("backend") + text(self.backend)
        out += text("manifest_root") + barr(self.manifest_root)
        out += text("proof_bytes") + barr(self.proof_bytes)
        out += text("meta") + _head(5, len(self.meta))
        for k in sorted(self.meta):
            v = self.meta[k]
            out += text(k) + (text(v) if isinstance(v, str) else _head(0, int(v)))
        return bytes(out)


def _head(major: int, v: int) -> bytes:
    if v < 24:
        return bytes([(major << 5) | v])
    for nb, ai in ((1, 24), (2, 25), (4, 26), (8, 27)):
        if v < 1 << (8 * nb):
            return bytes([(major << 5) | ai]) + v.to_bytes(nb, "big")
    raise ValueError(v)


def _meta(proof: bytes, tau: int, streaming: bool) -> dict:
    m = {"proto": "stark-v1", "domain_n": struct.unpack_from("<Q", proof, 0)[0], "tau": tau}
    if streaming:
        m["mode"] = "streaming"
    return m


class StarkV1:
    """`impl ProvingBackend for StarkV1` on MI355X (stateless associated functions)."""

    @staticmethod
    def prove(blocks: BlockSoA, manifest_root: bytes) -> ProofArtifact:
        return StarkV1._prove(blocks, manifest_root, False)

    @staticmethod
    def prove_streaming(blocks: BlockSoA, manifest_root: bytes) -> ProofArtifact:
        """StarkV1::prove_streaming (lib.rs:170-190): same bytes, meta gains mode=streaming."""
        return StarkV1._prove(blocks, manifest_root, True)

    @staticmethod
    def _prove(blocks: BlockSoA, manifest_root: bytes, streaming: bool) -> ProofArtifact:
        if len(manifest_root) != 32:
            raise SezkpError(-1, "manifest_root must be 32 bytes")
        blocks.check_shape()
        pb, mb = Buf(), Buf()
        err = C.create_string_buffer(1024)
        rc = lib.sezkp_stark_v1_prove(C.byref(blocks.view()), bytes(manifest_root),
                                      SEZKP_FLAG_STREAMING if streaming else 0, C.byref(pb), C.byref(mb), err, 1024)
        check(rc, err)
        proof = take_buf(pb)
        meta = json.loads(take_buf(mb).decode())
        return ProofArtifact("stark", bytes(manifest_root), proof, meta)

    @staticmethod
    def verify(artifact: ProofArtifact, blocks: BlockSoA, manifest_root: bytes) -> None:
        """StarkV1::verify (lib.rs:144-162 -> v1/verify.rs:60-196), host CPU."""
        if artifact.backend != "stark":
            raise SezkpError(-5, "backend kind mismatch: expected STARK")
        if bytes(artifact.manifest_root) != bytes(manifest_root):
            raise SezkpError(-5, "manifest root mismatch")
        blocks.check_shape()
        err = C.create_string_buffer(1024)
        rc = lib.sezkp_stark_v1_verify(artifact.proof_bytes, len(artifact.proof_bytes), C.byref(blocks.view()),
                                       bytes(manifest_root), err, 1024)
        check(rc, err)


class ProverContext:
    """Resident-input prover: upload once (trace image in HBM), prove many times."""

    def __init__(self, device: int = 0):
        err = C.create_string_buffer(1024)
        self._h = lib.sezkp_ctx_create(device, err, 1024)
        if not self._h:
            raise SezkpError(-2, err.value.decode())
        self.tau = 0
        self.rank, self.world = 0, 1

    def upload(self, blocks: BlockSoA) -> None:
        blocks.check_shape()
        err = C.create_string_buffer(1024)
        check(lib.sezkp_ctx_upload(self._h, C.byref(blocks.view()), err, 1024), err)
        self.tau = blocks.tau

    def upload_rows(self, blocks: BlockSoA, row0: int, nrows: int) -> None:
        """Upload from a view whose step arrays hold only rows [row0, row0 +
        nrows) (a sharded rank's slice, sezkp_ctx_upload_rows)."""
        if row0 < 0 or nrows < 0:
            raise SezkpError(-1, "row0 and nrows must be non-negative")
        blocks.check_shape(nrows)
        if blocks.step_start[-1] < row0 + nrows:
            raise SezkpError(-1, "rows [row0, row0 + nrows) exceed the trace")
        err = C.create_string_buffer(1024)
        check(lib.sezkp_ctx_upload_rows(self._h, C.byref(blocks.view()), row0, nrows, err, 1024), err)
        self.tau = blocks.tau

    def stage(self, blocks: BlockSoA) -> None:
        """Pipelined upload of the next trace (same shape as the uploaded one):
        async H2D into the spare trace image, allowed while a proof is in
        flight; the next prove uses it (sezkp_ctx_stage). `blocks` must stay
        alive and unchanged until that prove has started."""
        blocks.check_shape()
        err = C.create_string_buffer(1024)
        check(lib.sezkp_ctx_stage(self._h, C.byref(blocks.view()), err, 1024), err)
        self._staged = blocks  # keep the arrays alive

    def prove(self, manifest_root: bytes, streaming: bool = False) -> ProofArtifact:
        pb = Buf()
        err = C.create_string_buffer(1024)
        check(lib.sezkp_ctx_prove(self._h, bytes(manifest_root), SEZKP_FLAG_STREAMING if streaming else 0,
                                  C.byref(pb), err, 1024), err)
        proof = take_buf(pb)
        return ProofArtifact("stark", bytes(manifest_root), proof, _meta(proof, self.tau, streaming))

    def prove_view(self, manifest_root: bytes) -> memoryview:
        """The proof bytes as a read-only view of the context's pinned host
        buffer (no copy); valid until the next prove/upload/close."""
        ptr = C.POINTER(C.c_uint8)()
        n = C.c_size_t()
        err = C.create_string_buffer(1024)
        check(lib.sezkp_ctx_prove_borrow(self._h, bytes(manifest_root), 0, C.byref(ptr), C.byref(n), err, 1024), err)
        return memoryview((C.c_uint8 * n.value).from_address(C.addressof(ptr.contents))).cast("B").toreadonly()

    def prove_async(self, manifest_root: bytes) -> None:
        """Start a proof on the context's worker thread (sezkp_ctx_prove_async)."""
        err = C.create_string_buffer(1024)
        check(lib.sezkp_ctx_prove_async(self._h, bytes(manifest_root), 0, err, 1024), err)

    def wait_view(self) -> memoryview:
        """Wait for the proof started by prove_async; a borrowed view as prove_view."""
        ptr = C.POINTER(C.c_uint8)()
        n = C.c_size_t()
        err = C.create_string_buffer(1024)
        check(lib.sezkp_ctx_wait(self._h, C.byref(ptr), C.byref(n), err, 1024), err)
        return memoryview((C.c_uint8 * n.value).from_address(C.addressof(ptr.contents))).cast("B").toreadonly()

    def stage_times_ms(self) -> dict:
        buf = (C.c_double * 32)()
        n = lib.sezkp_ctx_stage_times(self._h, buf, 32)
        return {STAGES[i]: buf[i] for i in range(min(n, len(STAGES)))}

    def comm_stats(self) -> list:
        """Per-collective stats of the last sharded prove: [{name, bytes, ms,
        GBs}] (sezkp_ctx_comm_stats; bytes = what this rank sent over links)."""
        from ._lib import CommStat
        buf = (CommStat * 64)()
        n = lib.sezkp_ctx_comm_stats(self._h, buf, 64)
        out = []
        for i in range(n):
            b, ms = int(buf[i].bytes), float(buf[i].ms)
            out.append({"name": buf[i].name.decode(), "bytes": b, "ms": ms,
                        "GBs": (b / ms / 1e6) if ms > 0 else None})
        return out

    def dist_ntt(self, local, scratch=None, inverse: bool = False, sync: bool = True):
        """Distributed four-step NTT of n = world * local.numel() points, in
        place on `local` (a device u64/i64 tensor; layouts in sezkp_stark.h,
        sezkp_ctx_dist_ntt). Every rank calls it together."""
        import torch
        if local.dtype not in (torch.int64, torch.uint64) or not local.is_cuda or not local.is_contiguous():
            raise SezkpError(-1, "local must be a contiguous 64-bit device tensor")
        m = local.numel()
        if m & (m - 1):
            raise SezkpError(-1, "local length must be a power of two")
        if scratch is None:
            scratch = torch.empty_like(local)
        log_n = (m * self.world).bit_length() - 1
        if sync:
            torch.cuda.current_stream(local.device).synchronize()
        err = C.create_string_buffer(1024)
        check(lib.sezkp_ctx_dist_ntt(self._h, local.data_ptr(), scratch.data_ptr(), log_n, -1 if inverse else 1,
                                     err, 1024), err)
        if sync:
            torch.cuda.ExternalStream(self.stream, device=local.device).synchronize()
        return local

    @property
    def stream(self) -> int:
        return lib.sezkp_ctx_stream(self._h) or 0

    def close(self):
        if self._h:
            lib.sezkp_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardedProverContext(ProverContext):
    """One STARK v1 proof over `world` GPUs (one process per GPU).

    Every rank uploads the same blocks and calls prove() with the same root;
    every rank gets the identical proof bytes. comm="rccl": the exchanges run
    over RCCL (xGMI) inside the library; the communicator id is created on
    rank 0 and broadcast over the torch.distributed `group`. comm="host":
    the exchanges are staged through host memory and run over the (gloo)
    `group` by `sezkp_amd.dist.HostCollectives` — for tests on one GPU.
    comm="solo": this rank alone on `device` with its own contributions only
    (no group): the per-rank cost model; timings real, proof bytes not.
    """

    def __init__(self, rank: int, world: int, device: int = 0, comm: str = "rccl", group=None):
        import torch.distributed as dist
        err = C.create_string_buffer(1024)
        self.tau = 0
        self.rank, self.world = rank, world
        self._hc = None
        if comm == "rccl":
            uid = C.create_string_buffer(128)
            if rank == 0:
                check(lib.sezkp_comm_unique_id(uid, err, 1024), err)
            obj = [bytes(uid.raw)]
            if world > 1:
                dist.broadcast_object_list(obj, src=0, group=group)
            self._h = lib.sezkp_ctx_create_sharded(device, rank, world, obj[0], err, 1024)
        elif comm == "solo":
            self._h = lib.sezkp_ctx_create_sharded_solo(device, rank, world, err, 1024)
        elif comm == "host":
            from .dist import HostCollectives
            self._coll = HostCollectives(group)
            self._hc = self._coll.c_struct()
            self._h = lib.sezkp_ctx_create_sharded_host(device, rank, world, C.byref(self._hc), err, 1024)
        else:
            raise ValueError(f"unknown comm {comm!r}")
        if not self._h:
            raise SezkpError(-2, err.value.decode())

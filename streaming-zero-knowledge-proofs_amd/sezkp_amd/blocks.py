"""Block summaries as struct-of-arrays (the `sezkp_block_view` of the C ABI).

`BlockSoA` mirrors `Vec<BlockSummary>` (crates/sezkp-core/src/types.rs:116-151).
`simulate()` + `partition()` restate the input producer of the reference
(`sezkp-cli simulate`: crates/sezkp-trace/src/generator.rs:38-73 and
partition.rs:43-150) with numpy: same distributions (input/tape moves uniform
in {-1,0,1}, writes with p=0.4 of a symbol in 0..=15) and the same partition
semantics, but a numpy PCG64 stream (any seed, fast) instead of rand 0.9's
ChaCha12 StdRng. `reference_trace()` / `reference_blocks()` are the bit-exact
restatement of the reference's own generator (tracegen.cpp), pinned by the
reference's trace.cbor / blocks.cbor fixtures.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import VIEW_FIELDS, BlockView, Buf, SezkpError, lib, take_buf

_NP = {C.c_uint16: np.uint16, C.c_uint32: np.uint32, C.c_uint64: np.uint64, C.c_int64: np.int64,
       C.c_int8: np.int8, C.c_uint8: np.uint8}


class BlockSoA:
    """Struct-of-arrays block summaries; per-step tape arrays are step-major."""

    def __init__(self, tau: int, **arrays):
        self.tau = int(tau)
        for f, t in VIEW_FIELDS:
            setattr(self, f, np.ascontiguousarray(arrays[f], dtype=_NP[t]))
        self.n_blocks = int(self.version.size)
        self._view = None

    def __getstate__(self):  # pickled across ranks (sliced ingest): arrays only, no ctypes view
        return {"tau": self.tau, **{f: getattr(self, f) for f, _ in VIEW_FIELDS}}

    def __setstate__(self, st):
        self.__init__(st.pop("tau"), **st)

    # total trace rows n = sum(step_hi - step_lo + 1)
    @property
    def n_rows(self) -> int:
        return int((self.step_hi - self.step_lo + 1).sum()) if self.n_blocks else 0

    def check_shape(self, nrows: int | None = None) -> None:
        """Raise SezkpError unless the arrays have the sizes the C ABI reads
        (sezkp_block_view carries no lengths): per-block fields n_blocks,
        per-(block, tape) fields n_blocks * tau, step_start n_blocks + 1, and
        step arrays of `nrows` rows (default: every row, step_start[-1])."""
        nb, tau = self.n_blocks, self.tau
        want = {f: nb for f, _ in VIEW_FIELDS}
        for f in ("win_left", "win_right", "off_in", "off_out"):
            want[f] = nb * tau
        want["step_start"] = nb + 1
        ss = self.step_start
        if ss.size and (ss[0] != 0 or (ss.size > 1 and bool((ss[1:] < ss[:-1]).any()))):
            raise SezkpError(-1, "blocks.step_start must start at 0 and never decrease")
        if self.step_start.size == nb + 1:
            S = int(self.step_start[-1]) if nrows is None else int(nrows)
            want.update(input_mv=S, mv=S * tau, has_write=S * tau, wsym=S * tau)
        for f, _ in VIEW_FIELDS:
            if getattr(self, f).size != want[f]:
                raise SezkpError(-1, f"blocks.{f} holds {getattr(self, f).size} values, expected {want[f]}"
                                 + (" (a metadata-only or sliced view: use upload_rows with its row range)"
                                    if f in ("input_mv", "mv", "has_write", "wsym") else ""))

    def view(self) -> BlockView:
        v = BlockView()
        v.n_blocks = self.n_blocks
        v.tau = self.tau
        for f, t in VIEW_FIELDS:
            a = getattr(self, f)
            if a.size == 0:  # keep a valid pointer for empty arrays
                a = np.zeros(1, dtype=_NP[t])
                setattr(self, "_empty_" + f, a)
            setattr(v, f, a.ctypes.data_as(C.POINTER(t)))
        self._view = v
        return v

    def pin(self) -> "BlockSoA":
        """Page-lock the per-step arrays (sezkp_host_register) so staged uploads
        (ProverContext.stage) are DMA that overlaps other proofs' kernels."""
        if getattr(self, "_pinned", None) is None:
            self._pinned = []
            for f in ("input_mv", "mv", "has_write", "wsym"):
                a = getattr(self, f)
                if a.nbytes and lib.sezkp_host_register(a.ctypes.data, a.nbytes) == 0:
                    self._pinned.append(a)
        return self

    def unpin(self) -> None:
        for a in getattr(self, "_pinned", None) or []:
            lib.sezkp_host_unregister(a.ctypes.data)
        self._pinned = None

    def __del__(self):
        try:
            self.unpin()
        except Exception:
            pass

    def manifest_root(self) -> bytes:
        """commit_blocks (sezkp-merkle lib.rs:214-222): the batch merkle_root."""
        out = C.create_string_buffer(32)
        lib.sezkp_manifest_root(C.byref(self.view()), out)
        return out.raw

    def manifest_frontier_root(self) -> bytes:
        """The streaming Frontier root (lib.rs:167-208) that the reference
        commits and prechecks for .jsonl/.ndjson files (lib.rs:259-330)."""
        out = C.create_string_buffer(32)
        lib.sezkp_manifest_frontier_root(C.byref(self.view()), out)
        return out.raw

    def file_root(self, path: str) -> bytes:
        """The manifest root the reference computes for a blocks file at `path`:
        Frontier for .jsonl/.ndjson, batch merkle_root for .json/.cbor."""
        ext = path.rsplit(".", 1)[-1].lower() if "." in path else ""
        return self.manifest_frontier_root() if ext in ("jsonl", "ndjson") else self.manifest_root()

    @classmethod
    def from_cbor(cls, data: bytes) -> "BlockSoA":
        """Decode CBOR Vec<BlockSummary> (crates/sezkp-core/src/io.rs:57-65) via the C ABI."""
        return cls._decode(lib.sezkp_blocks_decode_cbor, data)

    @classmethod
    def from_jsonl(cls, data: bytes) -> "BlockSoA":
        """Decode JSON Lines, one BlockSummary per line (io_jsonl.rs:43-84)."""
        return cls._decode(lib.sezkp_blocks_decode_jsonl, data)

    @classmethod
    def from_file(cls, path: str) -> "BlockSoA":
        """.cbor / .jsonl / .ndjson block files (by extension)."""
        data = open(path, "rb").read()
        ext = path.rsplit(".", 1)[-1].lower() if "." in path else ""
        if ext == "cbor":
            return cls.from_cbor(data)
        if ext in ("jsonl", "ndjson"):
            return cls.from_jsonl(data)
        raise SezkpError(-1, f"unsupported blocks extension: {ext or '(none)'} (supported: .cbor, .jsonl, .ndjson)")

    def to_jsonl(self) -> bytes:
        """write_block_summaries_jsonl (io_jsonl.rs:93-106) via the C ABI."""
        b = Buf()
        rc = lib.sezkp_blocks_encode_jsonl(C.byref(self.view()), C.byref(b))
        if rc != 0:
            raise SezkpError(rc, "encode jsonl")
        return take_buf(b)

    def to_cbor(self) -> bytes:
        """Vec<BlockSummary> as the reference writes blocks.cbor (ciborium), via the C ABI."""
        b = Buf()
        rc = lib.sezkp_blocks_encode_cbor(C.byref(self.view()), C.byref(b))
        if rc != 0:
            raise SezkpError(rc, "encode cbor")
        return take_buf(b)

    @classmethod
    def _decode(cls, fn, data: bytes) -> "BlockSoA":
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        rc = fn(data, len(data), C.byref(h), err, 512)
        if rc != 0:
            raise SezkpError(rc, err.value.decode())
        return cls._take(h)

    def leaf_hashes(self) -> bytes:
        """The manifest leaf hash of every block (sezkp-merkle lib.rs:85-117),
        32 bytes each: needs the blocks' fields and step counts only."""
        out = C.create_string_buffer(32 * max(1, self.n_blocks))
        rc = lib.sezkp_manifest_leaf_hashes(C.byref(self.view()), out)
        if rc != 0:
            raise SezkpError(rc, "leaf hashes")
        return out.raw[:32 * self.n_blocks]

    @classmethod
    def from_jsonl_meta(cls, data, lo: int, hi: int, steps: bool = False) -> tuple:
        """The metadata of the JSONL lines starting in bytes [lo, hi) of `data`
        (bytes or a uint8 numpy array / memmap; cut at line ends): every field
        and step count, no steps (empty step arrays); steps=True: the same
        lines decoded in full. Returns (BlockSoA, line byte offsets)
        (sezkp_blocks_decode_jsonl_lines)."""
        ptr, n = _addr(data)
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        rc = lib.sezkp_blocks_decode_jsonl_lines(ptr, n, lo, hi, int(steps), C.byref(h), err, 512)
        if rc != 0:
            raise SezkpError(rc, err.value.decode())
        p = C.POINTER(C.c_uint64)()
        cnt = C.c_size_t()
        lib.sezkp_blocks_line_offsets(h, C.byref(p), C.byref(cnt))
        offs = np.ctypeslib.as_array(p, shape=(cnt.value,)).copy() if cnt.value else np.zeros(0, np.uint64)
        return cls._take(h, meta=not steps), offs

    def meta_only(self) -> "BlockSoA":
        """These blocks' fields and step counts without the step arrays."""
        arr = {f: getattr(self, f) for f, _ in VIEW_FIELDS}
        for f in ("input_mv", "mv", "has_write", "wsym"):
            arr[f] = arr[f][:0]
        return BlockSoA(self.tau, **arr)

    @classmethod
    def from_jsonl_range(cls, data, lo: int, hi: int) -> "BlockSoA":
        """Full decode of the whole lines in bytes [lo, hi) of `data`."""
        ptr, n = _addr(data)
        if not 0 <= lo <= hi <= n:
            raise SezkpError(-1, "bad byte range")
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        rc = lib.sezkp_blocks_decode_jsonl(C.cast(C.c_void_p(ptr + lo), C.c_char_p), hi - lo, C.byref(h), err, 512)
        if rc != 0:
            raise SezkpError(rc, err.value.decode())
        return cls._take(h)

    @classmethod
    def concat_meta(cls, parts: list) -> "BlockSoA":
        """Blocks of several metadata-only parts, in order (step_start rebuilt
        from the parts' step counts)."""
        parts = [p for p in parts if p.n_blocks]
        tau = parts[0].tau if parts else 0
        arr = {}
        for f, t in VIEW_FIELDS:
            if f == "step_start":
                counts = np.concatenate([np.diff(p.step_start) for p in parts]) if parts else np.zeros(0, np.uint64)
                arr[f] = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
            elif f in ("input_mv", "mv", "has_write", "wsym"):
                arr[f] = np.zeros(0, _NP[t])
            else:
                arr[f] = np.concatenate([getattr(p, f) for p in parts]) if parts else np.zeros(0, _NP[t])
        return cls(tau, **arr)

    def with_steps(self, slice_blocks: "BlockSoA") -> "BlockSoA":
        """These (global) block fields with the step arrays of `slice_blocks`
        (a run of whole blocks): the view sezkp_ctx_upload_rows takes."""
        arr = {f: getattr(self, f) for f, _ in VIEW_FIELDS}
        for f in ("input_mv", "mv", "has_write", "wsym"):
            arr[f] = getattr(slice_blocks, f)
        return BlockSoA(self.tau, **arr)

    @classmethod
    def _take(cls, h, meta: bool = False) -> "BlockSoA":
        """Copy a library-owned sezkp_blocks into numpy arrays and free it
        (meta: the step arrays are empty, step_start holds the step counts)."""
        try:
            v = lib.sezkp_blocks_view(h).contents
            nb, tau = v.n_blocks, v.tau
            counts = {"step_start": nb + 1}
            arr = {}
            base = {f: nb for f, _ in VIEW_FIELDS}
            for f in ("win_left", "win_right", "off_in", "off_out"):
                base[f] = nb * tau
            step_start = np.ctypeslib.as_array(v.step_start, shape=(nb + 1,)).copy() if nb else np.zeros(1, np.uint64)
            S = 0 if meta else int(step_start[-1])
            base.update(step_start=nb + 1, input_mv=S, mv=S * tau, has_write=S * tau, wsym=S * tau)
            for f, t in VIEW_FIELDS:
                cnt = base[f]
                arr[f] = (np.ctypeslib.as_array(getattr(v, f), shape=(cnt,)).copy() if cnt
                          else np.zeros(0, _NP[t]))
            del counts
            return cls(tau, **arr)
        finally:
            lib.sezkp_blocks_free(h)


def _addr(data) -> tuple:
    """(address, length) of bytes or a contiguous uint8 numpy array / memmap."""
    if isinstance(data, bytes):  # no copy: the caller keeps `data` alive
        return C.cast(C.c_char_p(data), C.c_void_p).value or 0, len(data)
    a = np.frombuffer(data, dtype=np.uint8) if isinstance(data, bytearray) else data
    if not (isinstance(a, np.ndarray) and a.dtype == np.uint8 and a.flags.c_contiguous):
        raise SezkpError(-1, "data must be bytes or a contiguous uint8 array")
    return a.ctypes.data, a.size


def merkle_root_of_leaves(leaves: bytes, frontier: bool) -> bytes:
    """The batch merkle_root (lib.rs:140-157) or the Frontier root (lib.rs:
    167-208) over 32-byte leaf hashes (sezkp_merkle_root_of_leaves)."""
    out = C.create_string_buffer(32)
    rc = lib.sezkp_merkle_root_of_leaves(leaves, len(leaves) // 32, 1 if frontier else 0, out)
    if rc != 0:
        raise SezkpError(rc, "merkle root of leaves")
    return out.raw


def shard_rows(step_start, rank: int, world: int) -> tuple:
    """The rows (row0, nrows) rank `rank` of a `world`-GPU sharded prove reads
    (whole blocks; sezkp_shard_rows)."""
    ss = np.ascontiguousarray(step_start, dtype=np.uint64)
    r0, nr = C.c_uint64(), C.c_uint64()
    rc = lib.sezkp_shard_rows(ss.ctypes.data, ss.size - 1, rank, world, C.byref(r0), C.byref(nr))
    if rc != 0:
        raise SezkpError(rc, "shard_rows: n must be a power of two >= 4096 * world")
    return r0.value, nr.value


def simulate(t: int, tau: int, seed: int = 42):
    """Synthetic trace (generator.rs:38-73 distribution): returns
    (input_mv[t], mv[t,tau], has_write[t,tau], wsym[t,tau])."""
    rng = np.random.Generator(np.random.PCG64(seed))
    input_mv = rng.integers(-1, 2, size=t, dtype=np.int8)
    has_write = (rng.random((t, tau)) < 0.4).astype(np.uint8)
    wsym = rng.integers(0, 16, size=(t, tau), dtype=np.uint16) * has_write
    mv = rng.integers(-1, 2, size=(t, tau), dtype=np.int8)
    return input_mv, mv, has_write, wsym.astype(np.uint16)


def partition(input_mv, mv, has_write, wsym, b: int) -> BlockSoA:
    """partition_trace (partition.rs:43-150): contiguous blocks of b steps,
    per-tape windows covering the post-move heads (relative, starting at 0)."""
    t = int(input_mv.size)
    tau = int(mv.shape[1]) if mv.ndim == 2 else 0
    nb = (t + b - 1) // b
    starts = np.arange(nb, dtype=np.int64) * b
    ends = np.minimum(starts + b, t)
    lens = ends - starts
    gin = np.concatenate([[0], np.cumsum(input_mv.astype(np.int64))])
    win_left = np.zeros((nb, tau), np.int64)
    win_right = np.zeros((nb, tau), np.int64)
    off_out = np.zeros((nb, tau), np.int64)
    for k in range(nb):  # per block (vectorised over steps and tapes)
        heads = np.cumsum(mv[starts[k]:ends[k]].astype(np.int64), axis=0)
        lo = np.minimum(heads.min(axis=0), 0) if heads.size else np.zeros(tau, np.int64)
        hi = np.maximum(heads.max(axis=0), 0) if heads.size else np.zeros(tau, np.int64)
        win_left[k], win_right[k] = lo, hi
        off_out[k] = (heads[-1] if heads.size else 0) - lo
    off_in = -win_left
    clamp = lambda x: np.where((x >= 0) & (x <= 0xFFFFFFFF), x, 0xFFFFFFFF).astype(np.uint32)
    return BlockSoA(
        tau,
        version=np.ones(nb, np.uint16), block_id=np.arange(1, nb + 1, dtype=np.uint32),
        step_lo=(starts + 1).astype(np.uint64), step_hi=ends.astype(np.uint64),
        ctrl_in=np.zeros(nb, np.uint16), ctrl_out=np.zeros(nb, np.uint16),
        in_head_in=gin[starts], in_head_out=gin[ends],
        win_left=win_left.reshape(-1), win_right=win_right.reshape(-1),
        off_in=clamp(off_in).reshape(-1), off_out=clamp(off_out).reshape(-1),
        step_start=np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64),
        input_mv=input_mv, mv=mv.reshape(-1), has_write=has_write.reshape(-1), wsym=wsym.reshape(-1),
    )


def reference_trace(t: int, tau: int, seed: int = 42):
    """The reference's own `generate_trace(t, tau)` (generator.rs:38-73, rand
    0.9.2 StdRng, bit-exact; the reference fixes seed 42), in the same
    (input_mv[t], mv[t,tau], has_write[t,tau], wsym[t,tau]) form as simulate()."""
    im = np.zeros(t, np.int8)
    mv = np.zeros((t, tau), np.int8)
    hw = np.zeros((t, tau), np.uint8)
    ws = np.zeros((t, tau), np.uint16)
    rc = lib.sezkp_simulate_trace(t, tau, seed, im.ctypes.data, mv.ctypes.data, hw.ctypes.data, ws.ctypes.data)
    if rc != 0:
        raise SezkpError(rc, "simulate_trace: tau must be <= 255")
    return im, mv, hw, ws


def reference_blocks(t: int, b: int = 512, tau: int = 8, seed: int = 42) -> BlockSoA:
    """Exactly what `sezkp-cli simulate --t T --b b --tau tau` writes
    (main.rs:317-350: generate_trace + partition_trace), built natively."""
    h = C.c_void_p()
    err = C.create_string_buffer(512)
    rc = lib.sezkp_simulate_blocks(t, b, tau, seed, C.byref(h), err, 512)
    if rc != 0:
        raise SezkpError(rc, err.value.decode())
    return BlockSoA._take(h)


def synthetic_blocks(t: int, b: int = 512, tau: int = 8, seed: int = 42) -> BlockSoA:
    """`sezkp-cli simulate --t T --b b --tau tau` stand-in (b = steps per block)."""
    return partition(*simulate(t, tau, seed), b)

/*
 * sezkp_stark.h — C ABI of the MI355X-native STARK v1 prover hot path.
 *
 * Drop-in boundary for logannye/streaming-zero-knowledge-proofs:
 *   - top level: replaces `impl ProvingBackend for StarkV1`
 *     (crates/sezkp-core/src/backend.rs:41-61, crates/sezkp-stark/src/lib.rs:126-190);
 *   - version symbols: crates/sezkp-ffi/src/lib.rs:65-79 (ABI bumped 1 -> 4);
 *   - kernel level: the hot loops of crates/sezkp-ffts (ntt.rs:79-177,
 *     coset.rs:85-102), crates/sezkp-stark/src/v1/{lde.rs:42-97,
 *     fri_stream.rs:37-121, merkle.rs:46-160, prover.rs:200-239}.
 * Plain pointers and sizes only; no exceptions or aborts cross this boundary:
 * every entry point returns 0 on success or a negative SEZKP_E_* code and
 * writes a NUL-terminated message into `err` (when err_len > 0).
 * Outputs of type sezkp_buf are library-allocated; release with sezkp_buf_free.
 * Thread safety: calls on distinct sezkp_ctx objects may run concurrently.
 */
#ifndef SEZKP_STARK_H
#define SEZKP_STARK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 4 (round 6): sezkp_fs_xof runs on the host and ignores `stream`;
 * sezkp_ctx_stage_times writes 17 values (the three fs_point slots of ABI 3
 * are gone) and col_openings is the openings kernel's own time; blocks of
 * zero steps (step_hi = step_lo - 1) are accepted as the reference does. */
#define SEZKP_ABI_VERSION 4u

#define SEZKP_OK 0
#define SEZKP_E_INVALID (-1)   /* malformed input (shape, non power-of-two n, ...) */
#define SEZKP_E_DEVICE (-2)    /* HIP runtime / kernel failure */
#define SEZKP_E_NOMEM (-3)
#define SEZKP_E_DECODE (-4)    /* CBOR/bincode decode failure */
#define SEZKP_E_VERIFY (-5)    /* proof rejected */

#define SEZKP_FLAG_STREAMING 1u /* meta gains "mode":"streaming" (StarkV1::prove_streaming, lib.rs:170-190) */

/* crates/sezkp-ffi/src/lib.rs:65-79 */
uint32_t sezkp_abi_version(void);
const char* sezkp_version(void);

typedef struct sezkp_buf {
    uint8_t* data;
    size_t len;
} sezkp_buf;
void sezkp_buf_free(sezkp_buf* b);

/* Struct-of-arrays view of &[BlockSummary] (crates/sezkp-core/src/types.rs:116-151).
 * Every block has exactly `tau` windows / head offsets; every step has exactly
 * `tau` tape ops (tape-op arrays are step-major: [step*tau + r]). */
typedef struct sezkp_block_view {
    uint32_t n_blocks;
    uint32_t tau;
    const uint16_t* version;     /* [n_blocks] */
    const uint32_t* block_id;    /* [n_blocks] */
    const uint64_t* step_lo;     /* [n_blocks] */
    const uint64_t* step_hi;     /* [n_blocks] */
    const uint16_t* ctrl_in;     /* [n_blocks] */
    const uint16_t* ctrl_out;    /* [n_blocks] */
    const int64_t* in_head_in;   /* [n_blocks] */
    const int64_t* in_head_out;  /* [n_blocks] */
    const int64_t* win_left;     /* [n_blocks*tau] */
    const int64_t* win_right;    /* [n_blocks*tau] */
    const uint32_t* off_in;      /* [n_blocks*tau] head_in_offsets */
    const uint32_t* off_out;     /* [n_blocks*tau] head_out_offsets */
    const uint64_t* step_start;  /* [n_blocks+1] prefix offsets into the step arrays */
    const int8_t* input_mv;      /* [total_steps] */
    const int8_t* mv;            /* [total_steps*tau] */
    const uint8_t* has_write;    /* [total_steps*tau] */
    const uint16_t* wsym;        /* [total_steps*tau] (symbol when has_write) */
} sezkp_block_view;

/* ---------------------------------------------------------------- top level
 * StarkV1::prove / prove_streaming (lib.rs:129-141, 170-190): proof_bytes is
 * bincode(ProofV1) (proof.rs:80-98), meta_json the artifact meta. */
int32_t sezkp_stark_v1_prove(const sezkp_block_view* blocks, const uint8_t manifest_root[32], uint32_t flags,
                             sezkp_buf* proof_bytes, sezkp_buf* meta_json, char* err, size_t err_len);
/* Same, returning the whole ProofArtifact as CBOR (io.rs:176-183). */
int32_t sezkp_stark_v1_prove_artifact_cbor(const sezkp_block_view* blocks, const uint8_t manifest_root[32],
                                           uint32_t flags, sezkp_buf* artifact_cbor, char* err, size_t err_len);
/* StarkV1::verify (lib.rs:144-162 -> v1/verify.rs:60-196) on the host CPU. */
int32_t sezkp_stark_v1_verify(const uint8_t* proof_bytes, size_t len, const sezkp_block_view* blocks,
                              const uint8_t manifest_root[32], char* err, size_t err_len);

/* ------------------------------------------------ resident-input context
 * One context = one device + one stream + a workspace sized on upload.
 * upload() builds the device trace image (HBM) from the block view; a
 * re-upload of a trace with the same shape (n, tau, block boundaries) reuses the
 * previous workspace and allocates nothing;
 * prove() then runs the whole prover with inputs resident in HBM. */
typedef struct sezkp_ctx sezkp_ctx;
sezkp_ctx* sezkp_ctx_create(int32_t device, char* err, size_t err_len);
void sezkp_ctx_destroy(sezkp_ctx* ctx);
int32_t sezkp_ctx_upload(sezkp_ctx* ctx, const sezkp_block_view* blocks, char* err, size_t err_len);
/* Upload from a view whose step arrays (input_mv, mv, has_write, wsym) hold
 * only rows [row0, row0 + nrows) (index 0 = row row0; block metadata and
 * step_start stay global): a sharded rank's slice of the trace, as the sliced
 * JSONL ingest decodes it. The slice must contain every row the context reads
 * (sezkp_shard_rows); one device needs the whole trace. */
int32_t sezkp_ctx_upload_rows(sezkp_ctx* ctx, const sezkp_block_view* blocks, uint64_t row0, uint64_t nrows,
                              char* err, size_t err_len);
/* The rows [*row0, *row0 + *nrows) (whole blocks) that rank `rank` of a
 * `world`-GPU sharded prove reads, from the global block boundaries
 * (step_start[0..n_blocks], n = step_start[n_blocks] a power of two). */
int32_t sezkp_shard_rows(const uint64_t* step_start, uint32_t n_blocks, int32_t rank, int32_t world, uint64_t* row0,
                         uint64_t* nrows);
int32_t sezkp_ctx_prove(sezkp_ctx* ctx, const uint8_t manifest_root[32], uint32_t flags, sezkp_buf* proof_bytes,
                        char* err, size_t err_len);
/* Pipelined upload of the NEXT trace: same shape as the uploaded one (tau,
 * block count and block boundaries; the values may all differ). The block
 * tables and step arrays go over PCIe on the context's copy stream into a
 * second (spare) trace image and the call returns at once; the next prove on
 * this context switches to it: that call checks on the host that the copies
 * are done (they normally are) and transposes the step arrays on its own
 * stream, so the copy stream never holds a packet that waits on a copy. Allowed while a proof is in flight on the context (that is the
 * point: the upload of proof i+1 overlaps proof i). The view's arrays must
 * stay valid and unchanged until the proof that consumes them has completed
 * (sezkp_ctx_prove / sezkp_ctx_prove_borrow returned, or sezkp_ctx_wait for
 * sezkp_ctx_prove_async): from pinned or registered memory
 * (sezkp_host_register) the copies are DMA that may still be reading them
 * after the prove call that takes the staged trace has returned. The trace a
 * proof reads is fixed when its prove call is made: a stage() issued right
 * after sezkp_ctx_prove_async fills the other image and feeds the NEXT proof.
 * A trace of another shape: SEZKP_E_INVALID (use sezkp_ctx_upload). */
int32_t sezkp_ctx_stage(sezkp_ctx* ctx, const sezkp_block_view* blocks, char* err, size_t err_len);
/* Page-lock (hipHostRegister) / release caller memory, e.g. the SoA arrays a
 * ProvingBackend shim fills from &[BlockSummary], so staging copies are DMA. */
int32_t sezkp_host_register(void* p, size_t bytes);
int32_t sezkp_host_unregister(void* p);
/* Same proof, borrowed: *data points into the context's pinned host buffer
 * (valid until the next prove/upload/destroy of this context); no copy. */
int32_t sezkp_ctx_prove_borrow(sezkp_ctx* ctx, const uint8_t manifest_root[32], uint32_t flags,
                               const uint8_t** data, size_t* len, char* err, size_t err_len);
/* Per-stage device times (ms) of the last prove, measured with HIP events on
 * the context's stream when SEZKP_STAGE_EVENTS=1 (or SEZKP_KERNEL_EVENTS=1) is
 * set, else 0 (timed events lengthen a proof). Order: expand, col_commit,
 * col_outer, compose, intt, lde_ntt, deep, layer0_tree, layer0_upper,
 * fri_fold_trees, col_openings (the openings kernel alone, on the side
 * stream: it overlaps fri_paths; the query round trip before both is only in
 * total), fri_paths, total, then host wall / sync-wait /
 * final-wait / serialize (always measured),
 * then the FRI forest launch (k_forest16), timed only when
 * SEZKP_KERNEL_EVENTS=1 is set (else 0).
 * Returns the number of values written. */
int32_t sezkp_ctx_stage_times(const sezkp_ctx* ctx, double* out_ms, int32_t max);
/* Asynchronous proving: the context's worker thread runs the proof; wait
 * returns the borrowed proof bytes (as sezkp_ctx_prove_borrow). One proof in
 * flight per context; keep several contexts (one per trace, same device) in
 * flight to overlap one proof's VALU-bound trees with another's memory- and
 * latency-bound stages. Other calls on a context with a proof in flight fail
 * with SEZKP_E_INVALID; destroy waits for it. When a staged trace is
 * pending, this call (like sezkp_ctx_prove) first waits on the host until that
 * trace's copies have finished (a hipStreamQuery poll of the copy stream: no
 * event packet sits in a shared hardware queue) and only then returns; in a
 * pipeline the copies finish long before, but a prove issued right after a
 * stage() of a 67 MB trace blocks for the rest of that upload (a few ms). */
int32_t sezkp_ctx_prove_async(sezkp_ctx* ctx, const uint8_t manifest_root[32], uint32_t flags, char* err,
                              size_t err_len);
int32_t sezkp_ctx_wait(sezkp_ctx* ctx, const uint8_t** data, size_t* len, char* err, size_t err_len);
/* Device hipStream_t of the context (as void*), for external timing. */
void* sezkp_ctx_stream(const sezkp_ctx* ctx);

/* ------------------------------------------------ sharded proving (one proof, P GPUs)
 * One process per GPU; every rank uploads the same blocks and calls prove()
 * with the same manifest root; every rank returns the identical proof bytes.
 * P must be a power of two <= 8 with n >= 4096 * P rows. The LDE domain is
 * split into P cosets (no communication), one all-to-all moves it to a run
 * layout (rank d owns indices i with (i mod 4096P) / 4096 == d), Merkle
 * leaves are hashed per GPU and the tree caps are built from allgathered
 * subtree roots. Replaces nothing in the reference (its prover
 * is single-threaded); the ProvingBackend shim calls it when a communicator
 * is configured. */
/* ncclUniqueId of a new RCCL communicator (rank 0 creates, the caller broadcasts). */
int32_t sezkp_comm_unique_id(uint8_t out[128], char* err, size_t err_len);
sezkp_ctx* sezkp_ctx_create_sharded(int32_t device, int32_t rank, int32_t world, const uint8_t unique_id[128],
                                    char* err, size_t err_len);
/* The same over caller-provided host collectives (buffers are host memory;
 * return 0 on success). */
typedef struct sezkp_host_comm {
  void* user;
  int32_t (*allgather)(void* user, const void* send, void* recv, size_t bytes_per_rank);
  int32_t (*alltoall)(void* user, const void* send, void* recv, size_t bytes_per_rank);
  int32_t (*allreduce_sum_u8)(void* user, void* buf, size_t bytes);
} sezkp_host_comm;
sezkp_ctx* sezkp_ctx_create_sharded_host(int32_t device, int32_t rank, int32_t world, const sezkp_host_comm* comm,
                                         char* err, size_t err_len);
/* Rank `rank` of a `world`-GPU sharded prove ALONE on `device` (the per-rank
 * cost model of a multi-GPU run measured on one GPU): each collective keeps
 * only this rank's own contribution, so the rank's kernels run with their
 * real shapes while the proof bytes are meaningless; sezkp_ctx_comm_stats
 * still reports the bytes every collective would put on the links. */
sezkp_ctx* sezkp_ctx_create_sharded_solo(int32_t device, int32_t rank, int32_t world, char* err, size_t err_len);
/* Failure handling of sharded proving: a rank that fails after the first
 * collective of a prove (a HIP error, a guard trip, a peer that stops
 * answering) aborts its RCCL communicator (ncclCommAbort) and returns
 * SEZKP_E_DEVICE; a rank waiting on a stream that holds collectives polls
 * ncclCommGetAsyncError and gives up after SEZKP_COLL_TIMEOUT_S seconds
 * (default 60), aborting as well, so every rank returns an error instead of
 * blocking. The context is then unusable (every later prove fails): destroy
 * it and create a new communicator.
 * Per-collective device time of the last sharded prove (HIP events around
 * each call on the prover stream) and the bytes this rank sent over the links
 * (allgather (P-1) x its part, all-to-all (P-1) x the per-peer part, allreduce
 * 2 (P-1)/P x the buffer). Returns the number of entries written. */
typedef struct sezkp_comm_stat {
  char name[32];
  uint64_t bytes;
  double ms;
} sezkp_comm_stat;
int32_t sezkp_ctx_comm_stats(const sezkp_ctx* ctx, sezkp_comm_stat* out, int32_t max);

/* Distributed four-step NTT of n = 2^log_n points over the context's P ranks
 * (BASELINE config 4: 2^26 points across 8 GPUs, the transpose as one RCCL
 * all-to-all). Rank g's `local` holds M = n/P elements. Forward (dir=+1):
 * in  local[j] = x[g + P j] (cyclic),
 * out local[k1 Q + q] = X[g Q + q + M k1]  (Q = M/P; rank g owns the k with
 *     (k mod M) / Q == g).
 * Inverse (dir=-1, incl. n^-1) maps the output layout back to the input one.
 * X_k = sum_t x_t w_n^(tk) as in ntt.rs:79-155. `scratch` holds M elements.
 * Asynchronous on sezkp_ctx_stream(ctx); needs 2^(8 + log P) <= n <= 2^32.
 * Any context works (P = 1 for sezkp_ctx_create). Extends the reference:
 * its NTT is single-threaded CPU code with no sharded form. */
int32_t sezkp_ctx_dist_ntt(sezkp_ctx* ctx, uint64_t* local, uint64_t* scratch, uint32_t log_n, int32_t dir,
                           char* err, size_t err_len);

/* ------------------------------------------------ kernel-level entry points
 * Device pointers (u64 canonical Goldilocks, natural order), 32-byte digests
 * (16-byte aligned), stream = hipStream_t (NULL = default stream).
 * Asynchronous on `stream`. Digest counts and lengths up to 2^38. */
/* In-place NTT (dir=+1 forward, -1 inverse incl. n^-1), natural -> natural:
 * ntt.rs:79-155. `scratch` (2^log_n elements, clobbered) is required below 2^8 points and
 * may be null from 2^8 up; given at 2^19..2^22, the transform runs out of place through it
 * and needs no bit-reversal pass (distinct from d). Null device pointers are rejected (SEZKP_E_INVALID) here and in
 * every kernel-level entry point below, before anything is launched. */
int32_t sezkp_gl_ntt(uint64_t* d, uint64_t* scratch, uint32_t log_n, int32_t dir, void* stream);
/* Coset LDE + DEEP (deep_coset_lde_stream, lde.rs:42-97): evals[2^log_n]
 * (base-domain values) -> interpolate (ntt.rs:117-155) -> coset evaluation
 * on shift * <w_N> (coset.rs:85-102) -> out[i] = y_i / (shift * w_N^i - z),
 * N = 2^(log_n + log_blowup), log_blowup <= 3 (the prover: 3, shift 3,
 * prover.rs:119). leaves32 != NULL also writes the N layer-0 leaf digests
 * BLAKE3(out[i] LE) (fri_stream.rs:37-41), 16-byte aligned. `evals` is
 * overwritten. SEZKP_E_INVALID when a denominator vanishes ((z/shift)^N = 1;
 * the prover nudges z off the coset, prover.rs:119-135), shift = 0, or
 * N = 1 (log_n + log_blowup = 0). */
int32_t sezkp_gl_coset_lde_deep(uint64_t* evals, uint32_t log_n, uint32_t log_blowup, uint64_t shift, uint64_t z,
                                uint64_t* out, uint8_t* leaves32, void* stream);
/* FRI fold (prover.rs:208-230): out[i] = in[i] + beta*in[i+n_out], i < n_out
 * (a power of two); inputs canonical. */
int32_t sezkp_fri_fold(const uint64_t* in, uint64_t n_out, uint64_t beta, uint64_t* out, void* stream);
/* The same fold, also hashing the folded leaves into a Merkle tree whose root
 * lands in root32 (host memory; the call synchronises `stream`). */
int32_t sezkp_fri_fold_commit(const uint64_t* in, uint64_t n_out, uint64_t beta, uint64_t* out, uint8_t* root32,
                              void* stream);
/* BLAKE3 leaves of 8-byte LE field values (merkle.rs:150-160) -> Merkle root
 * (merkle.rs:46-71), n a power of two; root32 in host memory (synchronises). */
int32_t sezkp_merkle_root_u64(const uint64_t* vals, uint64_t n, uint8_t* root32, void* stream);
/* hash_field_leaves (merkle.rs:150-160): leaves32[i] = BLAKE3(vals[i] as 8 LE
 * bytes), one 32-byte digest per value. */
int32_t sezkp_blake3_leaves_u64(const uint64_t* vals, uint64_t n, uint8_t* leaves32, void* stream);
/* hash_field_leaves_labeled (merkle.rs:132-147): BLAKE3("col_leaf" || u32 LE
 * label_len || label || vals[i] LE), label_len <= 44 (one BLAKE3 block; the
 * prover's labels are at most 20 bytes, openings.rs:89-116). */
int32_t sezkp_blake3_leaves_labeled(const uint64_t* vals, uint64_t n, const char* label, uint32_t label_len,
                                    uint8_t* leaves32, void* stream);
/* MerkleTree::from_leaves (merkle.rs:46-71): nodes32 receives every level
 * bottom -> top (level 0 = the n leaves, then ceil(len/2) per level, odd
 * promotion carries the last node up), the root last:
 * sezkp_merkle_node_count(n) digests. n = 0 is one all-zero leaf (merkle.rs:48-50).
 * nodes32 may equal leaves32 when it has room for every level. */
uint64_t sezkp_merkle_node_count(uint64_t n);
int32_t sezkp_merkle_build(const uint8_t* leaves32, uint64_t n, uint8_t* nodes32, void* stream);
/* MerkleTree::open (merkle.rs:80-108) of q leaf indices idx[q] (device) in the
 * tree sezkp_merkle_build wrote for n leaves: out32[i * depth + l] = sibling at
 * level l (bottom -> top) of leaf idx[i] % n; a node without a sibling is its
 * own. depth = ceil(log2 n) (0 for n <= 1). */
int32_t sezkp_merkle_paths(const uint8_t* nodes32, uint64_t n, const uint64_t* idx, uint32_t q, uint8_t* out32,
                           void* stream);

/* ------------------------------------------------ host helpers (CPU)
 * Manifest leaf_hash + merkle_root (crates/sezkp-merkle/src/lib.rs:85-157). */
int32_t sezkp_manifest_root(const sezkp_block_view* blocks, uint8_t out[32]);
/* The streaming Frontier root (crates/sezkp-merkle/src/lib.rs:167-208) that
 * commit_block_file / verify_block_file_against_manifest (lib.rs:259-330) use
 * for .jsonl/.ndjson block files; .json/.cbor files use sezkp_manifest_root.
 * The two differ at 7, 11, 13, 14, 15, 19, ... blocks (the reference's own
 * frontier/batch mismatch, kept bit-exact). */
int32_t sezkp_manifest_frontier_root(const sezkp_block_view* blocks, uint8_t out[32]);
/* Decode a CBOR Vec<BlockSummary> (io.rs:57-65). The returned handle owns the
 * arrays a view points to; free with sezkp_blocks_free. */
typedef struct sezkp_blocks sezkp_blocks;
int32_t sezkp_blocks_decode_cbor(const uint8_t* data, size_t len, sezkp_blocks** out, char* err, size_t err_len);
/* JSON Lines, one BlockSummary per line (crates/sezkp-core/src/io_jsonl.rs:43-84;
 * an empty line is an error naming its line number), and its writer
 * (write_block_summaries_jsonl, io_jsonl.rs:93-106). */
int32_t sezkp_blocks_decode_jsonl(const uint8_t* data, size_t len, sezkp_blocks** out, char* err, size_t err_len);
int32_t sezkp_blocks_encode_jsonl(const sezkp_block_view* blocks, sezkp_buf* out);
const sezkp_block_view* sezkp_blocks_view(const sezkp_blocks* b);
void sezkp_blocks_free(sezkp_blocks* b);
/* Sliced ingest (a multi-GPU launcher's rank reads its part of one file):
 * the metadata of the JSONL lines that start in bytes [lo, hi) (cut just past
 * the first newline at or after lo and hi; 0 and len map to themselves, so
 * ranges [len g/P, len (g+1)/P) cover each line exactly once). Every field
 * and each block's step count (step_start) are decoded, the steps are not:
 * the view's step arrays are empty. Line byte offsets via
 * sezkp_blocks_line_offsets, to fully decode a run of lines later with
 * sezkp_blocks_decode_jsonl on data + off[a] .. data + off[b]. */
int32_t sezkp_blocks_decode_jsonl_meta(const uint8_t* data, size_t len, uint64_t lo, uint64_t hi, sezkp_blocks** out,
                                       char* err, size_t err_len);
/* The same lines decoded in full when steps != 0 (the blocks of
 * sezkp_blocks_decode_jsonl on those lines, plus their offsets): a rank
 * decodes its own byte range once and takes its row slice from it. */
int32_t sezkp_blocks_decode_jsonl_lines(const uint8_t* data, size_t len, uint64_t lo, uint64_t hi, int32_t steps,
                                        sezkp_blocks** out, char* err, size_t err_len);
int32_t sezkp_blocks_line_offsets(const sezkp_blocks* b, const uint64_t** offsets, size_t* n);
/* The manifest leaf hashes (sezkp-merkle lib.rs:85-117, 32 bytes per block)
 * and a root over given leaves: the batch merkle_root (frontier = 0,
 * lib.rs:140-157) or the Frontier (frontier = 1, lib.rs:167-208). A sharded
 * launcher hashes each rank's blocks and reduces the gathered leaves. */
int32_t sezkp_manifest_leaf_hashes(const sezkp_block_view* blocks, uint8_t* out);
int32_t sezkp_merkle_root_of_leaves(const uint8_t* leaves, size_t n, int32_t frontier, uint8_t out[32]);
/* Vec<BlockSummary> as CBOR, byte-identical to the reference's writer
 * (io.rs, ciborium; pins: the reference's blocks.cbor fixtures). */
int32_t sezkp_blocks_encode_cbor(const sezkp_block_view* blocks, sezkp_buf* out);
/* The reference's input producer, bit-exact (`sezkp-cli simulate`, main.rs:317-350):
 * generate_trace (sezkp-trace generator.rs:38-73, rand 0.9.2 StdRng seeded by
 * seed_from_u64(seed); the reference always uses 42) into step-major arrays
 * input_mv[t], mv/has_write/wsym[t][tau] ... */
int32_t sezkp_simulate_trace(uint64_t t, uint32_t tau, uint64_t seed, int8_t* input_mv, int8_t* mv,
                             uint8_t* has_write, uint16_t* wsym);
/* ... and partition_trace (partition.rs:43-150) into blocks of b steps;
 * free with sezkp_blocks_free. */
int32_t sezkp_simulate_blocks(uint64_t t, uint32_t b, uint32_t tau, uint64_t seed, sezkp_blocks** out, char* err,
                              size_t err_len);
/* Decode a manifest file (sezkp-merkle commit output: {root: [32], n_leaves}),
 * CBOR or JSON (is_json != 0). */
int32_t sezkp_manifest_decode(const uint8_t* data, size_t len, int32_t is_json, uint8_t root[32],
                              uint32_t* n_leaves, char* err, size_t err_len);
/* BLAKE3 hash with extendable output (host). */
void sezkp_blake3(const uint8_t* data, size_t len, uint8_t* out, size_t out_len);

/* Fiat-Shamir transcript challenges, the core of
 * Blake3Transcript::challenge_bytes (crates/sezkp-crypto/src/lib.rs:102-123)
 * for a batch, on the host with the prover's BLAKE3:
 * out_i = BLAKE3-XOF(stream[0..pos[i]) || suffix_i, out_len[i]) with suffix_i
 * the next sfx_len[i] bytes of `suffixes` (a transcript passes "challenge" ||
 * u32 LE len || label). Outputs are concatenated in `out` (sum of out_len
 * bytes). The known-answer interface of the prover's transcript. `stream` is
 * ignored (ABI 3 ran a device kernel on it; ABI 4 answers on the host). */
int32_t sezkp_fs_xof(const uint8_t* stream_bytes, size_t stream_len, const uint32_t* pos, const uint8_t* suffixes,
                     const uint32_t* sfx_len, const uint32_t* out_len, uint32_t nchal, uint8_t* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SEZKP_STARK_H */

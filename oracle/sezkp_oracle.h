/*
 * sezkp_oracle.h — CPU ORACLE (test infrastructure only).
 *
 * This is a plain-C restatement of the reference STARK v1 prover path of
 * logannye/streaming-zero-knowledge-proofs (Rust; unbuildable here: no cargo,
 * no crates.io cache — see DESIGN.md §Oracle).  It exists ONLY to check the
 * MI355X product path: tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product library never links or calls it.
 *
 * Every function cites the reference file:line it restates.  Field arithmetic
 * deliberately mirrors the reference (u128 `%` reduction, Fermat inversion),
 * BLAKE3 is restated from its published spec (crates.io blake3 1.8.2 is the
 * pinned dependency, Cargo.lock:125).
 *
 * Pinning: BLAKE3 known-answer vectors, the reference's committed manifest
 * roots (blocks.cbor / examples/minimal-riscv) and the two committed v0 proof
 * envelopes (transcript framing + XOF) — tests/test_oracle_fixtures.py.
 */
#ifndef SEZKP_ORACLE_H
#define SEZKP_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Flattened, struct-of-arrays view of Vec<BlockSummary>
 * (crates/sezkp-core/src/types.rs:116-151). All per-block vectors
 * (windows, offsets, pre/post tags) have exactly `tau` entries; every step
 * has exactly `tau` tape ops. */
typedef struct {
    uint32_t n_blocks;
    uint32_t tau;
    const uint16_t *version;     /* [n_blocks] */
    const uint32_t *block_id;    /* [n_blocks] */
    const uint64_t *step_lo;     /* [n_blocks] */
    const uint64_t *step_hi;     /* [n_blocks] */
    const uint16_t *ctrl_in;     /* [n_blocks] */
    const uint16_t *ctrl_out;    /* [n_blocks] */
    const int64_t *in_head_in;   /* [n_blocks] */
    const int64_t *in_head_out;  /* [n_blocks] */
    const int64_t *win_left;     /* [n_blocks*tau] */
    const int64_t *win_right;    /* [n_blocks*tau] */
    const uint32_t *off_in;      /* [n_blocks*tau] */
    const uint32_t *off_out;     /* [n_blocks*tau] */
    const uint64_t *step_start;  /* [n_blocks+1] prefix offsets into step arrays */
    const int8_t *input_mv;      /* [total_steps] */
    const int8_t *mv;            /* [total_steps*tau] */
    const uint8_t *has_write;    /* [total_steps*tau] */
    const uint16_t *wsym;        /* [total_steps*tau] (value when has_write) */
} orc_blocks;

/* ---- Goldilocks (crates/sezkp-ffts/src/lib.rs:57-133, 229-242) ---- */
uint64_t orc_gl_mul(uint64_t a, uint64_t b);
uint64_t orc_gl_inv(uint64_t a);
uint64_t orc_gl_root_2exp(uint32_t k);

/* ---- NTT (crates/sezkp-ffts/src/ntt.rs:79-155, coset.rs:85-102) ---- */
void orc_ntt_forward(uint64_t *a, size_t n);
void orc_ntt_inverse(uint64_t *a, size_t n);
void orc_coset_lde(const uint64_t *coeffs, size_t m, uint32_t k_log2, uint64_t shift, uint64_t *out);
void orc_det_vec(uint64_t *out, size_t n, uint64_t seed); /* benches/ntt.rs:21-34 */
void orc_lde_deep(const uint64_t *base_vals, size_t n, unsigned blow_log2, uint64_t z, uint64_t *out); /* lde.rs:42-97 */

/* ---- BLAKE3 (spec restatement of crates.io blake3 1.8.2) ---- */
void orc_blake3(const uint8_t *in, size_t len, uint8_t *out, size_t out_len);

/* ---- Transcript (crates/sezkp-crypto/src/lib.rs:74-123) ---- */
typedef struct orc_transcript orc_transcript;
orc_transcript *orc_tr_new(const char *domain);
void orc_tr_free(orc_transcript *t);
void orc_tr_absorb(orc_transcript *t, const char *label, const uint8_t *bytes, size_t len);
void orc_tr_absorb_u64(orc_transcript *t, const char *label, uint64_t x);
void orc_tr_challenge(orc_transcript *t, const char *label, uint8_t *out, size_t n);

/* ---- Merkle (stark v1 merkle.rs:46-126; sezkp-merkle lib.rs:85-208) ---- */
void orc_merkle_root(const uint8_t *leaves32, size_t n, uint8_t root[32]);        /* v1 MerkleTree::from_leaves().root() */
void orc_manifest_leaf_hash(const orc_blocks *b, uint32_t k, uint8_t out[32]);   /* sezkp-merkle leaf_hash */
void orc_manifest_root(const orc_blocks *b, uint8_t out[32]);                    /* commit_blocks / merkle_root */
void orc_manifest_frontier_root(const uint8_t *leaves32, size_t n, uint8_t out[32]); /* Frontier (JSONL path) */
size_t orc_merkle_nodes(const uint8_t *leaves32, size_t n, uint8_t *out);            /* from_leaves: all levels */
size_t orc_merkle_open(const uint8_t *leaves32, size_t n, const uint64_t *idx, size_t q, uint8_t *sibs); /* open */
void orc_lde_deep_shift(const uint64_t *base_vals, size_t n, unsigned blow_log2, uint64_t shift, uint64_t z,
                        uint64_t *out);                                                   /* lde.rs:42-97 */
void orc_hash_leaf_u64(uint64_t v, uint8_t out[32]);                             /* merkle.rs:150-160 */
void orc_hash_leaf_labeled(uint64_t v, const char *label, uint8_t out[32]);     /* merkle.rs:132-147 */

/* ---- v0 StarkIOP transcript (sezkp-stark/src/lib.rs:66-95, commit.rs:47-90) ---- */
int orc_v0_proof(const orc_blocks *b, const uint8_t manifest_root[32], uint8_t out64[64], uint64_t *n_rows);

/* ---- v1 prover (sezkp-stark/src/v1/prover.rs:61-462) ----
 * mode 0: compute-once (identical bytes, no recomputation).
 * mode 1: reference-faithful recomputation structure (CPU timing only).
 * Returns 0 on success, <0 on error (message in err). *out is malloc'd. */
int orc_prove_v1(const orc_blocks *b, const uint8_t manifest_root[32], int mode,
                 uint8_t **out, size_t *out_len, char *err, size_t err_len);
/* Intermediate views for tests (compute-once): column roots [(3+7tau)*32],
 * layer-0 LDE values [8n], fri roots [(k+1)*32]. Any pointer may be NULL. */
int orc_prove_v1_debug(const orc_blocks *b, const uint8_t manifest_root[32],
                       uint8_t *col_roots, uint64_t *base_evals, uint64_t *lde_vals,
                       uint8_t *fri_roots, char *err, size_t err_len);
void orc_free(void *p);
/* OpenMP threads of the compute-once path (libsezkp_oracle_mt.so); returns the count in use (1 without OpenMP) */
int orc_set_threads(int n);

/* Time one reference-faithful LDE+layer-0 pass (the unit the reference
 * repeats 1+60k times, prover.rs:312-398); returns seconds. */
double orc_time_lde_pass(const orc_blocks *b, const uint8_t manifest_root[32]);

#ifdef __cplusplus
}
#endif
#endif

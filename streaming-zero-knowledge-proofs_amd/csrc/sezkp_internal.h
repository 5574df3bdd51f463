// sezkp_internal.h — structures shared by the HIP kernels and the host
// orchestrator of the MI355X STARK v1 prover (not part of the public C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace sezkp {

struct DevChal;        // transcript-derived values in device memory (below)
struct ComposeTerms;   // per-row composition sums (below)

// w_{2^K}^e = hi[e >> S] * lo[e & (2^S - 1)]; p3_* likewise for 3^e.
struct NttTables {
  const uint64_t* hi;
  const uint64_t* lo;
  const uint64_t* p3_hi;
  const uint64_t* p3_lo;
  int K;
  int S;
};

struct NttPassArgs {
  uint64_t* a;
  const uint64_t* src;  // replicated LDE load source (bit-reversed coeffs), or null
  NttTables tw;
  uint64_t inv_n;
  uint64_t coset_e;  // LDE load: extra factor w_{2^K}^(coset_e * bitrev(k)) (sharded coset), 0 = none
  int m, sL, logC, inverse, skip, log_src;
  // src layout: 0 = the n coefficients bit-reversed (one n-point DIF INTT);
  // s > 0 = the sharded INTT's allgather: coefficient e at
  // (e mod 2^s) * (n >> s) + bitrev_{log n - s}(e >> s)
  int src_logP;
  // fused DEEP on the last forward pass (k_ntt4<..., DEEP = true>)
  uint64_t deep_z;
  int deep_logN, deep_logP;
  uint32_t deep_g;
  // DEEP quotient LDE (first DIT pass, SKIP = 0): position p loads
  // h_e = [e < n] src[p >> 3] n^-1 3^e + rhi[e >> 12] rlo[e & 4095], e = bitrev(p)
  const uint64_t* dp_rlo;
  const uint64_t* dp_rhi;
  const uint64_t* dp_rhk;
  int dp_logN;
  // out-of-place DIF store (null = in place); nat_out: the last (narrow) DIF
  // pass writes position p to out[bitrev_{nat_logN}(p)] * out_scale, i.e. the
  // transform leaves in natural order without a bit-reversal pass
  uint64_t* out;
  int nat_out, nat_logN;
  uint64_t out_scale;
  // nat_tr: the last (narrow, m <= 8) DIF pass gathers the 16 blocks whose
  // outputs share 128-B lines and stores them transposed into natural order
  // (ntt.hip gather_to_lds / lds_to_transposed)
  int nat_tr;
};
// DEEP division y_i / (3 w_N^(g + P i) - z) fused into the LDE's last pass
struct DeepFuse {
  uint64_t z;
  int logN, logP;
  uint32_t g;
};
// DEEP as a polynomial: y_i / (x_i - z) = H(x_i) with H = q + c S,
// q = (f - f(z)) / (X - z), S = sum_k z^(N-1-k) X^k and c = f(z) / (3^N - z^N)
// (x_i^N = 3^N on the coset), so the LDE of H's coefficients
// h_k = q_k 3^k + c' r^k (r = 3/z, c' = c z^(N-1)) IS the DEEP layer: no
// per-point inversion. f(z) is the barycentric sum (1 - z^n)/n *
// sum_j C_j w^j / (w^j - z). The INTT does not wait for f(z): on the base
// domain q(w^j) = D_j - f(z) / (w^j - z) with D_j = C_j / (w^j - z), and the
// interpolant of 1 / (w^j - z) has the coefficients z^(n-1-k) / (1 - z^n), so
// q_k = d_k - f(z) z^(n-1-k) / (1 - z^n), and q_k 3^k = d_k 3^k - kappa r^k
// with kappa = f(z) z^(n-1) / (1 - z^n) = K3 S. The INTT runs on D and the
// LDE's first pass subtracts kappa r^k for k < n; f(z) (the partial sums) is
// needed only there, so sharded ranks gather it with the INTT coefficients.
struct DeepPoly {
  const uint64_t* rlo;  // 4096 entries: r^t
  const uint64_t* rhi;  // N >> 12 entries: c' r^(4096 t)
  const uint64_t* rhk;  // max(1, n >> 12) entries: kappa r^(4096 t)
};
// over a block of base rows [row0, row0 + nrows) (row0 a multiple of per):
// D_j = C_j / (w^j - z) into D, C_j = compose_value of the row's terms (one
// Montgomery batch inversion per `per` rows), and this block's partial sums
// of C_j w^j / (w^j - z) at partial[row0 / per ...] (z, alphas, mask from ch)
// (partials of `per` rows each: dq_rows_per_part of the block's row count,
// the same on every rank)
uint64_t dq_rows_per_part(uint64_t nrows);
hipError_t launch_inv_base(hipStream_t st, const ComposeTerms& Tm, uint64_t* D, uint64_t* partial, int logn,
                           const DevChal* ch, const NttTables& T, uint64_t row0, uint64_t nrows, uint64_t per);
// once every partial of the n rows is in `partial`: f(z) = K1 S, the DeepPoly
// tables rlo / rhi / rhk (K1, K2, K3, rho, rho^4096 from ch)
hipError_t launch_q_tables(hipStream_t st, const uint64_t* partial, int logn, int logN, const DevChal* ch,
                           uint64_t* rlo, uint64_t* rhi, uint64_t* rhk, uint64_t per);

hipError_t ntt_dif(hipStream_t st, uint64_t* a, int logN, bool inverse, const NttTables& T);
// natural order in and out through `scratch` (n words): the first pass reads a
// and writes scratch, the last scatters scratch back to a in natural order
// (times scale). False = this size takes ntt_dif + a bit reversal instead.
bool ntt_dif_natural(hipStream_t st, uint64_t* a, uint64_t* scratch, int logN, bool inverse, const NttTables& T,
                     uint64_t scale, hipError_t* err);
// deep != nullptr: fuse the DEEP division into the last pass when its shape
// allows; *fused says whether it did (else the caller runs launch_deep).
hipError_t ntt_dit(hipStream_t st, uint64_t* a, int logN, bool inverse, const NttTables& T,
                   const uint64_t* src, int log_src, uint64_t inv_n, uint64_t coset_e = 0,
                   const DeepFuse* deep = nullptr, bool* fused = nullptr, const DeepPoly* dpoly = nullptr,
                   int src_logP = 0);
hipError_t bitrev_permute(hipStream_t st, const uint64_t* in, uint64_t* out, int logN, uint64_t scale,
                          bool do_scale);
hipError_t bitrev_inplace(hipStream_t st, uint64_t* a, int logN, uint64_t scale, bool do_scale);  // logN >= 8
// distributed four-step NTT pieces (ntt.hip)
hipError_t dntt_permute_twiddle(hipStream_t st, const uint64_t* in, uint64_t* out, int logM, const NttTables& T,
                                uint64_t e_step, bool inverse, bool tw_src, uint64_t scale);
hipError_t dntt_dft(hipStream_t st, uint64_t* r, int P, uint64_t Q, bool inverse);
// sharded INTT (block layout in): after the first all-to-all rank d holds
// r[g Q + t] = x[g m + d Q + t] (m = n / P, Q = m / P); in place
// r[k1 Q + t] = w_n^-(j k1) sum_g w_P^-(g k1) r[g Q + t], j = d Q + t
hipError_t bintt_dft_twiddle(hipStream_t st, uint64_t* r, int P, uint64_t Q, uint32_t d, int logn,
                             const NttTables& T);

// A binary Merkle tree over 2^logLen leaves whose levels >= lstore are kept
// in HBM: level l (lstore <= l <= logLen) starts at node
// off(l) = 2^(logLen-lstore+1) - 2^(logLen-l+1); 8 u32 words per node.
// Lower levels are recomputed from the leaf values when a path is opened.
struct TreeDev {
  uint32_t* nodes;
  uint32_t* root;   // 8 words
  int logLen;
  int lstore;
};
__host__ __device__ inline uint64_t tree_level_off(int logLen, int lstore, int l) {
  return (1ULL << (logLen - lstore + 1)) - (1ULL << (logLen - l + 1));
}
__host__ __device__ inline uint64_t tree_stored_nodes(int logLen, int lstore) {
  return logLen >= lstore ? (1ULL << (logLen - lstore + 1)) - 1 : 0;
}

// Device image of the trace (struct-of-arrays, tape-major), built by upload.
struct TraceDev {
  uint64_t n;
  int tau;
  uint32_t nblk;
  const int8_t* input_mv;     // [n]
  const int8_t* mv;           // [tau][n]
  const uint8_t* wflag;       // [tau][n]
  const uint16_t* wsym;       // [tau][n]  (0 when no write)
  const uint64_t* blk_start;  // [nblk+1] row offsets
  const uint64_t* blk_winlen; // [tau][nblk] canonical field values
  const uint64_t* blk_offin;  // [tau][nblk]
  const uint64_t* blk_offout; // [tau][nblk]
  uint32_t* row_blk;          // [n]   (derived)
  uint8_t* row_flags;         // [n]   bit0 first, bit1 last (derived)
  int32_t* head;              // [tau][n] post-move head (derived; block-local; k_expand rejects |head| >= 2^31)
  int64_t* head_rng;          // [tau][nblk][2] per-block min / max of head (derived by k_expand)
};

// Per-row constraint sums of the composition (k_compose_terms): everything
// of C(i) that does not depend on the transcript, summed over the tapes
// exactly (integers where they are small, canonical field values otherwise).
// Rows [row0, row_end) of this device; the boundary sums once per block.
struct ComposeTerms {
  uint64_t* hr;               // [n] sum of head - (head & 0xFFFF) over written tapes
  uint64_t* sl;               // [n] sum of slack - (slack & 0xFFFF) over written tapes
  int64_t* c3;                // [n] head-update sum (1 - is_last) (head' - head - mv')
  int32_t* c2;                // [n] mv domain sum mv^3 - mv
  int32_t* sy;                // [n] symbol sum sym & ~0xF over written tapes
  uint64_t* bf;               // [nblk] boundary_first sum of the block's first row
  uint64_t* bl;               // [nblk] boundary_last sum of the block's last row
  const uint8_t* row_flags;   // = TraceDev::row_flags
  const uint32_t* row_blk;    // = TraceDev::row_blk
};

// guard word bits (d_err): a kernel saw input it cannot represent
constexpr uint32_t GUARD_HEAD_RANGE = 0x100u;  // k_expand: a head outside i32

struct Alphas {
  uint64_t bool_flag, mv_domain, head_update, head_bits_bool, head_reconstruct, slack_bits_bool,
      slack_reconstruct, sym_bits_bool, sym_reconstruct, boundary_first, boundary_last;
};

// Per-column BLAKE3 message template for labelled leaves
// BLAKE3("col_leaf" || u32 len || label || v LE)  (merkle.rs:132-147).
struct ColTemplate {
  uint32_t words[16];
  uint32_t block_len;  // 20 + len(label)
  uint32_t kind;       // 0 input_mv,1 is_first,2 is_last,3+k: per-tape kind k
  uint32_t tape;
  uint32_t off;        // byte offset of the value = 12 + len(label)
  uint64_t tab;        // node offset of this column's leaf/uniform table, or NO_TAB
  uint32_t tab_log;    // leaf table: log2(entries) (8 or 16); 0 otherwise
  uint32_t pad;
};
constexpr uint64_t NO_TAB = ~0ULL;
constexpr int U_LEVELS = 11;  // uniform-subtree hashes U_0..U_10 (chunk = 2^10 rows)

// Column kinds whose leaf depends on a small raw domain (i8 / u8 / u16):
// leaves come from a per-column table of all possible labelled leaves.
__host__ __device__ inline bool kind_has_leaf_table(uint32_t kind) { return kind == 0 || kind == 3 || kind == 4 || kind == 5; }
// Columns that are piecewise constant along the trace (per-block constants and
// the block-boundary flags): committed from uniform-subtree hashes.
__host__ __device__ inline bool kind_piecewise(uint32_t kind) { return kind == 1 || kind == 2 || kind >= 7; }

// Dictionary (memoized subtree) commitment of dense small-range columns.
constexpr int DICT_LEVELS = 5;          // tables T_0..T_4
constexpr uint32_t DICT_CAP = 65536;    // entries per table level
struct DictCol {
  uint32_t col;
  uint32_t mv;   // head columns: dictionary index of the same tape's mv column (delta plan), else NO_DICT
  uint64_t tab;  // node offset of this column's DICT_LEVELS x DICT_CAP tables
};
struct DictPlan {
  int64_t min;
  uint32_t R;    // range size (codes = raw - min < R)
  int32_t K;     // table level used by the commit kernel; -1 = leaves computed
  uint32_t pw[DICT_LEVELS];  // entries of T_k = R^(2^k) (0 above K)
  uint32_t delta;  // head delta plan: K = 2 and slot 2 holds TD (below)
  int64_t dmin;    // delta plan: range of the tape's moves
  uint32_t dR;
  uint32_t a;      // rows per commit lane = 2^(6 + a): dict_extra(K), lowered for few rows (k_dict_plan)
};
// Head delta plan: inside a block head[r] = head[r-1] + mv[r], so an aligned
// 4-row head group is a function of (head[g], mv[g+1], mv[g+2], mv[g+3]):
// TD[c0 + R (d1 + dR d2 + dR^2 d3)] = H(T_1[c0 + R c1], T_1[c2 + R c3]) with
// c_j = c_{j-1} + mv_j (codes). Groups with a block start at g+1..g+3 use
// the two T_1 nodes directly. Needs R^2 <= DICT_CAP and R dR^3 <= DICT_CAP.
__host__ __device__ inline bool kind_dict(uint32_t kind) { return kind == 0 || (kind >= 3 && kind <= 6); }
// Chunk levels 6..9 of every dictionary column (16 + 8 + 4 + 2 nodes per
// 1024-row chunk), written by the commitment, read by the openings.
constexpr int DICT_LANE_LOG = 6;  // rows per lane of the dictionary commitment (level-6 nodes)
constexpr int DLEV_NODES = 30;
__host__ __device__ inline int dlev_base(int level) { return level == 6 ? 0 : level == 7 ? 16 : level == 8 ? 24 : 28; }
constexpr uint32_t NO_DICT = 0xFFFFFFFFu;
// extra lane rows (log2) of the dictionary commitment for table level K:
// high K leaves few table nodes per 64 rows, so lanes take 2^(6+a) rows
__host__ __device__ inline int dict_extra(int K) { return K >= 3 ? 2 : (K == 2 ? 1 : 0); }
constexpr int OPEN_REQ_WORDS = 5;  // column, row lo, row hi, ordinal, dictionary index

constexpr int LSTORE_FRI = 6;
constexpr int COL_CHUNK_LOG2 = 10;
// Device image of the bincode ProofV1 body (proof.rs:80-98) after the
// column-root header: every record there is 8-byte aligned and fixed-size,
// so the opening and path kernels write proof bytes in place.
//   0                 u64 #queries
//   8 + q*q_bytes     u64 row, u64 tau, then open_per_q openings of open_bytes
//   fr_off            u64 k+1, (k+1) x 32 B FRI roots            (host)
//   fq_off            u64 #queries
//   fq_off+8+q*fq_bytes  u64 k+1, k+1 positions, u64 k, 2k path records
//   tail_off          final value (8 B), manifest root (32 B)     (root: host)
struct ProofLayout {
  uint32_t* base;          // device pointer, 8-byte aligned
  uint64_t open_bytes;     // 80 + 32*log2(n)
  uint64_t q_bytes;        // 16 + open_per_q * open_bytes
  uint64_t fr_off, fq_off, fq_bytes, tail_off, total;
  uint32_t open_per_q;     // 9*tau + 3
  uint32_t nq;             // queries (params.rs:31)
  int k;                   // log2(N)
  uint32_t tau;
};

// ------------------------------------------------- Fiat-Shamir challenges
// The transcript-derived values every challenge-dependent kernel reads from
// device memory, written by the host transcript (one H2D copy per point).
constexpr int FS_MAX_BETAS = 64;
struct DevChal {
  uint64_t alpha[8];                // derive_alphas (params.rs:82-92); reuse of prover.rs:86-98 in the kernels
  uint64_t mask[4];                 // derive_mask_coeffs (masking.rs:56-79)
  uint64_t z, zn, K1, K2, rho, rho4096;  // OOD point (nudged) and the DEEP-polynomial constants
  uint64_t K3;                      // z^(n-1) / n: kappa = K3 S (DeepPoly, the q correction)
  uint64_t beta[FS_MAX_BETAS];      // derive_betas_for_fri (params.rs:109-119)
};

// kernels launched by the host orchestrator (prover.cpp)
// blocks [blk_lo, blk_lo + blk_cnt) only (a sharded rank's rows + one row of halo)
// row-major step arrays [n][tau] -> tape-major trace image [tau][n], rows [r0, r1)
hipError_t launch_trace_image(hipStream_t st, const int8_t* raw_mv, const uint8_t* raw_hw, const uint16_t* raw_ws,
                              uint64_t n, int tau, int8_t* mv, uint8_t* wf, uint16_t* ws, uint64_t r0 = 0,
                              uint64_t r1 = ~0ull);
// d_err: guard word, GUARD_HEAD_RANGE is or-ed in when a head leaves the i32 range
hipError_t launch_expand(hipStream_t st, const TraceDev& T, uint32_t blk_lo, uint32_t blk_cnt, uint32_t* d_err);
hipError_t launch_col_tables(hipStream_t st, const TraceDev& T, const ColTemplate* d_tmpl, const uint32_t* d_tab_cols,
                             int n_tab_cols, uint64_t tab_entries, uint32_t* tabs, uint32_t blk_lo, uint32_t blk_cnt);
hipError_t launch_col_commit(hipStream_t st, const TraceDev& T, const ColTemplate* d_tmpl, const uint32_t* d_work,
                             int nwork, const uint32_t* tabs, uint32_t* outer_nodes, uint64_t outer_stride_nodes);
// rows [row0, row0 + nrows) of every dictionary column (row0, nrows multiples of 4096 or the whole trace)
hipError_t launch_dict_commit(hipStream_t st, const TraceDev& T, const ColTemplate* d_tmpl, const DictCol* d_dcols,
                              int ndict, int64_t* d_part, DictPlan* d_plans, uint32_t* d_dtabs, uint32_t* outer_nodes,
                              uint64_t outer_stride_nodes, uint64_t row0, uint64_t nrows, uint32_t* d_dlev,
                              uint32_t tab_cap = DICT_CAP);
// the same in three steps, so the commit of the columns whose table level K
// is built early can run beside the later levels: ranges + plans, table
// levels [lvl_lo, lvl_hi), and the commit of the columns with kmin <= K <= kmax
hipError_t launch_dict_prepare(hipStream_t st, const TraceDev& T, const ColTemplate* d_tmpl, const DictCol* d_dcols,
                               int ndict, int64_t* d_part, DictPlan* d_plans, uint64_t row0, uint64_t nrows,
                               uint32_t tab_cap = DICT_CAP);
hipError_t launch_dict_levels(hipStream_t st, const ColTemplate* d_tmpl, const DictCol* d_dcols, int ndict,
                              const DictPlan* d_plans, uint32_t* d_dtabs, int lvl_lo, int lvl_hi);
hipError_t launch_dict_commit_cols(hipStream_t st, const TraceDev& T, const ColTemplate* d_tmpl,
                                   const DictCol* d_dcols, int ndict, const DictPlan* d_plans,
                                   const uint32_t* d_dtabs, uint32_t* outer_nodes, uint64_t outer_stride_nodes,
                                   uint64_t row0, uint64_t nrows, uint32_t* d_dlev, int kmin, int kmax);
hipError_t launch_col_commit_pw(hipStream_t st, const TraceDev& T, const ColTemplate* d_tmpl, const uint32_t* d_pw_cols,
                                int n_pw_cols, const uint32_t* d_chunks, int nchunks, const uint32_t* tabs,
                                uint32_t* outer_nodes, uint64_t outer_stride_nodes, uint32_t* d_err);
// composition, rows [row0, row0 + nrows) (nrows = n for the whole trace):
// the transcript-independent row sums (ComposeTerms), then C(i) from them
// with the alphas and mask coefficients of ch (device memory)
hipError_t launch_compose_terms(hipStream_t st, const TraceDev& T, const ComposeTerms& Tm, uint64_t row0,
                                uint64_t nrows);
hipError_t launch_compose_combine(hipStream_t st, const ComposeTerms& Tm, const DevChal* ch, const NttTables& tw,
                                  int logn, uint64_t* out, uint64_t row0, uint64_t nrows);
// DEEP divide of y[j] at x = shift * w_{2^logN}^(g + (j << logP)) (logP = 0, g = 0: natural layout)
hipError_t launch_deep(hipStream_t st, uint64_t* y, int logN, uint64_t z, const NttTables& tw, int logP = 0,
                       uint32_t g = 0, uint64_t shift = 3);
// a[p] *= base^bitrev_logn(p) (tables lo[2048] | hi[max(1, n >> 11)] in `scratch`)
hipError_t launch_scale_pow_bitrev(hipStream_t st, uint64_t* a, int logn, uint64_t base, uint64_t* scratch);
// kernel-level ABI helpers (api_kernels.hip); digests are 8 u32 words
hipError_t launch_fold_any(hipStream_t st, const uint64_t* in, uint64_t* out, uint64_t n_out, uint64_t beta);
hipError_t launch_leaves_u64(hipStream_t st, const uint64_t* v, uint64_t n, uint32_t* out);
hipError_t launch_leaves_labeled(hipStream_t st, const uint64_t* v, uint64_t n, const ColTemplate& ct, uint32_t* out);
// one MerkleTree level with odd promotion: out[i] = H(in[2i] || in[2i+1]), or in[2i] when 2i+1 == len
hipError_t launch_merkle_level(hipStream_t st, const uint32_t* in, uint64_t len, uint32_t* out);
struct MerkleLevels {
  uint64_t off[64];  // node offset of level l (level 0 = the leaves)
  uint64_t len[64];
  int depth;         // levels above the leaves
};
// q paths of `depth` siblings: path i, level l = sibling of (idx[i] % len[0]) >> l
hipError_t launch_merkle_paths(hipStream_t st, const uint32_t* nodes, const MerkleLevels& L, const uint64_t* idx,
                               uint32_t q, uint32_t* out);
// Sharded LDE layout change (see prover.cpp, prove_sharded): cyclic coset
// values of rank g (index g + P*j) <-> runs of S = 2^12 consecutive indices.
hipError_t launch_cyc_pack(hipStream_t st, const uint64_t* cyc, uint64_t* send, uint64_t M, int logP);
hipError_t launch_cyc_unpack(hipStream_t st, const uint64_t* recv, uint64_t* local, uint64_t M, int logP);
// gathered[d][k1] (run roots of rank d) -> level-12 node k1*P + d of `cap`
// rank g's runs of 4096 (local index k1 S + t = global (k1 P + g) S + t) out
// of the whole N-point LDE (sharded P = 2)
hipError_t launch_runs_extract(hipStream_t st, const uint64_t* full, uint64_t* local, uint64_t M, int logP,
                               uint32_t g);
constexpr int RR_BATCH_MAX = 40;
struct RunRootsBatch {
  const uint32_t* gathered[RR_BATCH_MAX];
  TreeDev cap[RR_BATCH_MAX];
  uint64_t nrun[RR_BATCH_MAX];  // runs per rank
  int n, logP;
};
hipError_t launch_runroots_scatter_multi(hipStream_t st, const RunRootsBatch& B);
hipError_t launch_runroots_scatter(hipStream_t st, const uint32_t* gathered, TreeDev cap, uint64_t nrun_per_rank,
                                   int logP);
// dbeta != null: the fold challenge is read from device memory instead of `beta`
hipError_t launch_leaf_subtree(hipStream_t st, const uint64_t* in, uint64_t* out_vals, int logLen, int fold,
                               uint64_t beta, TreeDev tree, const uint64_t* dbeta = nullptr);
hipError_t launch_tree_upper(hipStream_t st, TreeDev* trees, int ntrees_same_shape, uint64_t tree_stride_nodes,
                             uint64_t root_stride_words, int from_level);
// A FRI layer as seen by the path kernel. Unsharded: vals/tree hold the
// whole layer and cap == tree. Sharded run layers: vals/tree are this rank's
// runs (global index i -> local ((i >> (12+logP)) << 12) | (i & 4095), tree
// levels < 12 valid) and cap holds levels >= 12 with global indices.
struct FriLayerDev {
  const uint64_t* vals;
  TreeDev tree;
  TreeDev cap;
  uint32_t sharded;
  uint32_t logP;
};
// Upper-level reduction job: one WG reduces <= 1024 stored nodes of `tree`
// from level `from` (WG index wg within that level).
struct UpperJob {
  TreeDev tree;
  int from;
  uint32_t wg;
  int to;  // last level to build (0: up to the root)
  uint32_t pad;
  // sharded cap of a run layer: level `from` (12) comes from the allgathered
  // run roots (rank-major: rank d's nrun roots at [d nrun, (d + 1) nrun)),
  // cap node g = root g >> logP of rank g & (P - 1); the job stores it too
  const uint32_t* gath = nullptr;
  uint64_t nrun = 0;
  int logP = 0;
  int pad2 = 0;
};
void plan_upper_jobs(const TreeDev& T, int from, std::vector<std::vector<UpperJob>>& passes, int to = 0,
                     const uint32_t* gath = nullptr, uint64_t nrun = 0, int logP = 0);
hipError_t launch_upper_jobs(hipStream_t st, const UpperJob* d_jobs, int njobs);

constexpr int L16_LOG = 12;  // leaves per WG of the 16-leaves-per-lane layer kernel
constexpr int L16S_LOG = 10; // leaves per WG of its 4-leaves-per-lane form (small trees)
constexpr int L16M_LOG = 11; // leaves per WG of its 8-leaves-per-lane form
// stop: highest level the WG reduces to (L16_LOG = its run root; LSTORE_FRI
// leaves levels 7..12 to the upper jobs, whose lanes are all busy)
// wg_log: leaves per WG (L16_LOG, or L16S_LOG for trees too small to fill
// the chip with 4096-leaf WGs); stop <= wg_log
hipError_t launch_layer16(hipStream_t st, const uint64_t* in, uint64_t* out_vals, int logLen, int fold, uint64_t beta,
                          TreeDev tree, int stop = L16_LOG, const uint64_t* dbeta = nullptr, int wg_log = L16_LOG);
// Fold chain kernel (values only) and the one-launch forest of layer trees.
hipError_t launch_fold(hipStream_t st, const uint64_t* in, uint64_t* out, int logLen, uint64_t beta,
                       const uint64_t* dbeta = nullptr);
// F = 2..FOLD_MAX folds in one pass (k_foldm): out[m-1] = layer r + m, beta[m-1] its challenge
constexpr int FOLD_MAX = 4;
struct FoldOuts {
  uint64_t* out[FOLD_MAX];
  const uint64_t* beta;  // device: beta[m - 1] folds layer r + m - 1 (the pass's first challenge)
};
hipError_t launch_foldm(hipStream_t st, const uint64_t* in, const FoldOuts& outs, int F, int logLenF);
struct ForestLayer {
  const uint64_t* vals;
  TreeDev tree;
  uint32_t wg_start;  // first WG of this layer in the forest launch
  uint32_t stop;      // level the WG reduces to (see launch_layer16)
};

// Small FRI layers (logLen <= Ls <= 11) in one launch; layer Ls - j is
// folded from layer Ls - j + 1 with beta[j]; src = layer Ls + 1.
constexpr int TAIL_MAX = 12;
struct TailArgs {
  const uint64_t* src;
  int Ls;
  const uint64_t* beta;  // device: beta[j] folds into layer Ls - j
  uint64_t* vals[TAIL_MAX];
  TreeDev tree[TAIL_MAX];
};
hipError_t launch_fri_tail(hipStream_t st, const TailArgs& a);
// the forest of layer trees >= 4096 leaves; tail != null: its first workgroups
// also build the small layers (fri_tail_wg), tailbuf = TAIL_MAX x 4096 u64 scratch
hipError_t launch_forest16(hipStream_t st, const ForestLayer* d_layers, int nlayers, uint32_t total_wgs,
                           const TailArgs* tail = nullptr, uint64_t* tailbuf = nullptr, uint32_t wg_base = 0,
                           int wg_log = L16_LOG);
// requests: (layer, index, ordinal in the proof's FRI records) triples
// d_count != null: the number of requests is read on the device (grid = nreq, the most possible)
hipError_t launch_fri_paths(hipStream_t st, const FriLayerDev* d_layers, const uint32_t* d_req, int nreq,
                            const ProofLayout& P, const uint32_t* d_count = nullptr);
// requests: OPEN_REQ_WORDS words each
hipError_t launch_col_open(hipStream_t st, const TraceDev& T, const ColTemplate* d_tmpl, const uint32_t* outer_nodes,
                           uint64_t outer_stride_nodes, int logChunks, const uint32_t* d_req, int nreq,
                           const ProofLayout& P, const uint32_t* tabs, const uint32_t* d_dlev,
                           const DictPlan* d_plans, const uint32_t* d_dtabs, const DictCol* d_dcols,
                           const uint32_t* d_count = nullptr);

}  // namespace sezkp

// transcript.hip — the Fiat-Shamir transcript of the STARK v1 prover on the
// device (crates/sezkp-crypto/src/lib.rs:74-123, schedule of
// crates/sezkp-stark/src/v1/prover.rs:67-70,78-81,85,103,120,187,198,248,297).
//
// The transcript state is BLAKE3 over one growing byte stream S (absorb
// framing, "after_challenge" ratchets); every challenge is the BLAKE3 XOF of
// S[0..pos) || "challenge" || u32 len || label. The layout of S is fixed by
// the proof's shape (labels, lengths), so the host builds a template at
// upload and the device only fills in the Merkle roots and the manifest root.
// One workgroup per transcript point:
//   phase 0  S -> LDS, roots filled in;
//   phase 1  the chaining values of S's new 64-byte blocks, one 1024-byte
//            chunk per quad of lanes (chunks are independent in BLAKE3);
//   phase 2  per challenge: the message tail (the partial block of S plus the
//            suffix), the chunk-CV stack merges and the root node;
//   phase 3  the XOF output blocks, one quad each;
//   phase 4  the derived values: alphas / masks / z / DEEP constants, betas,
//            query rows, the path and opening requests and the proof-body
//            fields the host used to write.
// A compression runs on a quad of lanes (lane i holds the state words i,
// 4 + i, 8 + i, 12 + i): the column step is four G functions in parallel, the
// diagonal step the same after rotating rows 1-3 with quad_perm DPP moves, so
// a compression's dependency chain is ~2 x 12 VALU ops per round instead of
// a single lane's ~8 x 12.
#include <hip/hip_runtime.h>

#include "dev_common.h"
#include "sezkp_internal.h"

namespace sezkp {

namespace {

constexpr uint32_t FS_CHUNK_START = 1, FS_CHUNK_END = 2, FS_PARENT = 4, FS_ROOT = 8;
constexpr int FS_THREADS = 256;
constexpr int FS_QUADS = FS_THREADS / 4;

// message word index of lane i's two column-step and two diagonal-step words
// in round r (BLAKE3's per-round permutation applied r times), packed as
// bytes: col_x | col_y << 8 | diag_x << 16 | diag_y << 24
__constant__ uint32_t FS_MIDX[7][4] = {
    {0x09080100u, 0x0b0a0302u, 0x0d0c0504u, 0x0f0e0706u},
    {0x0b010602u, 0x050c0a03u, 0x0e090007u, 0x080f0d04u},
    {0x05060403u, 0x00090c0au, 0x0f0b020du, 0x01080e07u},
    {0x0004070au, 0x020b090cu, 0x0805030eu, 0x06010f0du},
    {0x02070d0cu, 0x03050b09u, 0x01000a0fu, 0x0406080eu},
    {0x030d0e09u, 0x0a00050bu, 0x06020c08u, 0x0704010fu},
    {0x0a0e0f0bu, 0x0c020005u, 0x04030901u, 0x0d070608u}};

__device__ __forceinline__ uint32_t fs_rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, false);
}
constexpr int ROT1 = 0x39, ROT2 = 0x4E, ROT3 = 0x93;  // lane i <- lane i + 1 / + 2 / + 3 (mod 4)

#define FS_G(a, b, c, d, x, y)                 \
  a = a + b + (x); d = fs_rotr(d ^ a, 16);     \
  c = c + d;       b = fs_rotr(b ^ c, 12);     \
  a = a + b + (y); d = fs_rotr(d ^ a, 8);      \
  c = c + d;       b = fs_rotr(b ^ c, 7);

// One BLAKE3 compression on a quad. m: the quad's 16 message words (LDS);
// midx: this lane's FS_MIDX row, loaded once per kernel. In: h0 = cv[li],
// h1 = cv[4 + li]. Out: words li, 4 + li, 8 + li, 12 + li of the 16-word
// output (the first two are the next chaining value). All 28 message words
// of the lane are read from LDS before the first round, so the rounds are a
// pure ALU / DPP chain.
__device__ __forceinline__ void b3q(const uint32_t* m, int li, const uint32_t (&midx)[7], uint32_t& h0,
                                    uint32_t& h1, uint32_t& h2, uint32_t& h3, uint64_t ctr, uint32_t blen,
                                    uint32_t flags) {
  const uint32_t IVQ[4] = {B3_IV0, B3_IV1, B3_IV2, B3_IV3};
  uint32_t a = h0, b = h1, c = IVQ[li];
  uint32_t d = li == 0 ? (uint32_t)ctr : li == 1 ? (uint32_t)(ctr >> 32) : li == 2 ? blen : flags;
  const uint32_t cv0 = h0, cv1 = h1;
  uint32_t mw[28];
#pragma unroll
  for (int r = 0; r < 7; r++) {
    const uint32_t mi = midx[r];
    mw[4 * r] = m[mi & 0xff];
    mw[4 * r + 1] = m[(mi >> 8) & 0xff];
    mw[4 * r + 2] = m[(mi >> 16) & 0xff];
    mw[4 * r + 3] = m[mi >> 24];
  }
#pragma unroll
  for (int r = 0; r < 7; r++) {
    const uint32_t cx = mw[4 * r], cy = mw[4 * r + 1], dx = mw[4 * r + 2], dy = mw[4 * r + 3];
    FS_G(a, b, c, d, cx, cy)
    b = qperm<ROT1>(b);
    c = qperm<ROT2>(c);
    d = qperm<ROT3>(d);
    FS_G(a, b, c, d, dx, dy)
    b = qperm<ROT3>(b);
    c = qperm<ROT2>(c);
    d = qperm<ROT1>(d);
  }
  h0 = a ^ c;
  h1 = b ^ d;
  h2 = c ^ cv0;
  h3 = d ^ cv1;
}

// byte j of the virtual message S[0..pos) || sfx[0..slen)
__device__ __forceinline__ uint32_t msg_byte(const uint8_t* S, uint32_t pos, uint32_t sfx, uint32_t slen, uint32_t j) {
  if (j < pos) return S[j];
  if (j < pos + slen) return S[sfx + (j - pos)];
  return 0;
}
// the quad's message words = virtual-message bytes [o, o + 64) (zero padded)
__device__ __forceinline__ void load_block(uint32_t* m, const uint8_t* S, uint32_t pos, uint32_t sfx, uint32_t slen,
                                           uint32_t o, int li) {
#pragma unroll
  for (int w = 0; w < 4; w++) {
    const uint32_t j = o + 16 * li + 4 * w;
    m[4 * li + w] = msg_byte(S, pos, sfx, slen, j) | msg_byte(S, pos, sfx, slen, j + 1) << 8 |
                    msg_byte(S, pos, sfx, slen, j + 2) << 16 | msg_byte(S, pos, sfx, slen, j + 3) << 24;
  }
}
__device__ __forceinline__ void qsync() { __builtin_amdgcn_wave_barrier(); }

__device__ __forceinline__ uint64_t rd64(const uint8_t* p) {
  uint64_t x = 0;
#pragma unroll
  for (int i = 7; i >= 0; i--) x = (x << 8) | p[i];
  return x;
}
__device__ __forceinline__ uint64_t gl_pow2k_dev(uint64_t x, int k) {
  for (int i = 0; i < k; i++) x = gl_sqr(x);
  return x;
}
__device__ __forceinline__ uint64_t gl_canon_mod(uint64_t x) { return x >= GL_P ? x - GL_P : x; }

struct RootNode {
  uint32_t cv[8];
  uint32_t block[16];
  uint32_t blen, flags;
};

}  // namespace

// Point 3: query rows (mod n) and FRI positions (mod N), the path and
// opening requests this rank owns, in proof order, and the proof-body fields
// the host used to write (counts, query headers, FRI roots, positions, final
// value, manifest root; prover.rs:242-297, proof.rs:80-98). Items run in
// canonical order, one contiguous run per thread; a workgroup scan of the
// owned counts places them (every item is owned on one device).
// FRI item i: query q = i / 2k, layer r, side (the ordinal is i); opening item
// j: query q = j / (9 tau + 3), slot t = j % (9 tau + 3) (the ordinal is j).
__device__ __forceinline__ void fri_item(const FsQueryArgs& Q, const uint64_t* pos0, int k, uint64_t N, uint32_t i,
                                         uint32_t& r, uint64_t& idx, bool& own) {
  const uint32_t q = i / (2 * k), rem = i % (2 * k), side = rem & 1;
  r = rem >> 1;
  const uint64_t p = pos0[q] & ((N >> r) - 1), half = N >> (r + 1);  // p_r = p_0 mod 2^(k - r)
  idx = side ? (p ^ half) : p;
  own = ((Q.sharded && (int)r <= Q.rR) ? (uint32_t)((idx >> L16_LOG) & (Q.world - 1)) : 0u) == Q.rank;
}
__device__ __forceinline__ void open_item(const FsQueryArgs& Q, const uint64_t* rows, uint64_t n, int logn,
                                          uint32_t j, uint32_t& c, uint64_t& row, bool& own) {
  const uint32_t tau = Q.tau, nopen = 9 * tau + 3, q = j / nopen, t = j % nopen;
  const uint64_t rw = rows[q], ip1 = rw + 1 < n ? rw + 1 : 0;  // next_wrap
  if (t < 9 * tau) {  // per tape: mv, next_mv, wflag, wsym, head, next_head, winlen, in_off, out_off
    const uint32_t tp = t / 9, kd = t % 9;
    const uint32_t kind = kd == 0 || kd == 1 ? 0 : kd == 2 ? 1 : kd == 3 ? 2 : kd == 4 || kd == 5 ? 3 : kd - 2;
    c = 3 + kind * tau + tp;
    row = (kd == 1 || kd == 5) ? ip1 : rw;
  } else {  // is_first, is_last, input_mv
    c = t == 9 * tau ? 1u : t == 9 * tau + 1 ? 2u : 0u;
    row = rw;
  }
  const uint64_t chn = logn >= COL_CHUNK_LOG2 ? row >> COL_CHUNK_LOG2 : 0;
  own = chn >= Q.ch_lo && chn < Q.ch_hi;
}
// exclusive workgroup scan of one count per thread
__device__ __forceinline__ uint32_t wg_scan(uint32_t v, uint32_t* sm, uint32_t& total) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sm[wave] = x;
  __syncthreads();
  uint32_t base = 0;
  total = 0;
  for (int w = 0; w < FS_THREADS / 64; w++) {
    if (w < wave) base += sm[w];
    total += sm[w];
  }
  __syncthreads();
  return base + x - v;
}
__device__ void fs_queries(const FsArgs& A, DevChal* D, int tid) {
  __shared__ uint64_t s_row[FS_NQ], s_pos[FS_NQ];
  __shared__ uint32_t s_sum[FS_THREADS / 64];
  const FsQueryArgs& Q = A.q;
  const uint64_t n = 1ULL << A.logn, N = 1ULL << A.logN;
  const int k = A.logN;
  if (tid < FS_NQ) {
    s_row[tid] = rd64(A.out + A.out_rowq + 8 * tid) & (n - 1);
    s_pos[tid] = rd64(A.out + A.out_rowq + 8 * FS_NQ + 8 * tid) & (N - 1);
    D->rows[tid] = s_row[tid];
    D->frows[tid] = s_pos[tid];
  }
  __syncthreads();
  // FRI path requests (layer, index, ordinal)
  const uint32_t MF = FS_NQ * 2 * (uint32_t)k, perF = (MF + FS_THREADS - 1) / FS_THREADS;
  const uint32_t f0 = tid * perF, f1 = min(MF, f0 + perF);
  uint32_t cnt = 0, total;
  for (uint32_t i = f0; i < f1; i++) {
    uint32_t r;
    uint64_t idx;
    bool own;
    fri_item(Q, s_pos, k, N, i, r, idx, own);
    cnt += own;
  }
  uint32_t at = wg_scan(cnt, s_sum, total);
  for (uint32_t i = f0; i < f1; i++) {
    uint32_t r;
    uint64_t idx;
    bool own;
    fri_item(Q, s_pos, k, N, i, r, idx, own);
    if (!own) continue;
    uint32_t* rq = Q.req + 3 * (uint64_t)at++;
    rq[0] = r;
    rq[1] = (uint32_t)idx;
    rq[2] = i;
  }
  if (tid == 0) D->counts[0] = total;
  // column openings (column, row lo, row hi, ordinal, dictionary index)
  const uint32_t MO = FS_NQ * (9 * Q.tau + 3), perO = (MO + FS_THREADS - 1) / FS_THREADS;
  const uint32_t o0 = tid * perO, o1 = min(MO, o0 + perO);
  cnt = 0;
  for (uint32_t j = o0; j < o1; j++) {
    uint32_t c;
    uint64_t row;
    bool own;
    open_item(Q, s_row, n, A.logn, j, c, row, own);
    cnt += own;
  }
  at = wg_scan(cnt, s_sum, total);
  uint32_t* orq = Q.req + 3 * Q.max_fri_req;
  for (uint32_t j = o0; j < o1; j++) {
    uint32_t c;
    uint64_t row;
    bool own;
    open_item(Q, s_row, n, A.logn, j, c, row, own);
    if (!own) continue;
    uint32_t* rq = orq + OPEN_REQ_WORDS * (uint64_t)at++;
    rq[0] = c;
    rq[1] = (uint32_t)row;
    rq[2] = (uint32_t)(row >> 32);
    rq[3] = j;
    rq[4] = Q.dict_of[c];
  }
  if (tid == 0) D->counts[1] = total;
  if (Q.rank != 0) return;  // sharded: one writer per byte (the image is byte-summed)
  // body fields (proof.rs:80-98)
  uint64_t* body = reinterpret_cast<uint64_t*>(Q.PL.base);
  for (uint32_t i = tid; i < FS_NQ * ((uint32_t)k + 1); i += FS_THREADS) {  // FRI positions
    const uint32_t q = i / (k + 1), r = i % (k + 1);
    body[(Q.PL.fq_off + 8 + q * Q.PL.fq_bytes) / 8 + 1 + r] = s_pos[q] & ((N >> r) - 1);
  }
  if (tid < FS_NQ) {
    uint64_t* fq = body + (Q.PL.fq_off + 8 + tid * Q.PL.fq_bytes) / 8;
    fq[0] = (uint64_t)k + 1;
    fq[2 + k] = (uint64_t)k;
    uint64_t* qh = body + (8 + tid * Q.PL.q_bytes) / 8;
    qh[0] = s_row[tid];
    qh[1] = Q.tau;
  }
  if (tid == 0) {
    body[0] = FS_NQ;
    body[Q.PL.fr_off / 8] = (uint64_t)k + 1;
    body[Q.PL.fq_off / 8] = FS_NQ;
    body[Q.PL.tail_off / 8] = Q.final_val[0];
  }
  uint32_t* b32 = Q.PL.base;
  for (int i = tid; i < 8 * (k + 1); i += FS_THREADS) b32[(Q.PL.fr_off + 8) / 4 + i] = A.friroots[i];
  if (tid < 8) b32[(Q.PL.tail_off + 8) / 4 + tid] = A.mroot[tid];
}

__global__ void __launch_bounds__(FS_THREADS) k_fs_point(FsArgs A) {
  __shared__ __attribute__((aligned(16))) uint8_t S[FS_S_MAX];
  __shared__ uint32_t qm[FS_QUADS][16];
  __shared__ uint32_t qstack[FS_MAX_CHAL][10][8];
  __shared__ RootNode rn[FS_MAX_CHAL];
  const int tid = threadIdx.x, li = tid & 3, quad = tid >> 2;
  uint32_t* m = qm[quad];
  uint32_t midx[7];
#pragma unroll
  for (int r = 0; r < 7; r++) midx[r] = FS_MIDX[r][li];
  // phase timestamps (100 MHz realtime clock) for SEZKP_HOST_TRACE
  uint64_t* tmark = (A.point >= 1 && A.point <= 3) ? A.ch->fs_t[A.point - 1] : nullptr;
  auto stamp = [&](int i) {
    if (tmark && tid == 0) tmark[i] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);

  // ---- phase 0: the stream template into LDS, the roots filled in
  {
    const uint32_t nw = (A.s_bytes + 15) / 16;
    const uint4* src = reinterpret_cast<const uint4*>(A.S);
    uint4* dst = reinterpret_cast<uint4*>(S);
    for (uint32_t i = tid; i < nw; i += FS_THREADS) dst[i] = src[i];
  }
  __syncthreads();
  for (uint32_t i = tid; i < A.nfill * 32; i += FS_THREADS) {
    const FsFill f = A.fills[i >> 5];
    const uint32_t byte = i & 31;
    uint32_t w;
    if (f.src == FS_SRC_MROOT) w = A.mroot[byte >> 2];
    else if (f.src < FS_SRC_FRI) w = A.colroots[8 * (f.src - FS_SRC_COL) + (byte >> 2)];
    else w = A.friroots[8 * (f.src - FS_SRC_FRI) + (byte >> 2)];
    S[f.s_off + byte] = (uint8_t)(w >> (8 * (byte & 3)));
  }
  __syncthreads();
  stamp(1);

  // ---- phase 1: chaining values of blocks [B0, B1), one chunk per quad
  if (A.B1 > A.B0) {
    const uint32_t c_first = A.B0 >> 4, c_last = (A.B1 - 1) >> 4;
    for (uint32_t c = c_first + quad; c <= c_last; c += FS_QUADS) {
      const uint32_t b0 = c * 16 > A.B0 ? c * 16 : A.B0;
      const uint32_t b1 = c * 16 + 16 < A.B1 ? c * 16 + 16 : A.B1;
      uint32_t h0, h1, h2, h3;
      if (b0 & 15) {
        h0 = A.cvs[8 * b0 + li];
        h1 = A.cvs[8 * b0 + 4 + li];
      } else {
        const uint32_t IV8[8] = {B3_IV0, B3_IV1, B3_IV2, B3_IV3, B3_IV4, B3_IV5, B3_IV6, B3_IV7};
        h0 = IV8[li];
        h1 = IV8[4 + li];
      }
      for (uint32_t b = b0; b < b1; b++) {
        A.cvs[8 * b + li] = h0;
        A.cvs[8 * b + 4 + li] = h1;
        const uint32_t* sw = reinterpret_cast<const uint32_t*>(S + 64 * b);
#pragma unroll
        for (int w = 0; w < 4; w++) m[4 * li + w] = sw[4 * li + w];
        qsync();
        const uint32_t fl = ((b & 15) == 0 ? FS_CHUNK_START : 0) | ((b & 15) == 15 ? FS_CHUNK_END : 0);
        b3q(m, li, midx, h0, h1, h2, h3, c, 64, fl);
        qsync();
        if ((b & 15) == 15) {
          A.ccv[8 * c + li] = h0;
          A.ccv[8 * c + 4 + li] = h1;
        }
      }
      if (b1 & 15) {  // the state in front of the next (not yet known) block
        A.cvs[8 * b1 + li] = h0;
        A.cvs[8 * b1 + 4 + li] = h1;
      }
    }
  }
  __syncthreads();

  stamp(2);
  // ---- phase 2: per challenge, the root node of S[0..pos) || suffix
  if (quad < (int)A.nchal) {
    const FsChal ch = A.chal[quad];
    const uint32_t L = ch.pos + ch.sfx_len;
    const uint32_t J = ch.pos >> 10, bi = (ch.pos >> 6) & 15;
    const uint32_t IV8[8] = {B3_IV0, B3_IV1, B3_IV2, B3_IV3, B3_IV4, B3_IV5, B3_IV6, B3_IV7};
    uint32_t h0, h1, h2, h3;
    if (bi) {
      h0 = A.cvs[8 * (16 * J + bi) + li];
      h1 = A.cvs[8 * (16 * J + bi) + 4 + li];
    } else {
      h0 = IV8[li];
      h1 = IV8[4 + li];
    }
    uint32_t o = (16 * J + bi) * 64, c = J, idx = bi;
    uint32_t tail_cv0 = 0, tail_cv1 = 0;  // chunk J's CV when the tail completes it
    bool crossed = false;
    uint32_t blen = 0, flags = 0;
    for (;;) {
      load_block(m, S, ch.pos, ch.sfx_off, ch.sfx_len, o, li);
      qsync();
      const uint32_t cend = 1024 * (c + 1);
      const uint32_t st = idx == 0 ? FS_CHUNK_START : 0;
      if (L <= cend && o + 64 >= L) {  // final block of the final chunk: the output node
        blen = L - o;
        flags = st | FS_CHUNK_END;
        break;
      }
      const bool last_in_chunk = o + 64 == cend;
      b3q(m, li, midx, h0, h1, h2, h3, c, 64, st | (last_in_chunk ? FS_CHUNK_END : 0));
      qsync();
      o += 64;
      if (last_in_chunk) {  // chunk c complete (only chunk J can be: the suffix is < 1 KB)
        tail_cv0 = h0;
        tail_cv1 = h1;
        crossed = true;
        h0 = IV8[li];
        h1 = IV8[4 + li];
        c++;
        idx = 0;
      } else {
        idx++;
      }
    }
    const uint32_t C = c + 1;  // chunks of the message
    // the output node of the last chunk: cv (h0, h1), block m, counter c
    if (C == 1) {
      rn[quad].cv[li] = h0;
      rn[quad].cv[4 + li] = h1;
#pragma unroll
      for (int w = 0; w < 4; w++) rn[quad].block[4 * li + w] = m[4 * li + w];
      rn[quad].blen = blen;
      rn[quad].flags = flags;
    } else {
      // its chaining value (non-root)
      uint32_t n0 = h0, n1 = h1, x2, x3;
      b3q(m, li, midx, n0, n1, x2, x3, c, blen, flags);
      qsync();
      // stack of merged subtrees over chunks 0..C-2 (push_chunk_cv)
      uint32_t(*stk)[8] = qstack[quad];
      int depth = 0;
      for (uint32_t j = 0; j + 1 < C; j++) {
        uint32_t c0, c1;
        if (j < J || !crossed) {
          c0 = A.ccv[8 * j + li];
          c1 = A.ccv[8 * j + 4 + li];
        } else {
          c0 = tail_cv0;
          c1 = tail_cv1;
        }
        uint32_t total = j + 1;
        while ((total & 1) == 0) {  // parent(stack top, cur)
          depth--;
          m[2 * li] = stk[depth][2 * li];
          m[2 * li + 1] = stk[depth][2 * li + 1];
          m[8 + li] = c0;
          m[12 + li] = c1;
          qsync();
          uint32_t p0 = IV8[li], p1 = IV8[4 + li], y2, y3;
          b3q(m, li, midx, p0, p1, y2, y3, 0, 64, FS_PARENT);
          qsync();
          c0 = p0;
          c1 = p1;
          total >>= 1;
        }
        stk[depth][li] = c0;
        stk[depth][4 + li] = c1;
        depth++;
        qsync();
      }
      // finalize: fold the stack from the top onto the last chunk's CV
      for (int i = depth - 1; i >= 0; i--) {
        m[2 * li] = stk[i][2 * li];
        m[2 * li + 1] = stk[i][2 * li + 1];
        m[8 + li] = n0;
        m[12 + li] = n1;
        qsync();
        if (i == 0) break;  // the root node: cv = IV, block m, PARENT
        uint32_t p0 = IV8[li], p1 = IV8[4 + li], y2, y3;
        b3q(m, li, midx, p0, p1, y2, y3, 0, 64, FS_PARENT);
        qsync();
        n0 = p0;
        n1 = p1;
      }
      rn[quad].cv[li] = IV8[li];
      rn[quad].cv[4 + li] = IV8[4 + li];
#pragma unroll
      for (int w = 0; w < 4; w++) rn[quad].block[4 * li + w] = m[4 * li + w];
      rn[quad].blen = 64;
      rn[quad].flags = FS_PARENT;
    }
  }
  __syncthreads();

  stamp(3);
  // ---- phase 3: XOF output blocks, one quad per (challenge, block)
  {
    uint32_t item = 0;
    for (uint32_t i = 0; i < A.nchal; i++) {
      const FsChal ch = A.chal[i];
      const uint32_t nb = (ch.out_len + 63) / 64;
      for (uint32_t t = 0; t < nb; t++, item++) {
        if ((int)(item % FS_QUADS) != quad) continue;
        const RootNode& R = rn[i];
#pragma unroll
        for (int w = 0; w < 4; w++) m[4 * li + w] = R.block[4 * li + w];
        qsync();
        uint32_t h0 = R.cv[li], h1 = R.cv[4 + li], h2, h3;
        b3q(m, li, midx, h0, h1, h2, h3, t, R.blen, R.flags | FS_ROOT);
        qsync();
        const uint32_t words[4] = {h0, h1, h2, h3};
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t wi = (uint32_t)(li + 4 * k);  // output word index
          const uint32_t at = 64 * t + 4 * wi;
          if (at < ch.out_len) *reinterpret_cast<uint32_t*>(A.out + ch.out_off + at) = words[k];
        }
      }
    }
  }
  __syncthreads();

  stamp(4);
  // ---- phase 4: derived values
  DevChal* D = A.ch;
  if (A.point == 1) {
    const uint8_t* o = A.out + A.out_alpha;
    if (tid >= 1 && tid < 9) D->alpha[tid - 1] = gl_canon_mod(rd64(o + 8 * (tid - 1)));
    else if (tid >= 9 && tid < 13) D->mask[tid - 9] = gl_canon_mod(rd64(o + 64 + 8 * (tid - 9)));
    if (tid == 0) {
      // OOD point + coset nudge (prover.rs:119-135): while (z / 3)^N == 1, z += 1.
      // The DEEP constants follow in k_fs_deep, beside the composition.
      uint64_t z = gl_canon_mod(rd64(o + 96));
      for (;;) {
        const uint64_t t = gl_pow2k_dev(gl_mul(z, A.inv3), A.logN);
        if (t != 1) break;
        z = gl_add(z, 1);
      }
      D->z = z;
    }
  } else if (A.point == 2) {
    const uint8_t* o = A.out + A.out_beta;
    for (int r = tid; r < A.logN; r += FS_THREADS) D->beta[r] = gl_canon_mod(rd64(o + 8 * r));
  } else if (A.point == 3) {
    fs_queries(A, D, tid);
  }
  __syncthreads();
  stamp(5);
}

// DEEP-polynomial constants from z (DeepPoly, sezkp_internal.h): z^n, K1 =
// (1 - z^n) / n, K2 = z^(N-1) / (3^N - z^N) * G, K3 = z^(n-1) / n, rho = (3 / z) w_N^rank,
// rho^4096 and the status flag for a z the polynomial form cannot use. One
// serial chain of ~130 products: it runs on the side stream beside the
// composition kernel, which needs only the alphas and masks.
__global__ void __launch_bounds__(64) k_fs_deep(FsArgs A) {
  if (threadIdx.x != 0) return;
  DevChal* D = A.ch;
  const uint64_t z = D->z;
  const uint64_t zn = gl_pow2k_dev(z, A.logn);
  const uint64_t zN = gl_pow2k_dev(zn, A.logN - A.logn);
  const uint64_t Dd = gl_sub(A.threeN, zN);
  // one inversion for 1/z and 1/(3^N - z^N)
  const uint64_t inv_zD = (z == 0 || Dd == 0) ? 0 : gl_inv(gl_mul(z, Dd));
  const uint64_t inv_z = gl_mul(inv_zD, Dd), inv_D = gl_mul(inv_zD, z);
  uint64_t K2 = gl_mul(gl_mul(zN, inv_z), inv_D);  // z^(N-1) / (3^N - z^N)
  const uint64_t rho = gl_mul(gl_mul(3, inv_z), A.w_rank);
  const uint64_t rhoM = gl_pow2k_dev(rho, A.logN - A.logP);
  uint64_t G = 0, pw = 1;
  for (int t = 0; t < (1 << A.logP); t++) {
    G = gl_add(G, pw);
    pw = gl_mul(pw, rhoM);
  }
  D->zn = zn;
  D->K1 = gl_mul(gl_sub(1, zn), A.inv_n);
  D->K2 = gl_mul(K2, G);
  D->rho = rho;
  D->rho4096 = gl_pow2k_dev(rho, 12);
  D->K3 = gl_mul(gl_mul(zn, inv_z), A.inv_n);  // z^(n-1) / n
  // the polynomial form needs z off the base domain and z != 0: otherwise
  // the host proves again with its own transcript (per-point DEEP)
  A.status[1] = (z == 0 || zn == 1 || Dd == 0) ? 1u : 0u;
}

hipError_t launch_fs_point(hipStream_t st, const FsArgs& a) {
  if (a.s_bytes > FS_S_MAX || a.nchal > FS_MAX_CHAL || (a.point == 3 && a.logN > 63)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_fs_point, dim3(1), dim3(FS_THREADS), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_fs_deep(hipStream_t st, const FsArgs& a) {
  hipLaunchKernelGGL(k_fs_deep, dim3(1), dim3(64), 0, st, a);
  return hipGetLastError();
}

}  // namespace sezkp

// dev_common.h — CDNA4 (gfx950) device primitives for the STARK v1 hot path:
// Goldilocks arithmetic and single-block BLAKE3 compressions.
//
// Field: p = 2^64 - 2^32 + 1 (crates/sezkp-ffts/src/lib.rs:229). Every value
// leaving a helper is canonical (< p), which is what the reference hashes and
// serialises (to_le_bytes of the canonical u64, lib.rs:123).
//
// BLAKE3: all hot-path messages fit one 64-byte block (8-byte field leaves,
// 64-byte parent l||r, <= 44-byte labelled column leaves), so one compression
// with flags CHUNK_START|CHUNK_END|ROOT, counter 0, cv = IV is the whole hash
// (crates/sezkp-stark/src/v1/merkle.rs:58-61,132-160; fri_stream.rs:37-50).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sezkp {

constexpr uint64_t GL_P = 0xffffffff00000001ULL;
constexpr uint64_t GL_EPS = 0xffffffffULL;  // 2^64 mod p

// ------------------------------------------------------------------ Goldilocks
// Carry-chain forms: 64-bit adds/subs as v_add_co/v_addc (v_sub_co/v_subb)
// pairs whose carry feeds a select, instead of 64-bit compares + cndmask
// (which also cost s_nop hazards on gfx950). tools/micro/gl_variants.hip measures
// them bit-identical to the compare forms and 1.2-1.6x faster.
__device__ __forceinline__ uint64_t add64c(uint64_t a, uint64_t b, uint32_t& carry) {
  uint32_t c0;
  const uint32_t lo = __builtin_addc((uint32_t)a, (uint32_t)b, 0u, &c0);
  const uint32_t hi = __builtin_addc((uint32_t)(a >> 32), (uint32_t)(b >> 32), c0, &carry);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t sub64b(uint64_t a, uint64_t b, uint32_t& borrow) {
  uint32_t b0;
  const uint32_t lo = __builtin_subc((uint32_t)a, (uint32_t)b, 0u, &b0);
  const uint32_t hi = __builtin_subc((uint32_t)(a >> 32), (uint32_t)(b >> 32), b0, &borrow);
  return ((uint64_t)hi << 32) | lo;
}
// canonical a, b: s = a + b; t = s + eps = s - p (mod 2^64); the true sum is
// >= p exactly when either addition carried.
__device__ __forceinline__ uint64_t gl_add(uint64_t a, uint64_t b) {
  uint32_t c1, c2;
  const uint64_t s = add64c(a, b, c1);
  const uint64_t t = add64c(s, GL_EPS, c2);
  return (c1 | c2) ? t : s;
}
// canonical a, b: a - b, and on borrow + p (= - eps mod 2^64)
__device__ __forceinline__ uint64_t gl_sub(uint64_t a, uint64_t b) {
  uint32_t br;
  const uint64_t d = sub64b(a, b, br);
  return br ? d - GL_EPS : d;
}
// any r < 2^64 -> r mod p (r - p iff r + eps carries)
__device__ __forceinline__ uint64_t gl_canon(uint64_t r) {
  uint32_t c;
  const uint64_t t = add64c(r, GL_EPS, c);
  return c ? t : r;
}
// x = hi*2^64 + lo -> r < 2^64 with r = x mod p (2^64 = eps, 2^96 = -1), not
// necessarily canonical. Neither fix-up can wrap again: after a borrow t0 >=
// 2^64 - 2^32 > eps, after a carry r < 2^64 - 2^33.
__device__ __forceinline__ uint64_t gl_reduce128_weak(uint64_t lo, uint64_t hi) {
  const uint32_t h0 = (uint32_t)hi, h1 = (uint32_t)(hi >> 32);
  uint32_t br, c;
  uint64_t t0 = sub64b(lo, h1, br);
  if (br) t0 -= GL_EPS;
  const uint64_t t1 = ((uint64_t)h0 << 32) - h0;
  const uint64_t r = add64c(t0, t1, c);
  return c ? r + GL_EPS : r;
}
__device__ __forceinline__ uint64_t gl_reduce128(uint64_t lo, uint64_t hi) {
  return gl_canon(gl_reduce128_weak(lo, hi));
}
// 64x64 -> 128 with four v_mad_u64_u32 (the partial sums cannot overflow 64 bits)
__device__ __forceinline__ void gl_mul128(uint64_t a, uint64_t b, uint64_t& lo, uint64_t& hi) {
  const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
  const uint64_t p00 = (uint64_t)a0 * b0;
  const uint64_t t = (uint64_t)a0 * b1 + (p00 >> 32);
  const uint64_t u = (uint64_t)a1 * b0 + (uint32_t)t;
  hi = (uint64_t)a1 * b1 + ((t >> 32) + (u >> 32));
  lo = ((uint64_t)(uint32_t)u << 32) | (uint32_t)p00;
}
// any a, b < 2^64 -> canonical a*b mod p
__device__ __forceinline__ uint64_t gl_mul(uint64_t a, uint64_t b) {
  uint64_t lo, hi;
  gl_mul128(a, b, lo, hi);
  return gl_reduce128(lo, hi);
}
__device__ __forceinline__ uint64_t gl_sqr(uint64_t a) { return gl_mul(a, a); }
__device__ __forceinline__ uint64_t gl_from_i64(int64_t x) {
  return x >= 0 ? (uint64_t)x : GL_P - (uint64_t)(-x);   // |x| < 2^63 << p
}
// a^(p-2) via the 2^32-1 addition chain (72 mul/sqr)
__device__ __forceinline__ uint64_t gl_pow2k(uint64_t x, int k) {
  for (int i = 0; i < k; i++) x = gl_sqr(x);
  return x;
}
// tK = a^(2^K - 1);  p-2 = (2^32-2)*2^32 + (2^32-1)
__device__ inline uint64_t gl_inv(uint64_t a) {
  uint64_t t2 = gl_mul(gl_sqr(a), a);
  uint64_t t4 = gl_mul(gl_pow2k(t2, 2), t2);
  uint64_t t8 = gl_mul(gl_pow2k(t4, 4), t4);
  uint64_t t16 = gl_mul(gl_pow2k(t8, 8), t8);
  uint64_t t24 = gl_mul(gl_pow2k(t16, 8), t8);
  uint64_t t28 = gl_mul(gl_pow2k(t24, 4), t4);
  uint64_t t30 = gl_mul(gl_pow2k(t28, 2), t2);
  uint64_t t31 = gl_mul(gl_sqr(t30), a);
  uint64_t t32 = gl_mul(gl_sqr(t31), a);
  uint64_t hi = gl_pow2k(gl_sqr(t31), 32);        // a^((2^32-2) * 2^32)
  return gl_mul(hi, t32);
}

// ------------------------------------------------------------------ BLAKE3
#define B3_IV0 0x6A09E667u
#define B3_IV1 0xBB67AE85u
#define B3_IV2 0x3C6EF372u
#define B3_IV3 0xA54FF53Au
#define B3_IV4 0x510E527Fu
#define B3_IV5 0x9B05688Cu
#define B3_IV6 0x1F83D9ABu
#define B3_IV7 0x5BE0CD19u
#define B3_ROOT_FLAGS 11u  // CHUNK_START | CHUNK_END | ROOT

__device__ __forceinline__ uint32_t rotr32(uint32_t x, int n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}

// BLAKE3 message schedule: word i of round r is sigma_r(i), sigma_r = PERM^r
// (a compile-time function, so every message index below is a constant)
__host__ __device__ constexpr int b3_sigma(int r, int i) {
  constexpr int PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
  for (int k = 0; k < r; k++) i = PERM[i];
  return i;
}

// Empty asm over the 16 state words: a scheduling barrier. The four G
// functions of a half-round then issue step by step (4 add3, 4 xor, 4
// alignbit, 4 add, ...) instead of the compiler's interleave of half-rate
// (add3, alignbit) and full-rate (xor, add) instructions: on gfx950 a mix
// issues as if every instruction were half rate, runs of one kind do not
// (tools/micro/valu_mix.hip; tools/micro/b3_sched.hip: 57.3 -> 61.1 G parent
// compressions/s at 8 waves per SIMD, 57.0 -> 58.9 at 4).
#define B3_FENCE(v)                                                                                         \
  asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),   \
               "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]),     \
               "+v"(v[14]), "+v"(v[15]))

// one half-round of round R: G on the columns (DIAG = 0) or the diagonals,
// message words sigma_R(2g + 8 DIAG), sigma_R(2g + 1 + 8 DIAG) for G g.
// FENCE = 0 leaves round 0 to the compiler, so constant IV / message words
// still fold there (leaf hashes).
template <int R, bool DIAG, bool FENCE>
__device__ __forceinline__ void b3_half_round(uint32_t (&v)[16], const uint32_t (&m)[16]) {
#define B3_STEP(EXPR)                                                                     \
  _Pragma("unroll") for (int g = 0; g < 4; g++) {                                         \
    const int A = g, B = 4 + (DIAG ? (g + 1) & 3 : g), C = 8 + (DIAG ? (g + 2) & 3 : g), \
              D = 12 + (DIAG ? (g + 3) & 3 : g);                                          \
    (void)A; (void)B; (void)C; (void)D;                                                   \
    EXPR;                                                                                 \
  }                                                                                       \
  if (FENCE) B3_FENCE(v);
  B3_STEP(v[A] = v[A] + v[B] + m[b3_sigma(R, 2 * g + 8 * DIAG)])
  B3_STEP(v[D] = v[D] ^ v[A])
  B3_STEP(v[D] = rotr32(v[D], 16))
  B3_STEP(v[C] = v[C] + v[D])
  B3_STEP(v[B] = v[B] ^ v[C])
  B3_STEP(v[B] = rotr32(v[B], 12))
  B3_STEP(v[A] = v[A] + v[B] + m[b3_sigma(R, 2 * g + 1 + 8 * DIAG)])
  B3_STEP(v[D] = v[D] ^ v[A])
  B3_STEP(v[D] = rotr32(v[D], 8))
  B3_STEP(v[C] = v[C] + v[D])
  B3_STEP(v[B] = v[B] ^ v[C])
  B3_STEP(v[B] = rotr32(v[B], 7))
#undef B3_STEP
}
template <int R>
__device__ __forceinline__ void b3_rounds(uint32_t (&v)[16], const uint32_t (&m)[16]) {
  b3_half_round<R, false, (R > 0)>(v, m);
  b3_half_round<R, true, (R > 0)>(v, m);
  if constexpr (R < 6) b3_rounds<R + 1>(v, m);
}

// One-block root hash: out = first 32 bytes of BLAKE3(message of block_len bytes).
__device__ __forceinline__ void b3_hash_block(const uint32_t (&m)[16], uint32_t block_len, uint32_t (&out)[8]) {
  uint32_t v[16] = {B3_IV0, B3_IV1, B3_IV2, B3_IV3, B3_IV4, B3_IV5, B3_IV6, B3_IV7,
                    B3_IV0, B3_IV1, B3_IV2, B3_IV3, 0,      0,      block_len, B3_ROOT_FLAGS};
  b3_rounds<0>(v, m);
#pragma unroll
  for (int w = 0; w < 8; w++) out[w] = v[w] ^ v[8 + w];
}
// leaf = BLAKE3(8 LE bytes of v)  (merkle.rs:150-160, fri_stream.rs:37-41)
__device__ __forceinline__ void b3_leaf_u64(uint64_t v, uint32_t (&out)[8]) {
  uint32_t m[16] = {(uint32_t)v, (uint32_t)(v >> 32), 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  b3_hash_block(m, 8, out);
}
// parent = BLAKE3(l || r), a plain 64-byte message (merkle.rs:58-61)
__device__ __forceinline__ void b3_parent(const uint32_t (&l)[8], const uint32_t (&r)[8], uint32_t (&out)[8]) {
  uint32_t m[16] = {l[0], l[1], l[2], l[3], l[4], l[5], l[6], l[7], r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]};
  b3_hash_block(m, 64, out);
}

// ------------------------------------------------ BLAKE3 on a quad of lanes
// One parent compression by four lanes (q = lane & 3): lane q holds column q
// of the state (v[q], v[4 + q], v[8 + q], v[12 + q]) and runs the G of that
// column; rows 1..3 are then rotated left by 1..3 lanes (DPP quad_perm) so the
// same lane runs the G of diagonal q, and rotated back. For the narrow top
// levels of a tree (fewer parents than lanes) a dependent chain of
// compressions then costs a quarter of the instructions per lane of the
// one-lane form. Message word k of round R for this lane is word
// b3_quad_word(R, k, q) of the 16-word message (k = 0, 1: the column G,
// 2, 3: the diagonal G). Output: words q and 4 + q of the parent.
__host__ __device__ constexpr uint32_t b3_quad_pack(int R, int k) {  // 4-bit word index per q
  uint32_t p = 0;
  for (int q = 0; q < 4; q++) p |= (uint32_t)b3_sigma(R, (k >= 2 ? 8 : 0) + 2 * q + (k & 1)) << (4 * q);
  return p;
}
__device__ __forceinline__ int b3_quad_word(int R, int k, int q) {
  return (int)((b3_quad_pack(R, k) >> (4 * q)) & 15u);
}
template <int CTRL>
__device__ __forceinline__ uint32_t quad_rot(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
constexpr int DPP_QROT1 = 0x39;  // quad_perm(1,2,3,0): lane q reads lane q+1
constexpr int DPP_QROT2 = 0x4E;  // quad_perm(2,3,0,1)
constexpr int DPP_QROT3 = 0x93;  // quad_perm(3,0,1,2)
__device__ __forceinline__ void b3_g1(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t mx, uint32_t my) {
  a = a + b + mx;
  d = rotr32(d ^ a, 16);
  c = c + d;
  b = rotr32(b ^ c, 12);
  a = a + b + my;
  d = rotr32(d ^ a, 8);
  c = c + d;
  b = rotr32(b ^ c, 7);
}
// mw[R][k]: the message words of this lane (see b3_quad_word); whole quads
// must be active (DPP reads the other three lanes)
__device__ __forceinline__ void b3_parent_quad(const uint32_t (&mw)[7][4], int q, uint32_t& h_lo, uint32_t& h_hi) {
  const uint32_t iv_a = q == 0 ? B3_IV0 : q == 1 ? B3_IV1 : q == 2 ? B3_IV2 : B3_IV3;
  const uint32_t iv_b = q == 0 ? B3_IV4 : q == 1 ? B3_IV5 : q == 2 ? B3_IV6 : B3_IV7;
  uint32_t a = iv_a, b = iv_b, c = iv_a, d = q == 2 ? 64u : q == 3 ? B3_ROOT_FLAGS : 0u;
#pragma unroll
  for (int R = 0; R < 7; R++) {
    b3_g1(a, b, c, d, mw[R][0], mw[R][1]);
    b = quad_rot<DPP_QROT1>(b);
    c = quad_rot<DPP_QROT2>(c);
    d = quad_rot<DPP_QROT3>(d);
    b3_g1(a, b, c, d, mw[R][2], mw[R][3]);
    b = quad_rot<DPP_QROT3>(b);
    c = quad_rot<DPP_QROT2>(c);
    d = quad_rot<DPP_QROT1>(d);
  }
  h_lo = a ^ c;
  h_hi = b ^ d;
}

// Parent pq of the LDS image's nodes 2 pq, 2 pq + 1 on the quad of lanes
// q = lane & 3 (b3_parent_quad's rounds): words q and 4 + q in lo / hi.
// AHEAD: the 28 message words read up front (latency-bound chains); else the
// lane's 4 words of a round read at that round (a compiler barrier per round
// keeps the reads and their addresses there: 4 live message words, not 28,
// so the throughput-bound tree kernels keep their occupancy).
template <int W, bool AHEAD = true>
__device__ __forceinline__ void lds_parent_quad(uint32_t (*lds)[W], int pq, int q, uint32_t& lo, uint32_t& hi) {
  if constexpr (AHEAD) {  // latency-bound chains: all 28 words read up front
    uint32_t mw[7][4];
#pragma unroll
    for (int R = 0; R < 7; R++)
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int j = b3_quad_word(R, k, q);
        mw[R][k] = lds[j & 7][2 * pq + (j >> 3)];
      }
    b3_parent_quad(mw, q, lo, hi);
    return;
  }
  // qv / pv: copies of q / pq the compiler must treat as new each round, so
  // the 28 word addresses are not all computed (and held) up front
  int qv = q, pv = pq;
  auto word = [&](int R, int k) -> uint32_t {
    const int j = b3_quad_word(R, k, qv);  // message word j: word j & 7 of child j >> 3
    return lds[j & 7][2 * pv + (j >> 3)];
  };
  const uint32_t iv_a = q == 0 ? B3_IV0 : q == 1 ? B3_IV1 : q == 2 ? B3_IV2 : B3_IV3;
  const uint32_t iv_b = q == 0 ? B3_IV4 : q == 1 ? B3_IV5 : q == 2 ? B3_IV6 : B3_IV7;
  uint32_t a = iv_a, b = iv_b, c = iv_a, d = q == 2 ? 64u : q == 3 ? B3_ROOT_FLAGS : 0u;
#pragma unroll
  for (int R = 0; R < 7; R++) {
    const uint32_t m0 = word(R, 0), m1 = word(R, 1);
    const uint32_t m2 = word(R, 2), m3 = word(R, 3);
    b3_g1(a, b, c, d, m0, m1);
    b = quad_rot<DPP_QROT1>(b);
    c = quad_rot<DPP_QROT2>(c);
    d = quad_rot<DPP_QROT3>(d);
    b3_g1(a, b, c, d, m2, m3);
    b = quad_rot<DPP_QROT3>(b);
    c = quad_rot<DPP_QROT2>(c);
    d = quad_rot<DPP_QROT1>(d);
    asm volatile("" : "+v"(qv), "+v"(pv) : : "memory");  // the next round's reads stay after this round
  }
  lo = a ^ c;
  hi = b ^ d;
}

// ------------------------------------------------------------ node helpers
__device__ __forceinline__ void node_load(const uint32_t* __restrict__ p, uint32_t (&h)[8]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  h[0] = a.x; h[1] = a.y; h[2] = a.z; h[3] = a.w; h[4] = b.x; h[5] = b.y; h[6] = b.z; h[7] = b.w;
}
__device__ __forceinline__ void node_store(uint32_t* __restrict__ p, const uint32_t (&h)[8]) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(h[0], h[1], h[2], h[3]);
  q[1] = make_uint4(h[4], h[5], h[6], h[7]);
}

}  // namespace sezkp

// ntt.hip — Goldilocks NTT passes for CDNA4 (gfx950).
//
// Mathematically the reference's transforms (crates/sezkp-ffts/src/ntt.rs:79-155):
// forward y_k = sum_j a_j w_N^{jk}, inverse = (1/n) sum_k y_k w_N^{-jk}, with
// w_{2^s} = 7^((p-1)>>s) (lib.rs:237-242). Field arithmetic is exact, so any
// factorisation produces the reference's bits.
//
// Structure: a transform of 2^logN points is a sequence of LDS passes. A pass
// owns m consecutive radix-2 stages whose smallest half-size is L = 2^sL; it
// treats every group {base + low + t*L : t < 2^m} (low < L) as one 2^m-point
// sub-transform done in LDS with internal twiddles w_{2^m}, plus ONE element-
// wise twiddle w_{2^m L}^{low * bitrev_m(t)} (post-multiply for DIF, pre-
// multiply for DIT; the four-step identity). Tiles are C <= 16 groups with
// consecutive `low` (128-B row segments) or, when L < C, one contiguous run.
//   DIF: natural -> bit-reversed order.   DIT: bit-reversed -> natural order.
// Twiddles: w_{2^K}^e = tw_hi[e >> S] * tw_lo[e & (2^S-1)] (two small tables,
// L2-resident), inverse uses e -> 2^K - e.
#include <stdlib.h>

#include <algorithm>

#include "dev_common.h"
#include "sezkp_internal.h"
#include "compose.h"

namespace sezkp {

constexpr int NTT_THREADS = 256;
constexpr int NTT_CMAX = 16;
constexpr int NTT_PADC = NTT_CMAX + 1;   // LDS row stride (u64) -> conflict-free b64 access
constexpr int NTT_MMAX = 8;              // <= 256 rows per tile

__device__ __forceinline__ uint64_t tw_pow(const NttTables& T, uint64_t e, bool inverse) {
  uint64_t mask = (T.K >= 64) ? ~0ULL : ((1ULL << T.K) - 1);
  if (inverse) e = (0 - e) & mask;
  return gl_mul(T.hi[e >> T.S], T.lo[e & ((1ULL << T.S) - 1)]);
}
__device__ __forceinline__ uint64_t pow3(const NttTables& T, uint64_t e) {
  return gl_mul(T.p3_hi[e >> T.S], T.p3_lo[e & ((1ULL << T.S) - 1)]);
}

// slot of coefficient e (= bitrev of the load position k) in the replicated
// source: k itself after one n-point DIF INTT, or the sharded INTT's
// allgathered layout (NttPassArgs::src_logP)
__device__ __forceinline__ uint64_t src_slot(const NttPassArgs& P, uint64_t k, uint32_t e) {
  if (!P.src_logP) return k;
  const int lm = P.log_src - P.src_logP;
  const uint64_t hi = (uint64_t)e >> P.src_logP;
  return ((uint64_t)(e & ((1u << P.src_logP) - 1)) << lm) | (lm ? (__brev((uint32_t)hi) >> (32 - lm)) : 0);
}

// DEEP-quotient coefficient at bit-reversed position p of the N-point DIT
// input: e = bitrev(p); the q part only where p's low b = log(N/n) bits are 0
__device__ __forceinline__ uint64_t dp_load(const NttPassArgs& P, const NttTables& T, uint64_t p, int b) {
  const uint64_t e = (uint64_t)(__brev((uint32_t)p) >> (32 - P.dp_logN));
  uint64_t v = gl_mul(P.dp_rhi[e >> 12], P.dp_rlo[e & 4095]);
  if ((p & ((1ULL << b) - 1)) == 0) {
    const uint64_t k = p >> b;
    const uint32_t rk = P.log_src ? (__brev((uint32_t)k) >> (32 - P.log_src)) : 0;  // = e
    uint64_t qv = gl_mul(gl_mul(P.src[src_slot(P, k, rk)], P.inv_n), pow3(T, rk));
    if (P.coset_e) qv = gl_mul(qv, tw_pow(T, ((uint64_t)rk * P.coset_e) & ((1ULL << T.K) - 1), false));  // (w_N^g)^e
    // q_e = d_e - f(z) z^(n-1-e) / (1 - z^n): minus kappa r^e (DeepPoly)
    v = gl_sub(gl_add(v, qv), gl_mul(P.dp_rhk[e >> 12], P.dp_rlo[e & 4095]));
  }
  return v;
}

template <bool DIF>
__global__ void __launch_bounds__(NTT_THREADS) k_ntt_pass(NttPassArgs P) {
  __shared__ uint64_t sh[(1 << NTT_MMAX) * NTT_PADC];
  __shared__ uint64_t W[(1 << NTT_MMAX) / 2];
  const int m = P.m, R = 1 << m, sL = P.sL;
  const uint64_t L = 1ULL << sL;
  const int logC = P.logC, C = 1 << logC;
  const int tid = threadIdx.x;
  const uint64_t tile = blockIdx.x;
  const NttTables& T = P.tw;

  for (int x = tid; x < R / 2; x += NTT_THREADS) W[x] = tw_pow(T, (uint64_t)x << (T.K - m), P.inverse);

  const int nel = R << logC;
  const bool wide = L >= (uint64_t)C;  // tile = C consecutive `low` columns
  uint64_t blk_base = 0, low0 = 0;
  if (wide) {
    uint64_t tiles_per_blk = L >> logC;
    blk_base = (tile / tiles_per_blk) * ((uint64_t)R << sL);
    low0 = (tile % tiles_per_blk) << logC;
  }
  const int tw_shift = T.K - m - sL;  // exponent scale into w_{2^K}
  // ---- load (+ DIT pre-twiddle)
  for (int q = tid; q < nel; q += NTT_THREADS) {
    int t, c;
    uint64_t low, pos;
    if (wide) {
      t = q >> logC; c = q & (C - 1); low = low0 + c;
      pos = blk_base + low + ((uint64_t)t << sL);
    } else {
      low = q & (L - 1);
      t = (q >> sL) & (R - 1);
      c = ((q >> (sL + m)) << sL) | (int)low;
      pos = tile * (uint64_t)nel + q;
    }
    uint64_t v;
    if (P.dp_rlo) {
      v = dp_load(P, T, pos, P.dp_logN - P.log_src);
    } else if (P.src) {  // LDE replicated load: B[2^skip k + s] = A[k] * n^-1 * (3 w^g)^bitrev(k)
      uint64_t k = pos >> P.skip;
      uint32_t rk = P.log_src ? (__brev((uint32_t)k) >> (32 - P.log_src)) : 0;
      v = gl_mul(gl_mul(P.src[src_slot(P, k, rk)], P.inv_n), pow3(T, rk));
      if (P.coset_e) v = gl_mul(v, tw_pow(T, ((uint64_t)rk * P.coset_e) & ((1ULL << T.K) - 1), false));
    } else {
      v = P.a[pos];
    }
    if (!DIF && low != 0) {
      uint32_t bt = __brev((uint32_t)t) >> (32 - m);
      v = gl_mul(v, tw_pow(T, (low * bt) << tw_shift, P.inverse));
    }
    sh[t * NTT_PADC + c] = v;
  }
  __syncthreads();
  // ---- internal radix-2 stages over t
  const int nbf = (R / 2) << logC;
  for (int it = 0; it < m - P.skip; it++) {
    const int s = DIF ? (m - 1 - it) : (it + P.skip);
    const int h = 1 << s;
    for (int b = tid; b < nbf; b += NTT_THREADS) {
      const int c = b & (C - 1), u = b >> logC;
      const int j = u & (h - 1);
      const int t0 = ((u >> s) << (s + 1)) | j, t1 = t0 + h;
      const uint64_t w = W[j << (m - 1 - s)];
      uint64_t x = sh[t0 * NTT_PADC + c], y = sh[t1 * NTT_PADC + c];
      if (DIF) {
        sh[t0 * NTT_PADC + c] = gl_add(x, y);
        sh[t1 * NTT_PADC + c] = gl_mul(gl_sub(x, y), w);
      } else {
        y = gl_mul(y, w);
        sh[t0 * NTT_PADC + c] = gl_add(x, y);
        sh[t1 * NTT_PADC + c] = gl_sub(x, y);
      }
    }
    __syncthreads();
  }
  // ---- (DIF post-twiddle +) store
  for (int q = tid; q < nel; q += NTT_THREADS) {
    int t, c;
    uint64_t low, pos;
    if (wide) {
      t = q >> logC; c = q & (C - 1); low = low0 + c;
      pos = blk_base + low + ((uint64_t)t << sL);
    } else {
      low = q & (L - 1);
      t = (q >> sL) & (R - 1);
      c = ((q >> (sL + m)) << sL) | (int)low;
      pos = tile * (uint64_t)nel + q;
    }
    uint64_t v = sh[t * NTT_PADC + c];
    if (DIF && low != 0) {
      uint32_t bt = __brev((uint32_t)t) >> (32 - m);
      v = gl_mul(v, tw_pow(T, (low * bt) << tw_shift, P.inverse));
    }
    P.a[pos] = v;
  }
}

// ------------------------------------------------ four-step register passes
// A pass of m = M1 + M2 stages as ONE exchange through LDS instead of m
// LDS round trips: two register-resident radix-2^M FFTs (<= 16 points) whose
// internal twiddles are powers of w_16 = 2^156 (w_16^-1 = 2^36), i.e. shifts
// plus one 128->64 reduction instead of general products, and one general
// twiddle w_{2^m}^(j1*k2) between them (LDS table). Same tile geometry and
// per-pass twiddle as k_ntt_pass; the two kernels are interchangeable per pass.
//   DIT (bit-reversed in, natural out): position F1*u + r holds a[j1 + F2*j2],
//     j1 = rev_M2(u), j2 = rev_M1(r). Step 1 (thread per u): F1-point DIT over
//     j2 -> Y[j1][k2]; * w^(j1 k2); step 2 (thread per k2): F2-point DIT over
//     j1 (slot u holds j1 = rev(u)) -> X[k2 + F1*k1].
//   DIF (natural in, bit-reversed out): step 1 (thread per r): F2-point DIF
//     over x[F1*u + r] -> slot q holds k_lo = rev_M2(q); * w^(r k_lo);
//     step 2 (thread per q): F1-point DIF over r -> X[k_lo + F2*k_hi] lands at
//     position q*F1 + q' (k_hi = rev_M1(q')).
__device__ __forceinline__ uint64_t gl_neg(uint64_t x) { return x ? GL_P - x : 0; }
// x * 2^e mod p for 0 <= e < 96 with e a compile-time constant after
// unrolling, by 32-bit limb placement (2^64 = 2^32 - 1, 2^96 = -1) instead of
// a 128-bit reduction. gl_add(A, B) is exact for any A < 2^64 when B < p.
//   e < 32:  x 2^e = A + y2 2^64 = A + y2 eps,   A = x << e, y2 = x >> (64-e)
//   e < 64:  x 2^e = A 2^32 + y2 2^96 = (A_lo << 32) + A_hi eps - y2, A = x << (e-32)
//   e < 96:  x 2^e = (x 2^(e-64)) 2^64 = y 2^32 - y
__device__ __forceinline__ uint64_t mul_eps32(uint32_t h) { return ((uint64_t)h << 32) - h; }  // h * eps < p
__device__ __forceinline__ uint64_t gl_mul2e_lo(uint64_t x, int e) {  // 0 <= e < 32
  if (e == 0) return x;
  const uint64_t A = x << e;
  const uint32_t y2 = (uint32_t)(x >> (64 - e));
  return gl_add(A, mul_eps32(y2));
}
__device__ __forceinline__ uint64_t gl_mul2e(uint64_t x, int e) {
  if (e < 32) return gl_mul2e_lo(x, e);
  if (e < 64) {
    const int r = e - 32;
    const uint64_t A = r ? x << r : x;
    const uint32_t y2 = r ? (uint32_t)(x >> (64 - r)) : 0u;
    const uint64_t t = gl_add(A << 32, mul_eps32((uint32_t)(A >> 32)));
    return r ? gl_sub(t, y2) : t;
  }
  const uint64_t y = gl_mul2e_lo(x, e - 64);
  return gl_sub(gl_add(y << 32, mul_eps32((uint32_t)(y >> 32))), y);
}
// x * 2^e mod p, 0 <= e < 192 (2^96 = -1)
__device__ __forceinline__ uint64_t gl_mul_pow2(uint64_t x, int e) {
  return e >= 96 ? gl_neg(gl_mul2e(x, e - 96)) : gl_mul2e(x, e);
}
// exponent of w_{2h}^j as a power of two: w_32 = 2^78 (w_32^-1 = 2^114), so
// w_16 = 2^156 (w_16^-1 = 2^36); 2 has order 192 mod p, every w_{2^k} with
// k <= 6 is a power of two (w_64 = 2^39), the reference's roots included
template <bool INV>
__device__ __forceinline__ constexpr int tw_exp(int j, int h) { return ((INV ? 114 : 78) * j * (16 / h)) % 192; }
// x * w_{2h}^j for 2h <= 32
template <bool INV>
__device__ __forceinline__ uint64_t tw_small(uint64_t x, int j, int h) {
  return gl_mul_pow2(x, tw_exp<INV>(j, h));
}
// Butterflies take the sign of w^j = -2^(e-96) into the add/sub instead of negating.
template <int LOGF, bool INV, int SKIP>
__device__ __forceinline__ void fft_dit_regs(uint64_t (&x)[1 << LOGF]) {
#pragma unroll
  for (int s = SKIP; s < LOGF; s++) {
    const int h = 1 << s;
#pragma unroll
    for (int t0 = 0; t0 < (1 << LOGF); t0++) {
      if (!(t0 & h)) {
        const int j = t0 & (h - 1);
        const int e = j ? tw_exp<INV>(j, h) : 0;
        const bool neg = e >= 96;
        const uint64_t y = gl_mul2e(x[t0 + h], neg ? e - 96 : e);
        const uint64_t a = x[t0];
        x[t0] = neg ? gl_sub(a, y) : gl_add(a, y);
        x[t0 + h] = neg ? gl_add(a, y) : gl_sub(a, y);
      }
    }
  }
}
template <int LOGF, bool INV>
__device__ __forceinline__ void fft_dif_regs(uint64_t (&x)[1 << LOGF]) {
#pragma unroll
  for (int s = LOGF - 1; s >= 0; s--) {
    const int h = 1 << s;
#pragma unroll
    for (int t0 = 0; t0 < (1 << LOGF); t0++) {
      if (!(t0 & h)) {
        const int j = t0 & (h - 1);
        const int e = j ? tw_exp<INV>(j, h) : 0;
        const bool neg = e >= 96;
        const uint64_t a = x[t0], b = x[t0 + h];
        x[t0] = gl_add(a, b);
        x[t0 + h] = gl_mul2e(neg ? gl_sub(b, a) : gl_sub(a, b), neg ? e - 96 : e);
      }
    }
  }
}
template <int M>
__device__ __forceinline__ constexpr int rev(int x) {
  int r = 0;
  for (int i = 0; i < M; i++) r |= ((x >> i) & 1) << (M - 1 - i);
  return r;
}

struct Tile {
  uint64_t blk_base, low0, tile;
  int sL, m;
  bool wide;
};
// global position of (sub-transform row t, tile column c); low = its `low` index
__device__ __forceinline__ uint64_t tile_pos(const Tile& G, int t, int c, uint64_t& low) {
  if (G.wide) {
    low = G.low0 + c;
    return G.blk_base + low + ((uint64_t)t << G.sL);
  }
  low = (uint64_t)c & ((1ULL << G.sL) - 1);
  const uint64_t cb = (uint64_t)c >> G.sL;
  return G.tile * ((uint64_t)NTT_CMAX << G.m) + (cb << (G.sL + G.m)) + ((uint64_t)t << G.sL) + low;
}

// Fused DEEP (last forward DIT pass of the LDE only): out_i = y_i / (x_i - z),
// x_i = 3 w_N^(g + P i) (merkle.hip k_deep, lde.rs:76-93). A thread's F2
// outputs sit F1 << sL apart, so consecutive x differ by w_F2 (a power of
// two: a shift); one Montgomery batch inversion per workgroup (4096 points).
template <int F, class Emit>
__device__ __forceinline__ void deep_tile(uint64_t x, uint64_t z, Emit emit) {
  __shared__ uint64_t wtot[NTT_THREADS / 64];
  __shared__ uint64_t s_inv;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint64_t d[F], a[F];
  uint64_t Pp = 1;
#pragma unroll
  for (int j = 0; j < F; j++) {
    d[j] = gl_sub(x, z);
    Pp = j ? gl_mul(Pp, d[j]) : d[j];
    a[j] = Pp;
    if (j + 1 < F) x = tw_small<false>(x, 1, F / 2);  // * w_F
  }
  uint64_t S = Pp, Tq = Pp;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t u = __shfl_up(S, o, 64);
    if (lane >= o) S = gl_mul(S, u);
    const uint64_t v = __shfl_down(Tq, o, 64);
    if (lane + o < 64) Tq = gl_mul(Tq, v);
  }
  uint64_t Q = __shfl_down(Tq, 1, 64);
  if (lane == 63) Q = 1;
  uint64_t Sprev = __shfl_up(S, 1, 64);
  if (lane == 0) Sprev = 1;
  if (lane == 63) wtot[wave] = S;
  __syncthreads();
  if (tid == 0) {
    uint64_t t = wtot[0];
#pragma unroll
    for (int w = 1; w < NTT_THREADS / 64; w++) t = gl_mul(t, wtot[w]);
    s_inv = gl_inv(t);
  }
  __syncthreads();
  uint64_t invW = s_inv;
#pragma unroll
  for (int w = 0; w < NTT_THREADS / 64; w++)
    if (w != wave) invW = gl_mul(invW, wtot[w]);
  uint64_t inv_run = gl_mul(gl_mul(invW, Q), Sprev);  // 1 / (this thread's product)
#pragma unroll
  for (int j = F - 1; j >= 0; j--) {
    emit(j, j ? gl_mul(inv_run, a[j - 1]) : inv_run);  // 1 / d_j
    if (j) inv_run = gl_mul(inv_run, d[j]);
  }
}

// NARROW (sL = 0, the first DIT / last DIF pass): a tile is 16 contiguous
// sub-transforms of R elements, so a thread's R points are consecutive and
// the lanes of one load or store instruction are R elements apart (64 cache
// lines per wave instruction). Those passes move the tile between HBM and the
// LDS image with lane-consecutive addresses (element e = j * 256 + tid of the
// tile: row e mod R, column e / R) and the register FFTs read / write the LDS.
template <int R>
__device__ __forceinline__ void narrow_to_lds(uint64_t* sh, const uint64_t* __restrict__ a, uint64_t tile) {
  constexpr int m = __builtin_ctz(R);
  const uint64_t* src = a + tile * (uint64_t)(NTT_CMAX * R);
#pragma unroll
  for (int j = 0; j < NTT_CMAX * R / NTT_THREADS; j++) {
    const int e = j * NTT_THREADS + threadIdx.x;
    sh[(e & (R - 1)) * NTT_PADC + (e >> m)] = src[e];
  }
}
template <int R>
__device__ __forceinline__ void lds_to_narrow(const uint64_t* sh, uint64_t* __restrict__ a, uint64_t tile) {
  constexpr int m = __builtin_ctz(R);
  uint64_t* dst = a + tile * (uint64_t)(NTT_CMAX * R);
#pragma unroll
  for (int j = 0; j < NTT_CMAX * R / NTT_THREADS; j++) {
    const int e = j * NTT_THREADS + threadIdx.x;
    dst[e] = sh[(e & (R - 1)) * NTT_PADC + (e >> m)];
  }
}

// nat_out: the tile's point p = tile * 16R + e holds frequency bitrev(p); it
// goes straight to out[bitrev(p)] (one word per 128-B line per tile; the 16
// tiles sharing those lines run back to back on one XCD, see nat_tile, so the
// partial lines merge in its L2 before they are written back)
template <int R>
__device__ __forceinline__ void lds_to_natural(const uint64_t* sh, const NttPassArgs& P, uint64_t tile) {
  constexpr int m = __builtin_ctz(R);
  const uint64_t p0 = tile * (uint64_t)(NTT_CMAX * R);
  const int sh_r = 32 - P.nat_logN;
#pragma unroll
  for (int j = 0; j < NTT_CMAX * R / NTT_THREADS; j++) {
    const int e = j * NTT_THREADS + threadIdx.x;
    uint64_t v = sh[(e & (R - 1)) * NTT_PADC + (e >> m)];
    if (P.out_scale != 1) v = gl_mul(v, P.out_scale);
    P.out[__brev((uint32_t)(p0 + e)) >> sh_r] = v;
  }
}
// nat_tr (the last, narrow DIF pass of a natural-order transform, 2^m-point
// sub-transforms, m <= 8): after the earlier passes block B (2^m contiguous
// points) holds the sub-transforms whose outputs land at
// X[k 2^(N-m) + bitrev_{N-m}(B)], k = bitrev_m(row). Tile T takes the 16
// blocks B_i = bitrev_{N-m}(16 T + i), i < 16, so for every k its 16 outputs
// are one contiguous 128-B segment: whole-segment loads (each block is 2^m
// contiguous points) and whole-segment stores, no bit-reversal pass.
template <int R>
__device__ __forceinline__ void gather_to_lds(uint64_t* sh, const uint64_t* __restrict__ a, uint64_t tile, int logN) {
  constexpr int m = __builtin_ctz(R);
  const int sb = 32 - (logN - m);
#pragma unroll
  for (int j = 0; j < NTT_CMAX * R / NTT_THREADS; j++) {
    const int e = j * NTT_THREADS + threadIdx.x, i = e >> m, row = e & (R - 1);
    const uint64_t B = __brev((uint32_t)(tile * NTT_CMAX + i)) >> sb;
    sh[row * NTT_PADC + i] = a[(B << m) + row];
  }
}
template <int R>
__device__ __forceinline__ void lds_to_transposed(const uint64_t* sh, const NttPassArgs& P, uint64_t tile) {
  constexpr int m = __builtin_ctz(R);
  const int lo = P.nat_logN - m;
#pragma unroll
  for (int j = 0; j < NTT_CMAX * R / NTT_THREADS; j++) {
    // lanes walk consecutive LDS rows (conflict-free reads; consecutive k =
    // rows R/4 apart put a wave's four k on the same banks); each k's 16
    // outputs stay one 128-B segment
    const int e = j * NTT_THREADS + threadIdx.x, i = e & (NTT_CMAX - 1), row = e >> 4;
    const uint64_t k = __brev((uint32_t)row) >> (32 - m);
    uint64_t v = sh[row * NTT_PADC + i];
    if (P.out_scale != 1) v = gl_mul(v, P.out_scale);
    P.out[(k << lo) + tile * NTT_CMAX + i] = v;
  }
}

// nat_tr on the DIT side (the first, narrow pass of a natural-order DIT
// transform, m <= 8): slot p of the DIT input holds x[bitrev_N(p)]. Tile T
// takes the 16 blocks B_i = bitrev_{N-m}(16 T + i): for every in-block slot e
// their inputs x[bitrev_m(e) 2^(N-m) + 16 T + i] are one contiguous 128-B
// segment; the blocks go back to their own slots (2^m contiguous points
// each). (An X16 tile, one 2^(m+4)-point sub-transform, would read single
// points 2^(N-m-4) apart and rely on L2 sharing between 16 tiles: measured
// 2^25 1267 vs 1053 us and 2^26 2493 vs 2109 us per round trip against the DIF
// transposed store, so it is not built.)
template <int R>
__device__ __forceinline__ void gather_dit_to_lds(uint64_t* sh, const uint64_t* __restrict__ x, uint64_t tile,
                                                  int logN) {
  constexpr int m = __builtin_ctz(R);
#pragma unroll
  for (int j = 0; j < NTT_CMAX * R / NTT_THREADS; j++) {
    const int e = j * NTT_THREADS + threadIdx.x, i = e & (NTT_CMAX - 1), row = e >> 4;
    sh[row * NTT_PADC + i] = x[((uint64_t)(__brev((uint32_t)row) >> (32 - m)) << (logN - m)) + tile * NTT_CMAX + i];
  }
}
template <int R>
__device__ __forceinline__ void lds_to_blocks(const uint64_t* sh, uint64_t* __restrict__ a, uint64_t tile, int logN) {
  constexpr int m = __builtin_ctz(R);
  const int sb = 32 - (logN - m);
#pragma unroll
  for (int j = 0; j < NTT_CMAX * R / NTT_THREADS; j++) {
    const int e = j * NTT_THREADS + threadIdx.x, i = e >> m, row = e & (R - 1);
    const uint64_t B = __brev((uint32_t)(tile * NTT_CMAX + i)) >> sb;
    a[(B << m) + row] = sh[row * NTT_PADC + i];
  }
}

// dispatch order of a nat_out pass: tiles T and T + j G (G = tiles / 16)
// write the same output lines; 16 consecutive workgroups of one XCD
// (workgroup b runs on XCD b mod 8) take one such group
__device__ __forceinline__ uint64_t nat_tile(uint32_t b, uint32_t tiles) {
  if (tiles % 128) return b;
  const uint32_t xcd = b % 8, k = b / 8;
  return (uint64_t)((k / 16) * 8 + xcd) + (uint64_t)(k % 16) * (tiles / 16);
}

// X16 (a NARROW pass extended by one radix-16 step inside its tile): a
// NARROW tile is 16 * R contiguous points, so it also holds every 16-point
// sub-transform {row + R t : t < 16} of the neighbouring pass with sL = log R.
// One thread per row runs it on the LDS image (element (row, t) at
// sh[row * NTT_PADC + t]) with the pass twiddle w_{16R}^(row * rev4(t)),
// pre-multiplied for DIT (after the R-point stages), post-multiplied for DIF
// (before them). A 2^12 tile then does 12 stages with one HBM round trip.
template <int R, bool DIF, bool INV>
__device__ __forceinline__ void tile_radix16(uint64_t* sh, const NttTables& T) {
  constexpr int m = __builtin_ctz(R);
  const int row = threadIdx.x;
  if (row >= R) return;
  uint64_t x[16];
#pragma unroll
  for (int t = 0; t < 16; t++) x[t] = sh[row * NTT_PADC + t];
  if constexpr (DIF) fft_dif_regs<4, INV>(x);
  if (row) {  // x[rev4(q)] *= w^(row q), the chain applied as it goes
    const uint64_t s1 = tw_pow(T, (uint64_t)row << (T.K - m - 4), INV);
    uint64_t t = s1;
#pragma unroll
    for (int q = 1; q < 16; q++) {
      x[rev<4>(q)] = gl_mul(x[rev<4>(q)], t);
      if (q + 1 < 16) t = gl_mul(t, s1);
    }
  }
  if constexpr (!DIF) fft_dit_regs<4, INV, 0>(x);
#pragma unroll
  for (int t = 0; t < 16; t++) sh[row * NTT_PADC + t] = x[t];
}

template <bool DIF, bool INV, int M1, int M2, int SKIP, bool DEEP = false, bool NARROW = false,
          bool X16 = false>
__global__ void __launch_bounds__(NTT_THREADS, 4) k_ntt4(NttPassArgs P) {
  constexpr int F1 = 1 << M1, F2 = 1 << M2, m = M1 + M2, R = 1 << m;
  static_assert(!(NARROW && DEEP), "the fused DEEP pass is a wide pass");
  static_assert(!X16 || (NARROW && SKIP == 0), "the in-tile radix-16 step extends a plain NARROW pass");
  __shared__ uint64_t sh[R * NTT_PADC];
  __shared__ uint64_t W[R];
  const int tid = threadIdx.x;
  const NttTables& T = P.tw;
  for (int x = tid; x < R; x += NTT_THREADS) W[x] = tw_pow(T, (uint64_t)x << (T.K - m), INV);
  Tile G;
  G.sL = P.sL;
  G.m = m;
  G.tile = (NARROW && P.nat_out) ? nat_tile(blockIdx.x, gridDim.x) : blockIdx.x;
  G.wide = (1ULL << G.sL) >= (uint64_t)NTT_CMAX;
  G.blk_base = 0;
  G.low0 = 0;
  if (G.wide) {
    const uint64_t tiles_per_blk = (1ULL << G.sL) / NTT_CMAX;
    G.blk_base = (G.tile / tiles_per_blk) * ((uint64_t)R << G.sL);
    G.low0 = (G.tile % tiles_per_blk) * NTT_CMAX;
  }
  const int tw_shift = T.K - m - G.sL;
  const int c = tid & (NTT_CMAX - 1), g = tid / NTT_CMAX;
  // a plain NARROW load stages the tile through the LDS image first
  const bool staged_load = NARROW && !P.dp_rlo && !P.src;
  if constexpr (NARROW && DIF && !X16) {
    if (P.nat_tr) gather_to_lds<R>(sh, P.a, G.tile, P.nat_logN);
    else if (staged_load) narrow_to_lds<R>(sh, P.a, G.tile);
  } else if constexpr (NARROW && !DIF && SKIP == 0 && !X16) {
    if (staged_load && P.nat_tr) gather_dit_to_lds<R>(sh, P.a, G.tile, P.nat_logN);
    else if (staged_load) narrow_to_lds<R>(sh, P.a, G.tile);
  } else if (staged_load) {
    narrow_to_lds<R>(sh, P.a, G.tile);
  }
  __syncthreads();
  if constexpr (X16 && DIF) {  // the previous DIF pass's 4 stages, in the tile
    tile_radix16<R, true, INV>(sh, T);
    __syncthreads();
  }
  if constexpr (!DIF) {
    uint64_t x[F1];
    if (g < F2) {  // step 1: thread (c, u), registers r
      const int u = g;
      uint64_t low = 0;
      if (P.dp_rlo) {  // DEEP-quotient LDE load (first pass, sL = 0, low = 0, SKIP = 0)
        const uint64_t p0 = tile_pos(G, F1 * u, c, low);
        const int b = P.dp_logN - P.log_src;
#pragma unroll
        for (int r = 0; r < F1; r++) x[r] = dp_load(P, T, p0 + r, b);
      } else if (P.src) {  // LDE replicated load (first pass, sL = 0, low = 0)
        const uint64_t p0 = tile_pos(G, F1 * u, c, low);
#pragma unroll
        for (int r = 0; r < F1; r += (1 << SKIP)) {
          const uint64_t k = (p0 + r) >> P.skip;
          const uint32_t rk = P.log_src ? (__brev((uint32_t)k) >> (32 - P.log_src)) : 0;
          uint64_t v = gl_mul(gl_mul(P.src[src_slot(P, k, rk)], P.inv_n), pow3(T, rk));
          if (P.coset_e) v = gl_mul(v, tw_pow(T, ((uint64_t)rk * P.coset_e) & ((1ULL << T.K) - 1), false));
#pragma unroll
          for (int s = 0; s < (1 << SKIP); s++) x[r + s] = v;
        }
      } else if (NARROW) {
#pragma unroll
        for (int r = 0; r < F1; r++) x[r] = sh[(F1 * u + r) * NTT_PADC + c];
      } else {
#pragma unroll
        for (int r = 0; r < F1; r++) x[r] = P.a[tile_pos(G, F1 * u + r, c, low)];
        // out_scale > 1 (the last pass of an inverse natural-order transform):
        // n^-1 rides on the pre-twiddle chain (one product per thread), the
        // rare low = 0 column is scaled point by point
        const bool scale = P.out_scale > 1;
        if (scale && low == 0) {
#pragma unroll
          for (int r = 0; r < F1; r++) x[r] = gl_mul(x[r], P.out_scale);
        }
        if (low != 0) {  // pre-twiddle w^(low * (j1 + F2 j2)), j2 = rev(r)
          const int j1 = rev<M2>(u);
          uint64_t t = tw_pow(T, (low * (uint64_t)j1) << tw_shift, INV);
          if (scale) t = gl_mul(t, P.out_scale);
          const uint64_t s1 = tw_pow(T, (low * (uint64_t)F2) << tw_shift, INV);
#pragma unroll
          for (int q = 0; q < F1; q++) {  // x[rev(q)] *= t s1^q, the chain applied as it goes
            x[rev<M1>(q)] = gl_mul(x[rev<M1>(q)], t);
            if (q + 1 < F1) t = gl_mul(t, s1);
          }
        }
      }
      fft_dit_regs<M1, INV, SKIP>(x);
    }
    if (staged_load) __syncthreads();  // every thread has read its points from the image
    if (g < F2) {
      const int u = g, j1 = rev<M2>(u);
#pragma unroll
      for (int k2 = 0; k2 < F1; k2++) {
        const uint64_t v = k2 && j1 ? gl_mul(x[k2], W[j1 * k2]) : x[k2];
        sh[(u * F1 + k2) * NTT_PADC + c] = v;
      }
    }
    __syncthreads();
    uint64_t y[F2];
    if (g < F1) {  // step 2: thread (c, k2), registers u
      const int k2 = g;
#pragma unroll
      for (int u = 0; u < F2; u++) y[u] = sh[(u * F1 + k2) * NTT_PADC + c];
      fft_dit_regs<M2, INV, 0>(y);
      uint64_t low;
      if constexpr (DEEP) {
        static_assert(F1 * NTT_CMAX == NTT_THREADS && !INV && !DIF, "fused DEEP needs every thread in step 2");
        // park y in this thread's own LDS slots (read above) to free registers
#pragma unroll
        for (int k1 = 0; k1 < F2; k1++) sh[(k1 * F1 + k2) * NTT_PADC + c] = y[k1];
        const uint64_t pos0 = tile_pos(G, k2, c, low);
        const uint64_t e = ((uint64_t)P.deep_g + (pos0 << P.deep_logP)) << (T.K - P.deep_logN);
        const uint64_t x0 = gl_mul(gl_mul(T.hi[e >> T.S], T.lo[e & ((1ULL << T.S) - 1)]), 3);
        deep_tile<F2>(x0, P.deep_z, [&](int k1, uint64_t inv) {
          P.a[tile_pos(G, k2 + F1 * k1, c, low)] = gl_mul(sh[(k1 * F1 + k2) * NTT_PADC + c], inv);
        });
      } else if (!NARROW) {
        uint64_t* dst = P.out ? P.out : P.a;
#pragma unroll
        for (int k1 = 0; k1 < F2; k1++) dst[tile_pos(G, k2 + F1 * k1, c, low)] = y[k1];
      }
    }
    if constexpr (NARROW) {  // rows k2 + F1 k1 back through the image, lane-consecutive stores
      __syncthreads();
      if (g < F1) {
#pragma unroll
        for (int k1 = 0; k1 < F2; k1++) sh[(g + F1 * k1) * NTT_PADC + c] = y[k1];
      }
      __syncthreads();
      if constexpr (X16) {  // the next DIT pass's 4 stages, in the tile
        tile_radix16<R, false, INV>(sh, T);
        __syncthreads();
      }
      if (!X16 && P.nat_tr) lds_to_blocks<R>(sh, P.out ? P.out : P.a, G.tile, P.nat_logN);
      else lds_to_narrow<R>(sh, P.out ? P.out : P.a, G.tile);
    }
  } else {
    uint64_t x[F2];
    if (g < F1) {  // step 1: thread (c, r), registers u (natural)
      const int r = g;
      uint64_t low;
#pragma unroll
      for (int u = 0; u < F2; u++)
        x[u] = NARROW ? sh[(F1 * u + r) * NTT_PADC + c] : P.a[tile_pos(G, F1 * u + r, c, low)];
      fft_dif_regs<M2, INV>(x);
    }
    if (NARROW) __syncthreads();
    if (g < F1) {
      const int r = g;
#pragma unroll
      for (int q = 0; q < F2; q++) {
        const int klo = rev<M2>(q);
        const uint64_t v = klo && r ? gl_mul(x[q], W[r * klo]) : x[q];
        sh[(q * F1 + r) * NTT_PADC + c] = v;
      }
    }
    __syncthreads();
    uint64_t y[F1];
    if (g < F2) {  // step 2: thread (c, q), registers r
      const int q = g;
#pragma unroll
      for (int r = 0; r < F1; r++) y[r] = sh[(q * F1 + r) * NTT_PADC + c];
      fft_dif_regs<M1, INV>(y);
      uint64_t low;
      (void)tile_pos(G, q * F1, c, low);
      if (low != 0) {  // post-twiddle w^(low * (k_lo + F2 k_hi)), k_hi = rev(q')
        uint64_t t = tw_pow(T, (low * (uint64_t)rev<M2>(q)) << tw_shift, INV);
        const uint64_t s1 = tw_pow(T, (low * (uint64_t)F2) << tw_shift, INV);
#pragma unroll
        for (int kh = 0; kh < F1; kh++) {
          y[rev<M1>(kh)] = gl_mul(y[rev<M1>(kh)], t);
          if (kh + 1 < F1) t = gl_mul(t, s1);
        }
      }
      if (!NARROW) {
        uint64_t* dst = P.out ? P.out : P.a;
#pragma unroll
        for (int qq = 0; qq < F1; qq++) dst[tile_pos(G, q * F1 + qq, c, low)] = y[qq];
      }
    }
    if constexpr (NARROW) {
      __syncthreads();
      if (g < F2) {
#pragma unroll
        for (int qq = 0; qq < F1; qq++) sh[(g * F1 + qq) * NTT_PADC + c] = y[qq];
      }
      __syncthreads();
      if (!X16 && P.nat_tr) lds_to_transposed<R>(sh, P, G.tile);
      else if (P.nat_out) lds_to_natural<R>(sh, P, G.tile);
      else lds_to_narrow<R>(sh, P.a, G.tile);
    }
  }
}

// Wide DIF pass of m = 9 stages for the natural-order transforms of 2^25 and
// 2^26 points: their last pass stays at 8 stages (the transposed store of
// nat_tr needs a 16-block tile), so the other 17 / 18 stages take passes of 9,
// keeping 3 passes. Tile = 16 columns x 512 rows (70 KB of LDS, 512 threads,
// two workgroups per CU: 16 waves, as four k_ntt4 workgroups). Four-step
// 512 = 32 x 16: step 1, thread (c, r) for r < 32, a 16-point DIF over u
// (x[32 u + r]), then * w_512^(r k_lo); step 2, thread (c, q) for q < 16, a
// 32-point DIF over r (w_32 = 2^78: shifts). Same row order, pass twiddle and
// out-of-place store as k_ntt4's wide DIF pass.
// LDS slot of (q, r, c): 16 u64 (32 banks) of padding after every q-block. A
// q-block is 32 rows = 64 * NTT_PADC dwords, so without it the four q of a
// step-2 wave hit the same 32 banks (a 2x serialised read).
template <int F1>
__device__ __forceinline__ int dif9_slot(int q, int r, int c) {
  return (q * F1 + r) * NTT_PADC + c + (q << 4);
}
template <bool INV>
__global__ void __launch_bounds__(512, 2) k_ntt_dif9(NttPassArgs P) {
  constexpr int M1 = 5, M2 = 4, F1 = 1 << M1, F2 = 1 << M2, m = M1 + M2, R = 1 << m, NT = 512;
  __shared__ uint64_t sh[R * NTT_PADC + 16 * (1 << M2)];
  __shared__ uint64_t W[R];
  const int tid = threadIdx.x;
  const NttTables& T = P.tw;
  for (int x = tid; x < R; x += NT) W[x] = tw_pow(T, (uint64_t)x << (T.K - m), INV);
  Tile G;
  G.sL = P.sL;
  G.m = m;
  G.tile = blockIdx.x;
  G.wide = true;
  const uint64_t tiles_per_blk = (1ULL << G.sL) / NTT_CMAX;
  G.blk_base = (G.tile / tiles_per_blk) * ((uint64_t)R << G.sL);
  G.low0 = (G.tile % tiles_per_blk) * NTT_CMAX;
  const int tw_shift = T.K - m - G.sL;
  const int c = tid & (NTT_CMAX - 1), g = tid / NTT_CMAX;  // g < F1
  uint64_t low;
  {  // step 1: thread (c, r), registers u
    const int r = g;
    uint64_t x[F2];
#pragma unroll
    for (int u = 0; u < F2; u++) x[u] = P.a[tile_pos(G, F1 * u + r, c, low)];
    fft_dif_regs<M2, INV>(x);
    __syncthreads();  // W
#pragma unroll
    for (int q = 0; q < F2; q++) {
      const int klo = rev<M2>(q);
      sh[dif9_slot<F1>(q, r, c)] = klo && r ? gl_mul(x[q], W[r * klo]) : x[q];
    }
  }
  __syncthreads();
  {  // step 2: the 32-point DIF over r of column q as two threads (c, q, h):
     // its first radix-2 stage (pairs r, r + 16; twiddle w_32^r, a shift) is
     // split by output half, h = 0 the sums, h = 1 the differences, then each
     // thread runs a 16-point DIF. Slot s of thread h is slot s + 16 h of
     // the 32-point output, i.e. k_hi = 2 rev4(s) + h. All 512 threads busy.
    const int q = g & (F2 - 1), h = g >> M2;
    uint64_t y[16];
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const uint64_t a = sh[dif9_slot<F1>(q, r, c)], b = sh[dif9_slot<F1>(q, r + 16, c)];
      if (h == 0) {
        y[r] = gl_add(a, b);
      } else {
        const int e = r ? tw_exp<INV>(r, 16) : 0;
        const bool neg = e >= 96;
        y[r] = gl_mul2e(neg ? gl_sub(b, a) : gl_sub(a, b), neg ? e - 96 : e);
      }
    }
    fft_dif_regs<4, INV>(y);
    (void)tile_pos(G, q * F1, c, low);
    if (low != 0) {  // post-twiddle w^(low * (k_lo + F2 k_hi)), k_hi = 2 k' + h, slot rev4(k')
      uint64_t t = tw_pow(T, (low * ((uint64_t)rev<M2>(q) + (uint64_t)F2 * h)) << tw_shift, INV);
      const uint64_t s2 = tw_pow(T, (low * (uint64_t)(2 * F2)) << tw_shift, INV);
#pragma unroll
      for (int kp = 0; kp < 16; kp++) {
        y[rev<4>(kp)] = gl_mul(y[rev<4>(kp)], t);
        if (kp + 1 < 16) t = gl_mul(t, s2);
      }
    }
    uint64_t* dst = P.out ? P.out : P.a;
#pragma unroll
    for (int s = 0; s < 16; s++) dst[tile_pos(G, q * F1 + 16 * h + s, c, low)] = y[s];
  }
}

// ---- 512-thread radix-8 DIF passes (8 points per lane, two waves per SIMD)
// The two passes of a 2^20-point DIF ([8, 12] stages) and the 12-stage
// narrow pass of other DIFs launch 256 workgroups of 4096 points: one
// workgroup per CU. With 256 lanes (16 points each, k_ntt4) that is one wave
// per SIMD and ~45% of its cycles wait on memory (round 3 PMC); with 512 lanes
// each SIMD holds two waves. Radix-8 steps: a lane loads 8 points L apart,
// runs an 8-point DIF (w_8 powers: shifts), multiplies slot q by
// w_{8L}^(low * rev3(q)) and stores them back (the four-step identity of
// k_ntt4's DIF, three stages per LDS exchange).
constexpr int R8_NT = 512;
// LDS hand-off between lanes of ONE wave: a wave's LDS instructions execute
// in issue order, so only the compiler has to keep its reads after its writes
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ int r8_pad(int e) { return e + (e >> 3); }  // conflict-free strides 64 / 8 / 1
// w_64 = 2^39, w_64^-1 = 2^153 (2 has order 192)
template <bool INV>
__device__ __forceinline__ constexpr int tw_exp64(int j) { return ((INV ? 153 : 39) * j) % 192; }
// slot rev3(k) *= w1^k, k = 1..7 (w1 = w_{8L}^low)
__device__ __forceinline__ void r8_twiddle(uint64_t (&x)[8], uint64_t w1) {
  uint64_t t = w1;
#pragma unroll
  for (int k = 1; k < 8; k++) {
    x[rev<3>(k)] = gl_mul(x[rev<3>(k)], t);
    if (k < 7) t = gl_mul(t, w1);
  }
}

// Wide DIF pass of 8 stages (tile = 16 columns x 256 rows, rows 2^sL apart),
// 256 = 8 x 8 x 4: lane (c, g), g < 32. Same pass twiddle and out-of-place
// store as k_ntt4's wide DIF pass.
template <bool INV>
__global__ void __launch_bounds__(R8_NT, 2) k_ntt_w8r8(NttPassArgs P) {
  __shared__ uint64_t sh[256 * NTT_PADC];
  const int tid = threadIdx.x, c = tid & (NTT_CMAX - 1), g = tid >> 4;
  const NttTables& T = P.tw;
  Tile G;
  G.sL = P.sL;
  G.m = 8;
  G.tile = blockIdx.x;
  G.wide = true;
  const uint64_t tiles_per_blk = (1ULL << G.sL) / NTT_CMAX;
  G.blk_base = (G.tile / tiles_per_blk) * (256ULL << G.sL);
  G.low0 = (G.tile % tiles_per_blk) * NTT_CMAX;
  const int tw_shift = T.K - 8 - G.sL;
  uint64_t low;
  (void)tile_pos(G, 0, c, low);
  // stages 1..0 take rows 4h..4h+3, h = h0 and h0 + 4: the 32 rows stages
  // 4..2 of this wave (g >> 2) wrote, so the last exchange stays in the wave.
  // Every table twiddle depends on the lane only: fetched beside the data.
  const int h0 = 8 * (g >> 2) + (g & 3);
  const uint64_t w1 = tw_pow(T, (uint64_t)g << (T.K - 8), INV);  // w_256^g
  uint64_t ta[2], tb = 1;
  if (low) {  // pass twiddle w_{2^(8+sL)}^(low rev8(t)), rev8(4h + rev2(k)) = 64 k + rev6(h)
#pragma unroll
    for (int hh = 0; hh < 2; hh++)
      ta[hh] = tw_pow(T, (low * (uint64_t)(__brev((uint32_t)(h0 + 4 * hh)) >> 26)) << tw_shift, INV);
    tb = tw_pow(T, (low * 64ULL) << tw_shift, INV);
  }
  uint64_t x[8];
  // stages 7..5 (stride 32), straight from HBM
#pragma unroll
  for (int d = 0; d < 8; d++) x[d] = P.a[tile_pos(G, g + 32 * d, c, low)];
  fft_dif_regs<3, INV>(x);
  if (g) r8_twiddle(x, w1);  // w_256^(g k)
#pragma unroll
  for (int q = 0; q < 8; q++) sh[(g + 32 * q) * NTT_PADC + c] = x[q];
  __syncthreads();
  {  // stages 4..2 (stride 4) on rows 32 (g >> 2) + ..., twiddles w_32^(lo k): shifts
    const int lo = g & 3, base = (g >> 2) * 32 + lo;
#pragma unroll
    for (int d = 0; d < 8; d++) x[d] = sh[(base + 4 * d) * NTT_PADC + c];
    fft_dif_regs<3, INV>(x);
    if (lo) {
#pragma unroll
      for (int k = 1; k < 8; k++) x[rev<3>(k)] = tw_small<INV>(x[rev<3>(k)], lo * k, 16);
    }
#pragma unroll
    for (int d = 0; d < 8; d++) sh[(base + 4 * d) * NTT_PADC + c] = x[d];
  }
  wave_lds_sync();
  uint64_t* dst = P.out ? P.out : P.a;
#pragma unroll
  for (int hh = 0; hh < 2; hh++) {
    const int h = h0 + 4 * hh;
    uint64_t y[4];
#pragma unroll
    for (int d = 0; d < 4; d++) y[d] = sh[(4 * h + d) * NTT_PADC + c];
    fft_dif_regs<2, INV>(y);
    if (low) {
      uint64_t t = ta[hh];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        y[rev<2>(k)] = gl_mul(y[rev<2>(k)], t);
        if (k < 3) t = gl_mul(t, tb);
      }
    }
#pragma unroll
    for (int d = 0; d < 4; d++) dst[tile_pos(G, 4 * h + d, c, low)] = y[d];
  }
}

// LDS slot of point e = 512 a + 64 b + 8 c + d of the 4096-point tile: the XOR
// swizzle 512 a + 64 b + 8 (c ^ (b & 3)) + (d ^ c) (a permutation, no padding).
// Every access of k_ntt_n12r8 is then conflict-free: a ds_read_b64 serves 32
// lanes per LDS cycle (bank = slot mod 32 must differ) and a ds_write_b64 16
// lanes (slot mod 16); the half-wave sets are (c low 2 bits, d), (b low 2
// bits, d) and (b low 2 bits, c), each mapped one to one onto the bank bits
// (round 5's pad e + e / 8 cost 31% of the LDS cycles in conflicts).
__device__ __forceinline__ int n12_slot(int e) {
  const int b = (e >> 6) & 7, c = (e >> 3) & 7, d = e & 7;
  return (e & ~63) | ((c ^ (b & 3)) << 3) | (d ^ c);
}

// Narrow DIF pass of 12 stages on 4096 contiguous points (sL = 0),
// 4096 = 8^4: lane g < 512; the natural-order store (nat_out): position
// p = 4096 tile + e goes to out[bitrev(p)] * out_scale (workgroup order as
// k_ntt4's nat_out).
template <bool INV>
__global__ void __launch_bounds__(R8_NT, 2) k_ntt_n12r8(NttPassArgs P) {
  __shared__ uint64_t sh[4096];
  const int g = threadIdx.x;
  const NttTables& T = P.tw;
  const uint64_t tile = nat_tile(blockIdx.x, gridDim.x);
  const uint64_t p0 = tile << 12;
  uint64_t x[8];
  // both table twiddles depend on the lane only: fetched beside the data
  const int lo2 = g & 63;
  const uint64_t w1 = tw_pow(T, (uint64_t)g << (T.K - 12), INV);    // w_4096^g
  const uint64_t w2 = tw_pow(T, (uint64_t)lo2 << (T.K - 9), INV);   // w_512^lo
  // stages 11..9 (stride 512), straight from HBM
#pragma unroll
  for (int d = 0; d < 8; d++) x[d] = P.a[p0 + g + 512 * d];
  fft_dif_regs<3, INV>(x);
  if (g) r8_twiddle(x, w1);
#pragma unroll
  for (int q = 0; q < 8; q++) sh[n12_slot(g + 512 * q)] = x[q];
  __syncthreads();
  // stages 8..0 stay inside 512-point block g >> 6: wave w's own block, so
  // the exchanges below are between lanes of one wave
  {  // stages 8..6 (stride 64)
    const int base = (g >> 6) * 512 + lo2;
#pragma unroll
    for (int d = 0; d < 8; d++) x[d] = sh[n12_slot(base + 64 * d)];
    fft_dif_regs<3, INV>(x);
    if (lo2) r8_twiddle(x, w2);
#pragma unroll
    for (int d = 0; d < 8; d++) sh[n12_slot(base + 64 * d)] = x[d];
  }
  wave_lds_sync();
  {  // stages 5..3 (stride 8), twiddles w_64^(lo k): shifts
    const int lo = g & 7, base = (g >> 3) * 64 + lo;
#pragma unroll
    for (int d = 0; d < 8; d++) x[d] = sh[n12_slot(base + 8 * d)];
    fft_dif_regs<3, INV>(x);
    if (lo) {
#pragma unroll
      for (int k = 1; k < 8; k++) x[rev<3>(k)] = gl_mul_pow2(x[rev<3>(k)], tw_exp64<INV>(lo * k));
    }
#pragma unroll
    for (int d = 0; d < 8; d++) sh[n12_slot(base + 8 * d)] = x[d];
  }
  wave_lds_sync();
  // stages 2..0 on 8 consecutive points
#pragma unroll
  for (int d = 0; d < 8; d++) x[d] = sh[n12_slot(8 * g + d)];
  fft_dif_regs<3, INV>(x);
  const int sh_r = 32 - P.nat_logN;
  const bool scale = P.out_scale > 1;
#pragma unroll
  for (int q = 0; q < 8; q++)
    P.out[__brev((uint32_t)(p0 + 8 * g + q)) >> sh_r] = scale ? gl_mul(x[q], P.out_scale) : x[q];
}

// the radix-8 forms of the natural-order 2^20 DIF's passes (wide m = 8 with
// 16 columns, narrow m = 12 with the natural-order store), else false.
// Measured (round 4, profiles/r04/c2_ab.txt): 2^20 fwd + inv 72.7 -> 70.4 us;
// round 5 (wave-local exchanges, twiddle loads beside the data) 69.3 -> 65.7 us.
// The prover's in-place 12-stage INTT pass measured 2 us slower with it, so
// it keeps k_ntt4's X16 form.
static bool launch_r8(hipStream_t st, const NttPassArgs& P, bool inverse, unsigned tiles) {
  if (P.src || P.dp_rlo || P.nat_tr) return false;
  if (P.m == 8 && P.logC == 4 && P.sL >= 4 && !P.nat_out) {
    if (inverse) hipLaunchKernelGGL(k_ntt_w8r8<true>, dim3(tiles), dim3(R8_NT), 0, st, P);
    else hipLaunchKernelGGL(k_ntt_w8r8<false>, dim3(tiles), dim3(R8_NT), 0, st, P);
    return true;
  }
  if (P.m == 12 && P.sL == 0 && P.nat_out) {
    if (inverse) hipLaunchKernelGGL(k_ntt_n12r8<true>, dim3(tiles), dim3(R8_NT), 0, st, P);
    else hipLaunchKernelGGL(k_ntt_n12r8<false>, dim3(tiles), dim3(R8_NT), 0, st, P);
    return true;
  }
  return false;
}

// launch one pass with the register kernel when its shape allows, else false
template <bool DIF, bool INV>
static bool launch_ntt4(hipStream_t st, const NttPassArgs& P, unsigned tiles) {
  if (P.logC != 4) return false;
  const int skip = P.src ? P.skip : 0;
  if (DIF && skip) return false;
  // sL = 0 passes stage their tile through the LDS image (k_ntt4 NARROW)
#define SEZKP_NTT4(M1, M2, SK)                                                                                \
  do {                                                                                                         \
    if (P.sL == 0)                                                                                           \
      hipLaunchKernelGGL((k_ntt4<DIF, INV, M1, M2, SK, false, true>), dim3(tiles), dim3(NTT_THREADS), 0, st, P); \
    else                                                                                                       \
      hipLaunchKernelGGL((k_ntt4<DIF, INV, M1, M2, SK>), dim3(tiles), dim3(NTT_THREADS), 0, st, P);           \
  } while (0)
  if (P.m > NTT_MMAX) {  // NARROW + in-tile radix-16 (plan_passes_x16)
    // plain passes, or the LDE's DEEP-polynomial first pass (all its stages: no skip)
    if (P.sL != 0 || skip || (P.src && !P.dp_rlo)) return false;
#define SEZKP_NTT4X(M1, M2) \
  hipLaunchKernelGGL((k_ntt4<DIF, INV, M1, M2, 0, false, true, true>), dim3(tiles), dim3(NTT_THREADS), 0, st, P)
    switch (P.m) {
      case 12: SEZKP_NTT4X(4, 4); return true;
      case 11: SEZKP_NTT4X(4, 3); return true;
      case 10: SEZKP_NTT4X(3, 3); return true;
      default: return false;
    }
#undef SEZKP_NTT4X
  }
  switch (P.m * 4 + skip) {
    case 8 * 4 + 0: SEZKP_NTT4(4, 4, 0); return true;
    case 7 * 4 + 0: SEZKP_NTT4(4, 3, 0); return true;
    case 6 * 4 + 0: SEZKP_NTT4(3, 3, 0); return true;
    default: break;
  }
  if constexpr (!DIF) {
    switch (P.m * 4 + skip) {
      case 8 * 4 + 1: SEZKP_NTT4(4, 4, 1); return true;
      case 8 * 4 + 2: SEZKP_NTT4(4, 4, 2); return true;
      case 8 * 4 + 3: SEZKP_NTT4(4, 4, 3); return true;
      case 7 * 4 + 1: SEZKP_NTT4(4, 3, 1); return true;
      case 7 * 4 + 2: SEZKP_NTT4(4, 3, 2); return true;
      case 7 * 4 + 3: SEZKP_NTT4(4, 3, 3); return true;
      case 6 * 4 + 1: SEZKP_NTT4(3, 3, 1); return true;
      case 6 * 4 + 2: SEZKP_NTT4(3, 3, 2); return true;
      case 6 * 4 + 3: SEZKP_NTT4(3, 3, 3); return true;
      default: break;
    }
  }
#undef SEZKP_NTT4
  return false;
}

// Out-of-place bit-reversal permutation (optionally scaled), tiled so both the
// read and the write are 16-element (128-B) row segments:
// p = x*2^(a+b) + y*2^a + z  ->  rev(z)*2^(a+b) + rev(y)*2^a + rev(x), a = 4.
__global__ void __launch_bounds__(256) k_bitrev_permute(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                         int logN, uint64_t scale, int do_scale) {
  __shared__ uint64_t sh[16 * 17];
  const int a = 4, b = logN - 2 * a;
  const uint32_t y = blockIdx.x;   // middle bits
  const int tid = threadIdx.x;
  const int x = tid >> 4, z = tid & 15;
  uint32_t ry = b ? (__brev(y) >> (32 - b)) : 0;
  uint64_t src = ((uint64_t)x << (a + b)) | ((uint64_t)y << a) | z;
  uint64_t v = in[src];
  if (do_scale) v = gl_mul(v, scale);
  sh[x * 17 + z] = v;
  __syncthreads();
  // thread (x', z') writes out[rev(z')... ] : destination row = rev(z), column = rev(x)
  const int rz = tid >> 4, rx = tid & 15;        // destination coordinates (already reversed)
  const int zz = __brev((uint32_t)rz) >> 28, xx = __brev((uint32_t)rx) >> 28;
  uint64_t dst = ((uint64_t)rz << (a + b)) | ((uint64_t)ry << a) | rx;
  out[dst] = sh[xx * 17 + zz];
}

// In-place bit-reversal permutation (optionally scaled): the WG of middle bits
// y also owns tile rev(y) (y <= rev(y)); both S x S tiles (S = 2^A) are read
// into LDS before either is written, so tile pairs swap without a second
// buffer. p = x 2^(A+b) + y 2^A + z -> rev_A(z) 2^(A+b) + rev_b(y) 2^A + rev_A(x):
// reads and writes are S-element row segments (A = 4: 128 B, A = 5: 256 B;
// the wider segments pay once the array no longer sits in the MALL).
template <int A>
__global__ void __launch_bounds__(256) k_bitrev_inplace(uint64_t* __restrict__ a, int logN, uint64_t scale,
                                                        int do_scale) {
  constexpr int S = 1 << A, PER = S * S / 256;
  __shared__ uint64_t sh[2][S * (S + 1)];
  const int b = logN - 2 * A;
  const uint32_t y = blockIdx.x;
  const uint32_t ry = b ? (__brev(y) >> (32 - b)) : 0;
  if (y > ry) return;
  const int tid = threadIdx.x;
  uint64_t v0[PER], v1[PER];
#pragma unroll
  for (int j = 0; j < PER; j++) {
    const int e = j * 256 + tid, x = e >> A, z = e & (S - 1);
    v0[j] = a[((uint64_t)x << (A + b)) | ((uint64_t)y << A) | z];
    v1[j] = a[((uint64_t)x << (A + b)) | ((uint64_t)ry << A) | z];
  }
#pragma unroll
  for (int j = 0; j < PER; j++) {
    const int e = j * 256 + tid, x = e >> A, z = e & (S - 1);
    sh[0][x * (S + 1) + z] = do_scale ? gl_mul(v0[j], scale) : v0[j];
    sh[1][x * (S + 1) + z] = do_scale ? gl_mul(v1[j], scale) : v1[j];
  }
  __syncthreads();
  // destination (rz, ry', rx) <- source (rev(rx), y', rev(rz)): tile y lands in tile ry and back
#pragma unroll
  for (int j = 0; j < PER; j++) {
    const int e = j * 256 + tid, rz = e >> A, rx = e & (S - 1);
    const int zz = __brev((uint32_t)rz) >> (32 - A), xx = __brev((uint32_t)rx) >> (32 - A);
    a[((uint64_t)rz << (A + b)) | ((uint64_t)ry << A) | rx] = sh[0][xx * (S + 1) + zz];
    if (ry != y) a[((uint64_t)rz << (A + b)) | ((uint64_t)y << A) | rx] = sh[1][xx * (S + 1) + zz];
  }
}

// Small transforms (logN < 8) fall back to a plain in-LDS pass per call.
__global__ void k_bitrev_permute_small(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, int logN,
                                       uint64_t scale, int do_scale) {
  uint64_t N = 1ULL << logN;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t r = logN ? (__brev((uint32_t)i) >> (32 - logN)) : 0;
    uint64_t v = in[i];
    out[r] = do_scale ? gl_mul(v, scale) : v;
  }
}

// ------------------------------------------------ distributed four-step NTT
// N = P * M points over P ranks (BASELINE config 4). Rank g holds
// x[g + P j] (j < M) and, after a local M-point NTT Y_g (bit-reversed), this
// kernel writes s[k2] = Y_g[k2] * w_N^(+-g k2) (* scale) in natural k2 order:
// s is already the all-to-all send image (peer d gets k2 in [d M/P, (d+1) M/P)).
// 16x16 LDS tiles as k_bitrev_permute, TPW adjacent tiles per WG: a source
// row of the WG is then 16 * TPW contiguous elements (512 B at TPW = 4), and
// every lane has TPW loads in flight before the exchange. The inverse runs the
// pipeline backwards and twiddles by the SOURCE index (tw_src = 1).
template <int TPW>
__global__ void __launch_bounds__(256) k_dntt_permute_twiddle(const uint64_t* __restrict__ in,
                                                               uint64_t* __restrict__ out, int logM, NttTables T,
                                                               uint64_t e_step, int inverse, int tw_src,
                                                               uint64_t scale) {
  __shared__ uint64_t sh[TPW][16 * 17];
  const int a = 4, b = logM - 2 * a;
  const uint32_t y0 = blockIdx.x * TPW;
  const int tid = threadIdx.x;
  uint64_t v[TPW];
#pragma unroll
  for (int i = 0; i < TPW; i++) {  // element e = i*256 + tid: row x, tile y0 + t, column z
    const int e = i * 256 + tid, x = e / (16 * TPW), t = (e / 16) % TPW, z = e & 15;
    v[i] = in[((uint64_t)x << (a + b)) | ((uint64_t)(y0 + t) << a) | z];
  }
#pragma unroll
  for (int i = 0; i < TPW; i++) {
    const int e = i * 256 + tid, x = e / (16 * TPW), t = (e / 16) % TPW, z = e & 15;
    sh[t][x * 17 + z] = v[i];
  }
  __syncthreads();
  const int rz = tid >> 4, rx = tid & 15;
  const int zz = __brev((uint32_t)rz) >> 28, xx = __brev((uint32_t)rx) >> 28;
#pragma unroll
  for (int t = 0; t < TPW; t++) {
    const uint32_t y = y0 + t;
    const uint32_t ry = b ? (__brev(y) >> (32 - b)) : 0;
    const uint64_t k2 = ((uint64_t)rz << (a + b)) | ((uint64_t)ry << a) | rx;
    const uint64_t src = ((uint64_t)xx << (a + b)) | ((uint64_t)y << a) | zz;
    uint64_t w = sh[t][xx * 17 + zz];
    if (e_step) w = gl_mul(w, tw_pow(T, (tw_src ? src : k2) * e_step, inverse != 0));
    if (scale != 1) w = gl_mul(w, scale);
    out[k2] = w;
  }
}

// After the all-to-all r[g * Q + q] = rank g's s[d Q + q] (Q = M/P). In place:
// r[k1 * Q + q] = sum_g w_P^(+-g k1) r[g * Q + q] = X[d Q + q + M k1]. The
// P-point DFT uses only powers of two (w_8 = 2^120), i.e. shifts.
template <int P, bool INV>
__global__ void __launch_bounds__(256) k_dntt_dft(uint64_t* __restrict__ r, uint64_t Q) {
  const uint64_t q = blockIdx.x * 256ull + threadIdx.x;
  if (q >= Q) return;
  uint64_t v[P], o[P];
#pragma unroll
  for (int g = 0; g < P; g++) v[g] = r[g * Q + q];
#pragma unroll
  for (int k1 = 0; k1 < P; k1++) {
    uint64_t acc = v[0];
#pragma unroll
    for (int g = 1; g < P; g++) {
      const int j = (g * k1) % P;
      acc = gl_add(acc, j ? tw_small<INV>(v[g], j, P / 2) : v[g]);  // w_P^j
    }
    o[k1] = acc;
  }
#pragma unroll
  for (int k1 = 0; k1 < P; k1++) r[k1 * Q + q] = o[k1];
}

// Sharded INTT, first half (block layout in, see bintt_dft_twiddle): the
// inverse P-point DFT over g (shifts only) and the four-step twiddle
// w_n^-(j k1), j = d Q + q, generated from the tables per output.
template <int P>
__global__ void __launch_bounds__(256) k_bintt_dft_twiddle(uint64_t* __restrict__ r, uint64_t Q, uint64_t j0,
                                                           int logn, NttTables T) {
  const uint64_t q = blockIdx.x * 256ull + threadIdx.x;
  if (q >= Q) return;
  uint64_t v[P];
#pragma unroll
  for (int g = 0; g < P; g++) v[g] = r[g * Q + q];
  const uint64_t j = j0 + q;
#pragma unroll
  for (int k1 = 0; k1 < P; k1++) {
    uint64_t acc = v[0];
#pragma unroll
    for (int g = 1; g < P; g++) {
      const int jj = (g * k1) % P;
      acc = gl_add(acc, jj ? tw_small<true>(v[g], jj, P / 2) : v[g]);  // w_P^-jj
    }
    if (k1) acc = gl_mul(acc, tw_pow(T, ((j * (uint64_t)k1) << (T.K - logn)) & ((1ULL << T.K) - 1), true));
    r[k1 * Q + q] = acc;
  }
}

// ------------------------------------------- DEEP quotient (base domain)
// See DeepPoly (sezkp_internal.h). k_inv_base: D_j = C_j / (w_n^j - z) for the
// base points j in [row0, row0 + nrows), C_j the composition value of the
// row (compose.h, from k_compose_terms' sums: the composition's
// transcript-dependent half runs here), DQ_PER per lane, one Montgomery batch
// per WG, and the per-WG partial sums of D_j w_n^j; WG b of the range
// writes partial[b] (sharded ranks each own a block of rows and allgather
// their partials with the INTT coefficients, so every rank reduces the same sum).
template <int DQ_PER>
__global__ void __launch_bounds__(NTT_THREADS) k_inv_base(ComposeTerms Tm, uint64_t* __restrict__ Dout,
                                                          uint64_t* __restrict__ partial, int logn,
                                                          const DevChal* __restrict__ ch, NttTables T, uint64_t row0,
                                                          uint64_t nrows) {
  const uint64_t z = ch->z;
  __shared__ uint64_t wtot[NTT_THREADS / 64];
  __shared__ uint64_t s_inv;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // the WG's rows wg0 + j NTT_THREADS + tid (j < DQ_PER): every load and
  // store of a j step is one coalesced row range (lane-consecutive rows
  // touched 8x the cache lines per instruction)
  const uint64_t wg0 = row0 + (uint64_t)blockIdx.x * NTT_THREADS * DQ_PER, end = row0 + nrows;
  uint64_t d[DQ_PER], a[DQ_PER], cv[DQ_PER];
  uint64_t Pp = 1;
  {
    const ComposeCoef K = compose_coef(ch);
    // exponents mod 2^K (w^(2^K) = 1): rows past a small n stay inside the
    // twiddle tables (their values are never used)
    const uint64_t kmask = (1ULL << T.K) - 1;
    const uint64_t e = ((wg0 + tid) << (T.K - logn)) & kmask;
    uint64_t x = gl_mul(T.hi[e >> T.S], T.lo[e & ((1ULL << T.S) - 1)]);
    const uint64_t e1 = ((uint64_t)NTT_THREADS << (T.K - logn)) & kmask;
    const uint64_t ws = gl_mul(T.hi[e1 >> T.S], T.lo[e1 & ((1ULL << T.S) - 1)]);  // w_n^NTT_THREADS
#pragma unroll
    for (int j = 0; j < DQ_PER; j++) {
      const uint64_t row = wg0 + (uint64_t)j * NTT_THREADS + tid;
      if (row < end) {
        cv[j] = compose_value(Tm, K, row, x);  // C_row (air.rs:49-136 + mask)
        d[j] = gl_sub(x, z);
      } else {  // past the block: a unit factor in the batch
        cv[j] = 0;
        d[j] = 1;
      }
      Pp = j ? gl_mul(Pp, d[j]) : d[j];
      a[j] = Pp;
      x = gl_mul(x, ws);
    }
  }
  uint64_t S = Pp, Tq = Pp;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t u = __shfl_up(S, o, 64);
    if (lane >= o) S = gl_mul(S, u);
    const uint64_t v = __shfl_down(Tq, o, 64);
    if (lane + o < 64) Tq = gl_mul(Tq, v);
  }
  uint64_t Q = __shfl_down(Tq, 1, 64);
  if (lane == 63) Q = 1;
  uint64_t Sprev = __shfl_up(S, 1, 64);
  if (lane == 0) Sprev = 1;
  if (lane == 63) wtot[wave] = S;
  __syncthreads();
  if (tid == 0) {
    uint64_t t = wtot[0];
#pragma unroll
    for (int w = 1; w < NTT_THREADS / 64; w++) t = gl_mul(t, wtot[w]);
    s_inv = gl_inv(t);
  }
  __syncthreads();
  uint64_t invW = s_inv;
#pragma unroll
  for (int w = 0; w < NTT_THREADS / 64; w++)
    if (w != wave) invW = gl_mul(invW, wtot[w]);
  uint64_t inv_run = gl_mul(gl_mul(invW, Q), Sprev);
  uint64_t acc = 0;
#pragma unroll
  for (int j = DQ_PER - 1; j >= 0; j--) {
    const uint64_t ij = j ? gl_mul(inv_run, a[j - 1]) : inv_run;
    if (j) inv_run = gl_mul(inv_run, d[j]);
    const uint64_t row = wg0 + (uint64_t)j * NTT_THREADS + tid;
    if (row < end) {
      const uint64_t xj = gl_add(d[j], z);  // w_n^row
      const uint64_t Dj = gl_mul(cv[j], ij);
      Dout[row] = Dj;
      acc = gl_add(acc, gl_mul(Dj, xj));
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc = gl_add(acc, __shfl_xor(acc, o, 64));
  __syncthreads();
  if (lane == 0) wtot[wave] = acc;
  __syncthreads();
  if (tid == 0) {
    uint64_t t = wtot[0];
#pragma unroll
    for (int w = 1; w < NTT_THREADS / 64; w++) t = gl_add(t, wtot[w]);
    partial[blockIdx.x] = t;
  }
}

__device__ __forceinline__ uint64_t gl_pow_dev(uint64_t b, uint64_t e) {
  uint64_t r = 1;
  while (e) {
    if (e & 1) r = gl_mul(r, b);
    b = gl_sqr(b);
    e >>= 1;
  }
  return r;
}

// Coset scaling for a shift other than the prover's 3 (kernel-level ABI):
// a[p] *= base^e, e = bitrev_logn(p), from base^e = lo[e & 2047] hi[e >> 11].
__global__ void __launch_bounds__(NTT_THREADS) k_pow_tables(uint64_t* __restrict__ lo, uint64_t* __restrict__ hi,
                                                            uint64_t base, uint32_t nhi) {
  const uint32_t t = blockIdx.x * NTT_THREADS + threadIdx.x;
  if (t < 2048) lo[t] = gl_pow_dev(base, t);
  if (t < nhi) hi[t] = gl_pow_dev(base, 2048ull * t);
}
__global__ void __launch_bounds__(NTT_THREADS) k_scale_pow_bitrev(uint64_t* __restrict__ a, int logn,
                                                                  const uint64_t* __restrict__ lo,
                                                                  const uint64_t* __restrict__ hi) {
  const uint64_t p = blockIdx.x * (uint64_t)NTT_THREADS + threadIdx.x;
  if (p >> logn) return;
  const uint32_t e = logn ? __brev((uint32_t)p) >> (32 - logn) : 0;
  a[p] = gl_mul(a[p], gl_mul(lo[e & 2047], hi[e >> 11]));
}
hipError_t launch_scale_pow_bitrev(hipStream_t st, uint64_t* a, int logn, uint64_t base, uint64_t* scratch) {
  if (logn > 31) return hipErrorInvalidValue;
  const uint32_t nhi = logn > 11 ? 1u << (logn - 11) : 1u;
  uint64_t* lo = scratch;
  uint64_t* hi = scratch + 2048;
  const uint32_t nt = std::max<uint32_t>(2048, nhi);
  hipLaunchKernelGGL(k_pow_tables, dim3((nt + NTT_THREADS - 1) / NTT_THREADS), dim3(NTT_THREADS), 0, st, lo, hi, base,
                     nhi);
  const uint64_t n = 1ULL << logn;
  hipLaunchKernelGGL(k_scale_pow_bitrev, dim3((unsigned)((n + NTT_THREADS - 1) / NTT_THREADS)), dim3(NTT_THREADS), 0,
                     st, a, logn, lo, hi);
  return hipGetLastError();
}

// Every WG reduces the partials (S; f(z) = K1 S, c' = f(z) K2, kappa = K3 S),
// then grid-strides over the tables: rlo[t] = r^t, rhi[t] = c' r^(4096 t),
// rhk[t] = kappa r^(4096 t).
__global__ void __launch_bounds__(NTT_THREADS) k_q_tables(const uint64_t* __restrict__ partial, uint32_t nparts,
                                                          const DevChal* __restrict__ ch, uint64_t* __restrict__ rlo,
                                                          uint64_t* __restrict__ rhi, uint32_t nhi,
                                                          uint64_t* __restrict__ rhk, uint32_t nhk) {
  const uint64_t K1 = ch->K1, K2 = ch->K2, K3 = ch->K3, r = ch->rho, r4096 = ch->rho4096;
  __shared__ uint64_t wsum[NTT_THREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint64_t acc = 0;
  for (uint32_t i = tid; i < nparts; i += NTT_THREADS) acc = gl_add(acc, partial[i]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc = gl_add(acc, __shfl_xor(acc, o, 64));
  if (lane == 0) wsum[wave] = acc;
  __syncthreads();
  uint64_t S = wsum[0];
#pragma unroll
  for (int w = 1; w < NTT_THREADS / 64; w++) S = gl_add(S, wsum[w]);
  const uint64_t fz = gl_mul(K1, S), cp = gl_mul(fz, K2), kappa = gl_mul(K3, S);
  const uint64_t g0 = (uint64_t)blockIdx.x * NTT_THREADS + tid, gs = (uint64_t)gridDim.x * NTT_THREADS;
  for (uint64_t t = g0; t < 4096; t += gs) rlo[t] = gl_pow_dev(r, t);
  for (uint64_t t = g0; t < nhi; t += gs) rhi[t] = gl_mul(cp, gl_pow_dev(r4096, t));
  for (uint64_t t = g0; t < nhk; t += gs) rhk[t] = gl_mul(kappa, gl_pow_dev(r4096, t));
}

uint64_t dq_rows_per_part(uint64_t nrows) {
  // 8 rows per lane (the composition values of the lane stay in registers:
  // 16 took 158 VGPRs); 4 when that leaves fewer than 512 workgroups (a
  // sharded rank's block: its batch inversions then run twice as parallel)
  return (uint64_t)NTT_THREADS * (nrows >= 512ull * NTT_THREADS * 8 ? 8 : 4);
}

hipError_t launch_inv_base(hipStream_t st, const ComposeTerms& Tm, uint64_t* D, uint64_t* partial, int logn,
                           const DevChal* ch, const NttTables& T, uint64_t row0, uint64_t nrows, uint64_t per) {
  if (logn < 4 || (per != 8 * NTT_THREADS && per != 4 * NTT_THREADS) || nrows % 16 || row0 % per ||
      row0 + nrows > (1ULL << logn))
    return hipErrorInvalidValue;
  const dim3 grid((unsigned)((nrows + per - 1) / per));
  if (per == 8 * NTT_THREADS)
    hipLaunchKernelGGL(k_inv_base<8>, grid, dim3(NTT_THREADS), 0, st, Tm, D, partial + row0 / per, logn, ch, T, row0,
                       nrows);
  else
    hipLaunchKernelGGL(k_inv_base<4>, grid, dim3(NTT_THREADS), 0, st, Tm, D, partial + row0 / per, logn, ch, T, row0,
                       nrows);
  return hipGetLastError();
}

hipError_t launch_q_tables(hipStream_t st, const uint64_t* partial, int logn, int logN, const DevChal* ch,
                           uint64_t* rlo, uint64_t* rhi, uint64_t* rhk, uint64_t per) {
  if (logn < 4 || logN < logn || logN > 32 || !per) return hipErrorInvalidValue;
  const uint64_t n = 1ULL << logn;
  const uint32_t nparts = (uint32_t)((n + per - 1) / per);
  const uint32_t nhi = logN > 12 ? (1u << (logN - 12)) : 1u;
  const uint32_t nhk = logn > 12 ? (1u << (logn - 12)) : 1u;
  const uint64_t work = std::max<uint64_t>(4096, nhi);
  const unsigned grid = (unsigned)std::min<uint64_t>(1024, (work + NTT_THREADS - 1) / NTT_THREADS);
  hipLaunchKernelGGL(k_q_tables, dim3(grid), dim3(NTT_THREADS), 0, st, partial, nparts, ch, rlo, rhi, nhi, rhk, nhk);
  return hipGetLastError();
}

// ------------------------------------------------------------------ host side
static void plan_passes(int logN, int first_min, int* ms, int* np) {
  int passes = (logN + NTT_MMAX - 1) / NTT_MMAX;
  if (passes < 1) passes = 1;
  int base = logN / passes, rem = logN % passes;
  for (int i = 0; i < passes; i++) ms[i] = base + (i < rem ? 1 : 0);
  (void)first_min;
  *np = passes;
}

// Plan with the sL = 0 pass extended by an in-tile radix-16 step (X16: m =
// 10..12 in one 2^m-point tile) when that saves a pass: 2^17..2^20 take 2
// passes instead of 3, 2^25..2^28 take 3 instead of 4. The other passes keep
// m in [6, 8] (the register kernels). Returns false when it saves nothing.
// The sL = 0 pass is first for DIT and last for DIF.
static bool plan_passes_x16(int logN, bool dif, int* ms, int* np) {
  const int cur = std::max(1, (logN + NTT_MMAX - 1) / NTT_MMAX);
  for (int f = 12; f >= 10; f--) {
    const int r = logN - f;
    if (r < 0) continue;
    const int k = (r + 7) / 8;  // passes for the rest, each m in [6, 8]
    if (6 * k > r || 1 + k >= cur || 1 + k > 8) continue;
    const int base = k ? r / k : 0, rem = k ? r % k : 0;
    int o = 0;
    if (!dif) ms[o++] = f;
    for (int i = 0; i < k; i++) ms[o++] = base + (i < rem ? 1 : 0);
    if (dif) ms[o++] = f;
    *np = o;
    return true;
  }
  return false;
}

// A 2^21-point DIF (the prover's INTT at T = 2^21) as a 9-stage wide pass
// (k_ntt_dif9) + the 12-stage X16 narrow pass: 2 HBM round trips instead of
// 3 passes of 7 (round 3, tools/ab_intt_dif9.sh: intt stage 97 -> 91 us per
// proof, in flight +0.7-1.1%).
hipError_t ntt_dif(hipStream_t st, uint64_t* a, int logN, bool inverse, const NttTables& T) {
  if (logN == 0) return hipSuccess;
  int ms[8], np;
  const bool x16 = plan_passes_x16(logN, true, ms, &np);
  if (!x16) plan_passes(logN, 1, ms, &np);
  if (logN == 21) {
    NttPassArgs P{};
    P.a = a; P.tw = T; P.m = 9; P.sL = 12; P.inverse = inverse ? 1 : 0; P.logC = 4;
    const unsigned tiles = (unsigned)((1ULL << logN) >> (9 + 4));
    if (inverse) hipLaunchKernelGGL(k_ntt_dif9<true>, dim3(tiles), dim3(512), 0, st, P);
    else hipLaunchKernelGGL(k_ntt_dif9<false>, dim3(tiles), dim3(512), 0, st, P);
    P.m = 12; P.sL = 0;
    const bool ok = inverse ? launch_ntt4<true, true>(st, P, (unsigned)((1ULL << logN) >> 12))
                            : launch_ntt4<true, false>(st, P, (unsigned)((1ULL << logN) >> 12));
    if (!ok) return hipErrorInvalidValue;
    return hipGetLastError();
  }
  int sL = logN;
  for (int i = 0; i < np; i++) {
    NttPassArgs P{};
    P.a = a; P.src = nullptr; P.tw = T; P.m = ms[i]; sL -= ms[i]; P.sL = sL;
    P.inverse = inverse ? 1 : 0; P.skip = 0;
    int logC = logN - P.m; if (logC > 4) logC = 4; P.logC = logC;
    uint64_t tiles = (1ULL << logN) >> (P.m + logC);
    if (P.m > NTT_MMAX) {  // X16 tile: 2^m contiguous points
      P.logC = 4;
      tiles = (1ULL << logN) >> P.m;
      const bool ok = inverse ? launch_ntt4<true, true>(st, P, (unsigned)tiles)
                              : launch_ntt4<true, false>(st, P, (unsigned)tiles);
      if (!ok) return hipErrorInvalidValue;
      continue;
    }
    const bool fast = inverse ? launch_ntt4<true, true>(st, P, (unsigned)tiles)
                              : launch_ntt4<true, false>(st, P, (unsigned)tiles);
    if (!fast) hipLaunchKernelGGL(k_ntt_pass<true>, dim3((unsigned)tiles), dim3(NTT_THREADS), 0, st, P);
  }
  return hipGetLastError();
}

// DIT from bit-reversed input. If src != nullptr, the first pass loads the
// replicated, scaled coefficients (LDE) and skips the 3 stages replication
// makes trivial (blowup 8).
hipError_t ntt_dit(hipStream_t st, uint64_t* a, int logN, bool inverse, const NttTables& T,
                   const uint64_t* src, int log_src, uint64_t inv_n, uint64_t coset_e, const DeepFuse* deep,
                   bool* fused, const DeepPoly* dpoly, int src_logP) {
  if (src_logP < 0 || src_logP > 3 || (src_logP && (!src || log_src < src_logP))) return hipErrorInvalidValue;
  if (fused) *fused = false;
  if (logN == 0) return hipSuccess;
  if (dpoly && (!src || logN > 32 || log_src > logN)) return hipErrorInvalidValue;
  int ms[8], np;
  // X16 for plain transforms and for the DEEP-polynomial LDE (its first pass
  // loads all 2^m points: no replication skip); not for the replicated load
  const bool x16 = (!src || dpoly) && plan_passes_x16(logN, false, ms, &np);
  if (!x16) plan_passes(logN, src ? 3 : 1, ms, &np);
  // DIT order: smallest strides first; ensure the first pass holds >= 3 stages for the LDE skip
  if (src && ms[0] < logN - log_src) return hipErrorInvalidValue;
  int sL = 0;
  for (int i = 0; i < np; i++) {
    NttPassArgs P{};
    P.a = a; P.tw = T; P.m = ms[i]; P.sL = sL; P.inverse = inverse ? 1 : 0;
    P.src = (i == 0) ? src : nullptr;
    P.log_src = log_src; P.inv_n = inv_n; P.coset_e = (i == 0) ? coset_e : 0;
    P.src_logP = (i == 0) ? src_logP : 0;
    P.skip = (i == 0 && src && !dpoly) ? (logN - log_src) : 0;
    if (i == 0 && dpoly) { P.dp_rlo = dpoly->rlo; P.dp_rhi = dpoly->rhi; P.dp_rhk = dpoly->rhk; P.dp_logN = logN; }
    int logC = logN - P.m; if (logC > 4) logC = 4; P.logC = logC;
    uint64_t tiles = (1ULL << logN) >> (P.m + logC);
    if (P.m > NTT_MMAX) {  // X16 tile: 2^m contiguous points
      P.logC = 4;
      tiles = (1ULL << logN) >> P.m;
      const bool ok = inverse ? launch_ntt4<false, true>(st, P, (unsigned)tiles)
                              : launch_ntt4<false, false>(st, P, (unsigned)tiles);
      if (!ok) return hipErrorInvalidValue;
      sL += ms[i];
      continue;
    }
    // last pass, forward, 16 wide columns, M1 = 4 (m = 7 or 8), not the replicated first pass
    if (deep && fused && i == np - 1 && i > 0 && !inverse &&
        logC == 4 && P.sL >= 4 && (P.m == 8 || P.m == 7)) {
      P.deep_z = deep->z; P.deep_logN = deep->logN; P.deep_logP = deep->logP; P.deep_g = deep->g;
      if (P.m == 8)
        hipLaunchKernelGGL((k_ntt4<false, false, 4, 4, 0, true>), dim3((unsigned)tiles), dim3(NTT_THREADS), 0, st, P);
      else
        hipLaunchKernelGGL((k_ntt4<false, false, 4, 3, 0, true>), dim3((unsigned)tiles), dim3(NTT_THREADS), 0, st, P);
      *fused = true;
      sL += ms[i];
      continue;
    }
    const bool fast = inverse ? launch_ntt4<false, true>(st, P, (unsigned)tiles)
                              : launch_ntt4<false, false>(st, P, (unsigned)tiles);
    if (!fast) hipLaunchKernelGGL(k_ntt_pass<false>, dim3((unsigned)tiles), dim3(NTT_THREADS), 0, st, P);
    sL += ms[i];
  }
  return hipGetLastError();
}

// Natural order through the transposed last pass (nat_tr): passes of <= 9
// stages, then 8 (2^23: 8+7+8, 2^24: 8+8+8, 2^25: 9+8+8, 2^26: 9+9+8). The
// first pass reads `a` and writes `scratch`, the middle ones run in place on
// scratch, the last gathers from scratch and writes `a` in natural order.
static bool ntt_dif_natural_tr(hipStream_t st, uint64_t* a, uint64_t* scratch, int logN, bool inverse,
                               const NttTables& T, uint64_t scale, hipError_t* err) {
  if (logN < 23 || logN > 26) return false;
  int plan[3];
  plan[2] = 8;
  const int rest = logN - 8;              // 15..18
  plan[0] = (rest + 1) / 2;               // 8, 8, 9, 9
  plan[1] = rest - plan[0];               // 7, 8, 8, 9
  int sL = logN;
  for (int i = 0; i < 3; i++) {
    NttPassArgs P{};
    P.a = i == 0 ? a : scratch;
    P.out = i == 0 ? scratch : nullptr;
    P.tw = T; P.m = plan[i]; sL -= plan[i]; P.sL = sL;
    P.inverse = inverse ? 1 : 0;
    P.logC = 4;
    const uint64_t tiles = (1ULL << logN) >> (P.m + 4);
    if (i == 2) {
      P.a = scratch; P.out = a; P.nat_tr = 1; P.nat_logN = logN; P.out_scale = scale;
    }
    if (P.m == 9) {
      if (inverse) hipLaunchKernelGGL(k_ntt_dif9<true>, dim3((unsigned)tiles), dim3(512), 0, st, P);
      else hipLaunchKernelGGL(k_ntt_dif9<false>, dim3((unsigned)tiles), dim3(512), 0, st, P);
      continue;
    }
    const bool ok = inverse ? launch_ntt4<true, true>(st, P, (unsigned)tiles)
                            : launch_ntt4<true, false>(st, P, (unsigned)tiles);
    if (!ok) { *err = hipErrorInvalidValue; return true; }
  }
  *err = hipGetLastError();
  return true;
}

// Natural order as a DIT whose first (narrow) pass gathers its input in
// bit-reversed order (gather_dit_to_lds): the plain plans of 2^21..2^24, no
// bit-reversal pass. The first
// pass reads `a` and writes `scratch`, the middle ones run in place on
// scratch, the last one writes `a` (n^-1 on its pre-twiddle chain).
static bool ntt_dit_natural(hipStream_t st, uint64_t* a, uint64_t* scratch, int logN, bool inverse,
                            const NttTables& T, uint64_t scale, hipError_t* err) {
  // measured (round 3, profiles/r03/ntt_nat_ab2.txt, fwd + inv round trips):
  // 2^21 96.6 vs 129.0 us (DIF natural store), 2^22 164.9 vs 178.6, 2^23 275.9
  // vs 283.2, 2^24 498.5 vs 508.7 (584.8 with the bit-reversal pass); the
  // X16 plans' point gather loses (2^25 1267 vs 1053, 2^26 2493 vs 2109), so
  // those sizes keep the DIF forms
  if (logN < 21 || logN > 24) return false;
  int ms[8], np;
  if (plan_passes_x16(logN, false, ms, &np)) return false;
  plan_passes(logN, 1, ms, &np);
  if (np < 2 || ms[0] > NTT_MMAX) return false;
  int sL = 0;
  for (int i = 0; i < np; i++) {
    NttPassArgs P{};
    P.tw = T; P.m = ms[i]; P.sL = sL; P.inverse = inverse ? 1 : 0; P.logC = 4;
    P.a = i == 0 ? a : scratch;
    P.out = i == 0 ? scratch : (i == np - 1 ? a : nullptr);
    if (i == 0) { P.nat_tr = 1; P.nat_logN = logN; }
    if (i == np - 1) P.out_scale = scale;
    const unsigned tiles = (unsigned)(P.m > NTT_MMAX ? (1ULL << logN) >> P.m : (1ULL << logN) >> (P.m + 4));
    const bool ok = inverse ? launch_ntt4<false, true>(st, P, tiles) : launch_ntt4<false, false>(st, P, tiles);
    if (!ok) { *err = hipErrorInvalidValue; return true; }
    sL += ms[i];
  }
  *err = hipGetLastError();
  return true;
}

bool ntt_dif_natural(hipStream_t st, uint64_t* a, uint64_t* scratch, int logN, bool inverse, const NttTables& T,
                     uint64_t scale, hipError_t* err) {
  *err = hipSuccess;
  if (scratch && scratch != a && ntt_dit_natural(st, a, scratch, logN, inverse, T, scale, err)) return true;
  if (scratch && scratch != a && ntt_dif_natural_tr(st, a, scratch, logN, inverse, T, scale, err)) return true;
  // measured (profiles/r02_ntt_nat_ab.txt): 1-5% faster at 2^19..2^22, slower from 2^24 (where the
  // scattered lines no longer merge in L2 before write-back: 687 vs 577 us at 2^24)
  if (!scratch || scratch == a || logN < 19 || logN > 22)
    return false;
  int ms[8], np;
  const bool x16 = plan_passes_x16(logN, true, ms, &np);
  if (!x16) plan_passes(logN, 1, ms, &np);
  if (np < 2) return false;
  int sL = logN;
  for (int i = 0; i < np; i++) {
    NttPassArgs P{};
    P.a = i == 0 ? a : scratch;
    P.out = i == 0 ? scratch : nullptr;
    P.tw = T; P.m = ms[i]; sL -= ms[i]; P.sL = sL;
    P.inverse = inverse ? 1 : 0;
    P.logC = 4;
    uint64_t tiles = (1ULL << logN) >> (P.m + 4);
    if (i == np - 1) {  // the narrow pass: sL = 0, tile of 16 * 2^m' contiguous points
      P.out = a; P.nat_out = 1; P.nat_logN = logN; P.out_scale = scale;
      if (P.m > NTT_MMAX) tiles = (1ULL << logN) >> P.m;
    }
    const bool ok = (logN == 20 && launch_r8(st, P, inverse, (unsigned)tiles)) ||
                    (inverse ? launch_ntt4<true, true>(st, P, (unsigned)tiles)
                             : launch_ntt4<true, false>(st, P, (unsigned)tiles));
    if (!ok) { *err = hipErrorInvalidValue; return true; }
  }
  *err = hipGetLastError();
  return true;
}

hipError_t bitrev_permute(hipStream_t st, const uint64_t* in, uint64_t* out, int logN, uint64_t scale, bool do_scale) {
  if (logN >= 8) {
    hipLaunchKernelGGL(k_bitrev_permute, dim3(1u << (logN - 8)), dim3(256), 0, st, in, out, logN, scale,
                       do_scale ? 1 : 0);
  } else {
    hipLaunchKernelGGL(k_bitrev_permute_small, dim3(1), dim3(256), 0, st, in, out, logN, scale, do_scale ? 1 : 0);
  }
  return hipGetLastError();
}

// tile side 2^A; measured (round 2): 2^26 round trip 2910 / 2782 / 2819 us at
// A = 4 / 5 / 6; 2^24 (MALL-resident) best at 4
static int bitrev_tile_log(int logN) {
  int A = logN >= 25 ? 5 : 4;
  while (A > 4 && logN < 2 * A) A--;
  return A;
}
hipError_t bitrev_inplace(hipStream_t st, uint64_t* a, int logN, uint64_t scale, bool do_scale) {
  if (logN < 8) return hipErrorInvalidValue;
  const int A = bitrev_tile_log(logN);
  const dim3 grid(1u << (logN - 2 * A));
  if (A == 5) hipLaunchKernelGGL(k_bitrev_inplace<5>, grid, dim3(256), 0, st, a, logN, scale, do_scale ? 1 : 0);
  else hipLaunchKernelGGL(k_bitrev_inplace<4>, grid, dim3(256), 0, st, a, logN, scale, do_scale ? 1 : 0);
  return hipGetLastError();
}

hipError_t dntt_permute_twiddle(hipStream_t st, const uint64_t* in, uint64_t* out, int logM, const NttTables& T,
                                uint64_t e_step, bool inverse, bool tw_src, uint64_t scale) {
  if (logM < 8) return hipErrorInvalidValue;
  if (logM >= 10)
    hipLaunchKernelGGL(k_dntt_permute_twiddle<4>, dim3(1u << (logM - 10)), dim3(256), 0, st, in, out, logM, T, e_step,
                       inverse ? 1 : 0, tw_src ? 1 : 0, scale);
  else
    hipLaunchKernelGGL(k_dntt_permute_twiddle<1>, dim3(1u << (logM - 8)), dim3(256), 0, st, in, out, logM, T, e_step,
                       inverse ? 1 : 0, tw_src ? 1 : 0, scale);
  return hipGetLastError();
}
hipError_t bintt_dft_twiddle(hipStream_t st, uint64_t* r, int P, uint64_t Q, uint32_t d, int logn,
                             const NttTables& T) {
  if (Q == 0 || logn > T.K) return hipErrorInvalidValue;
  const dim3 g((unsigned)((Q + 255) / 256));
  const uint64_t j0 = (uint64_t)d * Q;
  switch (P) {
    case 2: hipLaunchKernelGGL(k_bintt_dft_twiddle<2>, g, dim3(256), 0, st, r, Q, j0, logn, T); break;
    case 4: hipLaunchKernelGGL(k_bintt_dft_twiddle<4>, g, dim3(256), 0, st, r, Q, j0, logn, T); break;
    case 8: hipLaunchKernelGGL(k_bintt_dft_twiddle<8>, g, dim3(256), 0, st, r, Q, j0, logn, T); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t dntt_dft(hipStream_t st, uint64_t* r, int P, uint64_t Q, bool inverse) {
  const dim3 g((unsigned)((Q + 255) / 256));
#define SEZKP_DFT(PP)                                                                              \
  if (P == PP) {                                                                                   \
    if (inverse) hipLaunchKernelGGL((k_dntt_dft<PP, true>), g, dim3(256), 0, st, r, Q);           \
    else hipLaunchKernelGGL((k_dntt_dft<PP, false>), g, dim3(256), 0, st, r, Q);                  \
    return hipGetLastError();                                                                      \
  }
  SEZKP_DFT(2) SEZKP_DFT(4) SEZKP_DFT(8)
#undef SEZKP_DFT
  return P == 1 ? hipSuccess : hipErrorInvalidValue;
}
}  // namespace sezkp

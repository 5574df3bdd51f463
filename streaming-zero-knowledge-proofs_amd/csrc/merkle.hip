// merkle.hip — DEEP division, FRI fold, BLAKE3 Merkle layers and path
// extraction for CDNA4 (gfx950).
//
// Reference semantics:
//  * DEEP: out_i = y_i * (3*w_N^i - z)^-1          (crates/sezkp-stark/src/v1/lde.rs:76-93)
//  * fold: y'_i = y_i + beta * y_{i+len/2}          (prover.rs:200-239)
//  * leaves BLAKE3(8 LE bytes), parents BLAKE3(l||r), odd promotion never
//    triggers because every FRI layer is a power of two (merkle.rs:46-71,150-160)
//  * paths: siblings bottom->top (merkle.rs:80-108; equal to
//    fri_stream.rs:357-409 on power-of-two layers)
//
// Layout: a workgroup of 256 lanes owns a 1024-leaf subtree. Each lane hashes 4
// consecutive leaves and folds them to one level-2 node in registers (all 64
// lanes busy), the remaining 8 levels reduce through an 8 KB struct-of-words
// LDS image read with ds_read_b64 pairs (conflict-free). Levels >= lstore are
// written to HBM for path extraction; lower levels are recomputed on demand.
#include "dev_common.h"
#include "sezkp_internal.h"

namespace sezkp {

constexpr int MK_THREADS = 256;

__device__ __forceinline__ void store_level(const TreeDev& T, int l, uint64_t idx, const uint32_t (&h)[8]) {
  if (l >= T.lstore && l <= T.logLen) node_store(T.nodes + 8 * (tree_level_off(T.logLen, T.lstore, l) + idx), h);
  if (l == T.logLen) node_store(T.root, h);
}

// LDS image: words-major [8][W]; nodes 2i and 2i+1 of word w are one b64.
template <int W>
__device__ __forceinline__ void lds_put(uint32_t (*lds)[W], int i, const uint32_t (&h)[8]) {
#pragma unroll
  for (int w = 0; w < 8; w++) lds[w][i] = h[w];
}
template <int W>
__device__ __forceinline__ void lds_pair(uint32_t (*lds)[W], int i, uint32_t (&l)[8], uint32_t (&r)[8]) {
#pragma unroll
  for (int w = 0; w < 8; w++) {
    uint2 p = *reinterpret_cast<const uint2*>(&lds[w][2 * i]);
    l[w] = p.x;
    r[w] = p.y;
  }
}

// words q and 4 + q of node idx at level l (a quad's share of store_level)
__device__ __forceinline__ void store_level_quad(const TreeDev& T, int l, uint64_t idx, int q, uint32_t lo,
                                                 uint32_t hi) {
  if (l >= T.lstore && l <= T.logLen) {
    uint32_t* p = T.nodes + 8 * (tree_level_off(T.logLen, T.lstore, l) + idx);
    p[q] = lo;
    p[4 + q] = hi;
  }
  if (l == T.logLen) {
    T.root[q] = lo;
    T.root[4 + q] = hi;
  }
}

// Reduce `cnt` level-`lvl` nodes in LDS to one; WG-local node i at level l has
// global index wg * (cnt_at_l) + i. A level of at most W / 4 parents runs one
// parent per quad of lanes (b3_parent_quad): the chain of the last levels is
// latency-bound, and a quad's compression is a quarter of the instructions
// per lane of a one-lane compression (round 6). QMAX: the largest level (in
// parents) that goes to quads: W / 4 in the latency-bound chains; 32 in the
// throughput-bound tree kernels, where a level of 64 parents is one full wave
// step of one-lane compressions but four of quad ones, while 32 or fewer
// parents leave most of a wave idle in the one-lane form (and when a small
// launch runs as a single round of workgroups in the same phase, the idle
// waves are not covered by other workgroups).
template <int W, int QMAX = 0>
__device__ __forceinline__ void wg_reduce(uint32_t (*lds)[W], int cnt, int lvl, uint64_t wg, const TreeDev& T,
                                          int stop = 64) {
  const int tid = threadIdx.x;
  while (cnt > 1 && lvl < stop) {
    const int half = cnt >> 1;
    if (half <= QMAX && 4 * half <= W) {
      const int pq = tid >> 2, q = tid & 3;
      const bool act = pq < half;  // whole quads
      uint32_t lo = 0, hi = 0;
      if (act) lds_parent_quad<W, (QMAX == W / 4)>(lds, pq, q, lo, hi);
      __syncthreads();
      lvl++;
      cnt = half;
      if (act) {
        lds[q][pq] = lo;
        lds[4 + q][pq] = hi;
        store_level_quad(T, lvl, wg * (uint64_t)cnt + pq, q, lo, hi);
      }
      __syncthreads();
      continue;
    }
    uint32_t h[8];
    const bool act = tid < half;
    if (act) {
      uint32_t l[8], r[8];
      lds_pair(lds, tid, l, r);
      b3_parent(l, r, h);
    }
    __syncthreads();
    lvl++;
    cnt = half;
    if (act) {
      lds_put(lds, tid, h);
      store_level(T, lvl, wg * (uint64_t)cnt + tid, h);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- DEEP
// 16 consecutive elements per lane, one Montgomery batch inversion per
// workgroup (4096 elements): wave prefix/suffix product scans + one Fermat
// inversion in lane 0 of wave 0.
constexpr int DEEP_PER = 16;
__global__ void __launch_bounds__(MK_THREADS) k_deep(uint64_t* __restrict__ y, int logN, uint64_t z, NttTables T,
                                                     int logP, uint32_t g, uint64_t shift) {
  __shared__ uint64_t wtot[MK_THREADS / 64];
  __shared__ uint64_t s_inv;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t i0 = ((uint64_t)blockIdx.x * MK_THREADS + tid) * DEEP_PER;
  const uint64_t N = 1ULL << (logN - logP);  // local length
  const bool act = i0 < N;
  uint64_t d[DEEP_PER], a[DEEP_PER];
  uint64_t P = 1;
  if (act) {
    // x_j = shift * w_N^(g + P j) (shift = 3 in the prover); first from the
    // two-level table, then incremental
    const uint64_t e = ((uint64_t)g + (i0 << logP)) << (T.K - logN);
    uint64_t x = gl_mul(gl_mul(T.hi[e >> T.S], T.lo[e & ((1ULL << T.S) - 1)]), shift);
    uint64_t wN;
    {
      const uint64_t e1 = 1ULL << (T.K - logN + logP);
      wN = gl_mul(T.hi[e1 >> T.S], T.lo[e1 & ((1ULL << T.S) - 1)]);
    }
#pragma unroll
    for (int j = 0; j < DEEP_PER; j++) {
      d[j] = i0 + j < N ? gl_sub(x, z) : 1;  // N < 16 (tiny kernel-level calls): neutral tail
      P = gl_mul(P, d[j]);
      a[j] = P;
      x = gl_mul(x, wN);
    }
  }
  // wave inclusive prefix S and exclusive suffix Q of the lane products
  uint64_t S = P, Tq = P;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t u = __shfl_up(S, o, 64);
    if (lane >= o) S = gl_mul(S, u);
    uint64_t v = __shfl_down(Tq, o, 64);
    if (lane + o < 64) Tq = gl_mul(Tq, v);
  }
  uint64_t Q = __shfl_down(Tq, 1, 64);
  if (lane == 63) Q = 1;
  uint64_t Sprev = __shfl_up(S, 1, 64);
  if (lane == 0) Sprev = 1;
  if (lane == 63) wtot[wave] = S;
  __syncthreads();
  if (tid == 0) {
    uint64_t t = 1;
#pragma unroll
    for (int w = 0; w < MK_THREADS / 64; w++) t = gl_mul(t, wtot[w]);
    s_inv = gl_inv(t);
  }
  __syncthreads();
  uint64_t invW = s_inv;  // inverse of this wave's total = inv(all) * prod(other waves)
#pragma unroll
  for (int w = 0; w < MK_THREADS / 64; w++)
    if (w != wave) invW = gl_mul(invW, wtot[w]);
  // inv(S_lane) = invW * Q ; inv(P_lane) = inv(S_lane) * S_{lane-1}
  uint64_t inv_run = gl_mul(gl_mul(invW, Q), Sprev);
  if (!act) return;
#pragma unroll
  for (int j = DEEP_PER - 1; j >= 0; j--) {
    uint64_t inv_dj = j ? gl_mul(inv_run, a[j - 1]) : inv_run;
    inv_run = gl_mul(inv_run, d[j]);
    if (i0 + j < N) y[i0 + j] = gl_mul(y[i0 + j], inv_dj);
  }
}

// ------------------------------------------------------- leaf + subtree
// fold == 0: leaves are in[i];  fold == 1: leaves y'_i = in[i] + beta*in[i+len],
// written to out (the next FRI layer). One WG = 1024 leaves (or the whole layer).
__global__ void __launch_bounds__(MK_THREADS) k_leaf_subtree(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                             int logLen, int fold, uint64_t beta,
                                                             const uint64_t* __restrict__ dbeta, TreeDev T) {
  __shared__ uint32_t lds[8][MK_THREADS];
  if (dbeta) beta = *dbeta;
  const int tid = threadIdx.x;
  const uint64_t len = 1ULL << logLen;
  const uint64_t wg = blockIdx.x;
  const int sub_log = logLen < 10 ? logLen : 10;
  const int logper = logLen < 2 ? logLen : 2;
  const int nact = 1 << (sub_log - logper);
  const uint64_t base = wg << sub_log;
  if (tid < nact) {
    const uint64_t i0 = base + ((uint64_t)tid << logper);
    uint64_t v[4] = {0, 0, 0, 0};
    if (logper == 2) {
      const ulonglong2* p = reinterpret_cast<const ulonglong2*>(in + i0);
      ulonglong2 a0 = p[0], a1 = p[1];
      v[0] = a0.x; v[1] = a0.y; v[2] = a1.x; v[3] = a1.y;
      if (fold) {
        const ulonglong2* q = reinterpret_cast<const ulonglong2*>(in + i0 + len);
        ulonglong2 b0 = q[0], b1 = q[1];
        v[0] = gl_add(v[0], gl_mul(beta, b0.x));
        v[1] = gl_add(v[1], gl_mul(beta, b0.y));
        v[2] = gl_add(v[2], gl_mul(beta, b1.x));
        v[3] = gl_add(v[3], gl_mul(beta, b1.y));
        ulonglong2* o = reinterpret_cast<ulonglong2*>(out + i0);
        o[0] = make_ulonglong2(v[0], v[1]);
        o[1] = make_ulonglong2(v[2], v[3]);
      }
    } else {
      for (int j = 0; j < (1 << logper); j++) {
        v[j] = in[i0 + j];
        if (fold) {
          v[j] = gl_add(v[j], gl_mul(beta, in[i0 + j + len]));
          out[i0 + j] = v[j];
        }
      }
    }
    uint32_t h[8];
    if (logper == 2) {
      uint32_t l0[8], l1[8], p0[8], p1[8];
      b3_leaf_u64(v[0], l0);
      b3_leaf_u64(v[1], l1);
      if (T.lstore == 0) { store_level(T, 0, i0, l0); store_level(T, 0, i0 + 1, l1); }
      b3_parent(l0, l1, p0);
      b3_leaf_u64(v[2], l0);
      b3_leaf_u64(v[3], l1);
      if (T.lstore == 0) { store_level(T, 0, i0 + 2, l0); store_level(T, 0, i0 + 3, l1); }
      b3_parent(l0, l1, p1);
      if (T.lstore <= 1) { store_level(T, 1, i0 >> 1, p0); store_level(T, 1, (i0 >> 1) + 1, p1); }
      b3_parent(p0, p1, h);
      store_level(T, 2, i0 >> 2, h);
    } else if (logper == 1) {
      uint32_t l0[8], l1[8];
      b3_leaf_u64(v[0], l0);
      b3_leaf_u64(v[1], l1);
      if (T.lstore == 0) { store_level(T, 0, i0, l0); store_level(T, 0, i0 + 1, l1); }
      b3_parent(l0, l1, h);
      store_level(T, 1, i0 >> 1, h);
    } else {
      b3_leaf_u64(v[0], h);
      store_level(T, 0, i0, h);
    }
    lds_put(lds, tid, h);
  }
  __syncthreads();
  wg_reduce(lds, nact, logper, wg, T);
}

// ------------------------------------------------------------ upper levels
// Input: stored level `from` (count 2^(logLen-from)); one WG reduces up to
// 1024 nodes (4 per lane, 2 levels in registers) and stores every level, up
// to level `to` (0: the root).
// node g of level `from`: stored, or (a sharded cap's first pass) taken from
// the allgathered run roots and stored at its cap position
struct GathSrc {  // a sharded cap's first pass: the allgathered run roots (UpperJob)
  const uint32_t* gath;
  uint64_t nrun;
  int logP;
};
__device__ __forceinline__ void upper_load(const uint32_t* src, const GathSrc& gs, uint64_t g, uint32_t (&h)[8]) {
  if (gs.gath) node_load(gs.gath + 8 * ((g & ((1ULL << gs.logP) - 1)) * gs.nrun + (g >> gs.logP)), h);
  else node_load(src + 8 * g, h);
}
__device__ __forceinline__ void upper_src(const TreeDev& T, const uint32_t* src, const GathSrc& gs, int from,
                                          uint64_t g, uint32_t (&h)[8]) {
  upper_load(src, gs, g, h);
  if (gs.gath) store_level(T, from, g, h);
}
__device__ __forceinline__ void upper_wg(const TreeDev& T, int from, uint64_t wg, uint32_t (*lds)[MK_THREADS],
                                         int to = 0, GathSrc gj = GathSrc{nullptr, 0, 0}) {
  const int tid = threadIdx.x;
  const int top = (to > 0 && to < T.logLen) ? to : T.logLen;
  const int cnt_log = top - from;
  const int sub_log = cnt_log < 10 ? cnt_log : 10;
  // up to 256 nodes: one per lane, every level in wg_reduce (its quad levels
  // take over from 64 parents down); more: 4 per lane, 2 levels in registers
  const int logper = cnt_log <= 8 ? 0 : 2;
  const int nact = 1 << (sub_log - logper);
  const uint32_t* src = T.nodes + 8 * tree_level_off(T.logLen, T.lstore, from);
  if (tid < nact) {
    const uint64_t g = (wg << (sub_log - logper)) + tid;  // node index at level from+logper
    uint32_t h[8];
    if (logper == 2) {
      // the four loads first, then (gathered caps) their stores: a store
      // between loads would serialise their latencies (the compiler cannot
      // tell the gathered roots from the cap apart)
      uint32_t a[8], b[8], c[8], d[8], p0[8], p1[8];
      upper_load(src, gj, 4 * g + 0, a);
      upper_load(src, gj, 4 * g + 1, b);
      upper_load(src, gj, 4 * g + 2, c);
      upper_load(src, gj, 4 * g + 3, d);
      if (gj.gath) {
        store_level(T, from, 4 * g + 0, a);
        store_level(T, from, 4 * g + 1, b);
        store_level(T, from, 4 * g + 2, c);
        store_level(T, from, 4 * g + 3, d);
      }
      b3_parent(a, b, p0);
      b3_parent(c, d, p1);
      store_level(T, from + 1, 2 * g, p0);
      store_level(T, from + 1, 2 * g + 1, p1);
      b3_parent(p0, p1, h);
      store_level(T, from + 2, g, h);
    } else if (logper == 1) {
      uint32_t a[8], b[8];
      upper_src(T, src, gj, from, 2 * g, a);
      upper_src(T, src, gj, from, 2 * g + 1, b);
      b3_parent(a, b, h);
      store_level(T, from + 1, g, h);
    } else {
      upper_src(T, src, gj, from, g, h);
      if (from == T.logLen) node_store(T.root, h);
    }
    lds_put(lds, tid, h);
  }
  __syncthreads();
  wg_reduce<MK_THREADS, MK_THREADS / 4>(lds, nact, from + logper, wg, T);
}

// grid.y indexes trees of identical shape spaced tree_stride nodes apart.
__global__ void __launch_bounds__(MK_THREADS) k_tree_upper(TreeDev T0, uint64_t tree_stride, uint64_t root_stride,
                                                           int from) {
  __shared__ uint32_t lds[8][MK_THREADS];
  TreeDev T = T0;
  T.nodes += 8 * tree_stride * blockIdx.y;
  T.root += root_stride * blockIdx.y;
  upper_wg(T, from, blockIdx.x, lds);
}

// One WG per job: trees of different shapes reduced in one launch.
__global__ void __launch_bounds__(MK_THREADS) k_upper_jobs(const UpperJob* __restrict__ jobs) {
  __shared__ uint32_t lds[8][MK_THREADS];
  const UpperJob J = jobs[blockIdx.x];
  upper_wg(J.tree, J.from, J.wg, lds, J.to, GathSrc{J.gath, J.nrun, J.logP});
}

// ------------------------------------------------- layers of >= 4096 leaves
// Depth-first subtree over v[B .. B + 2^LV) held in registers (static
// indices only); leaf i0 + j is global leaf index. Keeps at most LV pending
// left siblings live, like a binary counter.
template <int LV, int B>
__device__ __forceinline__ void subtree_regs(const uint64_t (&v)[16], uint64_t i0, const TreeDev& T, uint32_t (&h)[8]) {
  if constexpr (LV == 0) {
    b3_leaf_u64(v[B], h);
    store_level(T, 0, i0 + B, h);
  } else {
    uint32_t l[8];
    subtree_regs<LV - 1, B>(v, i0, T, l);
    subtree_regs<LV - 1, B + (1 << (LV - 1))>(v, i0, T, h);
    b3_parent(l, h, h);
    store_level(T, LV, (i0 + B) >> LV, h);
  }
}

// One WG = 256 << LPL leaves: 2^LPL consecutive leaves per lane folded to a
// level-LPL node in registers (binary counter; LPL = 4: 31 compressions per
// lane, all lanes busy), then levels LPL+1 .. 8+LPL through LDS. fold == 1
// computes the layer from the previous one first (y'_i = in[i] + beta*in[i+len])
// and writes it to out. Levels above `stop` are left to the upper-level jobs.
// LPL = 4 (4096-leaf WGs) for large trees; LPL = 2 (1024 leaves) when a
// launch has 512 or fewer 4096-leaf WGs (small shards and traces): a WG's 31
// dependent compressions per lane then ran at one or two waves per SIMD.
template <int LPL>
__device__ __forceinline__ void layer16_wg(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, int logLen,
                                           int fold, uint64_t beta, const TreeDev& T, uint64_t wg,
                                           uint32_t (*lds)[MK_THREADS], int stop) {
  const int tid = threadIdx.x;
  const uint64_t len = 1ULL << logLen;
  const uint64_t i0 = (wg << (8 + LPL)) + ((uint64_t)tid << LPL);
  uint64_t v[16];
  {
    const ulonglong2* p = reinterpret_cast<const ulonglong2*>(in + i0);
#pragma unroll
    for (int k = 0; k < (1 << LPL) / 2; k++) {
      const ulonglong2 a = p[k];
      v[2 * k] = a.x;
      v[2 * k + 1] = a.y;
    }
  }
  if (fold) {
    const ulonglong2* q = reinterpret_cast<const ulonglong2*>(in + i0 + len);
    ulonglong2* o = reinterpret_cast<ulonglong2*>(out + i0);
#pragma unroll
    for (int k = 0; k < (1 << LPL) / 2; k++) {
      const ulonglong2 b = q[k];
      v[2 * k] = gl_add(v[2 * k], gl_mul(beta, b.x));
      v[2 * k + 1] = gl_add(v[2 * k + 1], gl_mul(beta, b.y));
      o[k] = make_ulonglong2(v[2 * k], v[2 * k + 1]);
    }
  }
  uint32_t h[8];
  subtree_regs<LPL, 0>(v, i0, T, h);
  lds_put(lds, tid, h);
  __syncthreads();
  // quads for the levels of <= 32 parents only in the 1024-leaf form, which
  // small per-device LDEs (a sharded rank's, <= 2^21 points) launch as one
  // round of workgroups in the same phase (a P = 8 rank's layer-0 tree 0.099
  // -> 0.090 ms); with several rounds (the headline's 4096 / 2048-leaf forms,
  // three proofs in flight) the one-lane form measured 3-5% faster in flight
  wg_reduce<MK_THREADS, (LPL == L16S_LOG - 8 ? 32 : 0)>(lds, MK_THREADS, LPL, wg, T, stop);
}

template <int LPL>
__global__ void __launch_bounds__(MK_THREADS) k_layer16(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                        int logLen, int fold, uint64_t beta,
                                                        const uint64_t* __restrict__ dbeta, TreeDev T, int stop) {
  __shared__ uint32_t lds[8][MK_THREADS];
  if (dbeta) beta = *dbeta;
  layer16_wg<LPL>(in, out, logLen, fold, beta, T, blockIdx.x, lds, stop);
}

// FRI fold y'_i = y_i + beta * y_{i+len} (prover.rs:200-239), 4 per lane.
__global__ void __launch_bounds__(MK_THREADS) k_fold(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                     int logLen, uint64_t beta, const uint64_t* __restrict__ dbeta) {
  const uint64_t len = 1ULL << logLen;
  if (dbeta) beta = *dbeta;
  const uint64_t i = ((uint64_t)blockIdx.x * MK_THREADS + threadIdx.x) * 4;
  if (i >= len) return;
  const ulonglong2* p = reinterpret_cast<const ulonglong2*>(in + i);
  const ulonglong2* q = reinterpret_cast<const ulonglong2*>(in + i + len);
  ulonglong2* o = reinterpret_cast<ulonglong2*>(out + i);
  const ulonglong2 a0 = p[0], a1 = p[1], b0 = q[0], b1 = q[1];
  o[0] = make_ulonglong2(gl_add(a0.x, gl_mul(beta, b0.x)), gl_add(a0.y, gl_mul(beta, b0.y)));
  o[1] = make_ulonglong2(gl_add(a1.x, gl_mul(beta, b1.x)), gl_add(a1.y, gl_mul(beta, b1.y)));
}

// F folds per pass (F = 2..4): layer r + m (m = 1..F) at index i + j L, j <
// 2^(F-m), L = len(layer r + F), is y_m = y_{m-1}[i + j L] + b_m
// y_{m-1}[i + (j + 2^(F-m)) L]; a lane holds two adjacent i, reads its 2^F
// strided pairs of layer r once and writes every intermediate layer once.
template <int F>
__global__ void __launch_bounds__(MK_THREADS) k_foldm(const uint64_t* __restrict__ in, FoldOuts O, int logLenF) {
  constexpr int W = 1 << F;
  const uint64_t L = 1ULL << logLenF;
  const uint64_t i = ((uint64_t)blockIdx.x * MK_THREADS + threadIdx.x) * 2;
  if (i >= L) return;
  uint64_t x0[W], x1[W];
#pragma unroll
  for (int j = 0; j < W; j++) {
    const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(in + i + (uint64_t)j * L);
    x0[j] = v.x;
    x1[j] = v.y;
  }
#pragma unroll
  for (int m = 1; m <= F; m++) {
    const int half = W >> m;
    const uint64_t b = O.beta[m - 1];
    uint64_t* out = O.out[m - 1];
#pragma unroll
    for (int j = 0; j < half; j++) {
      x0[j] = gl_add(x0[j], gl_mul(b, x0[j + half]));
      x1[j] = gl_add(x1[j], gl_mul(b, x1[j + half]));
      *reinterpret_cast<ulonglong2*>(out + i + (uint64_t)j * L) = make_ulonglong2(x0[j], x1[j]);
    }
  }
}

// ------------------------------------------------------ small FRI layers
// All fold layers of <= 2048 leaves in one launch: WG j produces layer
// logLen = Ls - j. Each WG reloads the (<= 4096-element) layer above the
// first tail layer into LDS and replays the fold chain down to its own layer
// (a few thousand mulmods), so the trees of all small layers are built
// concurrently instead of as a dependent chain of tiny launches.
constexpr int TAIL_THREADS = 256;
// depth-first subtree over 2^LV leaves b[i0 ..] (LDS values), leaf index i0 + j
template <int LV>
__device__ __forceinline__ void tail_sub(const uint64_t* b, uint64_t i0, const TreeDev& T, uint32_t (&h)[8]) {
  if constexpr (LV == 0) {
    b3_leaf_u64(b[i0], h);
    store_level(T, 0, i0, h);
  } else {
    uint32_t l[8];
    tail_sub<LV - 1>(b, i0, T, l);
    tail_sub<LV - 1>(b, i0 + (1ULL << (LV - 1)), T, h);
    b3_parent(l, h, h);
    store_level(T, LV, i0 >> LV, h);
  }
}
__global__ void __launch_bounds__(TAIL_THREADS) k_fri_tail(TailArgs A) {
  __shared__ uint64_t buf[1 << (TAIL_MAX)];  // the 2^(Ls+1) <= 4096 source values
  __shared__ uint32_t lds[8][TAIL_THREADS];
  // these few workgroups share CUs with the forest's (VALU-saturating) waves;
  // their serial fold chain + tree would otherwise get a 1/7 share of issue
  // and outlast the forest. Top wave priority for the whole (short) kernel.
  __builtin_amdgcn_s_setprio(3);
  const int tid = threadIdx.x;
  const int j = blockIdx.x;
  const int L = A.Ls - j;
  int cur = A.Ls + 1;
  for (int i = tid; i < (1 << cur); i += TAIL_THREADS) buf[i] = A.src[i];
  __syncthreads();
  uint64_t* vals = nullptr;
  TreeDev T{};
#pragma unroll
  for (int s = 0; s < TAIL_MAX; s++) {
    if (s <= j) {
      const int half = 1 << (cur - 1);
      for (int i = tid; i < half; i += TAIL_THREADS) buf[i] = gl_add(buf[i], gl_mul(A.beta[s], buf[i + half]));
      __syncthreads();
      cur--;
    }
    if (s == j) {
      vals = A.vals[s];
      T = A.tree[s];
    }
  }
  const int len = 1 << L;
  for (int i = tid; i < len; i += TAIL_THREADS) vals[i] = buf[i];
  // 2^lp leaves per lane (lp <= 3), folded in registers, then LDS levels
  const int lp = L > 8 ? L - 8 : 0;
  const int nact = len >> lp;
  if (tid < nact) {
    uint32_t h[8];
    const uint64_t i0 = (uint64_t)tid << lp;
    switch (lp) {
      case 0: tail_sub<0>(buf, i0, T, h); break;
      case 1: tail_sub<1>(buf, i0, T, h); break;
      case 2: tail_sub<2>(buf, i0, T, h); break;
      default: tail_sub<3>(buf, i0, T, h); break;
    }
    lds_put(lds, tid, h);
  }
  __syncthreads();
  wg_reduce<TAIL_THREADS, TAIL_THREADS / 4>(lds, nact, lp, 0, T);
}

// The same small-layer job as k_fri_tail, run by the first workgroups of the
// forest launch: the fold replay goes through a per-workgroup global scratch
// (4096 values, L2-resident; workgroup-scope visibility after each barrier)
// instead of 32 KB of LDS, so these workgroups fit beside the forest's and are
// dispatched first. As a kernel of its own on the side stream the tail could
// only start once the forest's ~2K workgroups had all been placed (they fill
// every CU's VGPRs), and it ended ~60 us after the forest (round 2).
__device__ __forceinline__ void fri_tail_wg(const TailArgs& A, int j, uint64_t* __restrict__ gbuf,
                                            uint32_t (*lds)[MK_THREADS]) {
  __builtin_amdgcn_s_setprio(3);  // a serial chain beside VALU-saturating forest waves
  const int tid = threadIdx.x;
  const int L = A.Ls - j;
  uint64_t* buf = gbuf + ((uint64_t)j << TAIL_MAX);
  int cur = A.Ls + 1;
  {  // first fold straight from the source layer
    const int half = 1 << (cur - 1);
    for (int i = tid; i < half; i += MK_THREADS) buf[i] = gl_add(A.src[i], gl_mul(A.beta[0], A.src[i + half]));
    cur--;
    __syncthreads();
  }
  uint64_t* vals = A.vals[0];
  TreeDev T = A.tree[0];
#pragma unroll
  for (int s = 1; s < TAIL_MAX; s++) {
    if (s <= j) {
      const int half = 1 << (cur - 1);
      constexpr int PER = (1 << TAIL_MAX) / 2 / MK_THREADS;
      uint64_t y[PER];
#pragma unroll
      for (int q = 0; q < PER; q++) {
        const int i = tid + q * MK_THREADS;
        if (i < half) y[q] = gl_add(buf[i], gl_mul(A.beta[s], buf[i + half]));
      }
      __syncthreads();  // every read of this step before any write
#pragma unroll
      for (int q = 0; q < PER; q++) {
        const int i = tid + q * MK_THREADS;
        if (i < half) buf[i] = y[q];
      }
      __syncthreads();
      cur--;
    }
    if (s == j) {
      vals = A.vals[s];
      T = A.tree[s];
    }
  }
  const int len = 1 << L;
  for (int i = tid; i < len; i += MK_THREADS) vals[i] = buf[i];
  const int lp = L > 8 ? L - 8 : 0;
  const int nact = len >> lp;
  if (tid < nact) {
    uint32_t h[8];
    const uint64_t i0 = (uint64_t)tid << lp;
    switch (lp) {
      case 0: tail_sub<0>(buf, i0, T, h); break;
      case 1: tail_sub<1>(buf, i0, T, h); break;
      case 2: tail_sub<2>(buf, i0, T, h); break;
      default: tail_sub<3>(buf, i0, T, h); break;
    }
    lds_put(lds, tid, h);
  }
  __syncthreads();
  wg_reduce(lds, nact, lp, 0, T);
}

// All fold layers of >= 4096 leaves hashed in one launch (their values were
// produced by the fold chain first): the per-layer trees are independent, so
// the small layers no longer serialize behind each other's latency. The first
// `ntail` workgroups build the layers of <= 2048 leaves (fri_tail_wg).
// A launch may cover a sub-range of the layers: `layers` then points at its
// first one and wg_base is that layer's wg_start (wg_start values are global).
template <int LPL, bool TAIL>
__global__ void __launch_bounds__(MK_THREADS) k_forest16(const ForestLayer* __restrict__ layers, int nlayers,
                                                         TailArgs A, int ntail, uint64_t* __restrict__ tailbuf,
                                                         uint32_t wg_base) {
  __shared__ uint32_t lds[8][MK_THREADS];
  // TAIL = false (the sharded launches, whose small layers run in k_fri_tail):
  // without the tail's fold replay the kernel needs fewer VGPRs, so a small
  // launch that runs as one round of workgroups fits more of them per SIMD
  if constexpr (TAIL) {
    if ((int)blockIdx.x < ntail) {
      fri_tail_wg(A, (int)blockIdx.x, tailbuf, lds);
      return;
    }
  }
  const uint32_t b = blockIdx.x - (uint32_t)ntail + wg_base;
  int l = 0;
  while (l + 1 < nlayers && layers[l + 1].wg_start <= b) l++;
  const ForestLayer F = layers[l];
  layer16_wg<LPL>(F.vals, nullptr, F.tree.logLen, 0, 0, F.tree, b - F.wg_start, lds, (int)F.stop);
}

// ------------------------------------------------ sharded layout changes
// Rank g of P holds the coset values e[j] = f(3 w_N^(g + P j)), j < M = N/P.
// Target (run) layout: rank d owns every index i with (i mod P*S) in
// [d*S, (d+1)*S), S = 4096, stored as runs k1 = i / (P*S) of S consecutive
// indices. Source j = k1*S + d*(S/P) + t (t < S/P) goes to rank d, slot
// k1*(S/P) + t of the d-th send segment; on arrival from rank g it lands at
// local k1*S + P*t + g. Both kernels are one coalesced pass (8 B read + write).
constexpr uint64_t L16_TILE = 1ULL << L16_LOG;
__global__ void __launch_bounds__(256) k_cyc_pack(const uint64_t* __restrict__ cyc, uint64_t* __restrict__ send,
                                                  uint64_t M, int logP) {
  const uint64_t o = (uint64_t)blockIdx.x * 256 + threadIdx.x;  // send index
  if (o >= M) return;
  const int lsp = L16_LOG - logP;                               // log2(S/P)
  const uint64_t d = o / (M >> logP), r = o % (M >> logP);
  const uint64_t k1 = r >> lsp, t = r & ((1ULL << lsp) - 1);
  send[o] = cyc[(k1 << L16_LOG) + (d << lsp) + t];
}
// One workgroup per run k1 (S = 4096 values): they arrive as P segments of
// S/P, one per source rank g, at recv[g M/P + k1 S/P + t], and go to
// local[k1 S + t P + g]: both sides contiguous through an LDS transpose
// (segments padded by 32/P words: the transposed reads take distinct banks).
// Round 5's one-thread-per-value form wrote 8-byte words P apart (~16 us for
// a P = 8 rank's 2^21 values).
__global__ void __launch_bounds__(256) k_cyc_unpack(const uint64_t* __restrict__ recv, uint64_t* __restrict__ local,
                                                    uint64_t M, int logP) {
  __shared__ uint64_t sh[L16_TILE + 32 * 8];
  const uint64_t k1 = blockIdx.x;
  const int lsp = L16_LOG - logP, tid = threadIdx.x;
  const int seg = 1 << lsp, row = seg + (32 >> logP);
  const uint64_t MP = M >> logP;
  for (int i = tid; i < (int)L16_TILE; i += 256) {
    const int g = i >> lsp, t = i & (seg - 1);
    sh[g * row + t] = recv[(uint64_t)g * MP + k1 * (uint64_t)seg + t];
  }
  __syncthreads();
  for (int j = tid; j < (int)L16_TILE; j += 256) {
    const int g = j & ((1 << logP) - 1), t = j >> logP;
    local[(k1 << L16_LOG) + j] = sh[g * row + t];
  }
}
// rank g's runs out of the whole LDE (P = 2, full_lde): local[k1 S + t] =
// full[(k1 P + g) S + t], two values per lane
__global__ void __launch_bounds__(256) k_runs_extract(const uint64_t* __restrict__ full, uint64_t* __restrict__ local,
                                                      uint64_t M, int logP, uint32_t g) {
  const uint64_t o = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 2;  // local index
  if (o >= M) return;
  const uint64_t k1 = o >> L16_LOG, t = o & (L16_TILE - 1);
  *reinterpret_cast<ulonglong2*>(local + o) =
      *reinterpret_cast<const ulonglong2*>(full + (((k1 << logP) + g) << L16_LOG) + t);
}
// run roots allgathered as [rank d][run k1] -> cap level L16_LOG node k1*P + d
__global__ void __launch_bounds__(256) k_runroots_scatter(const uint32_t* __restrict__ gathered, TreeDev cap,
                                                          uint64_t nrun, int logP) {
  const uint64_t o = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (o >= (nrun << logP)) return;
  const uint64_t d = o / nrun, k1 = o % nrun;
  uint32_t h[8];
  node_load(gathered + 8 * o, h);
  store_level(cap, L16_LOG, (k1 << logP) + d, h);
}

// the same for every FRI run layer in one launch (a thread per cap node;
// the layers' node ranges are consecutive in the grid)
__global__ void __launch_bounds__(256) k_runroots_scatter_multi(const RunRootsBatch B) {
  uint64_t o = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  int j = 0;
  while (j < B.n && o >= (B.nrun[j] << B.logP)) o -= B.nrun[j++] << B.logP;
  if (j >= B.n) return;
  const uint64_t nrun = B.nrun[j];
  const uint64_t d = o / nrun, k1 = o % nrun;
  uint32_t h[8];
  node_load(B.gathered[j] + 8 * o, h);
  store_level(B.cap[j], L16_LOG, (k1 << B.logP) + d, h);
}

// ---------------------------------------------------------- path extraction
// One 64-lane workgroup per (layer, index): recompute the 64-leaf group that
// holds the index (levels < lstore), then read stored siblings above.
__global__ void __launch_bounds__(64) k_fri_paths(const FriLayerDev* __restrict__ layers, const uint32_t* __restrict__ req,
                                                  const uint32_t* __restrict__ count, ProofLayout P) {
  __shared__ uint32_t lds[8][64];
  const int lane = threadIdx.x;
  if (count && blockIdx.x >= *count) return;  // grid sized for the most requests a rank can own
  const uint32_t r = req[3 * blockIdx.x];
  const uint64_t idx = req[3 * blockIdx.x + 1];
  const uint32_t ord = req[3 * blockIdx.x + 2];  // q*2k + 2r + side
  const FriLayerDev Ly = layers[r];
  const TreeDev& T = Ly.tree;
  const TreeDev& C = Ly.cap;
  const int L = C.logLen;  // global layer length 2^L
  // local position of the global index (identity when unsharded)
  const uint64_t li = Ly.sharded ? (((idx >> (L16_LOG + Ly.logP)) << L16_LOG) | (idx & (L16_TILE - 1))) : idx;
  const int glog = L < T.lstore ? L : T.lstore;
  const uint64_t g = 1ULL << glog;
  const uint64_t base = li & ~(g - 1);
  // FriQuery (proof.rs:68-78): record = value, u64 path length, siblings
  const int k = P.k;
  const uint32_t qi = ord / (2 * k), side = ord & 1;
  uint32_t* fq = P.base + (P.fq_off + 8 + (uint64_t)qi * P.fq_bytes) / 4;
  const uint64_t off_r = 2 * (16 * (uint64_t)r + 32 * ((uint64_t)r * k - (uint64_t)r * (r - 1) / 2));
  uint32_t* o = fq + (8 + 8 * (uint64_t)(k + 1) + 8 + off_r + side * (16 + 32 * (uint64_t)L)) / 4;
  if (lane == 0) {
    const uint64_t v = Ly.vals[li];
    o[0] = (uint32_t)v;
    o[1] = (uint32_t)(v >> 32);
    o[2] = (uint32_t)L;
    o[3] = 0;
  }
  // stored siblings above the group: lane (j, w) takes word w of level
  // glog + 8 i + j. All loads issued up front, so their latency overlaps the
  // group's hashing instead of one dependent load/store round per level.
  constexpr int PATH_ROUNDS = (64 - LSTORE_FRI + 7) / 8;
  uint32_t sw[PATH_ROUNDS];
#pragma unroll
  for (int i = 0; i < PATH_ROUNDS; i++) {
    const int lvl = glog + 8 * i + (lane >> 3);
    if (lvl >= L) break;
    if (lvl < C.lstore) {  // inside this rank's run subtree (local tree)
      const uint64_t sib = (li >> lvl) ^ 1;
      sw[i] = T.nodes[8 * (tree_level_off(T.logLen, T.lstore, lvl) + sib) + (lane & 7)];
    } else {               // cap levels (global indices)
      const uint64_t sib = (idx >> lvl) ^ 1;
      sw[i] = C.nodes[8 * (tree_level_off(C.logLen, C.lstore, lvl) + sib) + (lane & 7)];
    }
  }
  if (lane < (int)g) {
    uint32_t h[8];
    b3_leaf_u64(Ly.vals[base + lane], h);
    for (int w = 0; w < 8; w++) lds[w][lane] = h[w];
  }
  __syncthreads();
  // the group's levels 1..glog-1 (its root, level glog, is not on the path):
  // 32 parents one per lane, then 16, 8, 4, 2 on quads of lanes (round 6)
  int cnt = (int)g;
  for (int lvl = 0; lvl < glog; lvl++) {
    const int sib = (int)(((li - base) >> lvl) ^ 1);
    if (lane < 8) o[4 + 8 * lvl + lane] = lds[lane][sib];
    if (lvl + 1 == glog) break;
    const int half = cnt >> 1;
    if (4 * half <= 64) {
      const int pq = lane >> 2, q = lane & 3;
      uint32_t lo = 0, hi = 0;
      if (pq < half) lds_parent_quad(lds, pq, q, lo, hi);
      __syncthreads();
      if (pq < half) {
        lds[q][pq] = lo;
        lds[4 + q][pq] = hi;
      }
    } else {
      uint32_t h[8];
      if (lane < half) {
        uint32_t a[8], b[8];
        for (int w = 0; w < 8; w++) { a[w] = lds[w][2 * lane]; b[w] = lds[w][2 * lane + 1]; }
        b3_parent(a, b, h);
      }
      __syncthreads();
      if (lane < half)
        for (int w = 0; w < 8; w++) lds[w][lane] = h[w];
    }
    __syncthreads();
    cnt = half;
  }
#pragma unroll
  for (int i = 0; i < PATH_ROUNDS; i++) {
    const int lvl = glog + 8 * i + (lane >> 3);
    if (lvl >= L) break;
    o[4 + 8 * lvl + (lane & 7)] = sw[i];
  }
}

// ------------------------------------------------------------------ host
hipError_t launch_deep(hipStream_t st, uint64_t* y, int logN, uint64_t z, const NttTables& tw, int logP, uint32_t g,
                       uint64_t shift) {
  if (logP > logN) return hipErrorInvalidValue;
  const uint64_t N = 1ULL << (logN - logP);
  const uint64_t per_wg = (uint64_t)MK_THREADS * DEEP_PER;
  const unsigned grid = (unsigned)((N + per_wg - 1) / per_wg);
  hipLaunchKernelGGL(k_deep, dim3(grid), dim3(MK_THREADS), 0, st, y, logN, z, tw, logP, g, shift);
  return hipGetLastError();
}

hipError_t launch_cyc_pack(hipStream_t st, const uint64_t* cyc, uint64_t* send, uint64_t M, int logP) {
  if (M % L16_TILE || (1 << logP) > (int)L16_TILE) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_cyc_pack, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, st, cyc, send, M, logP);
  return hipGetLastError();
}
hipError_t launch_cyc_unpack(hipStream_t st, const uint64_t* recv, uint64_t* local, uint64_t M, int logP) {
  if (M % L16_TILE || (1 << logP) > (int)L16_TILE) return hipErrorInvalidValue;
  if (logP > 3) return hipErrorInvalidValue;  // the LDS padding assumes P <= 8
  hipLaunchKernelGGL(k_cyc_unpack, dim3((unsigned)(M >> L16_LOG)), dim3(256), 0, st, recv, local, M, logP);
  return hipGetLastError();
}
hipError_t launch_runs_extract(hipStream_t st, const uint64_t* full, uint64_t* local, uint64_t M, int logP,
                               uint32_t g) {
  if (M % L16_TILE || (g >> logP)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_runs_extract, dim3((unsigned)((M / 2 + 255) / 256)), dim3(256), 0, st, full, local, M, logP, g);
  return hipGetLastError();
}
hipError_t launch_runroots_scatter(hipStream_t st, const uint32_t* gathered, TreeDev cap, uint64_t nrun_per_rank,
                                   int logP) {
  const uint64_t total = nrun_per_rank << logP;
  hipLaunchKernelGGL(k_runroots_scatter, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, gathered, cap,
                     nrun_per_rank, logP);
  return hipGetLastError();
}

hipError_t launch_runroots_scatter_multi(hipStream_t st, const RunRootsBatch& B) {
  if (B.n <= 0 || B.n > RR_BATCH_MAX) return hipErrorInvalidValue;
  uint64_t total = 0;
  for (int j = 0; j < B.n; j++) total += B.nrun[j] << B.logP;
  hipLaunchKernelGGL(k_runroots_scatter_multi, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, B);
  return hipGetLastError();
}

hipError_t launch_leaf_subtree(hipStream_t st, const uint64_t* in, uint64_t* out_vals, int logLen, int fold,
                               uint64_t beta, TreeDev tree, const uint64_t* dbeta) {
  if (logLen >= L16_LOG) {
    hipError_t e = launch_layer16(st, in, out_vals, logLen, fold, beta, tree, L16_LOG, dbeta);
    if (e != hipSuccess) return e;
    if (logLen == L16_LOG) return hipSuccess;  // the single WG wrote the root
    return launch_tree_upper(st, &tree, 1, 0, 0, L16_LOG);
  }
  const int sub_log = logLen < 10 ? logLen : 10;
  const unsigned grid = (unsigned)(1ULL << (logLen - sub_log));
  hipLaunchKernelGGL(k_leaf_subtree, dim3(grid), dim3(MK_THREADS), 0, st, in, out_vals, logLen, fold, beta, dbeta,
                     tree);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  int from = sub_log;
  while (from < logLen) {
    const int cnt_log = logLen - from;
    const int step = cnt_log < 10 ? cnt_log : 10;
    hipLaunchKernelGGL(k_tree_upper, dim3((unsigned)(1ULL << (cnt_log - step)), 1), dim3(MK_THREADS), 0, st, tree,
                       (uint64_t)0, (uint64_t)0, from);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    from += step;
  }
  return hipSuccess;
}

hipError_t launch_layer16(hipStream_t st, const uint64_t* in, uint64_t* out_vals, int logLen, int fold, uint64_t beta,
                          TreeDev tree, int stop, const uint64_t* dbeta, int wg_log) {
  if ((wg_log != L16_LOG && wg_log != L16M_LOG && wg_log != L16S_LOG) || logLen < wg_log || stop < tree.lstore ||
      stop > wg_log)
    return hipErrorInvalidValue;
  const dim3 grid((unsigned)(1ULL << (logLen - wg_log)));
  if (wg_log == L16_LOG)
    hipLaunchKernelGGL(k_layer16<4>, grid, dim3(MK_THREADS), 0, st, in, out_vals, logLen, fold, beta, dbeta, tree, stop);
  else if (wg_log == L16M_LOG)
    hipLaunchKernelGGL(k_layer16<3>, grid, dim3(MK_THREADS), 0, st, in, out_vals, logLen, fold, beta, dbeta, tree, stop);
  else
    hipLaunchKernelGGL(k_layer16<2>, grid, dim3(MK_THREADS), 0, st, in, out_vals, logLen, fold, beta, dbeta, tree, stop);
  return hipGetLastError();
}

hipError_t launch_fold(hipStream_t st, const uint64_t* in, uint64_t* out, int logLen, uint64_t beta,
                       const uint64_t* dbeta) {
  if (logLen < 2) return hipErrorInvalidValue;
  const uint64_t per = (uint64_t)MK_THREADS * 4;
  const unsigned grid = (unsigned)(((1ULL << logLen) + per - 1) / per);
  hipLaunchKernelGGL(k_fold, dim3(grid), dim3(MK_THREADS), 0, st, in, out, logLen, beta, dbeta);
  return hipGetLastError();
}

hipError_t launch_foldm(hipStream_t st, const uint64_t* in, const FoldOuts& outs, int F, int logLenF) {
  if (logLenF < 1 || F < 2 || F > FOLD_MAX) return hipErrorInvalidValue;
  const uint64_t per = (uint64_t)MK_THREADS * 2;
  const unsigned grid = (unsigned)(((1ULL << logLenF) + per - 1) / per);
  switch (F) {
    case 2: hipLaunchKernelGGL(k_foldm<2>, dim3(grid), dim3(MK_THREADS), 0, st, in, outs, logLenF); break;
    case 3: hipLaunchKernelGGL(k_foldm<3>, dim3(grid), dim3(MK_THREADS), 0, st, in, outs, logLenF); break;
    default: hipLaunchKernelGGL(k_foldm<4>, dim3(grid), dim3(MK_THREADS), 0, st, in, outs, logLenF); break;
  }
  return hipGetLastError();
}

hipError_t launch_forest16(hipStream_t st, const ForestLayer* d_layers, int nlayers, uint32_t total_wgs,
                           const TailArgs* tail, uint64_t* tailbuf, uint32_t wg_base, int wg_log) {
  if (nlayers <= 0) return tail ? hipErrorInvalidValue : hipSuccess;
  if (tail && (tail->Ls < 0 || tail->Ls >= TAIL_MAX || !tailbuf)) return hipErrorInvalidValue;
  const int ntail = tail ? tail->Ls + 1 : 0;
  const TailArgs none{};
#define SEZKP_FOREST(LPL)                                                                                      \
  do {                                                                                                         \
    if (tail)                                                                                                  \
      hipLaunchKernelGGL((k_forest16<LPL, true>), dim3(total_wgs + (uint32_t)ntail), dim3(MK_THREADS), 0, st,   \
                         d_layers, nlayers, *tail, ntail, tailbuf, wg_base);                                   \
    else                                                                                                       \
      hipLaunchKernelGGL((k_forest16<LPL, false>), dim3(total_wgs), dim3(MK_THREADS), 0, st, d_layers, nlayers, \
                         none, 0, tailbuf, wg_base);                                                           \
  } while (0)
  if (wg_log == L16_LOG) SEZKP_FOREST(4);
  else if (wg_log == L16M_LOG) SEZKP_FOREST(3);
  else if (wg_log == L16S_LOG) SEZKP_FOREST(2);
  else return hipErrorInvalidValue;
#undef SEZKP_FOREST
  return hipGetLastError();
}

hipError_t launch_fri_tail(hipStream_t st, const TailArgs& a) {
  if (a.Ls < 0 || a.Ls >= TAIL_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_fri_tail, dim3((unsigned)(a.Ls + 1)), dim3(TAIL_THREADS), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_upper_jobs(hipStream_t st, const UpperJob* d_jobs, int njobs) {
  if (njobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_upper_jobs, dim3((unsigned)njobs), dim3(MK_THREADS), 0, st, d_jobs);
  return hipGetLastError();
}

void plan_upper_jobs(const TreeDev& T, int from, std::vector<std::vector<UpperJob>>& passes, int to,
                     const uint32_t* gath, uint64_t nrun, int logP) {
  const int top = (to > 0 && to < T.logLen) ? to : T.logLen;
  if (gath && from == top) {  // a one-node cap (P = 1): the job copies the gathered root into it
    if (passes.empty()) passes.resize(1);
    UpperJob J{T, from, 0u, to, 0};
    J.gath = gath;
    J.nrun = nrun;
    J.logP = logP;
    passes[0].push_back(J);
    return;
  }
  int p = 0;
  while (from < top) {
    const int c = top - from;
    const int step = c < 10 ? c : 10;
    if ((int)passes.size() <= p) passes.resize(p + 1);
    for (uint64_t w = 0; w < (1ULL << (T.logLen - from - step)); w++) {
      UpperJob J{T, from, (uint32_t)w, to, 0};
      if (p == 0 && gath) {  // the first pass reads the gathered run roots (and stores them)
        J.gath = gath;
        J.nrun = nrun;
        J.logP = logP;
      }
      passes[p].push_back(J);
    }
    from += step;
    p++;
  }
}

hipError_t launch_tree_upper(hipStream_t st, TreeDev* trees, int ntrees, uint64_t tree_stride_nodes,
                             uint64_t root_stride_words, int from_level) {
  const TreeDev T = trees[0];
  int from = from_level;
  if (from == T.logLen) {  // single node: it is the root
    hipLaunchKernelGGL(k_tree_upper, dim3(1, ntrees), dim3(MK_THREADS), 0, st, T, tree_stride_nodes,
                       root_stride_words, from);
    return hipGetLastError();
  }
  while (from < T.logLen) {
    const int cnt_log = T.logLen - from;
    const int step = cnt_log < 10 ? cnt_log : 10;
    hipLaunchKernelGGL(k_tree_upper, dim3((unsigned)(1ULL << (cnt_log - step)), ntrees), dim3(MK_THREADS), 0, st, T,
                       tree_stride_nodes, root_stride_words, from);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    from += step;
  }
  return hipSuccess;
}

hipError_t launch_fri_paths(hipStream_t st, const FriLayerDev* d_layers, const uint32_t* d_req, int nreq,
                            const ProofLayout& P, const uint32_t* d_count) {
  if (nreq == 0) return hipSuccess;
  if ((uint64_t)nreq > (uint64_t)P.nq * 2 * P.k) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_fri_paths, dim3(nreq), dim3(64), 0, st, d_layers, d_req, d_count, P);
  return hipGetLastError();
}

}  // namespace sezkp

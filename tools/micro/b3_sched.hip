// Microbenchmark: BLAKE3 parent-compression throughput on gfx950 under
// different instruction schedules. The default is the compiler's schedule
// (dev_common.h b3_parent). The "grouped" variants put empty asm barriers on
// the state words between the twelve steps of a half-round, so the four G
// functions of a half-round issue step by step (4 add3, 4 xor, 4 alignbit,
// ...): runs of same-rate instructions instead of the compiler's interleave.
// "2add" splits each add3 into two full-rate adds; "x2" runs two independent
// compressions per lane through the same barriers (runs of 8).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../streaming-zero-knowledge-proofs_amd/csrc/dev_common.h"
using namespace sezkp;

#define FENCE16(s)                                                                                          \
  asm volatile("" : "+v"(s[0]), "+v"(s[1]), "+v"(s[2]), "+v"(s[3]), "+v"(s[4]), "+v"(s[5]), "+v"(s[6]),   \
               "+v"(s[7]), "+v"(s[8]), "+v"(s[9]), "+v"(s[10]), "+v"(s[11]), "+v"(s[12]), "+v"(s[13]),     \
               "+v"(s[14]), "+v"(s[15]))

__device__ __forceinline__ uint32_t rot(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }

// one half-round over NS independent states: columns (diag = false) or
// diagonals, message words mx[g], my[g] for G g
template <int NS, bool ADD3>
__device__ __forceinline__ void half_round(uint32_t (&v)[NS][16], const uint32_t (&m)[NS][16], const int (&ix)[8],
                                           bool diag) {
  int A[4], B[4], C[4], D[4];
  for (int g = 0; g < 4; g++) {
    A[g] = g;
    B[g] = 4 + (diag ? (g + 1) & 3 : g);
    C[g] = 8 + (diag ? (g + 2) & 3 : g);
    D[g] = 12 + (diag ? (g + 3) & 3 : g);
  }
#define STEP(EXPR)                                 \
  _Pragma("unroll") for (int s = 0; s < NS; s++) { \
    _Pragma("unroll") for (int g = 0; g < 4; g++) { EXPR; }  \
  }                                                \
  _Pragma("unroll") for (int s = 0; s < NS; s++) FENCE16(v[s]);
  if (ADD3) {
    STEP(v[s][A[g]] = v[s][A[g]] + v[s][B[g]] + m[s][ix[2 * g]])
  } else {
    STEP(v[s][A[g]] = v[s][A[g]] + v[s][B[g]])
    STEP(v[s][A[g]] = v[s][A[g]] + m[s][ix[2 * g]])
  }
  STEP(v[s][D[g]] = v[s][D[g]] ^ v[s][A[g]])
  STEP(v[s][D[g]] = rot(v[s][D[g]], 16))
  STEP(v[s][C[g]] = v[s][C[g]] + v[s][D[g]])
  STEP(v[s][B[g]] = v[s][B[g]] ^ v[s][C[g]])
  STEP(v[s][B[g]] = rot(v[s][B[g]], 12))
  if (ADD3) {
    STEP(v[s][A[g]] = v[s][A[g]] + v[s][B[g]] + m[s][ix[2 * g + 1]])
  } else {
    STEP(v[s][A[g]] = v[s][A[g]] + v[s][B[g]])
    STEP(v[s][A[g]] = v[s][A[g]] + m[s][ix[2 * g + 1]])
  }
  STEP(v[s][D[g]] = v[s][D[g]] ^ v[s][A[g]])
  STEP(v[s][D[g]] = rot(v[s][D[g]], 8))
  STEP(v[s][C[g]] = v[s][C[g]] + v[s][D[g]])
  STEP(v[s][B[g]] = v[s][B[g]] ^ v[s][C[g]])
  STEP(v[s][B[g]] = rot(v[s][B[g]], 7))
#undef STEP
}

__device__ constexpr int SIGMA[7][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
    {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1}, {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
    {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4}, {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
    {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13}};

template <int NS, bool ADD3>
__device__ __forceinline__ void parent_grouped(uint32_t (&l)[NS][8], const uint32_t (&r)[NS][8], uint32_t (&o)[NS][8]) {
  uint32_t m[NS][16], v[NS][16];
#pragma unroll
  for (int s = 0; s < NS; s++) {
#pragma unroll
    for (int w = 0; w < 8; w++) { m[s][w] = l[s][w]; m[s][8 + w] = r[s][w]; }
    v[s][0] = B3_IV0; v[s][1] = B3_IV1; v[s][2] = B3_IV2; v[s][3] = B3_IV3;
    v[s][4] = B3_IV4; v[s][5] = B3_IV5; v[s][6] = B3_IV6; v[s][7] = B3_IV7;
    v[s][8] = B3_IV0; v[s][9] = B3_IV1; v[s][10] = B3_IV2; v[s][11] = B3_IV3;
    v[s][12] = 0; v[s][13] = 0; v[s][14] = 64; v[s][15] = B3_ROOT_FLAGS;
  }
#pragma unroll
  for (int r = 0; r < 7; r++) {
    const int c[8] = {SIGMA[r][0], SIGMA[r][1], SIGMA[r][2], SIGMA[r][3], SIGMA[r][4], SIGMA[r][5], SIGMA[r][6], SIGMA[r][7]};
    const int d[8] = {SIGMA[r][8], SIGMA[r][9], SIGMA[r][10], SIGMA[r][11], SIGMA[r][12], SIGMA[r][13], SIGMA[r][14], SIGMA[r][15]};
    half_round<NS, ADD3>(v, m, c, false);
    half_round<NS, ADD3>(v, m, d, true);
  }
#pragma unroll
  for (int s = 0; s < NS; s++)
#pragma unroll
    for (int w = 0; w < 8; w++) o[s][w] = v[s][w] ^ v[s][8 + w];
}

// reference schedule: dev_common.h b3_parent, CH independent chains per lane
template <int CH>
__global__ void __launch_bounds__(256) k_default(uint32_t* out, int iters) {
  uint32_t h[CH][8];
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
#pragma unroll
  for (int c = 0; c < CH; c++)
    for (int w = 0; w < 8; w++) h[c][w] = t * 8 + w + c * 77;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < CH; c++) {
      uint32_t o[8];
      b3_parent(h[c], h[(c + 1) % CH], o);
#pragma unroll
      for (int w = 0; w < 8; w++) h[c][w] = o[w];
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int c = 0; c < CH; c++)
    for (int w = 0; w < 8; w++) x ^= h[c][w];
  out[t] = x;
}

template <int NS, bool ADD3>
__global__ void __launch_bounds__(256) k_grouped(uint32_t* out, int iters) {
  uint32_t h[NS][8], g[NS][8];
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
#pragma unroll
  for (int s = 0; s < NS; s++)
    for (int w = 0; w < 8; w++) { h[s][w] = t * 8 + w + s * 77; g[s][w] = t ^ (w * 0x9E3779B9u) ^ s; }
  for (int it = 0; it < iters; it++) {
    uint32_t o[NS][8];
    parent_grouped<NS, ADD3>(h, g, o);
#pragma unroll
    for (int s = 0; s < NS; s++)
#pragma unroll
      for (int w = 0; w < 8; w++) { g[s][w] = h[s][w]; h[s][w] = o[s][w]; }
  }
  uint32_t x = 0;
#pragma unroll
  for (int s = 0; s < NS; s++)
    for (int w = 0; w < 8; w++) x ^= h[s][w];
  out[t] = x;
}

// correctness: the grouped schedule must give b3_parent's bytes
__global__ void k_check(uint32_t* bad) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  uint32_t l[2][8], r[2][8], o[2][8], want[8], nbad = 0;
  for (int s = 0; s < 2; s++)
    for (int w = 0; w < 8; w++) { l[s][w] = t * 31 + w * 7 + s; r[s][w] = t ^ (w * 0x9E3779B9u) ^ (s << 20); }
  parent_grouped<2, true>(l, r, o);
  for (int s = 0; s < 2; s++) {
    b3_parent(l[s], r[s], want);
    for (int w = 0; w < 8; w++)
      nbad += want[w] != o[s][w];
  }
  parent_grouped<2, false>(l, r, o);
  for (int s = 0; s < 2; s++) {
    b3_parent(l[s], r[s], want);
    for (int w = 0; w < 8; w++)
      nbad += want[w] != o[s][w];
  }
  bad[t] = nbad;
}

template <class F>
double timeit(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; i++) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  uint32_t* out;
  uint32_t* bad;
  (void)hipMalloc(&out, 4 << 24);
  (void)hipMalloc(&bad, 4 * 64 * 256);
  hipLaunchKernelGGL(k_check, dim3(64), dim3(256), 0, 0, bad);
  static uint32_t hb[64 * 256];
  (void)hipMemcpy(hb, bad, sizeof hb, hipMemcpyDeviceToHost);
  uint32_t nb = 0;
  for (uint32_t x : hb) nb += x;
  printf("grouped schedule vs b3_parent: %u mismatching words\n", nb);
  const int iters = 128;
  for (int wps : {4, 8}) {
    const int blocks = 256 * wps;  // 4 waves per WG, one per SIMD
    auto run = [&](const char* name, void (*k)(uint32_t*, int), int per_lane) {
      const double ms = timeit([&] { hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters); }, 5);
      printf("waves/SIMD %d  %-22s %.2f G comp/s\n", wps, name, (double)blocks * 256 * iters * per_lane / ms / 1e6);
    };
    run("default x1", k_default<1>, 1);
    run("default x2", k_default<2>, 2);
    run("default x4", k_default<4>, 4);
    run("grouped add3 x1", k_grouped<1, true>, 1);
    run("grouped 2add x1", k_grouped<1, false>, 1);
    run("grouped add3 x2", k_grouped<2, true>, 2);
    run("grouped 2add x2", k_grouped<2, false>, 2);
  }
  return 0;
}

// Goldilocks butterfly chains in the LATENCY regime (1-2 waves per SIMD, a few
// independent chains per lane, as in a 2^20-point NTT pass: 4096 points per
// CU) and in the throughput regime (8 waves per SIMD), for gl_add variants:
//   cur   dev_common.h: s = a + b, t = s + eps, (c1 | c2) ? t : s  (the mask OR is SALU)
//   sub   a - (p - b): p - b in two VALU ops, then gl_sub's borrow select (no SALU)
//   sel2  two selects in turn, c2 ? t : s then c1 ? t : r  (no SALU)
// Also checks the variants bit-identical to gl_add on random canonical inputs.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/gl_latency.hip -o tools/micro/gl_latency
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../streaming-zero-knowledge-proofs_amd/csrc/dev_common.h"
using namespace sezkp;

__device__ __forceinline__ uint64_t add_sub_form(uint64_t a, uint64_t b) {
  // q = p - b (b < p: no wrap): lo = 1 - b_lo, hi = 0xffffffff - b_hi - borrow
  uint32_t br0, br1;
  const uint32_t qlo = __builtin_subc(1u, (uint32_t)b, 0u, &br0);
  const uint32_t qhi = __builtin_subc(0xffffffffu, (uint32_t)(b >> 32), br0, &br1);
  const uint64_t q = ((uint64_t)qhi << 32) | qlo;
  return gl_sub(a, q);
}
__device__ __forceinline__ uint64_t add_sel2(uint64_t a, uint64_t b) {
  uint32_t c1, c2;
  const uint64_t s = add64c(a, b, c1);
  const uint64_t t = add64c(s, GL_EPS, c2);
  const uint64_t r = c2 ? t : s;
  return c1 ? t : r;
}

template <int V>
__device__ __forceinline__ uint64_t addv(uint64_t a, uint64_t b) {
  if constexpr (V == 0) return gl_add(a, b);
  else if constexpr (V == 1) return add_sub_form(a, b);
  else return add_sel2(a, b);
}

// CH independent butterfly chains per lane, ITER rounds
template <int V, int CH>
__global__ void k_chain(uint64_t* io, int iters) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t x[CH], y[CH];
#pragma unroll
  for (int c = 0; c < CH; c++) {
    x[c] = io[(i * CH + c) * 2] % GL_P;
    y[c] = io[(i * CH + c) * 2 + 1] % GL_P;
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < CH; c++) {
      const uint64_t a = addv<V>(x[c], y[c]);
      const uint64_t b = gl_sub(x[c], y[c]);
      x[c] = a;
      y[c] = b;
    }
  }
#pragma unroll
  for (int c = 0; c < CH; c++) {
    io[(i * CH + c) * 2] = x[c];
    io[(i * CH + c) * 2 + 1] = y[c];
  }
}

template <int V>
__global__ void k_check(const uint64_t* in, uint32_t* bad, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t a = in[2 * i] % GL_P, b = in[2 * i + 1] % GL_P;
  if (addv<V>(a, b) != gl_add(a, b)) atomicAdd(bad, 1u);
}

static uint64_t rng = 0x243F6A8885A308D3ull;
static uint64_t next() {
  rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
  return rng;
}

template <int V, int CH>
static void run(const char* name, uint64_t* d, int waves_per_simd, int iters) {
  const int threads = 256;                       // 4 waves: one per SIMD
  const int blocks = 256 * waves_per_simd;       // 256 CUs
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  k_chain<V, CH><<<blocks, threads>>>(d, iters);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; r++) k_chain<V, CH><<<blocks, threads>>>(d, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double bfly = 5.0 * blocks * threads * (double)CH * iters;
  printf("%-5s waves/SIMD %d chains %d   %7.3f ms   %6.2f G butterflies/s\n", name, waves_per_simd, CH, ms / 5,
         bfly / (ms * 1e-3) / 1e9);
}

int main() {
  const size_t words = 256ull * 8 * 256 * 8 * 2;
  uint64_t* h = (uint64_t*)malloc(words * 8);
  for (size_t i = 0; i < words; i++) h[i] = next();
  for (size_t i = 0; i < 64; i++) h[i] = (i & 1) ? GL_P - 1 - (i >> 1) : (i >> 1);  // edge values
  uint64_t* d;
  uint32_t* bad;
  (void)hipMalloc(&d, words * 8);
  (void)hipMalloc(&bad, 4);
  (void)hipMemcpy(d, h, words * 8, hipMemcpyHostToDevice);
  const int n = 1 << 22;
  for (int v = 1; v <= 2; v++) {
    (void)hipMemset(bad, 0, 4);
    if (v == 1) k_check<1><<<n / 256, 256>>>(d, bad, n);
    else k_check<2><<<n / 256, 256>>>(d, bad, n);
    uint32_t b;
    (void)hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost);
    printf("variant %d vs gl_add: %u mismatches over %d pairs\n", v, b, n);
  }
  const int iters = 4096;
  for (int w : {1, 2, 8}) {
    run<0, 4>("cur", d, w, iters);
    run<1, 4>("sub", d, w, iters);
    run<2, 4>("sel2", d, w, iters);
    run<0, 8>("cur", d, w, iters);
    run<1, 8>("sub", d, w, iters);
    run<2, 8>("sel2", d, w, iters);
  }
  (void)hipFree(d);
  (void)hipFree(bad);
  free(h);
  return 0;
}

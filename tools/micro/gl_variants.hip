// Throughput + correctness microbenchmark of Goldilocks primitive variants on
// gfx950 (dev_common.h's canonical ops vs carry-chain / weakly reduced forms).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/gl_variants.hip -o tools/micro/gl_variants
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../streaming-zero-knowledge-proofs_amd/csrc/dev_common.h"
using namespace sezkp;

// 64-bit add/sub through 32-bit carry chains (v_add_co/v_addc, no 64-bit compares)
__device__ __forceinline__ uint64_t add64c(uint64_t a, uint64_t b, uint32_t& c) {
  uint32_t c0, c1;
  uint32_t lo = __builtin_addc((uint32_t)a, (uint32_t)b, 0u, &c0);
  uint32_t hi = __builtin_addc((uint32_t)(a >> 32), (uint32_t)(b >> 32), c0, &c1);
  c = c1;
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t sub64b(uint64_t a, uint64_t b, uint32_t& br) {
  uint32_t b0, b1;
  uint32_t lo = __builtin_subc((uint32_t)a, (uint32_t)b, 0u, &b0);
  uint32_t hi = __builtin_subc((uint32_t)(a >> 32), (uint32_t)(b >> 32), b0, &b1);
  br = b1;
  return ((uint64_t)hi << 32) | lo;
}
// canonical add: s = a+b; t = s+eps; result = (c1|c2) ? t : s
__device__ __forceinline__ uint64_t gl_add_v2(uint64_t a, uint64_t b) {
  uint32_t c1, c2;
  uint64_t s = add64c(a, b, c1);
  uint64_t t = add64c(s, GL_EPS, c2);
  return (c1 | c2) ? t : s;
}
__device__ __forceinline__ uint64_t gl_sub_v2(uint64_t a, uint64_t b) {
  uint32_t br;
  uint64_t d = sub64b(a, b, br);
  return br ? d - GL_EPS : d;
}
// 128-bit product with 4 v_mad_u64_u32
__device__ __forceinline__ void mul128(uint64_t a, uint64_t b, uint64_t& lo, uint64_t& hi) {
  const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
  const uint64_t p00 = (uint64_t)a0 * b0;
  const uint64_t t = (uint64_t)a0 * b1 + (p00 >> 32);
  const uint64_t u = (uint64_t)a1 * b0 + (uint32_t)t;
  hi = (uint64_t)a1 * b1 + ((t >> 32) + (u >> 32));
  lo = ((uint64_t)(uint32_t)u << 32) | (uint32_t)p00;
}
// weak reduction: x = lo + 2^64 hi -> r in [0, 2^64), r = x mod p (not canonical)
__device__ __forceinline__ uint64_t reduce_weak(uint64_t lo, uint64_t hi) {
  const uint32_t h0 = (uint32_t)hi, h1 = (uint32_t)(hi >> 32);
  uint32_t br;
  uint64_t t0 = sub64b(lo, h1, br);
  if (br) t0 -= GL_EPS;
  const uint64_t t1 = ((uint64_t)h0 << 32) - h0;
  uint32_t c;
  uint64_t r = add64c(t0, t1, c);
  return c ? r + GL_EPS : r;
}
__device__ __forceinline__ uint64_t canon(uint64_t r) {
  uint32_t c;
  uint64_t t = add64c(r, GL_EPS, c);
  return c ? t : r;
}
__device__ __forceinline__ uint64_t gl_mul_v2(uint64_t a, uint64_t b) {
  uint64_t lo, hi;
  mul128(a, b, lo, hi);
  return canon(reduce_weak(lo, hi));
}
__device__ __forceinline__ uint64_t gl_mul_weak(uint64_t a, uint64_t b) {
  uint64_t lo, hi;
  mul128(a, b, lo, hi);
  return reduce_weak(lo, hi);
}

template <int OP>
__global__ void __launch_bounds__(256) k(uint64_t* out, uint64_t seed, int iters) {
  uint64_t x0 = (seed ^ (threadIdx.x * 0x9E3779B97F4A7C15ULL)) % GL_P, x1 = gl_add(x0, 12345), x2 = gl_add(x0, 777), x3 = gl_add(x1, 99);
  const uint64_t c = (0x123456789abcdefULL * (blockIdx.x + 1)) % GL_P;
  for (int i = 0; i < iters; i++) {
    if constexpr (OP == 0) { x0 = gl_mul(x0, c); x1 = gl_mul(x1, c); x2 = gl_mul(x2, c); x3 = gl_mul(x3, c); }
    if constexpr (OP == 1) { x0 = gl_mul_v2(x0, c); x1 = gl_mul_v2(x1, c); x2 = gl_mul_v2(x2, c); x3 = gl_mul_v2(x3, c); }
    if constexpr (OP == 2) { x0 = gl_mul_weak(x0, c); x1 = gl_mul_weak(x1, c); x2 = gl_mul_weak(x2, c); x3 = gl_mul_weak(x3, c); }
    if constexpr (OP == 3) { x0 = gl_add(x0, x1); x1 = gl_add(x1, x2); x2 = gl_add(x2, x3); x3 = gl_add(x3, c); }
    if constexpr (OP == 4) { x0 = gl_add_v2(x0, x1); x1 = gl_add_v2(x1, x2); x2 = gl_add_v2(x2, x3); x3 = gl_add_v2(x3, c); }
    if constexpr (OP == 5) { x0 = gl_sub(x0, x1); x1 = gl_sub(x1, x2); x2 = gl_sub(x2, x3); x3 = gl_sub(x3, c); }
    if constexpr (OP == 6) { x0 = gl_sub_v2(x0, x1); x1 = gl_sub_v2(x1, x2); x2 = gl_sub_v2(x2, x3); x3 = gl_sub_v2(x3, c); }
  }
  if constexpr (OP == 2) { x0 = canon(x0); x1 = canon(x1); x2 = canon(x2); x3 = canon(x3); }
  out[blockIdx.x * 256 + threadIdx.x] = x0 ^ (x1 * 3) ^ (x2 * 5) ^ (x3 * 7);
}

template <int OP>
double run(uint64_t* d, int blocks, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  k<OP><<<blocks, 256>>>(d, 1, iters);
  hipEventRecord(a);
  k<OP><<<blocks, 256>>>(d, 1, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return (double)blocks * 256 * iters * 4 / (ms * 1e-3);
}
static bool same(uint64_t* d, uint64_t* h1, uint64_t* h2, size_t n) {
  hipMemcpy(h2, d, n * 8, hipMemcpyDeviceToHost);
  for (size_t i = 0; i < n; i++) if (h1[i] != h2[i]) return false;
  return true;
}

int main() {
  const int blocks = 256 * 8 * 4, iters = 1024;
  const size_t n = (size_t)blocks * 256;
  uint64_t* d; hipMalloc(&d, n * 8);
  uint64_t* h1 = (uint64_t*)malloc(n * 8);
  uint64_t* h2 = (uint64_t*)malloc(n * 8);
  double r;
  r = run<0>(d, blocks, iters); hipMemcpy(h1, d, n * 8, hipMemcpyDeviceToHost);
  printf("gl_mul        %.1f G/s\n", r / 1e9);
  r = run<1>(d, blocks, iters); printf("gl_mul_v2     %.1f G/s  same=%d\n", r / 1e9, same(d, h1, h2, n));
  r = run<2>(d, blocks, iters); printf("gl_mul_weak   %.1f G/s  same=%d\n", r / 1e9, same(d, h1, h2, n));
  r = run<3>(d, blocks, iters); hipMemcpy(h1, d, n * 8, hipMemcpyDeviceToHost);
  printf("gl_add        %.1f G/s\n", r / 1e9);
  r = run<4>(d, blocks, iters); printf("gl_add_v2     %.1f G/s  same=%d\n", r / 1e9, same(d, h1, h2, n));
  r = run<5>(d, blocks, iters); hipMemcpy(h1, d, n * 8, hipMemcpyDeviceToHost);
  printf("gl_sub        %.1f G/s\n", r / 1e9);
  r = run<6>(d, blocks, iters); printf("gl_sub_v2     %.1f G/s  same=%d\n", r / 1e9, same(d, h1, h2, n));
  return 0;
}

// Throughput microbenchmark: Goldilocks mul / add and v_mad_u64_u32 on gfx950.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/glmul_bench.hip -o tools/micro/glmul_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../streaming-zero-knowledge-proofs_amd/csrc/dev_common.h"
using namespace sezkp;

template <int OP>
__global__ void __launch_bounds__(256) k(uint64_t* out, uint64_t seed, int iters) {
  uint64_t x0 = seed ^ threadIdx.x, x1 = x0 * 3 + 1, x2 = x0 * 5 + 7, x3 = x0 * 11 + 13;
  const uint64_t c = 0x123456789abcdefULL + blockIdx.x;
  for (int i = 0; i < iters; i++) {
    if constexpr (OP == 0) { x0 = gl_mul(x0, c); x1 = gl_mul(x1, c); x2 = gl_mul(x2, c); x3 = gl_mul(x3, c); }
    if constexpr (OP == 1) { x0 = gl_add(x0, c); x1 = gl_add(x1, c); x2 = gl_add(x2, c); x3 = gl_add(x3, c); }
    if constexpr (OP == 2) {
      x0 = (uint64_t)(uint32_t)x0 * (uint32_t)c + (x0 >> 32); x1 = (uint64_t)(uint32_t)x1 * (uint32_t)c + (x1 >> 32);
      x2 = (uint64_t)(uint32_t)x2 * (uint32_t)c + (x2 >> 32); x3 = (uint64_t)(uint32_t)x3 * (uint32_t)c + (x3 >> 32);
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3;
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

int main() {
  const int blocks = 256 * 8 * 4, iters = 2048;
  uint64_t* d; hipMalloc(&d, (size_t)blocks * 256 * 8);
  printf("gl_mul  %.1f G/s\n", run<0>(d, blocks, iters) / 1e9);
  printf("gl_add  %.1f G/s\n", run<1>(d, blocks, iters) / 1e9);
  printf("mad_u64_u32 %.1f G/s\n", run<2>(d, blocks, iters) / 1e9);
  return 0;
}

// Microbenchmark: BLAKE3 single-block compression throughput ceiling on gfx950.
// Each lane runs a dependent chain of parent compressions (no HBM traffic),
// several independent chains per lane to expose ILP. Prints G compressions/s.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../streaming-zero-knowledge-proofs_amd/csrc/dev_common.h"
using namespace sezkp;

template <int CHAINS>
__global__ void __launch_bounds__(256) k_chain(uint32_t* out, int iters) {
  uint32_t h[CHAINS][8];
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
#pragma unroll
  for (int c = 0; c < CHAINS; c++)
    for (int w = 0; w < 8; w++) h[c][w] = t * 8 + w + c * 77;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) {
      uint32_t o[8];
      b3_parent(h[c], h[(c + 1) % CHAINS], o);
#pragma unroll
      for (int w = 0; w < 8; w++) h[c][w] = o[w];
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; c++)
    for (int w = 0; w < 8; w++) x ^= h[c][w];
  out[t] = x;
}
// 8-byte leaf hashing throughput (constant-folded message)
__global__ void __launch_bounds__(256) k_leaf(uint32_t* out, int iters) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  uint64_t v = t;
  uint32_t acc = 0;
  for (int it = 0; it < iters; it++) {
    uint32_t o[8];
    b3_leaf_u64(v, o);
    v = ((uint64_t)o[1] << 32) | o[0];
    acc ^= o[2];
  }
  out[t] = acc;
}

template <class F>
double timeit(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < reps; i++) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  uint32_t* out; hipMalloc(&out, 4 << 24);
  const int iters = 256;
  for (int blocks : {1024, 4096, 16384}) {
    double ms = timeit([&] { hipLaunchKernelGGL(k_chain<1>, dim3(blocks), dim3(256), 0, 0, out, iters); }, 5);
    printf("chain1 blocks=%d: %.2f G comp/s\n", blocks, blocks * 256.0 * iters / ms / 1e6);
    ms = timeit([&] { hipLaunchKernelGGL(k_chain<2>, dim3(blocks), dim3(256), 0, 0, out, iters); }, 5);
    printf("chain2 blocks=%d: %.2f G comp/s\n", blocks, blocks * 256.0 * iters * 2 / ms / 1e6);
    ms = timeit([&] { hipLaunchKernelGGL(k_chain<4>, dim3(blocks), dim3(256), 0, 0, out, iters); }, 5);
    printf("chain4 blocks=%d: %.2f G comp/s\n", blocks, blocks * 256.0 * iters * 4 / ms / 1e6);
    ms = timeit([&] { hipLaunchKernelGGL(k_leaf, dim3(blocks), dim3(256), 0, 0, out, iters); }, 5);
    printf("leaf8  blocks=%d: %.2f G comp/s\n", blocks, blocks * 256.0 * iters / ms / 1e6);
  }
  return 0;
}

// Microbenchmark: HBM efficiency of the NTT pass tile shapes on gfx950.
// A pass tile is R rows x C consecutive u64 columns of an N-element array
// viewed as [N/S][S] (row stride S elements). Each WG loads its tile into
// LDS, syncs, and stores it back (out of place), i.e. exactly the memory
// pattern of an LDS-staged NTT pass without the arithmetic. Reports
// effective GB/s (16 B per element) for
//   - the 3-pass shape  R=256,  C=16 (128-B segments)
//   - the 2-pass shapes R=4096, C=1 contiguous, and C=1/2/4/8 strided
// with natural and XCD-grouped WG->column-group maps (WGs sharing a 128-B
// line placed on one XCD, dispatched together: block b runs on XCD b % 8).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int R, int C, int THREADS, bool XCD>
__global__ void __launch_bounds__(THREADS) k_tile(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst,
                                                  uint64_t S, uint64_t ngroups) {
  extern __shared__ uint64_t sh[];
  uint64_t b = blockIdx.x;
  // column groups: S/C per row-block of R rows; tiles = (N/S/R) * (S/C)
  uint64_t g = b;
  if (XCD) {
    // lines hold 16/C groups; put the 16/C groups of one line on one XCD at
    // consecutive dispatch slots: b = 8*j + x -> XCD x, slot j
    constexpr int G = (16 / C) > 0 ? 16 / C : 1;
    const uint64_t x = b % 8, j = b / 8;
    // slot j of XCD x: line-set = (j / G) * 8 + x, member = j % G
    g = ((j / G) * 8 + x) * G + (j % G);
    if (g >= ngroups) g = b;  // tail (not hit for the sizes below)
  }
  const uint64_t gpr = S / C;  // groups per row block
  const uint64_t rb = g / gpr, cg = g % gpr;
  const uint64_t base = rb * R * S + cg * C;
  constexpr int NEL = R * C;
  for (int q = threadIdx.x; q < NEL; q += THREADS) {
    const int r = q / C, c = q % C;
    sh[q] = src[base + (uint64_t)r * S + c];
  }
  __syncthreads();
  for (int q = threadIdx.x; q < NEL; q += THREADS) {
    const int r = q / C, c = q % C;
    dst[base + (uint64_t)r * S + c] = sh[NEL - 1 - q] ^ 1;
  }
}

template <int R, int C, int THREADS, bool XCD>
static void run(const char* name, uint64_t* a, uint64_t* b, uint64_t N, uint64_t S) {
  const uint64_t ngroups = N / C / R;
  const size_t lds = (size_t)R * C * 8;
  auto k = k_tile<R, C, THREADS, XCD>;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  for (int i = 0; i < 3; i++) hipLaunchKernelGGL(k, dim3((unsigned)ngroups), dim3(THREADS), lds, 0, a, b, S, ngroups);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = 10;
  hipEventRecord(e0);
  for (int i = 0; i < reps; i++)
    hipLaunchKernelGGL(k, dim3((unsigned)ngroups), dim3(THREADS), lds, 0, (i & 1) ? b : a, (i & 1) ? a : b, S,
                       ngroups);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double per = ms / reps;
  printf("%-44s N=2^%d S=%6llu  %8.1f us  %7.0f GB/s  (%.2f of 8 TB/s)\n", name, 63 - __builtin_clzll(N),
         (unsigned long long)S, per * 1e3, 16.0 * N / (per * 1e-3) / 1e9, 16.0 * N / (per * 1e-3) / 8e12);
}

int main() {
  for (int lg : {24, 26}) {
    const uint64_t N = 1ULL << lg;
    uint64_t *a, *b;
    hipMalloc(&a, N * 8);
    hipMalloc(&b, N * 8);
    hipMemset(a, 1, N * 8);
    hipMemset(b, 2, N * 8);
    const uint64_t S12 = N >> 12;  // 2-pass: stride-S tiles of 4096 rows
    run<256, 16, 256, false>("3-pass R=256 C=16 stride 2^16", a, b, N, 1ULL << 16);
    run<256, 16, 256, false>("3-pass R=256 C=16 stride 2^8", a, b, N, 1ULL << 8);
    run<4096, 1, 512, false>("contig R=4096 (S=1 row)", a, b, N, 1);
    run<4096, 1, 1024, false>("strided R=4096 C=1", a, b, N, S12);
    run<4096, 1, 1024, true>("strided R=4096 C=1 xcd", a, b, N, S12);
    run<4096, 2, 1024, false>("strided R=4096 C=2", a, b, N, S12);
    run<4096, 2, 1024, true>("strided R=4096 C=2 xcd", a, b, N, S12);
    run<4096, 4, 1024, false>("strided R=4096 C=4", a, b, N, S12);
    run<4096, 4, 1024, true>("strided R=4096 C=4 xcd", a, b, N, S12);
    run<2048, 8, 1024, false>("strided R=2048 C=8", a, b, N, N >> 11);
    run<2048, 8, 1024, true>("strided R=2048 C=8 xcd", a, b, N, N >> 11);
    if (lg == 26) {
      const uint64_t S13 = N >> 13;
      run<8192, 1, 1024, false>("contig R=8192", a, b, N, 1);
      run<8192, 2, 1024, false>("strided R=8192 C=2", a, b, N, S13);
      run<8192, 2, 1024, true>("strided R=8192 C=2 xcd", a, b, N, S13);
    }
    hipFree(a);
    hipFree(b);
  }
  return 0;
}

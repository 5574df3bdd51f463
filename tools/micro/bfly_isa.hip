// ISA experiment: instruction cost of a 16-point register FFT (4 radix-2
// DIT stages, shift twiddles) under different Goldilocks formulations.
// Compile with --cuda-device-only -S and run tools/isa_hist.py on each kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../streaming-zero-knowledge-proofs_amd/csrc/dev_common.h"

using namespace sezkp;

// ---------------------------------------------------------------- variant A: current (canonical)
namespace va {
__device__ __forceinline__ uint64_t mul_eps32(uint32_t h) { return ((uint64_t)h << 32) - h; }
__device__ __forceinline__ uint64_t mul2e(uint64_t x, int e) {  // e < 32 only (test)
  if (e == 0) return x;
  const uint64_t A = x << e;
  const uint32_t y2 = (uint32_t)(x >> (64 - e));
  return gl_add(A, mul_eps32(y2));
}
}  // namespace va

// ---------------------------------------------------------------- variant B: weak, mad folds
namespace vb {
// x + c*eps for c in {0,1} given as a 32-bit value
__device__ __forceinline__ uint64_t mad32(uint32_t a, uint32_t b, uint64_t c) {
  return (uint64_t)a * b + c;  // v_mad_u64_u32
}
// weak a + b, with b canonical-ish (single fold)
__device__ __forceinline__ uint64_t add(uint64_t a, uint64_t b) {
  uint32_t c;
  const uint64_t s = add64c(a, b, c);
  return mad32(c, 0xffffffffu, s);
}
__device__ __forceinline__ uint64_t sub(uint64_t a, uint64_t b) {
  uint32_t br;
  const uint64_t d = sub64b(a, b, br);
  // d - br*eps = d + br*p (mod 2^64)
  return d + ((uint64_t)(0u - br) << 32) + br;
}
__device__ __forceinline__ uint64_t mul2e(uint64_t x, int e) {  // e < 32
  if (e == 0) return x;
  const uint64_t A = x << e;
  const uint32_t T = (uint32_t)(x >> (64 - e));
  // A + T*eps: carry -> + eps
  const uint64_t t = mad32(T, 0xffffffffu, A);
  const uint32_t c = t < A;  // carry
  return mad32(c, 0xffffffffu, t);
}
}  // namespace vb

template <class ADD, class SUB, class MUL2E>
__device__ __forceinline__ void fft16(uint64_t (&x)[16], ADD add, SUB sub, MUL2E m2e) {
#pragma unroll
  for (int s = 0; s < 4; s++) {
    const int h = 1 << s;
#pragma unroll
    for (int t0 = 0; t0 < 16; t0++) {
      if (!(t0 & h)) {
        const int j = t0 & (h - 1);
        const int e = j * (24 >> s) % 32;  // stand-in shift amounts < 32
        const uint64_t y = e ? m2e(x[t0 + h], e) : x[t0 + h];
        const uint64_t a = x[t0];
        x[t0] = add(a, y);
        x[t0 + h] = sub(a, y);
      }
    }
  }
}

__global__ void k_va(uint64_t* d) {
  uint64_t x[16];
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
#pragma unroll
  for (int r = 0; r < 16; r++) x[r] = d[i * 16 + r];
  fft16(x, [](uint64_t a, uint64_t b) { return gl_add(a, b); }, [](uint64_t a, uint64_t b) { return gl_sub(a, b); },
        [](uint64_t a, int e) { return va::mul2e(a, e); });
#pragma unroll
  for (int r = 0; r < 16; r++) d[i * 16 + r] = x[r];
}

__global__ void k_vb(uint64_t* d) {
  uint64_t x[16];
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
#pragma unroll
  for (int r = 0; r < 16; r++) x[r] = d[i * 16 + r];
  fft16(x, [](uint64_t a, uint64_t b) { return vb::add(a, b); }, [](uint64_t a, uint64_t b) { return vb::sub(a, b); },
        [](uint64_t a, int e) { return vb::mul2e(a, e); });
#pragma unroll
  for (int r = 0; r < 16; r++) d[i * 16 + r] = x[r];
}

// ---------------------------------------------------------------- variant C: 64-bit add + compare carries
namespace vc {
__device__ __forceinline__ uint64_t mad32(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }
// weak x + t, t <= p (single fold)
__device__ __forceinline__ uint64_t add(uint64_t x, uint64_t t) {
  const uint64_t s = x + t;
  return mad32((uint32_t)(s < t), 0xffffffffu, s);
}
// weak x - t, t <= p: x + (p - t)
__device__ __forceinline__ uint64_t sub(uint64_t x, uint64_t t) {
  const uint64_t nt = ~t + (GL_P + 1);  // p - t (t <= p)
  const uint64_t s = x + nt;
  return mad32((uint32_t)(s < nt), 0xffffffffu, s);
}
// y * 2^e (e < 32), result <= p? (weak; canonicalised below)
__device__ __forceinline__ uint64_t mul2e(uint64_t y, int e) {
  if (e == 0) return y;
  const uint64_t A = y << e;
  const uint32_t T = (uint32_t)(y >> (64 - e));
  const uint64_t t = mad32(T, 0xffffffffu, A);
  const uint64_t r = mad32((uint32_t)(t < A), 0xffffffffu, t);
  // canonical: r >= p -> r - p = r + eps
  const uint64_t r2 = r + 0xffffffffull;
  return r2 < r ? r2 : r;
}
}  // namespace vc

__global__ void k_vc(uint64_t* d) {
  uint64_t x[16];
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
#pragma unroll
  for (int r = 0; r < 16; r++) x[r] = d[i * 16 + r];
  fft16(x, [](uint64_t a, uint64_t b) { return vc::add(a, b); }, [](uint64_t a, uint64_t b) { return vc::sub(a, b); },
        [](uint64_t a, int e) { return vc::mul2e(a, e); });
#pragma unroll
  for (int r = 0; r < 16; r++) d[i * 16 + r] = x[r];
}

// Microbenchmark: does mixing full-rate (v_xor/v_add) and half-rate
// (v_alignbit/v_add3) VALU instructions cost more than the sum of their issue
// times on gfx950, and does grouping same-class instructions help? Each lane
// runs NCH independent chains; the body is written in inline asm so the
// compiler cannot reorder it. Reports wave64 instructions/s chip-wide and
// cycles per instruction per SIMD at 2.4 GHz, for 1..8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define X(r) "v_xor_b32 " r ", " r ", %[b]\n"
#define A(r) "v_alignbit_b32 " r ", " r ", " r ", 16\n"
#define D(r) "v_add_u32 " r ", " r ", %[b]\n"
#define T(r) "v_add3_u32 " r ", " r ", %[b], %[c]\n"
#define R8(M) M("%0") M("%1") M("%2") M("%3") M("%4") M("%5") M("%6") M("%7")
#define R4a(M) M("%0") M("%1") M("%2") M("%3")
#define R4b(M) M("%4") M("%5") M("%6") M("%7")
#define OUTS "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
#define INS [b] "v"(b), [c] "v"(c)

// bodies: 16 instructions each
#define B_XOR R8(X) R8(X)
#define B_ALIGN R8(A) R8(A)
#define B_XA8 R8(X) R8(A)
#define B_XA4 R4a(X) R4b(X) R4a(A) R4b(A)  /* same as XA8, kept for the pattern list */
#define B_XA1 X("%0") A("%1") X("%2") A("%3") X("%4") A("%5") X("%6") A("%7") \
              A("%0") X("%1") A("%2") X("%3") A("%4") X("%5") A("%6") X("%7")
#define B_XA2 X("%0") X("%1") A("%2") A("%3") X("%4") X("%5") A("%6") A("%7") \
              A("%0") A("%1") X("%2") X("%3") A("%4") A("%5") X("%6") X("%7")
#define B_XD R8(X) R8(D)
#define B_AT R8(A) R8(T)
#define B_G  R4a(T) R4a(X) R4a(A) R4a(D) R4b(T) R4b(X) R4b(A) R4b(D)   /* G-like, groups of 4 */
#define B_G2 R4a(D) R4a(D) R4a(X) R4a(A) R4b(D) R4b(D) R4b(X) R4b(A)   /* add3 as two adds: 12 full + 4 half */

#define DEF(NAME, BODY)                                                                        \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, int iters) {                      \
    uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, \
             a6 = a0 * 17, a7 = a0 * 19;                                                       \
    uint32_t b = blockIdx.x | 1, c = blockIdx.x * 7 + 1;                                       \
    for (int i = 0; i < iters; i++) {                                                          \
      asm volatile(BODY BODY BODY BODY : OUTS : INS);                                          \
    }                                                                                          \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;               \
  }
DEF(k_xor, B_XOR)
DEF(k_align, B_ALIGN)
DEF(k_xa8, B_XA8)
DEF(k_xa1, B_XA1)
DEF(k_xa2, B_XA2)
DEF(k_xd, B_XD)
DEF(k_at, B_AT)
DEF(k_g, B_G)
DEF(k_g2, B_G2)

int main() {
  uint32_t* out;
  hipMalloc(&out, 4u << 24);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct K { const char* name; void (*f)(uint32_t*, int); double full, half; };
  K ks[] = {{"16 xor", k_xor, 16, 0},          {"16 align", k_align, 0, 16},
            {"8 xor | 8 align", k_xa8, 8, 8},  {"xor/align alternating", k_xa1, 8, 8},
            {"xor/align pairs", k_xa2, 8, 8},  {"8 xor | 8 add", k_xd, 16, 0},
            {"8 align | 8 add3", k_at, 0, 16}, {"G-like groups of 4 (add3)", k_g, 8, 8},
            {"G-like add3 -> 2 add", k_g2, 12, 4}};
  const int iters = 2000, per = 64;  // 4 bodies x 16 instructions
  for (int wps : {1, 2, 4, 8}) {
    const int blocks = 256 * wps;  // 256 threads = 4 waves, one per SIMD of a CU
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 10);
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double winstr = (double)blocks * 4 * iters * per;  // wave64 instructions
      const double rate = winstr / (ms * 1e-3);
      const double cyc = 1024.0 * 2.4e9 / rate;  // cycles per wave64 instr per SIMD
      const double model = 2.0 * k.full / 16 + 4.0 * k.half / 16;  // 2 / 4 cycles
      printf("waves/SIMD %d  %-28s %.3f T wave-instr/s  %.2f cyc/instr/SIMD  (issue model %.2f)\n", wps, k.name,
             rate / 1e12, cyc, model);
    }
  }
  return 0;
}

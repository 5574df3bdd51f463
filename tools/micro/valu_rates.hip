// Microbenchmark: issue rate of the integer VALU instructions the hot path is
// built from (BLAKE3: xor / add / add3 / alignbit; Goldilocks: mad_u64_u32 …)
// on gfx950. Each lane runs 8 independent chains of one instruction; the grid
// fills every SIMD with 8 waves. Reports cycles per wave64 instruction per
// SIMD, using the shader clock (s_memtime) so DVFS does not enter.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CH8(OP)  OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)

#define DEF_KERNEL(NAME, ASM)                                                         \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint64_t* cyc, int iters) { \
    uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11,     \
             a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;                                  \
    uint32_t b = blockIdx.x | 1, c = blockIdx.x * 7 + 1;                                \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                                        \
    for (int i = 0; i < iters; i++) {                                                   \
      _Pragma("unroll") for (int k = 0; k < 8; k++) { CH8(ASM) }                      \
    }                                                                                   \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                                        \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;        \
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                   \
  }

#define OP_XOR(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define OP_ADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define OP_ADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define OP_ALIGN(x) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(x));
#define OP_PERM(x) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(x) : "v"(c));
#define OP_XOR3(x) asm volatile("v_xor3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define OP_XAD(x) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define OP_LSHLOR(x) asm volatile("v_lshl_or_b32 %0, %0, 16, %1" : "+v"(x) : "v"(b));
#define OP_XORE64(x) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(x) : "v"(b));
#define OP_BITOP3(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "v"(c));
#define OP_MULLO(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define OP_MULHI(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define OP_PKADD16(x) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(b));
#define OP_ADDCO(x) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x) : "v"(b) : "vcc");
#define OP_CND(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(b));

#define OP_SDWAX(x) asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0" : "+v"(x) : "v"(b));
#define OP_SDWAO(x) asm volatile("v_or_b32_sdwa %0, %0, %1 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0" : "+v"(x) : "v"(b));
#define OP_SDWAA(x) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0" : "+v"(x) : "v"(b));
#define OP_OR3(x) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define OP_ANDOR(x) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define OP_LSHLADD(x) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x) : "v"(b));
#define OP_LSHR(x) asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(x));
#define OP_ALIGNBYTE(x) asm volatile("v_alignbyte_b32 %0, %0, %0, 1" : "+v"(x));
#define OP_CNDE64(x) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[4:5]" : "+v"(x) : "v"(b) : "s4", "s5");
#define OP_ADDC(x) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(x) : "v"(b) : "vcc");
#define OP_MADU24(x) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define OP_MULU24(x) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(b));
#define OP_BFI(x) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define OP_SUBCO(x) asm volatile("v_sub_co_u32 %0, vcc, %0, %1" : "+v"(x) : "v"(b) : "vcc");
#define OP_MAX(x) asm volatile("v_max_u32 %0, %0, %1" : "+v"(x) : "v"(b));
DEF_KERNEL(k_sdwax, OP_SDWAX)
DEF_KERNEL(k_sdwao, OP_SDWAO)
DEF_KERNEL(k_sdwaa, OP_SDWAA)
DEF_KERNEL(k_or3, OP_OR3)
DEF_KERNEL(k_andor, OP_ANDOR)
DEF_KERNEL(k_lshladd, OP_LSHLADD)
DEF_KERNEL(k_lshr, OP_LSHR)
DEF_KERNEL(k_alignbyte, OP_ALIGNBYTE)
DEF_KERNEL(k_cnde64, OP_CNDE64)
DEF_KERNEL(k_addc, OP_ADDC)
DEF_KERNEL(k_madu24, OP_MADU24)
DEF_KERNEL(k_mulu24, OP_MULU24)
DEF_KERNEL(k_bfi, OP_BFI)
DEF_KERNEL(k_subco, OP_SUBCO)
DEF_KERNEL(k_max, OP_MAX)
DEF_KERNEL(k_xor, OP_XOR)
DEF_KERNEL(k_add, OP_ADD)
DEF_KERNEL(k_add3, OP_ADD3)
DEF_KERNEL(k_align, OP_ALIGN)
DEF_KERNEL(k_perm, OP_PERM)
DEF_KERNEL(k_xad, OP_XAD)
DEF_KERNEL(k_lshlor, OP_LSHLOR)
DEF_KERNEL(k_xore64, OP_XORE64)
DEF_KERNEL(k_bitop3, OP_BITOP3)
DEF_KERNEL(k_mullo, OP_MULLO)
DEF_KERNEL(k_mulhi, OP_MULHI)
DEF_KERNEL(k_pkadd16, OP_PKADD16)
DEF_KERNEL(k_addco, OP_ADDCO)
DEF_KERNEL(k_cnd, OP_CND)

// instruction mixes (per chain, per unrolled step): BLAKE3's G is
// 2 add3 + 2 add + 4 xor + 4 alignbit
#define MIX_XA(x) CH8(OP_XOR) CH8(OP_ALIGN)
#define MIX_XXA(x) CH8(OP_XOR) CH8(OP_XOR) CH8(OP_ALIGN)
#define MIX_G(x) CH8(OP_ADD3) CH8(OP_XOR) CH8(OP_ALIGN) CH8(OP_ADD) CH8(OP_XOR) CH8(OP_ALIGN)
#define MIX_G2(x) CH8(OP_ADD) CH8(OP_ADD) CH8(OP_XOR) CH8(OP_ALIGN) CH8(OP_ADD) CH8(OP_XOR) CH8(OP_ALIGN)
#define MIX_XADD(x) CH8(OP_XOR) CH8(OP_ADD)
#define MIX_AA(x) CH8(OP_ALIGN) CH8(OP_ADD3)
#define ONCE(OP) OP(a0)
#define DEF_MIX(NAME, BODY)                                                            \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint64_t* cyc, int iters) { \
    uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11,     \
             a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;                                  \
    uint32_t b = blockIdx.x | 1, c = blockIdx.x * 7 + 1;                                \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                                        \
    for (int i = 0; i < iters; i++) {                                                   \
      _Pragma("unroll") for (int k = 0; k < 8; k++) { BODY(0) }                        \
    }                                                                                   \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                                        \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;        \
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                   \
  }
DEF_MIX(k_mix_xa, MIX_XA)
DEF_MIX(k_mix_xxa, MIX_XXA)
DEF_MIX(k_mix_g, MIX_G)
DEF_MIX(k_mix_g2, MIX_G2)
DEF_MIX(k_mix_xadd, MIX_XADD)
DEF_MIX(k_mix_aa, MIX_AA)

// 64-bit: mad_u64_u32 chains
__global__ void __launch_bounds__(256) k_mad64(uint32_t* out, uint64_t* cyc, int iters) {
  uint64_t a[8];
  for (int j = 0; j < 8; j++) a[j] = threadIdx.x * (j + 3);
  uint32_t b = blockIdx.x | 1;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
#pragma unroll
      for (int j = 0; j < 8; j++)
        asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a[j]) : "v"(b) : "s0", "s1");
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
  for (int j = 0; j < 8; j++) x ^= (uint32_t)a[j];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}


#define DEF_K64(NAME, INSTR)                                                            \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint64_t* cyc, int iters) { \
    uint64_t a[8];                                                                      \
    for (int j = 0; j < 8; j++) a[j] = threadIdx.x * (j + 3);                            \
    uint64_t b = blockIdx.x | 1;                                                        \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                                        \
    for (int i = 0; i < iters; i++) {                                                   \
      _Pragma("unroll") for (int k = 0; k < 8; k++) {                                  \
        _Pragma("unroll") for (int j = 0; j < 8; j++) asm volatile(INSTR : "+v"(a[j]) : "v"(b)); \
      }                                                                                 \
    }                                                                                   \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                                        \
    uint32_t x = 0;                                                                     \
    for (int j = 0; j < 8; j++) x ^= (uint32_t)a[j] ^ (uint32_t)(a[j] >> 32);           \
    out[blockIdx.x * 256 + threadIdx.x] = x;                                            \
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                   \
  }
DEF_K64(k_lshladd64, "v_lshl_add_u64 %0, %0, 0, %1")
DEF_K64(k_lshr64, "v_lshrrev_b64 %0, 12, %0")
DEF_K64(k_mov64, "v_mov_b64 %0, %1")
DEF_K64(k_pkmov, "v_pk_mov_b32 %0, %0, %1 op_sel:[1,0]")
DEF_K64(k_pkaddf32, "v_pk_add_f32 %0, %0, %1")

typedef void (*KFn)(uint32_t*, uint64_t*, int);

int main() {
  const int blocks = 256 * 8;  // 8 WGs of 4 waves per CU -> 8 waves per SIMD
  const int iters = 4096;
  uint32_t* out;
  uint64_t* cyc;
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&cyc, blocks * 8);
  struct { const char* n; KFn f; } ks[] = {
      {"v_xor_b32", k_xor},       {"v_add_u32", k_add},         {"v_add3_u32", k_add3},
      {"v_alignbit_b32", k_align}, {"v_perm_b32", k_perm},      
      {"v_xad_u32", k_xad},       {"v_lshl_or_b32", k_lshlor},  {"v_xor_b32_e64", k_xore64},
      {"v_bitop3_b32", k_bitop3}, {"v_mul_lo_u32", k_mullo},    {"v_mul_hi_u32", k_mulhi},
      {"v_pk_add_u16", k_pkadd16}, {"v_add_co_u32", k_addco},   {"v_cndmask_b32", k_cnd},
      {"v_mad_u64_u32", k_mad64},
      {"v_xor_b32_sdwa w16", k_sdwax}, {"v_or_b32_sdwa byte", k_sdwao}, {"v_add_u32_sdwa", k_sdwaa},
      {"v_or3_b32", k_or3}, {"v_and_or_b32", k_andor}, {"v_lshl_add_u32", k_lshladd}, {"v_lshrrev_b32", k_lshr},
      {"v_alignbyte_b32", k_alignbyte}, {"v_cndmask_e64", k_cnde64}, {"v_addc_co_u32", k_addc},
      {"v_mad_u32_u24", k_madu24}, {"v_mul_u32_u24", k_mulu24}, {"v_bfi_b32", k_bfi}, {"v_sub_co_u32", k_subco},
      {"v_max_u32", k_max},
      {"mix xor+align (/2)", k_mix_xa}, {"mix 2xor+align (/3)", k_mix_xxa}, {"mix G-half add3 (/6)", k_mix_g},
      {"mix G-half 2add (/7)", k_mix_g2}, {"mix xor+add (/2)", k_mix_xadd}, {"mix align+add3 (/2)", k_mix_aa},
      {"v_lshl_add_u64", k_lshladd64}, {"v_lshrrev_b64", k_lshr64}, {"v_mov_b64", k_mov64},
      {"v_pk_mov_b32", k_pkmov}, {"v_pk_add_f32", k_pkaddf32},
  };
  uint64_t* h = (uint64_t*)malloc(blocks * 8);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, cyc, 16);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
    double mx = 0, sum = 0;
    for (int i = 0; i < blocks; i++) { sum += h[i]; mx = h[i] > mx ? h[i] : mx; }
    // per wave: iters*64 instructions; 8 waves share a SIMD concurrently
    double per_wave = (double)iters * 64;
    double cyc_per_instr_simd = (sum / blocks) / (per_wave * 8);
    double wall_rate = (double)blocks * 4 * per_wave / (ms * 1e-3) / 1e12;  // T wave-instr/s
    printf("%-16s %6.2f cycles/instr/SIMD (memtime, mean WG)  wall %.3f ms  %.3f T wave64-instr/s  (%.1f T lane-ops/s)\n",
           k.n, cyc_per_instr_simd, ms, wall_rate, wall_rate * 64);
  }
  return 0;
}

#!/bin/bash
# Build the NTT component-timing variants (see tools/ntt_parts_main.hip) into
# tools/ntt_parts/: a copy of csrc/ntt.hip with VAR_TW / VAR_W / VAR_FFT hooks
# around the pass twiddles, the W twiddle and the register FFTs. Run each
# binary on the GPU box; DESIGN.md §3 quotes the result.
set -euo pipefail
D=tools/ntt_parts
mkdir -p $D
python3 - <<'PY'
s = open("streaming-zero-knowledge-proofs_amd/csrc/ntt.hip").read()
rep = [
    ("if (low != 0) {  // pre-twiddle", "if (VAR_TW && low != 0) {  // pre-twiddle"),
    ("if (low != 0) {  // post-twiddle", "if (VAR_TW && low != 0) {  // post-twiddle"),
    ("const uint64_t v = k2 && j1 ? gl_mul(x[k2], W[j1 * k2]) : x[k2];",
     "const uint64_t v = k2 && j1 ? (VAR_W ? gl_mul(x[k2], W[j1 * k2]) : x[k2] ^ W[j1 * k2]) : x[k2];"),
    ("const uint64_t v = klo && r ? gl_mul(x[q], W[r * klo]) : x[q];",
     "const uint64_t v = klo && r ? (VAR_W ? gl_mul(x[q], W[r * klo]) : x[q] ^ W[r * klo]) : x[q];"),
    ("      fft_dit_regs<M1, INV, SKIP>(x);", "      if (VAR_FFT) fft_dit_regs<M1, INV, SKIP>(x);"),
    ("      fft_dit_regs<M2, INV, 0>(y);", "      if (VAR_FFT) fft_dit_regs<M2, INV, 0>(y);"),
    ("      fft_dif_regs<M2, INV>(x);", "      if (VAR_FFT) fft_dif_regs<M2, INV>(x);"),
    ("      fft_dif_regs<M1, INV>(y);", "      if (VAR_FFT) fft_dif_regs<M1, INV>(y);"),
]
rep.append(("  const int c = tid & (NTT_CMAX - 1), g = tid / NTT_CMAX;\n  // a plain NARROW load",
            "  const int c = tid & (NTT_CMAX - 1), g = tid / NTT_CMAX;\n#if VAR_SLEEP\n  if ((blockIdx.x & 1) && blockIdx.x < 1024) for (int i = 0; i < VAR_SLEEP; i++) __builtin_amdgcn_s_sleep(127);\n#endif\n  // a plain NARROW load"))
# VAR_NOMEM: loads replaced by values made from the address, stores kept only
# behind a compare that never holds (the arithmetic stays, the HBM traffic goes)
rep += [
    ("        for (int r = 0; r < F1; r++) x[r] = P.a[tile_pos(G, F1 * u + r, c, low)];",
     "        for (int r = 0; r < F1; r++) { const uint64_t p_ = tile_pos(G, F1 * u + r, c, low); x[r] = VAR_NOMEM ? (p_ | 1) : P.a[p_]; }"),
    ("        for (int k1 = 0; k1 < F2; k1++) P.a[tile_pos(G, k2 + F1 * k1, c, low)] = y[k1];",
     "        for (int k1 = 0; k1 < F2; k1++) { const uint64_t p_ = tile_pos(G, k2 + F1 * k1, c, low); if (!VAR_NOMEM || y[k1] == 0x123456789ull) P.a[p_] = y[k1]; }"),
    ("        x[u] = NARROW ? sh[(F1 * u + r) * NTT_PADC + c] : P.a[tile_pos(G, F1 * u + r, c, low)];",
     "        x[u] = NARROW ? sh[(F1 * u + r) * NTT_PADC + c] : (VAR_NOMEM ? (tile_pos(G, F1 * u + r, c, low) | 1) : P.a[tile_pos(G, F1 * u + r, c, low)]);"),
    ("        for (int qq = 0; qq < F1; qq++) P.a[tile_pos(G, q * F1 + qq, c, low)] = y[qq];",
     "        for (int qq = 0; qq < F1; qq++) { const uint64_t p_ = tile_pos(G, q * F1 + qq, c, low); if (!VAR_NOMEM || y[qq] == 0x123456789ull) P.a[p_] = y[qq]; }"),
    ("    sh[(e & (R - 1)) * NTT_PADC + (e >> m)] = src[e];",
     "    sh[(e & (R - 1)) * NTT_PADC + (e >> m)] = VAR_NOMEM ? (uint64_t)(e | 1) + tile : src[e];"),
    ("    dst[e] = sh[(e & (R - 1)) * NTT_PADC + (e >> m)];",
     "    { const uint64_t v_ = sh[(e & (R - 1)) * NTT_PADC + (e >> m)]; if (!VAR_NOMEM || v_ == 0x123456789ull) dst[e] = v_; }"),
]
# VAR_OCC2: 36 KB more static LDS per workgroup, so only 2 fit on a CU (2 waves per SIMD)
rep.append(("  __shared__ uint64_t W[R];\n  const int tid = threadIdx.x;\n  const NttTables& T = P.tw;",
            "  __shared__ uint64_t W[R];\n  const int tid = threadIdx.x;\n  const NttTables& T = P.tw;\n#if VAR_OCC2\n"
            "  __shared__ uint64_t occ_pad[4608];\n  if (P.m == 99) occ_pad[tid] = tid;\n  asm volatile(\"\" :: \"v\"(occ_pad[(tid * 7) & 4095]));\n#endif"))
for a, b in rep:
    assert a in s, a
    s = s.replace(a, b)
s = s.replace('#include "dev_common.h"', '#include "../../streaming-zero-knowledge-proofs_amd/csrc/dev_common.h"')
s = s.replace('#include "sezkp_internal.h"', '#include "../../streaming-zero-knowledge-proofs_amd/csrc/sezkp_internal.h"')
open("tools/ntt_parts/ntt_var.hip", "w").write(s)
PY
cp tools/ntt_parts_main.hip $D/main.hip
for v in "1 1 1" "0 1 1" "1 0 1" "1 1 0" "0 0 0"; do
  set -- $v
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -w -DVAR_TW=$1 -DVAR_W=$2 -DVAR_FFT=$3 -o $D/nv_$1$2$3 $D/main.hip
done
# arithmetic only: no HBM loads or stores (is the pass bound by its instructions?)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -w -DVAR_NOMEM=1 -o $D/nv_nomem $D/main.hip
# the same two at 2 workgroups per CU (what a double-buffered LDS tile would allow)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -w -DVAR_NOMEM=1 -DVAR_OCC2=1 -o $D/nv_nomem_occ2 $D/main.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -w -DVAR_OCC2=1 -o $D/nv_occ2 $D/main.hip
# odd workgroups of the first round (blockIdx < 4 x 256 CUs) start later (s_sleep), to offset the
# phases of the workgroups sharing a CU
for sl in 1 2 4; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -w -DVAR_SLEEP=$sl -o $D/nv_sleep$sl $D/main.hip
done
echo built $D

// compose.h — the AIR composition value C(i) (air.rs:49-136, prover.rs:142-158)
// from the per-row constraint sums of k_compose_terms (trace.hip), once the
// transcript has the alphas and the mask. Shared by k_compose_combine
// (trace.hip) and k_inv_base (ntt.hip, fused with the DEEP quotient).
#pragma once
#include "dev_common.h"
#include "sezkp_internal.h"

namespace sezkp {

// the alphas with the reuse of prover.rs:86-98 and the mask coefficients,
// from the transcript's device record
__device__ __forceinline__ Alphas alphas_of(const DevChal* ch) {
  const uint64_t* a = ch->alpha;
  return Alphas{a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[0], a[2], a[2]};
}

struct ComposeCoef {
  Alphas A;
  uint64_t m0, m1, m2, m3;
};
__device__ __forceinline__ ComposeCoef compose_coef(const DevChal* ch) {
  return ComposeCoef{alphas_of(ch), ch->mask[0], ch->mask[1], ch->mask[2], ch->mask[3]};
}

// C(i) = sum over constraint types of alpha * (its per-tape sum) + R(x),
// x = w_n^i, R(x) = m0 + m1 x + m2 x^2 + m3 x^3 (masking.rs:56-103). The
// zero sums are skipped exactly as the one-kernel composition did (a * 0 = 0).
__device__ __forceinline__ uint64_t compose_value(const ComposeTerms& Tm, const ComposeCoef& K, uint64_t i,
                                                  uint64_t x) {
  const uint8_t fl = Tm.row_flags[i];
  const int32_t c2 = Tm.c2[i], sy = Tm.sy[i];
  const int64_t c3 = Tm.c3[i];
  const uint64_t hr = Tm.hr[i], sl = Tm.sl[i];
  uint64_t acc = 0;
  if (c2) acc = gl_mul(K.A.mv_domain, gl_from_i64(c2));
  if (c3) acc = gl_add(acc, gl_mul(K.A.head_update, gl_from_i64(c3)));
  if (hr) acc = gl_add(acc, gl_mul(K.A.head_reconstruct, hr));
  if (sl) acc = gl_add(acc, gl_mul(K.A.slack_reconstruct, sl));
  if (sy) acc = gl_add(acc, gl_mul(K.A.sym_reconstruct, (uint64_t)sy));
  if (fl & 3) {  // a block's first / last row: its boundary sums (one per block)
    const uint32_t b = Tm.row_blk[i];
    if (fl & 1) acc = gl_add(acc, gl_mul(K.A.boundary_first, Tm.bf[b]));
    if (fl & 2) acc = gl_add(acc, gl_mul(K.A.boundary_last, Tm.bl[b]));
  }
  const uint64_t R = gl_add(gl_mul(gl_add(gl_mul(gl_add(gl_mul(K.m3, x), K.m2), x), K.m1), x), K.m0);
  return gl_add(acc, R);
}

}  // namespace sezkp

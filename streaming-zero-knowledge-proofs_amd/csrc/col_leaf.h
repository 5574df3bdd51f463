// col_leaf.h — labelled column leaf BLAKE3("col_leaf" || u32 LE len(label) ||
// label || v LE) (crates/sezkp-stark/src/v1/merkle.rs:132-147) for any
// label of <= 44 bytes (one 64-byte block), from a per-column message template.
#pragma once
#include "dev_common.h"
#include "sezkp_internal.h"

namespace sezkp {

// generic (any label length <= 44): value words inserted with runtime shifts
__device__ __forceinline__ void leaf_labeled_rt(const ColTemplate& ct, uint64_t v, uint32_t (&out)[8]) {
  uint32_t m[16];
  const int W = ct.off >> 2, B = ct.off & 3;
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  const uint32_t x0 = B ? lo << (8 * B) : lo;
  const uint32_t x1 = B ? (lo >> (32 - 8 * B)) | (hi << (8 * B)) : hi;
  const uint32_t x2 = B ? hi >> (32 - 8 * B) : 0;
#pragma unroll
  for (int i = 0; i < 16; i++)
    m[i] = ct.words[i] | (i == W ? x0 : 0) | (i == W + 1 ? x1 : 0) | (i == W + 2 ? x2 : 0);
  b3_hash_block(m, ct.off + 8, out);
}
}  // namespace sezkp

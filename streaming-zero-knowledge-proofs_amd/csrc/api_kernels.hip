// api_kernels.hip — kernels behind the kernel-level C ABI entry points that
// the prover itself runs in fused form (leaf hashing inside the tree kernels,
// stored-level trees): plain leaf digests, a full MerkleTree with odd
// promotion, and path gathers.
//
// Reference semantics:
//  * hash_field_leaves         crates/sezkp-stark/src/v1/merkle.rs:150-160
//  * hash_field_leaves_labeled merkle.rs:132-147
//  * MerkleTree::from_leaves   merkle.rs:46-71 (levels bottom -> top, odd
//    promotion carries the last node up unchanged)
//  * MerkleTree::open          merkle.rs:80-108 (idx %= n; a node without a
//    sibling is its own sibling)
// One lane per digest: 8-byte loads, 32-byte (2 x 16 B) stores, consecutive
// lanes on consecutive digests. These are HBM/VALU-streaming kernels; the
// prover's fused versions live in merkle.hip.
#include "col_leaf.h"

namespace sezkp {

constexpr int AK_THREADS = 256;

__global__ void __launch_bounds__(AK_THREADS) k_leaves_u64(const uint64_t* __restrict__ v, uint64_t n,
                                                           uint32_t* __restrict__ out) {
  const uint64_t i = blockIdx.x * (uint64_t)AK_THREADS + threadIdx.x;
  if (i >= n) return;
  uint32_t h[8];
  b3_leaf_u64(v[i], h);
  node_store(out + 8 * i, h);
}

__global__ void __launch_bounds__(AK_THREADS) k_leaves_labeled(const uint64_t* __restrict__ v, uint64_t n,
                                                               ColTemplate ct, uint32_t* __restrict__ out) {
  const uint64_t i = blockIdx.x * (uint64_t)AK_THREADS + threadIdx.x;
  if (i >= n) return;
  uint32_t h[8];
  leaf_labeled_rt(ct, v[i], h);
  node_store(out + 8 * i, h);
}

__global__ void __launch_bounds__(AK_THREADS) k_merkle_level(const uint32_t* __restrict__ in, uint64_t len,
                                                             uint32_t* __restrict__ out) {
  const uint64_t i = blockIdx.x * (uint64_t)AK_THREADS + threadIdx.x;
  if (i >= (len + 1) / 2) return;
  uint32_t l[8], h[8];
  node_load(in + 16 * i, l);
  if (2 * i + 1 < len) {
    uint32_t r[8];
    node_load(in + 16 * i + 8, r);
    b3_parent(l, r, h);
    node_store(out + 8 * i, h);
  } else {
    node_store(out + 8 * i, l);  // odd promotion (merkle.rs:59-62)
  }
}

__global__ void __launch_bounds__(AK_THREADS) k_merkle_paths(const uint32_t* __restrict__ nodes, MerkleLevels L,
                                                             const uint64_t* __restrict__ idx, uint32_t q,
                                                             uint32_t* __restrict__ out) {
  const uint64_t t = blockIdx.x * (uint64_t)AK_THREADS + threadIdx.x;
  if (t >= (uint64_t)q * L.depth) return;
  const uint64_t qi = t / L.depth;
  const int l = (int)(t % L.depth);
  const uint64_t i = (idx[qi] % L.len[0]) >> l;
  const uint64_t sib = (i ^ 1) < L.len[l] ? (i ^ 1) : i;
  uint32_t h[8];
  node_load(nodes + 8 * (L.off[l] + sib), h);
  node_store(out + 8 * t, h);
}

// FRI fold of any power-of-two length: out[i] = in[i] + beta in[i + n]
// (prover.rs:208-230); lengths >= 4 take the prover's 4-per-lane k_fold
__global__ void __launch_bounds__(AK_THREADS) k_fold1(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                      uint64_t n, uint64_t beta) {
  const uint64_t i = blockIdx.x * (uint64_t)AK_THREADS + threadIdx.x;
  if (i < n) out[i] = gl_add(in[i], gl_mul(beta, in[i + n]));
}

static unsigned grid_for(uint64_t n) { return (unsigned)((n + AK_THREADS - 1) / AK_THREADS); }

hipError_t launch_fold_any(hipStream_t st, const uint64_t* in, uint64_t* out, uint64_t n, uint64_t beta) {
  if (n >= 4) {
    int lg = 0;
    while ((1ULL << lg) < n) lg++;
    return launch_fold(st, in, out, lg, beta);
  }
  hipLaunchKernelGGL(k_fold1, dim3(1), dim3(AK_THREADS), 0, st, in, out, n, beta);
  return hipGetLastError();
}

hipError_t launch_leaves_u64(hipStream_t st, const uint64_t* v, uint64_t n, uint32_t* out) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_leaves_u64, dim3(grid_for(n)), dim3(AK_THREADS), 0, st, v, n, out);
  return hipGetLastError();
}

hipError_t launch_leaves_labeled(hipStream_t st, const uint64_t* v, uint64_t n, const ColTemplate& ct, uint32_t* out) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_leaves_labeled, dim3(grid_for(n)), dim3(AK_THREADS), 0, st, v, n, ct, out);
  return hipGetLastError();
}

hipError_t launch_merkle_level(hipStream_t st, const uint32_t* in, uint64_t len, uint32_t* out) {
  hipLaunchKernelGGL(k_merkle_level, dim3(grid_for((len + 1) / 2)), dim3(AK_THREADS), 0, st, in, len, out);
  return hipGetLastError();
}

hipError_t launch_merkle_paths(hipStream_t st, const uint32_t* nodes, const MerkleLevels& L, const uint64_t* idx,
                               uint32_t q, uint32_t* out) {
  const uint64_t work = (uint64_t)q * L.depth;
  if (work == 0) return hipSuccess;
  hipLaunchKernelGGL(k_merkle_paths, dim3(grid_for(work)), dim3(AK_THREADS), 0, st, nodes, L, idx, q, out);
  return hipGetLastError();
}

}  // namespace sezkp

// host_crypto.h — host-side BLAKE3 (streaming hasher + XOF) and the
// Fiat-Shamir transcript of crates/sezkp-crypto/src/lib.rs:74-123.
// The transcript is a few KB per proof and strictly sequential, so it stays
// on the CPU; only its outputs (alphas, masks, z, betas, queries) cross to HBM.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace sezkp {

class Blake3 {
 public:
  Blake3();
  void update(const void* data, size_t len);
  void finalize(uint8_t* out, size_t out_len) const;  // XOF, any length

 private:
  struct Node {
    uint32_t cv[8];
    uint32_t block[16];
    uint64_t counter;
    uint32_t len, flags;
  };
  void push_chunk_cv(const uint32_t cv[8], uint64_t total_chunks);
  Node chunk_node() const;
  uint32_t cv_[8];
  uint64_t chunk_ctr_ = 0;
  uint8_t buf_[64];
  uint32_t buf_len_ = 0;
  uint32_t blocks_done_ = 0;
  uint32_t stack_[64][8];
  int depth_ = 0;
};

void blake3_compress(const uint32_t cv[8], const uint32_t m[16], uint64_t ctr, uint32_t len, uint32_t flags,
                     uint32_t out[16]);
void blake3_oneshot(const void* data, size_t len, uint8_t out[32]);

class Transcript {
 public:
  explicit Transcript(const std::string& domain);
  void absorb(const std::string& label, const void* bytes, size_t len);
  void absorb_u64(const std::string& label, uint64_t x);
  std::vector<uint8_t> challenge(const std::string& label, size_t n);

 private:
  Blake3 st_;
};

// Host Goldilocks helpers (u128), used for constants and verification.
constexpr uint64_t GL_P_HOST = 0xffffffff00000001ULL;
uint64_t hgl_mul(uint64_t a, uint64_t b);
uint64_t hgl_add(uint64_t a, uint64_t b);
uint64_t hgl_sub(uint64_t a, uint64_t b);
uint64_t hgl_pow(uint64_t a, uint64_t e);
uint64_t hgl_inv(uint64_t a);
uint64_t hgl_root_2exp(uint32_t k);
uint64_t hgl_from_i64(int64_t x);

}  // namespace sezkp

// host_crypto.cpp — host BLAKE3 (hash mode + XOF, spec restatement) and the
// sezkp Blake3Transcript (crates/sezkp-crypto/src/lib.rs:74-123).
#include "host_crypto.h"

#include <string.h>

namespace sezkp {

namespace {
const uint32_t IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                        0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
const int SIGMA[7][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
    {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1}, {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
    {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4}, {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
    {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13}};
constexpr uint32_t CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8;
inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
inline void G(uint32_t* v, int a, int b, int c, int d, uint32_t x, uint32_t y) {
  v[a] += v[b] + x; v[d] = rotr(v[d] ^ v[a], 16);
  v[c] += v[d];     v[b] = rotr(v[b] ^ v[c], 12);
  v[a] += v[b] + y; v[d] = rotr(v[d] ^ v[a], 8);
  v[c] += v[d];     v[b] = rotr(v[b] ^ v[c], 7);
}
inline void load_words(const uint8_t* b, uint32_t* w) {
  for (int i = 0; i < 16; i++)
    w[i] = (uint32_t)b[4 * i] | (uint32_t)b[4 * i + 1] << 8 | (uint32_t)b[4 * i + 2] << 16 | (uint32_t)b[4 * i + 3] << 24;
}
}  // namespace

void blake3_compress(const uint32_t cv[8], const uint32_t m[16], uint64_t ctr, uint32_t len, uint32_t flags,
                     uint32_t out[16]) {
  uint32_t v[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7], IV[0], IV[1], IV[2], IV[3],
                    (uint32_t)ctr, (uint32_t)(ctr >> 32), len, flags};
  for (int r = 0; r < 7; r++) {
    const int* s = SIGMA[r];
    G(v, 0, 4, 8, 12, m[s[0]], m[s[1]]);
    G(v, 1, 5, 9, 13, m[s[2]], m[s[3]]);
    G(v, 2, 6, 10, 14, m[s[4]], m[s[5]]);
    G(v, 3, 7, 11, 15, m[s[6]], m[s[7]]);
    G(v, 0, 5, 10, 15, m[s[8]], m[s[9]]);
    G(v, 1, 6, 11, 12, m[s[10]], m[s[11]]);
    G(v, 2, 7, 8, 13, m[s[12]], m[s[13]]);
    G(v, 3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
  for (int i = 0; i < 8; i++) {
    out[i] = v[i] ^ v[i + 8];
    out[i + 8] = v[i + 8] ^ cv[i];
  }
}

Blake3::Blake3() { memcpy(cv_, IV, 32); memset(buf_, 0, 64); }

void Blake3::push_chunk_cv(const uint32_t cv[8], uint64_t total_chunks) {
  uint32_t cur[8];
  memcpy(cur, cv, 32);
  while ((total_chunks & 1) == 0) {  // merge completed subtrees
    uint32_t m[16], o[16];
    memcpy(m, stack_[--depth_], 32);
    memcpy(m + 8, cur, 32);
    blake3_compress(IV, m, 0, 64, PARENT, o);
    memcpy(cur, o, 32);
    total_chunks >>= 1;
  }
  memcpy(stack_[depth_++], cur, 32);
}

void Blake3::update(const void* data, size_t len) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  while (len) {
    if (buf_len_ == 64) {
      // a full block is only compressed once more input follows
      uint32_t m[16], o[16];
      load_words(buf_, m);
      if (blocks_done_ == 15) {  // last block of a 1024-byte chunk: close the chunk
        blake3_compress(cv_, m, chunk_ctr_, 64, CHUNK_END, o);
        push_chunk_cv(o, chunk_ctr_ + 1);
        chunk_ctr_++;
        memcpy(cv_, IV, 32);
        blocks_done_ = 0;
      } else {
        blake3_compress(cv_, m, chunk_ctr_, 64, blocks_done_ == 0 ? CHUNK_START : 0, o);
        memcpy(cv_, o, 32);
        blocks_done_++;
      }
      buf_len_ = 0;
      memset(buf_, 0, 64);
    }
    size_t take = 64 - buf_len_;
    if (take > len) take = len;
    memcpy(buf_ + buf_len_, p, take);
    buf_len_ += (uint32_t)take;
    p += take;
    len -= take;
  }
}

Blake3::Node Blake3::chunk_node() const {
  Node n;
  memcpy(n.cv, cv_, 32);
  load_words(buf_, n.block);
  n.counter = chunk_ctr_;
  n.len = buf_len_;
  n.flags = (blocks_done_ == 0 ? CHUNK_START : 0) | CHUNK_END;
  return n;
}

void Blake3::finalize(uint8_t* out, size_t out_len) const {
  Node node = chunk_node();
  for (int i = depth_ - 1; i >= 0; i--) {
    uint32_t o[16], m[16];
    blake3_compress(node.cv, node.block, node.counter, node.len, node.flags, o);
    memcpy(m, stack_[i], 32);
    memcpy(m + 8, o, 32);
    memcpy(node.cv, IV, 32);
    memcpy(node.block, m, 64);
    node.counter = 0;
    node.len = 64;
    node.flags = PARENT;
  }
  uint64_t t = 0;
  while (out_len) {
    uint32_t o[16];
    blake3_compress(node.cv, node.block, t++, node.len, node.flags | ROOT, o);
    for (int i = 0; i < 16 && out_len; i++)
      for (int k = 0; k < 4 && out_len; k++, out_len--) *out++ = (uint8_t)(o[i] >> (8 * k));
  }
}

void blake3_oneshot(const void* data, size_t len, uint8_t out[32]) {
  Blake3 h;
  h.update(data, len);
  h.finalize(out, 32);
}

// --------------------------------------------------------------- transcript
static void put_u32(Blake3& h, uint32_t x) {
  uint8_t b[4] = {(uint8_t)x, (uint8_t)(x >> 8), (uint8_t)(x >> 16), (uint8_t)(x >> 24)};
  h.update(b, 4);
}
Transcript::Transcript(const std::string& domain) {
  st_.update("sezkp.transcript.v0", 19);
  put_u32(st_, (uint32_t)domain.size());
  st_.update(domain.data(), domain.size());
}
void Transcript::absorb(const std::string& label, const void* bytes, size_t len) {
  st_.update("absorb", 6);
  put_u32(st_, (uint32_t)label.size());
  st_.update(label.data(), label.size());
  put_u32(st_, (uint32_t)len);
  st_.update(bytes, len);
}
void Transcript::absorb_u64(const std::string& label, uint64_t x) {
  uint8_t b[8];
  for (int i = 0; i < 8; i++) b[i] = (uint8_t)(x >> (8 * i));
  absorb(label, b, 8);
}
std::vector<uint8_t> Transcript::challenge(const std::string& label, size_t n) {
  Blake3 st = st_;
  st.update("challenge", 9);
  put_u32(st, (uint32_t)label.size());
  st.update(label.data(), label.size());
  std::vector<uint8_t> out(n);
  st.finalize(out.data(), n);
  st_.update("after_challenge", 15);
  put_u32(st_, (uint32_t)label.size());
  st_.update(label.data(), label.size());
  return out;
}

// ------------------------------------------------------------- goldilocks
typedef unsigned __int128 u128;
// a * b mod p without a 128-bit division: x = lo + 2^64 h0 + 2^96 h1 with
// 2^64 = 2^32 - 1 and 2^96 = -1 (mod p) (the device's gl_reduce128). The
// u128 % libcall cost ~35 ns per product, and the transcript round trips
// (inverses and powers of z) ran ~30 us of them per proof with the GPU idle.
uint64_t hgl_mul(uint64_t a, uint64_t b) {
  const u128 x = (u128)a * b;
  const uint64_t lo = (uint64_t)x, hi = (uint64_t)(x >> 64);
  const uint64_t h0 = hi & 0xFFFFFFFFull, h1 = hi >> 32;
  uint64_t t0;
  if (__builtin_sub_overflow(lo, h1, &t0)) t0 -= 0xFFFFFFFFull;  // + p (mod 2^64); t0 stays >= 2^64 - 2^32
  uint64_t r;
  if (__builtin_add_overflow(t0, h0 * 0xFFFFFFFFull, &r)) r += 0xFFFFFFFFull;  // cannot wrap again
  return r >= GL_P_HOST ? r - GL_P_HOST : r;
}
uint64_t hgl_add(uint64_t a, uint64_t b) {
  u128 s = (u128)a + b;
  return (uint64_t)(s >= GL_P_HOST ? s - GL_P_HOST : s);
}
uint64_t hgl_sub(uint64_t a, uint64_t b) { return a >= b ? a - b : (uint64_t)((u128)a + GL_P_HOST - b); }
uint64_t hgl_pow(uint64_t a, uint64_t e) {
  uint64_t r = 1;
  while (e) {
    if (e & 1) r = hgl_mul(r, a);
    a = hgl_mul(a, a);
    e >>= 1;
  }
  return r;
}
uint64_t hgl_inv(uint64_t a) { return hgl_pow(a, GL_P_HOST - 2); }
uint64_t hgl_root_2exp(uint32_t k) { return hgl_pow(7, (GL_P_HOST - 1) >> k); }
uint64_t hgl_from_i64(int64_t x) { return x >= 0 ? (uint64_t)x % GL_P_HOST : GL_P_HOST - ((0 - (uint64_t)x) % GL_P_HOST); }

}  // namespace sezkp

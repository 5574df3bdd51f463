// tracegen.cpp — `sezkp-cli simulate`'s input producer, bit-exact: the
// synthetic movement log of crates/sezkp-trace/src/generator.rs:38-73 drawn
// from rand 0.9.2's StdRng (Cargo.lock:842-870), restated from the crates'
// published algorithms (not vendored in the reference tree):
//   * rand_core 0.9.3 SeedableRng::seed_from_u64 — 8 PCG32 outputs
//     (MUL 6364136223846793005, INC 11634580027462260723) form the 32-B key;
//   * rand_chacha 0.9.0 ChaCha12Rng — ChaCha with 12 rounds, 64-bit block
//     counter (words 12-13) from 0, stream 0, consumed through rand_core's
//     BlockRng over a 64-word buffer of 4 consecutive blocks;
//   * rand 0.9 random_range(a..=b) on 32-bit-or-smaller ints — one u32 draw
//     widened by the range, plus Canon's correction draw when the low half
//     exceeds -range; random_bool(p) — one u64 draw < (u64)(p * 2^64).
// Host code (a caller of the hot path): the draw sequence is
// data-dependent, so it is one sequential stream, ~0.1 s at T = 2^21.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/sezkp_stark.h"
#include "codec.h"

namespace {

struct StdRng {
  uint32_t key[8];
  uint64_t ctr = 0;
  uint32_t buf[64];
  int idx = 64;

  explicit StdRng(uint64_t state) {
    for (int i = 0; i < 8; i++) {
      state = state * 6364136223846793005ULL + 11634580027462260723ULL;
      const uint32_t xs = (uint32_t)(((state >> 18) ^ state) >> 27);
      const uint32_t rot = (uint32_t)(state >> 59);
      key[i] = (xs >> rot) | (xs << ((32 - rot) & 31));
    }
  }
  static inline uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
  static inline void qr(uint32_t* s, int a, int b, int c, int d) {
    s[a] += s[b]; s[d] = rotl(s[d] ^ s[a], 16);
    s[c] += s[d]; s[b] = rotl(s[b] ^ s[c], 12);
    s[a] += s[b]; s[d] = rotl(s[d] ^ s[a], 8);
    s[c] += s[d]; s[b] = rotl(s[b] ^ s[c], 7);
  }
  void refill() {
    for (int blk = 0; blk < 4; blk++) {
      const uint64_t c = ctr + blk;
      uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                         key[4], key[5], key[6], key[7], (uint32_t)c, (uint32_t)(c >> 32), 0, 0};
      uint32_t s[16];
      memcpy(s, in, sizeof s);
      for (int r = 0; r < 6; r++) {
        qr(s, 0, 4, 8, 12); qr(s, 1, 5, 9, 13); qr(s, 2, 6, 10, 14); qr(s, 3, 7, 11, 15);
        qr(s, 0, 5, 10, 15); qr(s, 1, 6, 11, 12); qr(s, 2, 7, 8, 13); qr(s, 3, 4, 9, 14);
      }
      for (int i = 0; i < 16; i++) buf[16 * blk + i] = s[i] + in[i];
    }
    ctr += 4;
  }
  uint32_t next_u32() {
    if (idx >= 64) { refill(); idx = 0; }
    return buf[idx++];
  }
  uint64_t next_u64() {  // BlockRng::next_u64: low word first, straddling a refill at index 63
    if (idx < 63) { const uint64_t v = buf[idx] | ((uint64_t)buf[idx + 1] << 32); idx += 2; return v; }
    if (idx >= 64) { refill(); idx = 2; return buf[0] | ((uint64_t)buf[1] << 32); }
    const uint64_t lo = buf[63];
    refill();
    idx = 1;
    return lo | ((uint64_t)buf[0] << 32);
  }
  uint32_t range_incl(uint32_t lo, uint32_t hi) {  // UniformInt::sample_single_inclusive, u32 sampling
    const uint32_t range = hi - lo + 1;
    const uint64_t m = (uint64_t)next_u32() * range;
    uint32_t res = (uint32_t)(m >> 32);
    const uint32_t lo_order = (uint32_t)m;
    if (lo_order > (uint32_t)(0u - range)) {
      const uint32_t nh = (uint32_t)(((uint64_t)next_u32() * range) >> 32);
      if ((uint64_t)lo_order + nh > 0xFFFFFFFFull) res += 1;
    }
    return lo + res;
  }
};

}  // namespace

extern "C" int32_t sezkp_simulate_trace(uint64_t t, uint32_t tau, uint64_t seed, int8_t* input_mv, int8_t* mv,
                                        uint8_t* has_write, uint16_t* wsym) {
  if (tau > 255 || (t && (!input_mv || (tau && (!mv || !has_write || !wsym))))) return SEZKP_E_INVALID;
  // Bernoulli::new(0.4): p_int = (0.4 * 2^64) as u64 (f64 product, truncated)
  const uint64_t p_write = (uint64_t)(0.4 * 18446744073709551616.0);
  StdRng rng(seed);
  for (uint64_t s = 0; s < t; s++) {
    input_mv[s] = (int8_t)((int)rng.range_incl(0, 2) - 1);  // 0 -> -1, 1 -> 0, 2 -> +1
    for (uint32_t k = 0; k < tau; k++) {
      const uint64_t o = s * tau + k;
      const bool w = rng.next_u64() < p_write;
      has_write[o] = w;
      wsym[o] = w ? (uint16_t)rng.range_incl(0, 15) : 0;
      mv[o] = (int8_t)((int)rng.range_incl(0, 2) - 1);
    }
  }
  return SEZKP_OK;
}

namespace sezkp {

void partition_trace(BlockStore& s, uint64_t t, uint32_t tau, uint32_t b, const int8_t* input_mv, const int8_t* mv,
                     const uint8_t* has_write, const uint16_t* wsym) {
  s = BlockStore();
  s.tau = tau;
  const uint64_t nb = (t + b - 1) / b;
  s.step_start.assign(1, 0);
  s.input_mv.assign(input_mv, input_mv + t);
  s.mv.assign(mv, mv + t * tau);
  s.has_write.assign(has_write, has_write + t * tau);
  s.wsym.assign(wsym, wsym + t * tau);
  std::vector<int64_t> cur(tau), lo(tau), hi(tau);
  int64_t gin = 0;
  auto u32_or_max = [](int64_t x) { return (x >= 0 && x <= 0xFFFFFFFFll) ? (uint32_t)x : 0xFFFFFFFFu; };
  for (uint64_t k = 0; k < nb; k++) {
    const uint64_t a = k * b, e = std::min<uint64_t>(a + b, t);
    std::fill(cur.begin(), cur.end(), 0);
    std::fill(lo.begin(), lo.end(), 0);
    std::fill(hi.begin(), hi.end(), 0);
    const int64_t in_head_in = gin;
    for (uint64_t st = a; st < e; st++) {
      gin += input_mv[st];
      for (uint32_t r = 0; r < tau; r++) {
        cur[r] += mv[st * tau + r];
        lo[r] = std::min(lo[r], cur[r]);
        hi[r] = std::max(hi[r], cur[r]);
      }
    }
    s.version.push_back(1);
    s.block_id.push_back((uint32_t)(k + 1));
    s.step_lo.push_back(a + 1);  // 1-based inclusive
    s.step_hi.push_back(e);
    s.ctrl_in.push_back(0);
    s.ctrl_out.push_back(0);
    s.in_head_in.push_back(in_head_in);
    s.in_head_out.push_back(gin);
    for (uint32_t r = 0; r < tau; r++) {
      s.win_left.push_back(lo[r]);
      s.win_right.push_back(hi[r]);
      s.off_in.push_back(u32_or_max(-lo[r]));
      s.off_out.push_back(u32_or_max(cur[r] - lo[r]));
    }
    s.step_start.push_back(e);
  }
  s.bind();
}

}  // namespace sezkp

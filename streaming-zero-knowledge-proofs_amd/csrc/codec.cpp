// codec.cpp — CBOR/JSON decode of Vec<BlockSummary> and manifests, CBOR
// encode of ProofArtifact, manifest commitment. Pull parsers decode straight
// into the struct-of-arrays store (no DOM), so multi-GB block files stream.
#include "codec.h"

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <stdexcept>
#include <system_error>
#include <thread>
#include <type_traits>

#include <emmintrin.h>

#include "host_crypto.h"

namespace sezkp {

void BlockStore::bind() {
  view.n_blocks = (uint32_t)version.size();
  view.tau = tau;
  view.version = version.data();
  view.block_id = block_id.data();
  view.step_lo = step_lo.data();
  view.step_hi = step_hi.data();
  view.ctrl_in = ctrl_in.data();
  view.ctrl_out = ctrl_out.data();
  view.in_head_in = in_head_in.data();
  view.in_head_out = in_head_out.data();
  view.win_left = win_left.data();
  view.win_right = win_right.data();
  view.off_in = off_in.data();
  view.off_out = off_out.data();
  view.step_start = step_start.data();
  view.input_mv = input_mv.data();
  view.mv = mv.data();
  view.has_write = has_write.data();
  view.wsym = wsym.data();
}

namespace {

struct DecodeError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// A map key as it lies in the input (no allocation): compared with literals.
struct Key {
  const char* p = nullptr;
  size_t n = 0;
  bool operator==(const char* lit) const { return strlen(lit) == n && !memcmp(p, lit, n); }
  bool operator!=(const char* lit) const { return !(*this == lit); }
};

// ------------------------------------------------------------- CBOR pull
class Cbor {
 public:
  Cbor(const uint8_t* p, size_t n) : p_(p), e_(p + n) {}
  bool done() const { return p_ == e_; }
  // container start: returns count, or -1 for indefinite length
  int64_t begin_array() { return container(4); }
  int64_t begin_map() { return container(5); }
  bool more(int64_t& remaining) {  // iterate a container
    if (remaining >= 0) return remaining-- > 0;
    need(1);
    if (*p_ == 0xff) { p_++; return false; }
    return true;
  }
  Key key() {
    int mj; uint64_t v; bool ind;
    head(mj, v, ind);
    if (mj != 3 || ind) throw DecodeError("expected text key");
    need(v);
    Key k{(const char*)p_, (size_t)v};
    p_ += v;
    return k;
  }
  bool null() {
    need(1);
    if (*p_ == 0xf6 || *p_ == 0xf7) { p_++; return true; }
    return false;
  }
  int64_t sint() {
    int mj; uint64_t v; bool ind;
    head(mj, v, ind);
    if (mj == 0) { if (v > (uint64_t)INT64_MAX) throw DecodeError("int overflow"); return (int64_t)v; }
    if (mj == 1) { if (v > (uint64_t)INT64_MAX) throw DecodeError("int overflow"); return -1 - (int64_t)v; }
    throw DecodeError("expected integer");
  }
  uint64_t uint() {
    int mj; uint64_t v; bool ind;
    head(mj, v, ind);
    if (mj != 0) throw DecodeError("expected unsigned integer");
    return v;
  }
  std::string text() { const Key k = key(); return std::string(k.p, k.n); }
  void skip() {
    int mj; uint64_t v; bool ind;
    head(mj, v, ind);
    switch (mj) {
      case 0: case 1: case 7: return;
      case 2: case 3:
        if (ind) { while (!brk()) skip(); return; }
        need(v); p_ += v; return;
      case 4: case 5: {
        const int per = mj == 5 ? 2 : 1;
        if (ind) { while (!brk()) for (int i = 0; i < per; i++) skip(); return; }
        for (uint64_t i = 0; i < v * per; i++) skip();
        return;
      }
      case 6: skip(); return;
    }
  }

 private:
  void need(uint64_t k) { if ((uint64_t)(e_ - p_) < k) throw DecodeError("truncated CBOR"); }
  bool brk() { need(1); if (*p_ == 0xff) { p_++; return true; } return false; }
  void head(int& mj, uint64_t& v, bool& ind) {
    need(1);
    uint8_t b = *p_++;
    mj = b >> 5;
    int ai = b & 31;
    ind = false;
    if (ai < 24) { v = ai; return; }
    int nb = ai == 24 ? 1 : ai == 25 ? 2 : ai == 26 ? 4 : ai == 27 ? 8 : 0;
    if (ai == 31) { ind = true; v = 0; return; }
    if (!nb) throw DecodeError("bad CBOR head");
    need(nb);
    v = 0;
    for (int i = 0; i < nb; i++) v = (v << 8) | *p_++;
  }
  int64_t container(int want) {
    int mj; uint64_t v; bool ind;
    head(mj, v, ind);
    if (mj != want) throw DecodeError(want == 4 ? "expected array" : "expected map");
    return ind ? -1 : (int64_t)v;
  }
  const uint8_t* p_;
  const uint8_t* e_;
};

// ------------------------------------------------------------- JSON pull
inline bool js_space(char c) { return c == ' ' || c == '\n' || c == '\r' || c == '\t'; }
inline bool js_digit(char c) { return c >= '0' && c <= '9'; }
class Json {
 public:
  Json(const char* p, size_t n) : p_(p), e_(p + n) {}
  bool done() { ws(); return p_ == e_; }
  int64_t begin_array() { ws(); expect('['); first_ = true; return -1; }
  int64_t begin_map() { ws(); expect('{'); first_ = true; return -1; }
  bool more(int64_t&) {
    ws();
    if (p_ < e_ && (*p_ == ']' || *p_ == '}')) { p_++; first_ = false; return false; }
    if (!first_) { expect(','); ws(); }
    first_ = false;
    return true;
  }
  Key key() {
    ws();
    expect('"');
    const char* b = p_;
    while (p_ < e_ && *p_ != '"' && *p_ != '\\') p_++;
    Key k{b, (size_t)(p_ - b)};
    if (p_ < e_ && *p_ == '\\') {  // escaped key: decode into this parser's buffer
      keybuf_.assign(b, k.n);
      while (p_ < e_ && *p_ != '"') {
        if (*p_ == '\\') { p_++; if (p_ >= e_) break; }
        keybuf_.push_back(*p_++);
      }
      k = Key{keybuf_.data(), keybuf_.size()};
    }
    expect('"');
    ws();
    expect(':');
    first_ = false;
    return k;
  }
  bool null() {
    ws();
    if (e_ - p_ >= 4 && !memcmp(p_, "null", 4)) { p_ += 4; return true; }
    return false;
  }
  int64_t sint() {
    ws();
    bool neg = false;
    if (p_ < e_ && *p_ == '-') { neg = true; p_++; }
    uint64_t v = digits();
    if (v > (uint64_t)INT64_MAX + (neg ? 1 : 0)) throw DecodeError("int overflow");
    return neg ? (int64_t)(0 - v) : (int64_t)v;
  }
  uint64_t uint() { ws(); return digits(); }
  std::string text() { return str(); }
  // Skip an array, counting its elements, without decoding them (string- and
  // bracket-aware scan): the metadata pass of the sliced JSONL ingest.
  uint64_t skip_count_array() {
    ws();
    expect('[');
    ws();
    if (p_ < e_ && *p_ == ']') {
      p_++;
      first_ = false;
      return 0;
    }
    // 64 bytes per step: SSE2 byte masks of '"', '\\', '[' '{', ']' '}' and
    // ',', the in-string mask as the prefix XOR of the quotes (carried across
    // blocks), and only the structural bytes outside strings walked in order.
    // A backslash sends the array to the exact byte scan.
    const char* const start = p_;
    const char* p = p_;
    uint64_t carry = 0, commas = 0;
    int depth = 1;
    auto eq = [](__m128i v, char c) { return _mm_cmpeq_epi8(v, _mm_set1_epi8(c)); };
    while (e_ - p >= 64) {
      uint64_t Q = 0, B = 0, O = 0, C = 0, M = 0;
      for (int i = 0; i < 4; i++) {
        const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 16 * i));
        const int sh = 16 * i;
        Q |= (uint64_t)(uint32_t)_mm_movemask_epi8(eq(v, '"')) << sh;
        B |= (uint64_t)(uint32_t)_mm_movemask_epi8(eq(v, '\\')) << sh;
        O |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_or_si128(eq(v, '['), eq(v, '{'))) << sh;
        C |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_or_si128(eq(v, ']'), eq(v, '}'))) << sh;
        M |= (uint64_t)(uint32_t)_mm_movemask_epi8(eq(v, ',')) << sh;
      }
      if (B) return skip_count_exact(start);
      uint64_t S = Q;  // prefix XOR: bit i = parity of the quotes at or before i
      S ^= S << 1; S ^= S << 2; S ^= S << 4; S ^= S << 8; S ^= S << 16; S ^= S << 32;
      S ^= carry;
      carry = 0 - (S >> 63);
      uint64_t X = (O | C | M) & ~S;
      while (X) {
        const uint64_t bit = X & (0 - X);
        X ^= bit;
        if (O & bit) {
          depth++;
        } else if (C & bit) {
          if (--depth == 0) {
            p_ = p + __builtin_ctzll(bit) + 1;
            first_ = false;
            return commas + 1;
          }
        } else {
          commas += depth == 1;
        }
      }
      p += 64;
    }
    // the last < 64 bytes (no backslash so far): byte by byte from the state
    bool instr = carry & 1;
    while (p < e_) {
      const char c = *p++;
      if (c == '\\') return skip_count_exact(start);
      if (instr) {
        instr = c != '"';
      } else if (c == '"') {
        instr = true;
      } else if (c == '[' || c == '{') {
        depth++;
      } else if (c == ']' || c == '}') {
        if (--depth == 0) {
          p_ = p;
          first_ = false;
          return commas + 1;
        }
      } else if (c == ',') {
        commas += depth == 1;
      }
    }
    throw DecodeError("truncated JSON array");
  }
  // the same count byte by byte with escapes honoured, from the first element
  uint64_t skip_count_exact(const char* start) {
    p_ = start;
    uint64_t commas = 0;
    int depth = 1;
    while (p_ < e_) {
      const char c = *p_++;
      if (c == '"') {
        while (p_ < e_ && *p_ != '"') p_ += *p_ == '\\' ? 2 : 1;
        if (p_ >= e_) break;
        p_++;
      } else if (c == '[' || c == '{') {
        depth++;
      } else if (c == ']' || c == '}') {
        if (--depth == 0) {
          first_ = false;
          return commas + 1;
        }
      } else if (c == ',') {
        commas += depth == 1;
      }
    }
    throw DecodeError("truncated JSON array");
  }
  // Fast paths for the canonical step encoding (serde's field order, no
  // white space: what write_block_summaries_jsonl and the reference write).
  // Each reads one exact form or consumes nothing and returns false, and the
  // general parser then reads the same bytes (any other spacing, field
  // order, value range or a malformed value).
  // {"write":null|N,"mv":M} (a tape op, after more() of the tapes array)
  bool fast_tape_op(int64_t& mv, bool& has, uint64_t& sym) {
    const char* p = p_;
    if (e_ - p < 16 || memcmp(p, "{\"write\":", 9)) return false;
    p += 9;
    if (*p == 'n') {
      if (memcmp(p, "null", 4)) return false;
      p += 4;
      has = false;
      sym = 0;
    } else {
      uint64_t v = 0;
      int nd = 0;
      while (p < e_ && js_digit(*p) && nd < 6) { v = v * 10 + (uint64_t)(*p++ - '0'); nd++; }
      if (nd == 0 || nd == 6 || v > 0xffff) return false;
      has = true;
      sym = v;
    }
    if (e_ - p < 8 || memcmp(p, ",\"mv\":", 6)) return false;
    p += 6;
    const bool neg = *p == '-';
    p += neg;
    int64_t v = 0;
    int nd = 0;
    while (p < e_ && js_digit(*p) && nd < 4) { v = v * 10 + (*p++ - '0'); nd++; }
    if (nd == 0 || nd == 4 || p >= e_ || *p != '}') return false;
    v = neg ? -v : v;
    if (v < -128 || v > 127) return false;
    mv = v;
    p_ = p + 1;
    first_ = false;
    return true;
  }
  // {"input_mv":M,"tapes":[ (a step object up to its first tape op; the
  // tapes array is open as after begin_array)
  bool fast_step_head(int64_t& imv) {
    ws();
    const char* p = p_;
    if (e_ - p < 24 || memcmp(p, "{\"input_mv\":", 12)) return false;
    p += 12;
    const bool neg = *p == '-';
    p += neg;
    int64_t v = 0;
    int nd = 0;
    while (p < e_ && js_digit(*p) && nd < 4) { v = v * 10 + (*p++ - '0'); nd++; }
    if (nd == 0 || nd == 4 || e_ - p < 10 || memcmp(p, ",\"tapes\":[", 10)) return false;
    v = neg ? -v : v;
    if (v < -128 || v > 127) return false;
    imv = v;
    p_ = p + 10;
    first_ = true;
    return true;
  }
  void skip() {
    ws();
    if (p_ >= e_) throw DecodeError("truncated JSON");
    char c = *p_;
    if (c == '"') { str(); return; }
    if (c == '[' || c == '{') {
      int64_t r = c == '[' ? begin_array() : begin_map();
      while (more(r)) { if (c == '{') (void)key(); skip(); }
      return;
    }
    while (p_ < e_ && *p_ != ',' && *p_ != ']' && *p_ != '}' && !js_space(*p_)) p_++;
  }

 private:
  void ws() { while (p_ < e_ && js_space(*p_)) p_++; }
  void expect(char c) {
    ws();
    if (p_ >= e_ || *p_ != c) throw DecodeError(std::string("JSON: expected '") + c + "'");
    p_++;
  }
  uint64_t digits() {
    if (p_ >= e_ || !js_digit(*p_)) throw DecodeError("JSON: expected number");
    uint64_t v = 0;
    while (p_ < e_ && js_digit(*p_)) {
      uint64_t d = *p_++ - '0';
      if (v > (UINT64_MAX - d) / 10) throw DecodeError("JSON: number overflow");
      v = v * 10 + d;
    }
    if (p_ < e_ && (*p_ == '.' || *p_ == 'e' || *p_ == 'E')) throw DecodeError("JSON: non-integer number");
    return v;
  }
  std::string str() {
    ws();
    expect('"');
    std::string s;
    while (p_ < e_ && *p_ != '"') {
      if (*p_ == '\\') { p_++; if (p_ >= e_) break; }
      s.push_back(*p_++);
    }
    expect('"');
    return s;
  }
  const char* p_;
  const char* e_;
  bool first_ = false;
  std::string keybuf_;
};

template <class P>
void decode_tape_op(P& d, BlockStore& s) {
  bool has = false;
  uint64_t sym = 0;
  int64_t mv = 0;
  if constexpr (std::is_same_v<P, Json>) {
    if (d.fast_tape_op(mv, has, sym)) {
      s.mv.push_back((int8_t)mv);
      s.has_write.push_back(has ? 1 : 0);
      s.wsym.push_back(has ? (uint16_t)sym : 0);
      return;
    }
  }
  int64_t r = d.begin_map();
  while (d.more(r)) {
    const Key k = d.key();
    if (k == "write") {
      if (!d.null()) { has = true; sym = d.uint(); if (sym > 0xffff) throw DecodeError("write symbol > u16"); }
    } else if (k == "mv") {
      mv = d.sint();
      if (mv < -128 || mv > 127) throw DecodeError("mv out of i8 range");
    } else {
      d.skip();
    }
  }
  s.mv.push_back((int8_t)mv);
  s.has_write.push_back(has ? 1 : 0);
  s.wsym.push_back(has ? (uint16_t)sym : 0);
}

struct BlockShape {
  std::vector<uint32_t> nwin, nin, nout;
  std::vector<uint32_t> ntape;  // per step
};

// META: the block's fields and its step count only (movement_log.steps is
// counted, not decoded; JSON only)
template <class P, bool META = false>
void decode_block(P& d, BlockStore& s, BlockShape& sh) {
  int64_t r = d.begin_map();
  uint32_t nwin = 0, nin = 0, nout = 0;
  const uint64_t steps_before = s.input_mv.size();
  uint64_t meta_steps = 0;
  s.version.push_back(0); s.block_id.push_back(0); s.step_lo.push_back(0); s.step_hi.push_back(0);
  s.ctrl_in.push_back(0); s.ctrl_out.push_back(0); s.in_head_in.push_back(0); s.in_head_out.push_back(0);
  while (d.more(r)) {
    const Key k = d.key();
    if (k == "version") s.version.back() = (uint16_t)d.uint();
    else if (k == "block_id") s.block_id.back() = (uint32_t)d.uint();
    else if (k == "step_lo") s.step_lo.back() = d.uint();
    else if (k == "step_hi") s.step_hi.back() = d.uint();
    else if (k == "ctrl_in") s.ctrl_in.back() = (uint16_t)d.uint();
    else if (k == "ctrl_out") s.ctrl_out.back() = (uint16_t)d.uint();
    else if (k == "in_head_in") s.in_head_in.back() = d.sint();
    else if (k == "in_head_out") s.in_head_out.back() = d.sint();
    else if (k == "windows") {
      int64_t a = d.begin_array();
      while (d.more(a)) {
        int64_t m = d.begin_map();
        int64_t left = 0, right = 0;
        while (d.more(m)) {
          const Key wk = d.key();
          if (wk == "left") left = d.sint();
          else if (wk == "right") right = d.sint();
          else d.skip();
        }
        s.win_left.push_back(left);
        s.win_right.push_back(right);
        nwin++;
      }
    } else if (k == "head_in_offsets" || k == "head_out_offsets") {
      const bool in = k == "head_in_offsets";
      int64_t a = d.begin_array();
      while (d.more(a)) {
        uint64_t x = d.uint();
        if (x > 0xffffffffULL) throw DecodeError("offset > u32");
        (in ? s.off_in : s.off_out).push_back((uint32_t)x);
        (in ? nin : nout)++;
      }
    } else if (k == "movement_log") {
      int64_t m = d.begin_map();
      while (d.more(m)) {
        const Key mk = d.key();
        if (mk != "steps") { d.skip(); continue; }
        if constexpr (META) {
          meta_steps += d.skip_count_array();
          continue;
        }
        int64_t a = d.begin_array();
        while (d.more(a)) {
          int64_t imv = 0;
          uint32_t ntape = 0;
          int64_t sm = -1;
          bool fast = false;
          if constexpr (std::is_same_v<P, Json>) fast = d.fast_step_head(imv);
          if (fast) {
            int64_t ta = -1;
            while (d.more(ta)) { decode_tape_op(d, s); ntape++; }
          } else {
            sm = d.begin_map();
          }
          while (d.more(sm)) {
            const Key sk = d.key();
            if (sk == "input_mv") {
              imv = d.sint();
              if (imv < -128 || imv > 127) throw DecodeError("input_mv out of i8 range");
            } else if (sk == "tapes") {
              int64_t ta = d.begin_array();
              while (d.more(ta)) { decode_tape_op(d, s); ntape++; }
            } else {
              d.skip();
            }
          }
          s.input_mv.push_back((int8_t)imv);
          sh.ntape.push_back(ntape);
        }
      }
    } else {
      d.skip();  // pre_tags / post_tags / unknown fields
    }
  }
  sh.nwin.push_back(nwin);
  sh.nin.push_back(nin);
  sh.nout.push_back(nout);
  s.step_start.push_back(s.step_start.back() + (META ? meta_steps : s.input_mv.size() - steps_before));
}

void finish_blocks(BlockStore& s, const BlockShape& sh);

template <class P>
void decode_blocks(P& d, BlockStore& s) {
  s.step_start.assign(1, 0);
  BlockShape sh;
  int64_t r = d.begin_array();
  while (d.more(r)) decode_block(d, s, sh);
  if (!d.done()) throw DecodeError("trailing bytes after block array");
  finish_blocks(s, sh);
}

void finish_blocks(BlockStore& s, const BlockShape& sh) {
  // The prover reads tau = blocks[0].windows.len() and indexes every per-block
  // vector and every step's tapes by r < tau (openings.rs:195, columns.rs:258).
  s.tau = sh.nwin.empty() ? 0 : sh.nwin[0];
  for (size_t k = 0; k < sh.nwin.size(); k++)
    if (sh.nwin[k] != s.tau || sh.nin[k] != s.tau || sh.nout[k] != s.tau)
      throw DecodeError("block " + std::to_string(k) + ": windows/head offsets length != tau");
  for (uint32_t t : sh.ntape)
    if (t != s.tau) throw DecodeError("step with tapes.len() != tau");
  s.bind();
}

template <class P>
void decode_manifest(P& d, uint8_t root[32], uint32_t* n_leaves) {
  int64_t r = d.begin_map();
  bool got = false;
  while (d.more(r)) {
    const Key k = d.key();
    if (k == "root") {
      int64_t a = d.begin_array();
      int i = 0;
      while (d.more(a)) {
        uint64_t x = d.uint();
        if (i >= 32 || x > 255) throw DecodeError("manifest root must be 32 bytes");
        root[i++] = (uint8_t)x;
      }
      if (i != 32) throw DecodeError("manifest root must be 32 bytes");
      got = true;
    } else if (k == "n_leaves") {
      uint64_t x = d.uint();
      if (n_leaves) *n_leaves = (uint32_t)x;
    } else {
      d.skip();
    }
  }
  if (!got) throw DecodeError("manifest without root");
}

// ------------------------------------------------------------- CBOR out
void cb_head(std::vector<uint8_t>& o, int major, uint64_t v) {
  const uint8_t m = (uint8_t)(major << 5);
  if (v < 24) { o.push_back(m | (uint8_t)v); return; }
  int nb = v < 256 ? 1 : v < 65536 ? 2 : v < (1ULL << 32) ? 4 : 8;
  o.push_back(m | (uint8_t)(nb == 1 ? 24 : nb == 2 ? 25 : nb == 4 ? 26 : 27));
  for (int i = nb - 1; i >= 0; i--) o.push_back((uint8_t)(v >> (8 * i)));
}
void cb_text(std::vector<uint8_t>& o, const std::string& s) {
  cb_head(o, 3, s.size());
  o.insert(o.end(), s.begin(), s.end());
}
void cb_byte_array(std::vector<uint8_t>& o, const uint8_t* p, size_t n) {  // serde Vec<u8>/[u8;N] -> array of uints
  cb_head(o, 4, n);
  for (size_t i = 0; i < n; i++) {
    if (p[i] < 24) o.push_back(p[i]);
    else { o.push_back(0x18); o.push_back(p[i]); }
  }
}
void sort_meta(std::vector<MetaEntry>& meta) {
  std::sort(meta.begin(), meta.end(), [](const MetaEntry& a, const MetaEntry& b) { return a.key < b.key; });
}

}  // namespace

// Host threads for block-file decoding: SEZKP_HOST_THREADS, else the
// OpenMP budget of the process (OMP_NUM_THREADS), else the hardware, at most
// 64; one thread per >= 4 MB of input.
static unsigned decode_threads(size_t len) {
  unsigned t = 0;
  for (const char* v : {"SEZKP_HOST_THREADS", "OMP_NUM_THREADS"})
    if (!t && getenv(v)) t = (unsigned)atoi(getenv(v));
  if (!t) t = std::thread::hardware_concurrency();
  t = std::min<unsigned>(std::max<unsigned>(t, 1), 64);
  return (unsigned)std::min<size_t>(t, std::max<size_t>(1, len >> 22));
}

// Concatenate the per-range stores (blocks in range order) into `out`.
static void merge_stores(std::vector<BlockStore>& parts, std::vector<BlockShape>& shapes, BlockStore& out, BlockShape& sh) {
  auto cat = [&](auto field) {
    size_t total = 0;
    for (auto& b : parts) total += (b.*field).size();
    (out.*field).reserve(total);
    for (auto& b : parts) (out.*field).insert((out.*field).end(), (b.*field).begin(), (b.*field).end());
  };
  cat(&BlockStore::version); cat(&BlockStore::ctrl_in); cat(&BlockStore::ctrl_out);
  cat(&BlockStore::block_id); cat(&BlockStore::off_in); cat(&BlockStore::off_out);
  cat(&BlockStore::step_lo); cat(&BlockStore::step_hi);
  cat(&BlockStore::in_head_in); cat(&BlockStore::in_head_out);
  cat(&BlockStore::win_left); cat(&BlockStore::win_right);
  cat(&BlockStore::input_mv); cat(&BlockStore::mv); cat(&BlockStore::has_write); cat(&BlockStore::wsym);
  out.step_start.assign(1, 0);
  for (auto& b : parts) {
    const uint64_t base = out.step_start.back();
    for (size_t k = 1; k < b.step_start.size(); k++) out.step_start.push_back(base + b.step_start[k]);
  }
  for (auto& x : shapes) {
    sh.nwin.insert(sh.nwin.end(), x.nwin.begin(), x.nwin.end());
    sh.nin.insert(sh.nin.end(), x.nin.begin(), x.nin.end());
    sh.nout.insert(sh.nout.end(), x.nout.begin(), x.nout.end());
    sh.ntape.insert(sh.ntape.end(), x.ntape.begin(), x.ntape.end());
  }
}

// CBOR Vec<BlockSummary> (io.rs:57-65), one thread: finding the block
// boundaries of a CBOR array takes a pass as long as decoding it (measured:
// a skip pass + 8 decode threads 1.4 s against 0.65 s sequential at T = 2^21).
bool decode_blocks_cbor(const uint8_t* data, size_t len, BlockStore& out, std::string& err) {
  try {
    Cbor d(data, len);
    decode_blocks(d, out);
    return true;
  } catch (const std::exception& e) {
    err = std::string("deserialize CBOR block summaries: ") + e.what();
    return false;
  }
}
bool decode_blocks_json(const char* data, size_t len, BlockStore& out, std::string& err) {
  try {
    Json d(data, len);
    decode_blocks(d, out);
    return true;
  } catch (const std::exception& e) {
    err = std::string("deserialize JSON block summaries: ") + e.what();
    return false;
  }
}
// JSON Lines: one BlockSummary object per line (io_jsonl.rs:43-84); a
// trailing "\r" is trimmed, an empty line is an error naming its line number.
// The file is cut at line ends into one range per host thread; each range
// decodes into its own store, and the stores are concatenated in order. The
// error reported is the one of the lowest failing line, as a sequential
// reader would stop there.
bool decode_blocks_jsonl(const char* data, size_t len, BlockStore& out, std::string& err) {
  const unsigned T = decode_threads(len);
  std::vector<const char*> cut(T + 1, data + len);
  cut[0] = data;
  for (unsigned t = 1; t < T; t++) {
    const char* p = std::max(cut[t - 1], data + len / T * t);
    const char* nl = p < data + len ? static_cast<const char*>(memchr(p, '\n', (size_t)(data + len - p))) : nullptr;
    cut[t] = nl ? nl + 1 : data + len;
  }
  std::vector<BlockStore> parts(T);
  std::vector<BlockShape> shapes(T);
  std::vector<size_t> lines(T, 0), bad_line(T, 0);
  std::vector<std::string> msg(T);
  auto run = [&](unsigned t) {
    BlockStore& s = parts[t];
    s.step_start.assign(1, 0);
    const char* p = cut[t];
    const char* e = cut[t + 1];
    try {
      while (p < e) {
        const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(e - p)));
        const char* end = nl ? nl : e;
        lines[t]++;
        const char* le = end;
        if (le > p && le[-1] == '\r') le--;
        if (le == p) throw DecodeError("empty line");
        Json d(p, (size_t)(le - p));
        decode_block(d, s, shapes[t]);
        if (!d.done()) throw DecodeError("trailing bytes after the block object");
        p = nl ? nl + 1 : e;
      }
    } catch (const std::exception& ex) {
      bad_line[t] = lines[t];
      msg[t] = ex.what();
    }
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < T; t++) {
    try {
      th.emplace_back(run, t);
    } catch (const std::system_error&) {  // no thread to be had: decode the range here
      run(t);
    }
  }
  run(0);
  for (auto& x : th) x.join();
  size_t before = 0;
  for (unsigned t = 0; t < T; t++) {
    if (bad_line[t]) {
      err = "parse jsonl line " + std::to_string(before + bad_line[t]) + ": " + msg[t];
      return false;
    }
    before += lines[t];
  }
  try {
    BlockShape sh;
    merge_stores(parts, shapes, out, sh);
    parts.clear();
    finish_blocks(out, sh);
    return true;
  } catch (const std::exception& ex) {
    err = std::string("deserialize JSONL block summaries: ") + ex.what();
    return false;
  }
}

// Sliced ingest, metadata pass: the lines that START in [cut(lo), cut(hi))
// (cut(x) = just past the first newline at or after byte x; cut(0) = 0,
// cut(len) = len, so P ranks taking [len g/P, len (g+1)/P) cover every line
// once). Every block's fields and step count, not its steps; line_off gets
// each line's byte offset. Step arrays stay empty.
bool decode_blocks_jsonl_meta(const char* data, size_t len, size_t lo, size_t hi, BlockStore& out,
                              std::vector<uint64_t>& line_off, std::string& err, bool steps) {
  auto cut = [&](size_t x) -> size_t {
    if (x == 0) return 0;
    if (x >= len) return len;
    const char* nl = static_cast<const char*>(memchr(data + x, '\n', len - x));
    return nl ? (size_t)(nl - data) + 1 : len;
  };
  const size_t b = cut(lo), e = cut(std::max(lo, hi));
  out = BlockStore{};
  out.step_start.assign(1, 0);
  line_off.clear();
  // one range per host thread, cut at line ends (as decode_blocks_jsonl)
  const unsigned T = decode_threads(e - b);
  std::vector<size_t> rc(T + 1, e);
  rc[0] = b;
  for (unsigned t = 1; t < T; t++) {
    const size_t x = std::max(rc[t - 1], b + (e - b) / T * t);
    const char* nl = x < e ? static_cast<const char*>(memchr(data + x, '\n', e - x)) : nullptr;
    rc[t] = nl ? (size_t)(nl - data) + 1 : e;
  }
  std::vector<BlockStore> parts(T);
  std::vector<BlockShape> shapes(T);
  std::vector<std::vector<uint64_t>> offs(T);
  std::vector<size_t> lines(T, 0);
  std::vector<std::string> msg(T);
  auto run = [&](unsigned t) {
    BlockStore& s = parts[t];
    s.step_start.assign(1, 0);
    size_t p = rc[t];
    const size_t pe = rc[t + 1];
    try {
      while (p < pe) {
        const char* nl = static_cast<const char*>(memchr(data + p, '\n', pe - p));
        const size_t end = nl ? (size_t)(nl - data) : pe;
        lines[t]++;
        size_t le = end;
        if (le > p && data[le - 1] == '\r') le--;
        offs[t].push_back(p);
        if (le == p) throw DecodeError("empty line");
        Json d(data + p, le - p);
        if (steps) decode_block<Json, false>(d, s, shapes[t]);
        else decode_block<Json, true>(d, s, shapes[t]);
        if (!d.done()) throw DecodeError("trailing bytes after the block object");
        p = nl ? end + 1 : pe;
      }
    } catch (const std::exception& ex) {
      msg[t] = ex.what();
      if (msg[t].empty()) msg[t] = "decode error";
    }
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < T; t++) {
    try {
      th.emplace_back(run, t);
    } catch (const std::system_error&) {
      run(t);
    }
  }
  run(0);
  for (auto& x : th) x.join();
  size_t before = 0;
  for (unsigned t = 0; t < T; t++) {
    if (!msg[t].empty()) {
      err = "parse jsonl line at byte " + std::to_string(offs[t].empty() ? rc[t] : offs[t].back()) + " (line " +
            std::to_string(before + lines[t]) + " of the range): " + msg[t];
      return false;
    }
    before += lines[t];
  }
  try {
    BlockShape sh;
    merge_stores(parts, shapes, out, sh);
    for (auto& o : offs) line_off.insert(line_off.end(), o.begin(), o.end());
    if (steps) {
      finish_blocks(out, sh);
      return true;
    }
    out.tau = sh.nwin.empty() ? 0 : sh.nwin[0];
    for (size_t k = 0; k < sh.nwin.size(); k++)
      if (sh.nwin[k] != out.tau || sh.nin[k] != out.tau || sh.nout[k] != out.tau)
        throw DecodeError("block " + std::to_string(k) + ": windows/head offsets length != tau");
    out.bind();
    return true;
  } catch (const std::exception& ex) {
    err = std::string("deserialize JSONL block metadata: ") + ex.what();
    return false;
  }
}

// write_block_summaries_jsonl (io_jsonl.rs:93-106): serde field order, tags zeroed
std::string encode_blocks_jsonl(const sezkp_block_view& v) {
  std::string o;
  const uint32_t tau = v.tau;
  o.reserve((size_t)v.step_start[v.n_blocks] * (40 + 28 * tau) + (size_t)v.n_blocks * 400);
  std::string tag = "[";
  for (int i = 0; i < 16; i++) tag += i ? ",0" : "0";
  tag += "]";
  auto num = [&](long long x) { o += std::to_string(x); };
  for (uint32_t k = 0; k < v.n_blocks; k++) {
    o += "{\"version\":"; num(v.version[k]);
    o += ",\"block_id\":"; num(v.block_id[k]);
    o += ",\"step_lo\":"; o += std::to_string(v.step_lo[k]);
    o += ",\"step_hi\":"; o += std::to_string(v.step_hi[k]);
    o += ",\"ctrl_in\":"; num(v.ctrl_in[k]);
    o += ",\"ctrl_out\":"; num(v.ctrl_out[k]);
    o += ",\"in_head_in\":"; num(v.in_head_in[k]);
    o += ",\"in_head_out\":"; num(v.in_head_out[k]);
    o += ",\"windows\":[";
    for (uint32_t r = 0; r < tau; r++) {
      if (r) o += ",";
      o += "{\"left\":"; num(v.win_left[(size_t)k * tau + r]);
      o += ",\"right\":"; num(v.win_right[(size_t)k * tau + r]);
      o += "}";
    }
    o += "],\"head_in_offsets\":[";
    for (uint32_t r = 0; r < tau; r++) { if (r) o += ","; num(v.off_in[(size_t)k * tau + r]); }
    o += "],\"head_out_offsets\":[";
    for (uint32_t r = 0; r < tau; r++) { if (r) o += ","; num(v.off_out[(size_t)k * tau + r]); }
    o += "],\"movement_log\":{\"steps\":[";
    for (uint64_t s = v.step_start[k]; s < v.step_start[k + 1]; s++) {
      if (s != v.step_start[k]) o += ",";
      o += "{\"input_mv\":"; num(v.input_mv[s]);
      o += ",\"tapes\":[";
      for (uint32_t r = 0; r < tau; r++) {
        const size_t i = (size_t)s * tau + r;
        if (r) o += ",";
        o += "{\"write\":";
        if (v.has_write[i]) num(v.wsym[i]); else o += "null";
        o += ",\"mv\":"; num(v.mv[i]);
        o += "}";
      }
      o += "]}";
    }
    o += "]},\"pre_tags\":[";
    for (uint32_t r = 0; r < tau; r++) { if (r) o += ","; o += tag; }
    o += "],\"post_tags\":[";
    for (uint32_t r = 0; r < tau; r++) { if (r) o += ","; o += tag; }
    o += "]}\n";
  }
  return o;
}

// Vec<BlockSummary> as ciborium writes it (sezkp-core types.rs:116-151, io.rs
// write path): maps with serde field order, minimal-length ints, Option ->
// null, [u8;16] tags -> arrays of uints (zero).
std::vector<uint8_t> encode_blocks_cbor(const sezkp_block_view& v) {
  std::vector<uint8_t> o;
  const uint32_t tau = v.tau;
  o.reserve((size_t)v.step_start[v.n_blocks] * (24 + 12 * tau) + (size_t)v.n_blocks * (200 + 60 * tau));
  auto sint = [&](int64_t x) { if (x >= 0) cb_head(o, 0, (uint64_t)x); else cb_head(o, 1, (uint64_t)(-1 - x)); };
  auto key = [&](const char* k) { cb_text(o, k); };
  static const uint8_t zero_tag[16] = {0};
  cb_head(o, 4, v.n_blocks);
  for (uint32_t k = 0; k < v.n_blocks; k++) {
    cb_head(o, 5, 14);
    key("version"); cb_head(o, 0, v.version[k]);
    key("block_id"); cb_head(o, 0, v.block_id[k]);
    key("step_lo"); cb_head(o, 0, v.step_lo[k]);
    key("step_hi"); cb_head(o, 0, v.step_hi[k]);
    key("ctrl_in"); cb_head(o, 0, v.ctrl_in[k]);
    key("ctrl_out"); cb_head(o, 0, v.ctrl_out[k]);
    key("in_head_in"); sint(v.in_head_in[k]);
    key("in_head_out"); sint(v.in_head_out[k]);
    key("windows"); cb_head(o, 4, tau);
    for (uint32_t r = 0; r < tau; r++) {
      cb_head(o, 5, 2);
      key("left"); sint(v.win_left[(size_t)k * tau + r]);
      key("right"); sint(v.win_right[(size_t)k * tau + r]);
    }
    key("head_in_offsets"); cb_head(o, 4, tau);
    for (uint32_t r = 0; r < tau; r++) cb_head(o, 0, v.off_in[(size_t)k * tau + r]);
    key("head_out_offsets"); cb_head(o, 4, tau);
    for (uint32_t r = 0; r < tau; r++) cb_head(o, 0, v.off_out[(size_t)k * tau + r]);
    key("movement_log"); cb_head(o, 5, 1);
    key("steps"); cb_head(o, 4, v.step_start[k + 1] - v.step_start[k]);
    for (uint64_t st = v.step_start[k]; st < v.step_start[k + 1]; st++) {
      cb_head(o, 5, 2);
      key("input_mv"); sint(v.input_mv[st]);
      key("tapes"); cb_head(o, 4, tau);
      for (uint32_t r = 0; r < tau; r++) {
        const size_t i = (size_t)st * tau + r;
        cb_head(o, 5, 2);
        key("write");
        if (v.has_write[i]) cb_head(o, 0, v.wsym[i]); else o.push_back(0xf6);
        key("mv"); sint(v.mv[i]);
      }
    }
    key("pre_tags"); cb_head(o, 4, tau);
    for (uint32_t r = 0; r < tau; r++) cb_byte_array(o, zero_tag, 16);
    key("post_tags"); cb_head(o, 4, tau);
    for (uint32_t r = 0; r < tau; r++) cb_byte_array(o, zero_tag, 16);
  }
  return o;
}

bool decode_manifest_cbor(const uint8_t* data, size_t len, uint8_t root[32], uint32_t* n_leaves, std::string& err) {
  try {
    Cbor d(data, len);
    decode_manifest(d, root, n_leaves);
    return true;
  } catch (const std::exception& e) {
    err = std::string("deserialize CBOR manifest: ") + e.what();
    return false;
  }
}
bool decode_manifest_json(const char* data, size_t len, uint8_t root[32], uint32_t* n_leaves, std::string& err) {
  try {
    Json d(data, len);
    decode_manifest(d, root, n_leaves);
    return true;
  } catch (const std::exception& e) {
    err = std::string("deserialize JSON manifest: ") + e.what();
    return false;
  }
}

bool decode_artifact_cbor(const uint8_t* data, size_t len, Artifact& out, std::string& err) {
  try {
    Cbor d(data, len);
    int64_t r = d.begin_map();
    while (d.more(r)) {
      const Key k = d.key();
      if (k == "backend") out.backend = d.text();
      else if (k == "manifest_root" || k == "proof_bytes") {
        auto& v = k == "proof_bytes" ? out.proof_bytes : out.manifest_root;
        int64_t a = d.begin_array();
        while (d.more(a)) {
          uint64_t x = d.uint();
          if (x > 255) throw DecodeError("byte > 255");
          v.push_back((uint8_t)x);
        }
      } else d.skip();
    }
    return true;
  } catch (const std::exception& e) {
    err = std::string("deserialize CBOR proof artifact: ") + e.what();
    return false;
  }
}

std::vector<uint8_t> encode_artifact_cbor(const std::string& backend, const uint8_t manifest_root[32],
                                          const std::vector<uint8_t>& proof, std::vector<MetaEntry> meta) {
  std::vector<uint8_t> o;
  o.reserve(proof.size() * 2 + 256);
  cb_head(o, 5, 4);
  cb_text(o, "backend");
  cb_text(o, backend);
  cb_text(o, "manifest_root");
  cb_byte_array(o, manifest_root, 32);
  cb_text(o, "proof_bytes");
  cb_byte_array(o, proof.data(), proof.size());
  cb_text(o, "meta");
  sort_meta(meta);
  cb_head(o, 5, meta.size());
  for (auto& m : meta) {
    cb_text(o, m.key);
    if (m.is_str) cb_text(o, m.s);
    else cb_head(o, 0, m.u);
  }
  return o;
}

std::string meta_to_json(std::vector<MetaEntry> meta) {
  sort_meta(meta);
  std::string s = "{";
  for (size_t i = 0; i < meta.size(); i++) {
    if (i) s += ",";
    s += "\"" + meta[i].key + "\":";
    s += meta[i].is_str ? "\"" + meta[i].s + "\"" : std::to_string(meta[i].u);
  }
  return s + "}";
}

std::vector<uint8_t> encode_manifest_cbor(const uint8_t root[32], uint32_t n_leaves) {
  std::vector<uint8_t> o;
  cb_head(o, 5, 3);
  cb_text(o, "version");
  cb_head(o, 0, 1);
  cb_text(o, "root");
  cb_byte_array(o, root, 32);
  cb_text(o, "n_leaves");
  cb_head(o, 0, n_leaves);
  return o;
}

// ----------------------------------------------------------------- manifest
void manifest_leaf_hash(const sezkp_block_view& v, uint32_t k, uint8_t out[32]) {
  BinWriter w;  // raw little-endian fields (sezkp-merkle/src/lib.rs:85-117)
  const uint32_t tau = v.tau;
  auto u16 = [&](uint16_t x) { w.raw(&x, 2); };
  auto u32 = [&](uint32_t x) { w.raw(&x, 4); };
  u16(v.version[k]);
  u32(v.block_id[k]);
  w.u64(v.step_lo[k]);
  w.u64(v.step_hi[k]);
  u16(v.ctrl_in[k]);
  u16(v.ctrl_out[k]);
  w.u64((uint64_t)v.in_head_in[k]);
  w.u64((uint64_t)v.in_head_out[k]);
  w.u64(tau);
  for (uint32_t r = 0; r < tau; r++) {
    w.u64((uint64_t)v.win_left[(size_t)k * tau + r]);
    w.u64((uint64_t)v.win_right[(size_t)k * tau + r]);
  }
  for (uint32_t r = 0; r < tau; r++) u32(v.off_in[(size_t)k * tau + r]);
  for (uint32_t r = 0; r < tau; r++) u32(v.off_out[(size_t)k * tau + r]);
  w.u64(v.step_start[k + 1] - v.step_start[k]);
  blake3_oneshot(w.b.data(), w.b.size(), out);
}

void manifest_root(const sezkp_block_view& v, uint8_t out[32]) {  // lib.rs:140-157, odd promotion
  std::vector<uint8_t> lv(32ull * v.n_blocks);
  for (uint32_t k = 0; k < v.n_blocks; k++) manifest_leaf_hash(v, k, lv.data() + 32ull * k);
  merkle_root_of_leaves(lv.data(), v.n_blocks, false, out);
}

void merkle_root_of_leaves(const uint8_t* leaves, size_t nleaves, bool frontier, uint8_t out[32]) {
  if (frontier) {
    frontier_root_of_leaves(leaves, nleaves, out);
    return;
  }
  if (nleaves == 0) { memset(out, 0, 32); return; }
  std::vector<uint8_t> lv(leaves, leaves + 32 * nleaves);
  size_t n = nleaves;
  while (n > 1) {
    size_t m = 0;
    for (size_t i = 0; i < n; i += 2, m++) {
      if (i + 1 < n) blake3_oneshot(lv.data() + 32 * i, 64, lv.data() + 32 * m);
      else memmove(lv.data() + 32 * m, lv.data() + 32 * i, 32);
    }
    n = m;
  }
  memcpy(out, lv.data(), 32);
}

// The streaming commitment the reference uses for .jsonl/.ndjson block files
// (commit_block_file / verify_block_file_against_manifest, lib.rs:259-330):
// Frontier::push_leaf (lib.rs:173-193) carries a leaf up through the occupied
// levels like a binary counter; finalize_root (lib.rs:195-207) then folds the
// leftover levels top-down as parent(higher, lower). That equals the batch root
// only when every fold pairs equal-height subtrees; at 7, 11, 13, 14, 15, 19 ...
// leaves it does not, and the reference commits this value, so it
// is restated as written.
void manifest_frontier_root(const sezkp_block_view& v, uint8_t out[32]) {
  std::vector<uint8_t> lv(32ull * v.n_blocks);
  for (uint32_t k = 0; k < v.n_blocks; k++) manifest_leaf_hash(v, k, lv.data() + 32ull * k);
  frontier_root_of_leaves(lv.data(), v.n_blocks, out);
}

void frontier_root_of_leaves(const uint8_t* leaves, size_t nleaves, uint8_t out[32]) {
  uint8_t level[64][32];  // level[l]: the pending 2^l-leaf subtree root (bit l of the count)
  uint64_t occupied = 0;
  uint8_t node[64];       // left || right of one parent
  for (size_t k = 0; k < nleaves; k++) {
    uint8_t h[32];
    memcpy(h, leaves + 32 * k, 32);
    int l = 0;
    while (occupied >> l & 1) {  // a waiting left sibling: merge and carry
      memcpy(node, level[l], 32);
      memcpy(node + 32, h, 32);
      blake3_oneshot(node, 64, h);
      occupied &= ~(1ull << l);
      l++;
    }
    memcpy(level[l], h, 32);
    occupied |= 1ull << l;
  }
  if (!occupied) { memset(out, 0, 32); return; }
  int l = 63 - __builtin_clzll(occupied);
  uint8_t acc[32];
  memcpy(acc, level[l], 32);
  while (l-- > 0) {
    if (!(occupied >> l & 1)) continue;
    memcpy(node, acc, 32);
    memcpy(node + 32, level[l], 32);
    blake3_oneshot(node, 64, acc);
  }
  memcpy(out, acc, 32);
}

}  // namespace sezkp

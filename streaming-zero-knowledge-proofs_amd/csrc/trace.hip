// trace.hip — trace-column kernels for CDNA4 (gfx950): row expansion, chunked
// column commitments, AIR composition and column openings.
//
// Reference semantics:
//  * columns (3+7*tau, label order openings.rs:89-116) with RowIter values
//    (openings.rs:227-273; == TraceColumns::build columns.rs:252-365)
//  * labelled leaf BLAKE3("col_leaf"||u32 len||label||v LE) (merkle.rs:132-147)
//  * 1024-row chunk trees + outer tree over chunk roots (openings.rs:306-398)
//  * composition C(i) = compose_row + compose_boundary (air.rs:49-136) with the
//    alpha reuse of prover.rs:86-98, plus the cubic mask R(w_n^i)
//    (masking.rs:86-103, prover.rs:142-158)
//  * openings (openings.rs:403-497): value, chunk root, path in chunk, path of
//    the chunk root in the outer tree.
#include <type_traits>

#include "dev_common.h"
#include "col_leaf.h"
#include "sezkp_internal.h"
#include "compose.h"

namespace sezkp {

constexpr int TR_THREADS = 256;

// ------------------------------------------------------------ trace image
// The block view's step arrays are row-major [n][tau]; the kernels read them
// tape-major [tau][n]. One lane per row: the lane's tau cells are adjacent on
// the read side, and a wave's stores to one tape are 64 consecutive cells.
// wsym is zeroed where has_write is false (the reference reads the
// symbol only under the flag: `op.write.unwrap_or(0)`, columns.rs:71-72).
__global__ void __launch_bounds__(TR_THREADS) k_trace_image(const int8_t* __restrict__ raw_mv,
                                                          const uint8_t* __restrict__ raw_hw,
                                                          const uint16_t* __restrict__ raw_ws, uint64_t n, int tau,
                                                          int8_t* __restrict__ mv, uint8_t* __restrict__ wf,
                                                          uint16_t* __restrict__ ws, uint64_t r0, uint64_t r1) {
  const uint64_t s = r0 + (uint64_t)blockIdx.x * TR_THREADS + threadIdx.x;
  if (s >= r1) return;
  const size_t i0 = (size_t)s * tau;
  for (int r = 0; r < tau; r++) {
    const size_t o = (size_t)r * n + s;
    const bool w = raw_hw[i0 + r] != 0;
    mv[o] = raw_mv[i0 + r];
    wf[o] = w ? 1 : 0;
    ws[o] = w ? raw_ws[i0 + r] : 0;
  }
}

// tau = 8 (the headline shape): a lane takes 8 consecutive steps, loads their
// 64 + 64 + 128 raw bytes as 16-byte vectors, transposes the 8 x 8 byte /
// u16 matrices in registers (three XOR-swap stages, 64-bit words) and stores
// 8 bytes / 16 bytes per tape: the same image as k_trace_image with wide
// coalesced accesses instead of byte loads and stores.
__device__ __forceinline__ void swap_bits(uint64_t& a, uint64_t& b, int sh, uint64_t m) {
  const uint64_t t = ((a >> sh) ^ b) & m;
  a ^= t << sh;
  b ^= t;
}
__device__ __forceinline__ void transpose8x8_u8(uint64_t (&r)[8]) {
#pragma unroll
  for (int i = 0; i < 4; i++) swap_bits(r[i], r[i + 4], 32, 0x00000000FFFFFFFFull);
#pragma unroll
  for (int i = 0; i < 8; i++)
    if ((i & 2) == 0) swap_bits(r[i], r[i + 2], 16, 0x0000FFFF0000FFFFull);
#pragma unroll
  for (int i = 0; i < 8; i += 2) swap_bits(r[i], r[i + 1], 8, 0x00FF00FF00FF00FFull);
}
// rows of 8 u16 as (lo = elements 0..3, hi = 4..7)
__device__ __forceinline__ void transpose8x8_u16(uint64_t (&lo)[8], uint64_t (&hi)[8]) {
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t t = hi[i];
    hi[i] = lo[i + 4];
    lo[i + 4] = t;
  }
#pragma unroll
  for (int i = 0; i < 8; i++)
    if ((i & 2) == 0) {
      swap_bits(lo[i], lo[i + 2], 32, 0x00000000FFFFFFFFull);
      swap_bits(hi[i], hi[i + 2], 32, 0x00000000FFFFFFFFull);
    }
#pragma unroll
  for (int i = 0; i < 8; i += 2) {
    swap_bits(lo[i], lo[i + 1], 16, 0x0000FFFF0000FFFFull);
    swap_bits(hi[i], hi[i + 1], 16, 0x0000FFFF0000FFFFull);
  }
}
// bytes -> 0 / 1 (any nonzero byte is a write)
__device__ __forceinline__ uint64_t bytes_nonzero(uint64_t x) {
  x |= x >> 4;
  x |= x >> 2;
  x |= x >> 1;
  return x & 0x0101010101010101ull;
}
// 4 bytes of 0 / 1 (low half of b) -> 4 u16 masks of 0 / 0xFFFF
__device__ __forceinline__ uint64_t spread_mask16(uint32_t b) {
  const uint64_t s = (uint64_t)(b & 0xFF) | ((uint64_t)(b & 0xFF00) << 8) | ((uint64_t)(b & 0xFF0000) << 16) |
                     ((uint64_t)(b & 0xFF000000u) << 24);
  return (s << 16) - s;
}
__global__ void __launch_bounds__(TR_THREADS) k_trace_image8(const int8_t* __restrict__ raw_mv,
                                                           const uint8_t* __restrict__ raw_hw,
                                                           const uint16_t* __restrict__ raw_ws, uint64_t n,
                                                           int8_t* __restrict__ mv, uint8_t* __restrict__ wf,
                                                           uint16_t* __restrict__ ws, uint64_t r0, uint64_t r1) {
  // rows [r0, r1): r0 a multiple of 8
  const uint64_t s0 = r0 + ((uint64_t)blockIdx.x * TR_THREADS + threadIdx.x) * 8;
  if (s0 >= r1) return;
  if (s0 + 8 > r1) {  // ragged tail: element by element
    for (uint64_t s = s0; s < r1; s++)
      for (int r = 0; r < 8; r++) {
        const bool w = raw_hw[s * 8 + r] != 0;
        mv[(uint64_t)r * n + s] = raw_mv[s * 8 + r];
        wf[(uint64_t)r * n + s] = w ? 1 : 0;
        ws[(uint64_t)r * n + s] = w ? raw_ws[s * 8 + r] : 0;
      }
    return;
  }
  uint64_t m[8], h[8], wl[8], wh[8];
  {
    const uint4* pm = reinterpret_cast<const uint4*>(raw_mv + s0 * 8);
    const uint4* ph = reinterpret_cast<const uint4*>(raw_hw + s0 * 8);
    const uint4* pw = reinterpret_cast<const uint4*>(raw_ws + s0 * 8);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint4 a = pm[q], b = ph[q];
      m[2 * q] = (uint64_t)a.x | ((uint64_t)a.y << 32);
      m[2 * q + 1] = (uint64_t)a.z | ((uint64_t)a.w << 32);
      h[2 * q] = (uint64_t)b.x | ((uint64_t)b.y << 32);
      h[2 * q + 1] = (uint64_t)b.z | ((uint64_t)b.w << 32);
    }
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint4 c = pw[q];
      wl[q] = (uint64_t)c.x | ((uint64_t)c.y << 32);
      wh[q] = (uint64_t)c.z | ((uint64_t)c.w << 32);
    }
  }
  // mask the symbols of steps that write nothing (row = step here)
#pragma unroll
  for (int i = 0; i < 8; i++) {
    h[i] = bytes_nonzero(h[i]);
    wl[i] &= spread_mask16((uint32_t)h[i]);
    wh[i] &= spread_mask16((uint32_t)(h[i] >> 32));
  }
  transpose8x8_u8(m);
  transpose8x8_u8(h);
  transpose8x8_u16(wl, wh);
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const uint64_t o = (uint64_t)r * n + s0;
    *reinterpret_cast<uint64_t*>(mv + o) = m[r];
    *reinterpret_cast<uint64_t*>(wf + o) = h[r];
    *reinterpret_cast<uint4*>(ws + o) =
        make_uint4((uint32_t)wl[r], (uint32_t)(wl[r] >> 32), (uint32_t)wh[r], (uint32_t)(wh[r] >> 32));
  }
}

// ------------------------------------------------------------ expansion
// One workgroup per block: row -> block id, first/last flags, and the
// post-move head prefix sums per tape (head starts at 0 in every block).
// The head columns are stored as i32 (the reference keeps i64 heads,
// air.rs:54): a block whose head leaves the i32 range (more than ~2^24 rows of
// large moves) sets the guard word to GUARD_HEAD_RANGE and the proof fails.
__global__ void __launch_bounds__(TR_THREADS) k_expand(TraceDev T, uint32_t b0, uint32_t* __restrict__ err) {
  const uint32_t b = b0 + blockIdx.x;
  const uint64_t s = T.blk_start[b], e = T.blk_start[b + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (uint64_t r = s + tid; r < e; r += TR_THREADS) {
    T.row_blk[r] = b;
    T.row_flags[r] = (uint8_t)((r == s ? 1 : 0) | (r + 1 == e ? 2 : 0));
  }
  // head = block-local inclusive prefix sum of the tape's moves. One wave per
  // tape (no WG barriers): two rows per lane, 32-bit wave scan (|sum| <= 128
  // rows * 128), 64-bit carry from lane 63. The block's min / max head goes to
  // head_rng, so the dictionary plan need not re-read the head columns.
  for (int tp = wave; tp < T.tau; tp += TR_THREADS / 64) {
    const int8_t* mv = T.mv + (uint64_t)tp * T.n;
    int32_t* hd = T.head + (uint64_t)tp * T.n;
    int64_t carry = 0, lo = INT64_MAX, hi = INT64_MIN;
    // even block start (n is even): a lane's row pair is one 2-byte load and
    // one 8-byte store
    const bool paired = (s & 1) == 0;
    for (uint64_t r0 = s; r0 < e; r0 += 128) {
      const uint64_t r = r0 + 2 * (uint64_t)lane;
      int32_t m0 = 0, m1 = 0;
      if (paired && r + 1 < e) {
        const uint16_t w = *reinterpret_cast<const uint16_t*>(mv + r);
        m0 = (int8_t)(w & 0xFF);
        m1 = (int8_t)(w >> 8);
      } else {
        m0 = r < e ? (int32_t)mv[r] : 0;
        m1 = r + 1 < e ? (int32_t)mv[r + 1] : 0;
      }
      int32_t x = m0 + m1;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      const int64_t h1 = carry + (int64_t)x;  // through row r + 1
      if (r < e) {
        lo = min(lo, h1 - m1);
        hi = max(hi, h1 - m1);
      }
      if (r + 1 < e) {
        lo = min(lo, h1);
        hi = max(hi, h1);
      }
      if (paired && r + 1 < e) {
        *reinterpret_cast<int2*>(hd + r) = make_int2((int32_t)(h1 - m1), (int32_t)h1);
      } else {
        if (r < e) hd[r] = (int32_t)(h1 - m1);
        if (r + 1 < e) hd[r + 1] = (int32_t)h1;
      }
      carry += __shfl(x, 63, 64);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo = min(lo, __shfl_xor(lo, o, 64));
      hi = max(hi, __shfl_xor(hi, o, 64));
    }
    if (lane == 0) {
      T.head_rng[2 * ((uint64_t)tp * T.nblk + b)] = lo;
      T.head_rng[2 * ((uint64_t)tp * T.nblk + b) + 1] = hi;
      if (lo < (int64_t)INT32_MIN || hi > (int64_t)INT32_MAX) atomicOr(err, GUARD_HEAD_RANGE);
    }
  }
}

// ------------------------------------------------------------ column values
// value of column `ct` at `row` (canonical field element)
__device__ __forceinline__ uint64_t col_value(const TraceDev& T, const ColTemplate& ct, uint64_t row) {
  const uint64_t o = (uint64_t)ct.tape * T.n + row;
  switch (ct.kind) {
    case 0: return gl_from_i64(T.input_mv[row]);
    case 1: return T.row_flags[row] & 1;
    case 2: return (T.row_flags[row] >> 1) & 1;
    case 3: return gl_from_i64(T.mv[o]);
    case 4: return T.wflag[o];
    case 5: return T.wsym[o];
    case 6: return gl_from_i64(T.head[o]);
    case 7: return T.blk_winlen[(uint64_t)ct.tape * T.nblk + T.row_blk[row]];
    case 8: return T.blk_offin[(uint64_t)ct.tape * T.nblk + T.row_blk[row]];
    default: return T.blk_offout[(uint64_t)ct.tape * T.nblk + T.row_blk[row]];
  }
}
// 4 consecutive rows (row0 % 4 == 0): vector loads of the narrow columns
__device__ __forceinline__ void col_values4(const TraceDev& T, const ColTemplate& ct, uint64_t row0, uint64_t (&v)[4]) {
  const uint64_t o = (uint64_t)ct.tape * T.n + row0;
  switch (ct.kind) {
    case 0: {
      uint32_t w = *reinterpret_cast<const uint32_t*>(T.input_mv + row0);
#pragma unroll
      for (int j = 0; j < 4; j++) v[j] = gl_from_i64((int8_t)(w >> (8 * j)));
      return;
    }
    case 1:
    case 2: {
      uint32_t w = *reinterpret_cast<const uint32_t*>(T.row_flags + row0);
      const int sh = ct.kind - 1;
#pragma unroll
      for (int j = 0; j < 4; j++) v[j] = (w >> (8 * j + sh)) & 1;
      return;
    }
    case 3: {
      uint32_t w = *reinterpret_cast<const uint32_t*>(T.mv + o);
#pragma unroll
      for (int j = 0; j < 4; j++) v[j] = gl_from_i64((int8_t)(w >> (8 * j)));
      return;
    }
    case 4: {
      uint32_t w = *reinterpret_cast<const uint32_t*>(T.wflag + o);
#pragma unroll
      for (int j = 0; j < 4; j++) v[j] = (w >> (8 * j)) & 0xff;
      return;
    }
    case 5: {
      uint2 w = *reinterpret_cast<const uint2*>(T.wsym + o);
      v[0] = w.x & 0xffff; v[1] = w.x >> 16; v[2] = w.y & 0xffff; v[3] = w.y >> 16;
      return;
    }
    case 6: {
      const int4 a = *reinterpret_cast<const int4*>(T.head + o);
      v[0] = gl_from_i64(a.x); v[1] = gl_from_i64(a.y); v[2] = gl_from_i64(a.z); v[3] = gl_from_i64(a.w);
      return;
    }
    default: {
      const uint64_t* tab = ct.kind == 7 ? T.blk_winlen : (ct.kind == 8 ? T.blk_offin : T.blk_offout);
      tab += (uint64_t)ct.tape * T.nblk;
      uint4 bl = *reinterpret_cast<const uint4*>(T.row_blk + row0);
      v[0] = tab[bl.x]; v[1] = tab[bl.y]; v[2] = tab[bl.z]; v[3] = tab[bl.w];
      return;
    }
  }
}

// labelled leaf with the value at compile-time byte offset OFF (= 12 + len(label))
template <int OFF>
__device__ __forceinline__ void leaf_labeled_t(const ColTemplate& ct, uint64_t v, uint32_t (&out)[8]) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; i++) m[i] = ct.words[i];
  constexpr int W = OFF / 4, B = OFF % 4;
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  if (B == 0) {
    m[W] |= lo;
    m[W + 1] |= hi;
  } else {
    m[W] |= lo << (8 * B);
    m[W + 1] |= (lo >> (32 - 8 * B)) | (hi << (8 * B));
    m[W + 2] |= hi >> (32 - 8 * B);
  }
  b3_hash_block(m, OFF + 8, out);
}
template <int OFF>
__device__ __forceinline__ void leaf_labeled(const ColTemplate& ct, uint64_t v, uint32_t (&out)[8]) {
  if constexpr (OFF == 0) leaf_labeled_rt(ct, v, out);
  else leaf_labeled_t<OFF>(ct, v, out);
}

__device__ __forceinline__ void lds_put8(uint32_t (*lds)[TR_THREADS], int i, const uint32_t (&h)[8]) {
#pragma unroll
  for (int w = 0; w < 8; w++) lds[w][i] = h[w];
}

// 4 consecutive labelled leaves -> level-2 node
template <int OFF>
__device__ __forceinline__ void hash4_labeled(const ColTemplate& ct, const uint64_t (&v)[4], uint32_t (&h)[8]) {
  uint32_t a[8], b[8], p0[8], p1[8];
  leaf_labeled<OFF>(ct, v[0], a);
  leaf_labeled<OFF>(ct, v[1], b);
  b3_parent(a, b, p0);
  leaf_labeled<OFF>(ct, v[2], a);
  leaf_labeled<OFF>(ct, v[3], b);
  b3_parent(a, b, p1);
  b3_parent(p0, p1, h);
}

// -------------------------------------------------------- column tables
// grid (work/256, table columns). Leaf-table columns: entry e -> labelled leaf
// of the raw value e (i8 reinterpreted, u8, u16). Piecewise columns: one lane
// per run value computes U_0..U_10 with U_0 = leaf(v), U_{l+1} = H(U_l || U_l),
// the root of a 2^l-row subtree whose rows all hold v.
__global__ void __launch_bounds__(TR_THREADS) k_col_tables(TraceDev T, const ColTemplate* __restrict__ tmpl,
                                                           const uint32_t* __restrict__ cols, uint32_t* __restrict__ tabs,
                                                           uint32_t blk_lo, uint32_t blk_cnt) {
  const ColTemplate ct = tmpl[cols[blockIdx.y]];
  uint64_t i = (uint64_t)blockIdx.x * TR_THREADS + threadIdx.x;
  uint32_t h[8];
  if (kind_has_leaf_table(ct.kind)) {
    if (i >= (1ULL << ct.tab_log)) return;
    const uint64_t v = (ct.kind == 0 || ct.kind == 3) ? gl_from_i64((int8_t)(uint8_t)i) : i;
    leaf_labeled_rt(ct, v, h);
    node_store(tabs + 8 * (ct.tab + i), h);
    return;
  }
  // per-block constants: only blocks [blk_lo, blk_lo + blk_cnt) (this rank's rows)
  const bool flags = ct.kind == 1 || ct.kind == 2;
  if (flags ? i >= 2 : i >= blk_cnt) return;
  if (!flags) i += blk_lo;
  uint64_t v;
  if (ct.kind == 1 || ct.kind == 2) v = i;
  else {
    const uint64_t* tab = ct.kind == 7 ? T.blk_winlen : (ct.kind == 8 ? T.blk_offin : T.blk_offout);
    v = tab[(uint64_t)ct.tape * T.nblk + i];
  }
  leaf_labeled_rt(ct, v, h);
  uint32_t* o = tabs + 8 * (ct.tab + i * U_LEVELS);
  node_store(o, h);
  for (int l = 1; l < U_LEVELS; l++) {
    b3_parent(h, h, h);
    node_store(o + 8 * l, h);
  }
}

// raw table index of 4 consecutive rows (leaf-table kinds)
__device__ __forceinline__ void col_index4(const TraceDev& T, const ColTemplate& ct, uint64_t row0, uint32_t (&ix)[4]) {
  const uint64_t o = (uint64_t)ct.tape * T.n + row0;
  if (ct.kind == 5) {
    uint2 w = *reinterpret_cast<const uint2*>(T.wsym + o);
    ix[0] = w.x & 0xffff; ix[1] = w.x >> 16; ix[2] = w.y & 0xffff; ix[3] = w.y >> 16;
    return;
  }
  const uint8_t* src = ct.kind == 0 ? reinterpret_cast<const uint8_t*>(T.input_mv) + row0
                     : ct.kind == 3 ? reinterpret_cast<const uint8_t*>(T.mv) + o : T.wflag + o;
  uint32_t w = *reinterpret_cast<const uint32_t*>(src);
#pragma unroll
  for (int j = 0; j < 4; j++) ix[j] = (w >> (8 * j)) & 0xff;
}

// -------------------------------------------------------- column commit
// One 256-lane WG per work item (column, chunk): 1024 rows, 4 rows per lane
// folded to a level-2 node in registers, 8 LDS levels above. Leaf-table
// columns read their 4 leaves from the table (3 compressions per lane instead
// of 7). Writes the chunk root as leaf `chunk` of the column's outer tree.
template <int OFF>
__device__ __forceinline__ void commit_body(const TraceDev& T, const ColTemplate& ct, uint64_t row0, uint32_t (&h)[8]) {
  uint64_t v[4];
  col_values4(T, ct, row0, v);
  hash4_labeled<OFF>(ct, v, h);
}

__global__ void __launch_bounds__(TR_THREADS) k_col_commit(TraceDev T, const ColTemplate* __restrict__ tmpl,
                                                           const uint32_t* __restrict__ work,
                                                           const uint32_t* __restrict__ tabs,
                                                           uint32_t* __restrict__ outer, uint64_t outer_stride) {
  __shared__ uint32_t lds[8][TR_THREADS];
  const int c = work[2 * blockIdx.x];
  const uint64_t ch = work[2 * blockIdx.x + 1];
  const ColTemplate ct = tmpl[c];
  const int tid = threadIdx.x;
  const uint64_t n = T.n;
  const uint64_t cl = n < 1024 ? n : 1024;
  int logcl = 0;
  while ((1ULL << logcl) < cl) logcl++;
  const int logper = logcl < 2 ? logcl : 2;
  const int nact = (int)(cl >> logper);
  if (tid < nact) {
    const uint64_t row0 = (ch << COL_CHUNK_LOG2) + ((uint64_t)tid << logper);
    uint32_t h[8];
    if (logper == 2 && kind_has_leaf_table(ct.kind)) {
      uint32_t ix[4], a[8], b[8], p0[8], p1[8];
      col_index4(T, ct, row0, ix);
      const uint32_t* tb = tabs + 8 * ct.tab;
      node_load(tb + 8 * ix[0], a);
      node_load(tb + 8 * ix[1], b);
      b3_parent(a, b, p0);
      node_load(tb + 8 * ix[2], a);
      node_load(tb + 8 * ix[3], b);
      b3_parent(a, b, p1);
      b3_parent(p0, p1, h);
    } else if (logper == 2) {
      switch (ct.off) {
        case 16: commit_body<16>(T, ct, row0, h); break;
        case 17: commit_body<17>(T, ct, row0, h); break;
        case 18: commit_body<18>(T, ct, row0, h); break;
        case 19: commit_body<19>(T, ct, row0, h); break;
        case 20: commit_body<20>(T, ct, row0, h); break;
        case 21: commit_body<21>(T, ct, row0, h); break;
        case 22: commit_body<22>(T, ct, row0, h); break;
        case 23: commit_body<23>(T, ct, row0, h); break;
        default: commit_body<0>(T, ct, row0, h); break;
      }
    } else if (logper == 1) {
      uint32_t a[8], b[8];
      leaf_labeled_rt(ct, col_value(T, ct, row0), a);
      leaf_labeled_rt(ct, col_value(T, ct, row0 + 1), b);
      b3_parent(a, b, h);
    } else {
      leaf_labeled_rt(ct, col_value(T, ct, row0), h);
    }
    lds_put8(lds, tid, h);
  }
  __syncthreads();
  int cnt = nact;
  while (cnt > 1) {
    const int half = cnt >> 1;
    uint32_t h[8];
    const bool act = tid < half;
    if (act) {
      uint32_t l[8], r[8];
#pragma unroll
      for (int w = 0; w < 8; w++) {
        uint2 p = *reinterpret_cast<const uint2*>(&lds[w][2 * tid]);
        l[w] = p.x;
        r[w] = p.y;
      }
      b3_parent(l, r, h);
    }
    __syncthreads();
    if (act) lds_put8(lds, tid, h);
    __syncthreads();
    cnt = half;
  }
  if (tid < 8) outer[(uint64_t)c * outer_stride * 8 + ch * 8 + tid] = lds[tid][0];
}

// ------------------------------------------- piecewise-constant columns
// One 64-lane WG per chunk, looping over the piecewise columns. A node covering
// rows [a, a+2^l) is pure when its first and last rows lie in the same run
// (same block; for is_first/is_last also the same flag value) and then equals
// the uniform hash U_l(v); only nodes straddling a run boundary are hashed
// from their children, and a node is evaluated only if its parent straddles
// (or it is the chunk root).
// One lane per (piecewise column, chunk). The chunk's rows split into runs
// of one value (a block's rows; for is_first/is_last the flagged row is a run
// of its own); each run piece is cut into maximal aligned dyadic intervals
// [a, a+2^l), whose subtree hash is the table entry U_l(v), and these are
// pushed left to right on a Merkle stack that merges equal-level neighbours
// (always siblings for aligned intervals) — the streaming builder of
// fri_stream.rs:172-218 on pre-hashed uniform subtrees. Compressions per
// chunk = merges = O(run boundaries x levels); the stack lives in LDS.
constexpr int PW_THREADS = 64;
constexpr int PW_STACK = 12;
__global__ void __launch_bounds__(PW_THREADS) k_col_commit_pw(TraceDev T, const ColTemplate* __restrict__ tmpl,
                                                              const uint32_t* __restrict__ pw_cols, int n_pw,
                                                              const uint32_t* __restrict__ chunks, int nchunks,
                                                              const uint32_t* __restrict__ tabs,
                                                              uint32_t* __restrict__ outer, uint64_t outer_stride,
                                                              uint32_t* __restrict__ err) {
  __shared__ uint32_t stk[PW_STACK][8][PW_THREADS];
  const int lane = threadIdx.x;
  const uint64_t item = (uint64_t)blockIdx.x * PW_THREADS + lane;
  if (item >= (uint64_t)n_pw * nchunks) return;
  // column-major items: a wave holds one column, so its lanes walk the same
  // number of runs (flag columns cut every block into 2 runs, others do not)
  const uint32_t c = pw_cols[item / nchunks];
  const uint64_t ch = chunks[item % nchunks];
  const uint32_t kind = tmpl[c].kind;
  const uint32_t* U = tabs + 8 * tmpl[c].tab;
  const uint64_t n = T.n;
  const uint64_t cl = n < 1024 ? n : 1024;
  const uint64_t c0 = ch << COL_CHUNK_LOG2, c1 = c0 + cl;
  int logcl = 0;
  while ((1ULL << logcl) < cl) logcl++;
  uint64_t lvpack = 0;  // 4-bit level of each stack entry
  int sp = 0;
  uint32_t k = T.row_blk[c0];
  uint64_t row = c0;
  while (row < c1) {
    if (k >= T.nblk) { atomicOr(err, 4u); return; }
    const uint64_t bs = T.blk_start[k], be = T.blk_start[k + 1];
    if (be <= row) { k++; continue; }  // empty or finished block
    const uint64_t pe = be < c1 ? be : c1;
    // sub-piece [row, cut) holding one value u (table index)
    uint64_t cut = pe;
    uint32_t u = k;
    if (kind == 1) { u = row == bs ? 1u : 0u; cut = row == bs ? row + 1 : pe; }
    else if (kind == 2) { u = row + 1 == be ? 1u : 0u; cut = (row + 1 < be && pe == be) ? be - 1 : pe; }
    while (row < cut) {
      const uint64_t off = row - c0, len = cut - row;
      int l = off ? __builtin_ctzll(off) : logcl;
      if (l > logcl) l = logcl;
      while ((1ULL << l) > len) l--;
      const uint64_t step = 1ULL << l;
      uint32_t h[8];
      node_load(U + 8 * ((uint64_t)u * U_LEVELS + l), h);
      while (sp > 0 && (int)((lvpack >> (4 * (sp - 1))) & 15) == l) {  // merge with the left sibling
        uint32_t left[8];
#pragma unroll
        for (int w = 0; w < 8; w++) left[w] = stk[sp - 1][w][lane];
        b3_parent(left, h, h);
        sp--;
        l++;
      }
      if (sp >= PW_STACK) { atomicOr(err, 8u); return; }
#pragma unroll
      for (int w = 0; w < 8; w++) stk[sp][w][lane] = h[w];
      lvpack = (lvpack & ~(15ULL << (4 * sp))) | ((uint64_t)l << (4 * sp));
      sp++;
      row += step;
    }
  }
  if (sp != 1) { atomicOr(err, 16u); return; }
#pragma unroll
  for (int w = 0; w < 8; w++) outer[(uint64_t)c * outer_stride * 8 + ch * 8 + w] = stk[0][w][lane];
}

// ------------------------------------------------------------ composition
// C(i) per air.rs:49-136 in two steps. Exact simplifications (flags are 0/1
// by construction, bit columns are boolean): every alpha*flag*(flag-1) and
// alpha*flg*sum(b(b-1)) term is identically zero and is skipped; the bit
// reconstructions equal x & 0xFFFF / x & 0xF of the canonical value. Each
// constraint type shares one alpha across tapes, so its per-tape terms are
// summed first (exactly, as integers where they are small) and multiplied
// once: sum_r a*t_r = a * sum_r t_r in the field.
// k_compose_terms needs only the trace: it runs on the side stream beside
// the column commitments, before the transcript has the alphas, and stores
// the row sums (ComposeTerms); compose_value (compose.h) combines them with
// the alphas and the mask in k_inv_base (fused with the DEEP quotient) or
// k_compose_combine. RW adjacent rows per lane (1, 2 or 4): the lane's mv /
// wflag / wsym / head cells of one tape are single loads, the next row of all
// but the last comes from the group itself. Needs row0 and the row count to
// be multiples of RW (n >= RW).
template <int RW>
__global__ void __launch_bounds__(TR_THREADS) k_compose_terms(TraceDev T, ComposeTerms Tm, uint64_t row0,
                                                              uint64_t row_end) {
  static_assert(RW == 1 || RW == 2 || RW == 4, "1, 2 or 4 rows per lane");
  using Narrow = typename std::conditional<RW == 1, uint8_t,
                                           typename std::conditional<RW == 2, uint16_t, uint32_t>::type>::type;
  using Wide = typename std::conditional<RW == 1, uint16_t,
                                         typename std::conditional<RW == 2, uint32_t, uint64_t>::type>::type;
  const uint64_t n = T.n;
  const uint64_t i = row0 + RW * ((uint64_t)blockIdx.x * TR_THREADS + threadIdx.x);
  if (i >= row_end) return;
  const uint64_t inx = (i + RW) & (n - 1);
  const Narrow flw = *reinterpret_cast<const Narrow*>(T.row_flags + i);
  uint32_t blk[RW];
  bool is_first[RW], is_last[RW];
  if constexpr (RW == 1) {
    blk[0] = T.row_blk[i];
  } else {
#pragma unroll
    for (int j = 0; j < RW; j += 2) {
      const uint2 b2 = *reinterpret_cast<const uint2*>(T.row_blk + i + j);
      blk[j] = b2.x;
      blk[j + 1] = b2.y;
    }
  }
#pragma unroll
  for (int j = 0; j < RW; j++) {
    is_first[j] = (flw >> (8 * j)) & 1;
    is_last[j] = (flw >> (8 * j + 1)) & 1;
  }
  int32_t s_c2[RW], s_sy[RW];
  int64_t s_c3[RW];
  uint64_t s_bf[RW], s_bl[RW], hr_lo[RW], sl_lo[RW];
  uint32_t hr_hi[RW], sl_hi[RW];
#pragma unroll
  for (int j = 0; j < RW; j++) {
    s_c2[j] = s_sy[j] = 0;
    s_c3[j] = 0;
    s_bf[j] = s_bl[j] = hr_lo[j] = sl_lo[j] = 0;
    hr_hi[j] = sl_hi[j] = 0;
  }
  for (int r = 0; r < T.tau; r++) {
    const uint64_t o = (uint64_t)r * n;
    const Narrow mvw = *reinterpret_cast<const Narrow*>(T.mv + o + i);
    const Narrow wfw = *reinterpret_cast<const Narrow*>(T.wflag + o + i);
    const Wide wsw = *reinterpret_cast<const Wide*>(T.wsym + o + i);
    int64_t head[RW + 1];
    if constexpr (RW == 1) {
      head[0] = T.head[o + i];
    } else {
#pragma unroll
      for (int j = 0; j < RW; j += 2) {
        const int2 h2 = *reinterpret_cast<const int2*>(T.head + o + i + j);
        head[j] = h2.x;
        head[j + 1] = h2.y;
      }
    }
    head[RW] = T.head[o + inx];
    int32_t mv[RW + 1];
#pragma unroll
    for (int j = 0; j < RW; j++) mv[j] = (int8_t)((mvw >> (8 * j)) & 0xFF);
    mv[RW] = T.mv[o + inx];
#pragma unroll
    for (int j = 0; j < RW; j++) {
      const uint64_t head_f = gl_from_i64(head[j]);
      // C2: mv(mv-1)(mv+1) = mv^3 - mv  (|mv| <= 128: exact in i32, 8 tapes)
      s_c2[j] += mv[j] * mv[j] * mv[j] - mv[j];
      // C3: (1 - is_last) * (head' - head - mv'), |head| <= 128 n
      if (!is_last[j]) s_c3[j] += head[j + 1] - head[j] - (int64_t)mv[j + 1];
      if ((wfw >> (8 * j)) & 0xFF) {
        uint32_t c;
        // head - sum(head_bits * 2^k)
        hr_lo[j] = add64c(hr_lo[j], head_f & ~0xFFFFULL, c);
        hr_hi[j] += c;
        // slack = (win_len - 1) - head, reconstructed from 16 bits
        const uint64_t winlen = T.blk_winlen[(uint64_t)r * T.nblk + blk[j]];
        const uint64_t slack = gl_sub(gl_sub(winlen, 1), head_f);
        sl_lo[j] = add64c(sl_lo[j], slack & ~0xFFFFULL, c);
        sl_hi[j] += c;
        // symbol 4-bit decomposition
        const int32_t sym = (int32_t)((wsw >> (16 * j)) & 0xFFFF);
        s_sy[j] += sym & ~0xF;
      }
      if (is_first[j]) {
        const uint64_t offin = T.blk_offin[(uint64_t)r * T.nblk + blk[j]];
        s_bf[j] = gl_add(s_bf[j], gl_sub(gl_sub(head_f, gl_from_i64(mv[j])), offin));
      }
      if (is_last[j]) {
        const uint64_t offout = T.blk_offout[(uint64_t)r * T.nblk + blk[j]];
        s_bl[j] = gl_add(s_bl[j], gl_sub(head_f, offout));
      }
    }
  }
  uint64_t hr[RW], sl[RW];
#pragma unroll
  for (int j = 0; j < RW; j++) {
    hr[j] = gl_reduce128(hr_lo[j], hr_hi[j]);
    sl[j] = gl_reduce128(sl_lo[j], sl_hi[j]);
    if (is_first[j]) Tm.bf[blk[j]] = s_bf[j];
    if (is_last[j]) Tm.bl[blk[j]] = s_bl[j];
  }
  if constexpr (RW == 1) {
    Tm.hr[i] = hr[0];
    Tm.sl[i] = sl[0];
    Tm.c3[i] = s_c3[0];
    Tm.c2[i] = s_c2[0];
    Tm.sy[i] = s_sy[0];
  } else {
#pragma unroll
    for (int j = 0; j < RW; j += 2) {
      *reinterpret_cast<ulonglong2*>(Tm.hr + i + j) = make_ulonglong2(hr[j], hr[j + 1]);
      *reinterpret_cast<ulonglong2*>(Tm.sl + i + j) = make_ulonglong2(sl[j], sl[j + 1]);
      *reinterpret_cast<longlong2*>(Tm.c3 + i + j) = make_longlong2(s_c3[j], s_c3[j + 1]);
      *reinterpret_cast<int2*>(Tm.c2 + i + j) = make_int2(s_c2[j], s_c2[j + 1]);
      *reinterpret_cast<int2*>(Tm.sy + i + j) = make_int2(s_sy[j], s_sy[j + 1]);
    }
  }
}

// C(i) for rows [row0, row_end) from the terms (the path without the DEEP
// quotient: per-point DEEP, or fewer than 16 rows)
__global__ void __launch_bounds__(TR_THREADS) k_compose_combine(ComposeTerms Tm, const DevChal* __restrict__ ch,
                                                                NttTables tw, int logn, uint64_t* __restrict__ out,
                                                                uint64_t row0, uint64_t row_end) {
  const uint64_t i = row0 + (uint64_t)blockIdx.x * TR_THREADS + threadIdx.x;
  if (i >= row_end) return;
  const ComposeCoef K = compose_coef(ch);
  const uint64_t e0 = i << (tw.K - logn);
  const uint64_t x = gl_mul(tw.hi[e0 >> tw.S], tw.lo[e0 & ((1ULL << tw.S) - 1)]);  // w_n^i
  out[i] = compose_value(Tm, K, i, x);
}

// ------------------------------------------------ dictionary commitments
// Exact memoization for the dense columns (input_mv, mv, write_flag,
// write_sym, head). Their raw integers lie in a small range [min, min+R) on
// real traces (the AIR constrains mv/input_mv to {-1,0,1} and write_flag to
// {0,1}; symbols come from a small alphabet; heads are block-relative walks).
// The hash of an aligned 2^k-row subtree is a function of its k-tuple of
// codes (raw - min), so tables T_k[e], e = sum_i code_i * R^i (row i of the
// subtree), built level by level (T_0 = labelled leaves, T_{k+1} = H(T_k||T_k)),
// replace the bottom K levels of every chunk tree. K is chosen per column on
// the device from the measured range (cost = table entries + n / 2^K);
// R^(2^K) <= DICT_CAP. Columns whose range is too wide use K = -1 (leaves
// computed per row). The commitment is bit-identical either way.

template <typename Key>
__device__ __forceinline__ const Key* dict_keys(const TraceDev& T, const ColTemplate& ct) {
  const uint64_t o = (uint64_t)ct.tape * T.n;
  if constexpr (sizeof(Key) == 4) return reinterpret_cast<const Key*>(T.head + o);
  else if constexpr (sizeof(Key) == 2) return reinterpret_cast<const Key*>(T.wsym + o);
  else {
    if (ct.kind == 0) return reinterpret_cast<const Key*>(T.input_mv);
    if (ct.kind == 3) return reinterpret_cast<const Key*>(T.mv + o);
    return reinterpret_cast<const Key*>(T.wflag + o);
  }
}
// raw integer of a dense column at `row` (signed for i8 / i64 kinds)
__device__ __forceinline__ int64_t dict_key_at(const TraceDev& T, const ColTemplate& ct, uint64_t row) {
  const uint64_t o = (uint64_t)ct.tape * T.n + row;
  switch (ct.kind) {
    case 0: return T.input_mv[row];
    case 3: return T.mv[o];
    case 4: return T.wflag[o];
    case 5: return T.wsym[o];
    default: return T.head[o];
  }
}

template <typename Key, int CNT>
__device__ __forceinline__ void load_keys(const Key* __restrict__ p, int64_t (&k)[CNT]) {
  constexpr int BYTES = CNT * (int)sizeof(Key);
  if constexpr (BYTES >= 16) {
    constexpr int PER = 16 / (int)sizeof(Key);
#pragma unroll
    for (int q = 0; q < BYTES / 16; q++) {
      const uint4 w = reinterpret_cast<const uint4*>(p)[q];
      const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int i = 0; i < PER; i++) {
        const int bit = i * 8 * (int)sizeof(Key);
        uint64_t raw;
        if constexpr (sizeof(Key) == 8) raw = (uint64_t)ww[bit / 32] | ((uint64_t)ww[bit / 32 + 1] << 32);
        else if constexpr (sizeof(Key) == 4) raw = ww[bit / 32];
        else raw = (ww[bit / 32] >> (bit % 32)) & ((1u << (8 * sizeof(Key))) - 1u);
        k[q * PER + i] = (int64_t)(Key)raw;
      }
    }
  } else if constexpr ((BYTES == 8 || BYTES == 4) && sizeof(Key) < 8) {
    // one 8- or 4-byte load per table node instead of CNT narrow loads: the
    // lanes of a wave sit 2^(6+a) rows apart, so every load instruction
    // touches 64 cache lines and the commit was bound by load issue
    // (mv: 8 byte loads per node, wsym: 4 short loads)
    uint64_t w;
    if constexpr (BYTES == 8) w = *reinterpret_cast<const uint64_t*>(p);
    else w = *reinterpret_cast<const uint32_t*>(p);
#pragma unroll
    for (int i = 0; i < CNT; i++) {
      const int bit = i * 8 * (int)sizeof(Key);
      k[i] = (int64_t)(Key)((w >> bit) & ((1ull << (8 * sizeof(Key))) - 1ull));
    }
  } else {
#pragma unroll
    for (int i = 0; i < CNT; i++) k[i] = (int64_t)p[i];
  }
}

// Node providers for lane_tree: node j of the lane's 2^D nodes. The gathered
// providers also split get() into raw(j) (the node's key bytes, one load)
// and node(raw) (table index, node load) for lane_tree_pf.
template <typename Key, int K>
struct DictNodes {
  const Key* p;           // first row of the lane
  const uint32_t* tab;    // T_K
  int64_t mn;
  uint32_t R;
  static constexpr int CNT = 1 << K;
  static constexpr int BYTES = CNT * (int)sizeof(Key);
  static constexpr int NW = BYTES >= 4 ? BYTES / 4 : 1;
  struct Raw {
    uint32_t w[NW];
  };
  __device__ __forceinline__ void get(int j, uint32_t (&h)[8]) const {
    int64_t k[1 << K];
    load_keys<Key, (1 << K)>(p + ((uint64_t)j << K), k);
    uint32_t idx = 0;
#pragma unroll
    for (int i = (1 << K) - 1; i >= 0; i--) idx = idx * R + (uint32_t)(k[i] - mn);
    node_load(tab + 8 * (uint64_t)idx, h);
  }
  __device__ __forceinline__ Raw raw(int j) const {
    Raw r;
    const Key* q = p + ((uint64_t)j << K);
    if constexpr (BYTES >= 16) {
#pragma unroll
      for (int i = 0; i < BYTES / 16; i++) {
        const uint4 v = reinterpret_cast<const uint4*>(q)[i];
        r.w[4 * i] = v.x; r.w[4 * i + 1] = v.y; r.w[4 * i + 2] = v.z; r.w[4 * i + 3] = v.w;
      }
    } else if constexpr (BYTES == 8) {
      const uint2 v = *reinterpret_cast<const uint2*>(q);
      r.w[0] = v.x; r.w[1] = v.y;
    } else if constexpr (BYTES == 4) {
      r.w[0] = *reinterpret_cast<const uint32_t*>(q);
    } else if constexpr (BYTES == 2) {
      r.w[0] = *reinterpret_cast<const uint16_t*>(q);
    } else {
      r.w[0] = *reinterpret_cast<const uint8_t*>(q);
    }
    return r;
  }
  __device__ __forceinline__ void node(const Raw& r, int, uint32_t (&h)[8]) const {
    uint32_t idx = 0;
#pragma unroll
    for (int i = CNT - 1; i >= 0; i--) {
      int64_t k;
      if constexpr (sizeof(Key) == 8) {
        k = (int64_t)((uint64_t)r.w[2 * i] | ((uint64_t)r.w[2 * i + 1] << 32));
      } else if constexpr (sizeof(Key) == 4) {
        k = (int64_t)(int32_t)r.w[i];
      } else {
        const int bit = i * 8 * (int)sizeof(Key);
        k = (int64_t)(Key)((r.w[bit / 32] >> (bit % 32)) & ((1u << (8 * sizeof(Key))) - 1u));
      }
      idx = idx * R + (uint32_t)(k - mn);
    }
    node_load(tab + 8 * (uint64_t)idx, h);
  }
};
// head delta plan: node j = the 4-row group at row 4j of the lane
struct DeltaNodes {
  const int32_t* hp;      // head, first row of the lane
  const int8_t* mp;       // mv of the same tape
  const uint8_t* fp;      // row_flags (bit 0 = block start)
  const uint32_t* t1;     // T_1
  const uint32_t* td;     // TD
  int64_t mn, dmin;
  uint32_t R, dR;
  __device__ __forceinline__ void get(int j, uint32_t (&h)[8]) const {
    const uint64_t g = (uint64_t)j << 2;
    const uint32_t f = *reinterpret_cast<const uint32_t*>(fp + g);
    const int64_t c0 = hp[g] - mn;
    if (!(f & 0x01010100u)) {
      const uint32_t m = *reinterpret_cast<const uint32_t*>(mp + g);
      const int64_t d1 = (int64_t)(int8_t)(m >> 8) - dmin, d2 = (int64_t)(int8_t)(m >> 16) - dmin,
                    d3 = (int64_t)(int8_t)(m >> 24) - dmin;
      node_load(td + 8 * (uint64_t)(c0 + (int64_t)R * (d1 + (int64_t)dR * (d2 + (int64_t)dR * d3))), h);
    } else {  // a block starts inside the group: two T_1 nodes
      uint32_t a[8], b[8];
      node_load(t1 + 8 * (uint64_t)(c0 + (int64_t)R * (hp[g + 1] - mn)), a);
      node_load(t1 + 8 * (uint64_t)((hp[g + 2] - mn) + (int64_t)R * (hp[g + 3] - mn)), b);
      b3_parent(a, b, h);
    }
  }
  // lane_tree_pf split: flags, moves and the first head of the group (the
  // other three heads are read only in the rare block-start case)
  struct Raw {
    uint32_t f, m;
    int64_t h0;
  };
  __device__ __forceinline__ Raw raw(int j) const {
    const uint64_t g = (uint64_t)j << 2;
    return Raw{*reinterpret_cast<const uint32_t*>(fp + g), *reinterpret_cast<const uint32_t*>(mp + g), hp[g]};
  }
  __device__ __forceinline__ void node(const Raw& r, int j, uint32_t (&h)[8]) const {
    const int64_t c0 = r.h0 - mn;
    if (!(r.f & 0x01010100u)) {
      const int64_t d1 = (int64_t)(int8_t)(r.m >> 8) - dmin, d2 = (int64_t)(int8_t)(r.m >> 16) - dmin,
                    d3 = (int64_t)(int8_t)(r.m >> 24) - dmin;
      node_load(td + 8 * (uint64_t)(c0 + (int64_t)R * (d1 + (int64_t)dR * (d2 + (int64_t)dR * d3))), h);
    } else {
      const uint64_t g = (uint64_t)j << 2;
      uint32_t a[8], b[8];
      node_load(t1 + 8 * (uint64_t)(c0 + (int64_t)R * (hp[g + 1] - mn)), a);
      node_load(t1 + 8 * (uint64_t)((hp[g + 2] - mn) + (int64_t)R * (hp[g + 3] - mn)), b);
      b3_parent(a, b, h);
    }
  }
};
template <typename Key>
struct RawLeaves {
  const Key* p;
  const ColTemplate* ct;
  __device__ __forceinline__ void get(int j, uint32_t (&h)[8]) const {
    leaf_labeled_rt(*ct, gl_from_i64((int64_t)p[j]), h);
  }
};

// Binary-counter Merkle step: node x (index j of the lane's run) merges with
// the pending left siblings s[L], s[L+1], ... while bit L of j is set, then
// waits at its level (or is the root). Template recursion keeps every stack
// index static: the stack stays in registers.
template <int L, int D>
__device__ __forceinline__ void counter_push(uint32_t (&s)[D > 0 ? D : 1][8], uint32_t (&x)[8], int j,
                                             uint32_t (&h)[8]) {
  if constexpr (L == D) {
#pragma unroll
    for (int w = 0; w < 8; w++) h[w] = x[w];
  } else {
    if ((j >> L) & 1) {
      b3_parent(s[L], x, x);
      counter_push<L + 1, D>(s, x, j, h);
    } else {
#pragma unroll
      for (int w = 0; w < 8; w++) s[L][w] = x[w];
    }
  }
}

// Binary-counter Merkle reduction of 2^D consecutive nodes in a rolled loop:
// the stack is indexed statically (merges unrolled per level, branch on the
// uniform loop counter), so code size is D+1 compressions, not 2^(D+1).
template <int D, class Prov>
__device__ __forceinline__ void lane_tree(const Prov& P, uint32_t (&h)[8]) {
  uint32_t s[D > 0 ? D : 1][8];
  for (int j = 0; j < (1 << D); j++) {
    uint32_t x[8];
    P.get(j, x);
    counter_push<0, D>(s, x, j, h);
  }
}
// lane_tree with the gathers software-pipelined: while node j is merged, the
// table node of j + 1 and the key bytes of j + 2 are in flight, so a lane's
// dependent key -> index -> node chain is paid once per lane, not per node
// (the rolled loop of lane_tree issues each node's loads only after the
// previous node's compressions)
template <int D, class Prov>
__device__ __forceinline__ void lane_tree_pf(const Prov& P, uint32_t (&h)[8]) {
  constexpr int N = 1 << D;
  uint32_t s[D > 0 ? D : 1][8];
  uint32_t nx[8];
  typename Prov::Raw k1 = P.raw(0);
  P.node(k1, 0, nx);
  if (N > 1) k1 = P.raw(1);
  for (int j = 0; j < N; j++) {
    uint32_t x[8];
#pragma unroll
    for (int w = 0; w < 8; w++) x[w] = nx[w];
    if (j + 1 < N) P.node(k1, j + 1, nx);
    if (j + 2 < N) k1 = P.raw(j + 2);
    counter_push<0, D>(s, x, j, h);
  }
}

// -------------------------------------------------------- column openings
// Hash of the aligned range [r0, r0 + 2^lw) of a piecewise-constant column:
// the run pieces of k_col_commit_pw (maximal aligned dyadic intervals, U_l
// lookups) merged on this lane's LDS stack. False if the stack overflows or
// the block table is inconsistent (the commitment flags those chunks).
__device__ __forceinline__ bool pw_range_hash(const TraceDev& T, uint32_t kind, const uint32_t* __restrict__ U,
                                              uint64_t r0, int lw, uint32_t (*stk)[8][64], int slot,
                                              uint32_t (&out)[8]) {
  const uint64_t c1 = r0 + (1ULL << lw);
  uint64_t lvpack = 0;
  int sp = 0;
  uint32_t k = T.row_blk[r0];
  uint64_t row = r0;
  while (row < c1) {
    if (k >= T.nblk) return false;
    const uint64_t bs = T.blk_start[k], be = T.blk_start[k + 1];
    if (be <= row) { k++; continue; }
    const uint64_t pe = be < c1 ? be : c1;
    uint64_t cut = pe;
    uint32_t u = k;
    if (kind == 1) { u = row == bs ? 1u : 0u; cut = row == bs ? row + 1 : pe; }
    else if (kind == 2) { u = row + 1 == be ? 1u : 0u; cut = (row + 1 < be && pe == be) ? be - 1 : pe; }
    while (row < cut) {
      const uint64_t off = row - r0, len = cut - row;
      int l = off ? __builtin_ctzll(off) : lw;
      if (l > lw) l = lw;
      while ((1ULL << l) > len) l--;
      const uint64_t step = 1ULL << l;
      uint32_t h[8];
      node_load(U + 8 * ((uint64_t)u * U_LEVELS + l), h);
      while (sp > 0 && (int)((lvpack >> (4 * (sp - 1))) & 15) == l) {
        uint32_t left[8];
#pragma unroll
        for (int w = 0; w < 8; w++) left[w] = stk[sp - 1][w][slot];
        b3_parent(left, h, h);
        sp--;
        l++;
      }
      if (sp >= PW_STACK) return false;
#pragma unroll
      for (int w = 0; w < 8; w++) stk[sp][w][slot] = h[w];
      lvpack = (lvpack & ~(15ULL << (4 * sp))) | ((uint64_t)l << (4 * sp));
      sp++;
      row += step;
    }
  }
  if (sp != 1) return false;
#pragma unroll
  for (int w = 0; w < 8; w++) out[w] = stk[0][w][slot];
  return true;
}

// level-K node of a dictionary column covering rows [row, row + 2^K) (the
// commitment's DictNodes / DeltaNodes for one node)
__device__ __forceinline__ void dict_node_at(const TraceDev& T, const ColTemplate& ct, const DictPlan& P,
                                             const uint32_t* __restrict__ tab, uint64_t row, uint32_t (&h)[8]) {
  if (P.delta) {
    const uint64_t o = (uint64_t)ct.tape * T.n + row;
    DeltaNodes{T.head + o, T.mv + o, T.row_flags + row, tab + 8 * (uint64_t)DICT_CAP, tab + 16 * (uint64_t)DICT_CAP,
               P.min, P.dmin, P.R, P.dR}
        .get(0, h);
    return;
  }
#define SEZKP_DN(KEY)                                                                                           \
  {                                                                                                             \
    const KEY* p = dict_keys<KEY>(T, ct) + row;                                                                 \
    switch (P.K) {                                                                                              \
      case 0: DictNodes<KEY, 0>{p, tab, P.min, P.R}.get(0, h); break;                                           \
      case 1: DictNodes<KEY, 1>{p, tab + 8 * (uint64_t)DICT_CAP, P.min, P.R}.get(0, h); break;                  \
      case 2: DictNodes<KEY, 2>{p, tab + 16 * (uint64_t)DICT_CAP, P.min, P.R}.get(0, h); break;                 \
      case 3: DictNodes<KEY, 3>{p, tab + 24 * (uint64_t)DICT_CAP, P.min, P.R}.get(0, h); break;                 \
      default: DictNodes<KEY, 4>{p, tab + 32 * (uint64_t)DICT_CAP, P.min, P.R}.get(0, h); break;                \
    }                                                                                                           \
  }
  switch (ct.kind) {
    case 0: case 3: SEZKP_DN(int8_t) break;
    case 4: SEZKP_DN(uint8_t) break;
    case 5: SEZKP_DN(uint16_t) break;
    default: SEZKP_DN(int32_t) break;
  }
#undef SEZKP_DN
}

// path_in_chunk siblings at levels glog..9 of a dictionary column, stored by
// the commitment: thread (level, word), one round of loads
__device__ __forceinline__ void copy_dlev_siblings(const uint32_t* __restrict__ lev, uint64_t in, int glog,
                                                   uint32_t* __restrict__ o) {
  const int lvl = glog + (threadIdx.x >> 3), w = threadIdx.x & 7;
  if (lvl < COL_CHUNK_LOG2) o[18 + 8 * lvl + w] = lev[8 * (dlev_base(lvl) + ((in >> lvl) ^ 1)) + w];
}

// One 256-lane WG per request (column, row). Record words: [0,1] value,
// [2..9] chunk_root, [10..89] path_in (<= 10), [90..345] path_to_chunk (<= 32).
//  - piecewise columns: sibling at level l = hash of an aligned 2^l-row range
//    (one lane per level, U_l lookups + merges at run boundaries only);
//  - dictionary columns (K >= 0): siblings below K are table entries T_l,
//    levels K..(6+a)-1 reduce the group's 2^(6+a-K) level-K table nodes in
//    LDS, levels (6+a)..9 were stored by the commitment;
//  - other columns: the chunk (or 64-row group) rebuilt from leaves in LDS.
// Chunk roots come from the stored outer tree (its leaves) for every column
// kind but the rebuilt one, and path_to_chunk from the outer tree.
__global__ void __launch_bounds__(TR_THREADS) k_col_open(TraceDev T, const ColTemplate* __restrict__ tmpl,
                                                         const uint32_t* __restrict__ outer, uint64_t outer_stride,
                                                         int logChunks, const uint32_t* __restrict__ req,
                                                         ProofLayout P, const uint32_t* __restrict__ tabs,
                                                         const uint32_t* __restrict__ dlev,
                                                         const DictPlan* __restrict__ plans,
                                                         const uint32_t* __restrict__ dtabs,
                                                         const DictCol* __restrict__ dcols,
                                                         const uint32_t* __restrict__ count) {
  __shared__ uint32_t lds[8][1024];
  if (count && blockIdx.x >= *count) return;  // grid sized for the most requests a rank can own
  const uint32_t* rq = req + OPEN_REQ_WORDS * (uint64_t)blockIdx.x;
  const int c = rq[0];
  const uint64_t row = (uint64_t)rq[1] | ((uint64_t)rq[2] << 32);
  const uint32_t q = rq[3];     // ordinal of this opening in the proof
  const uint32_t dsel = rq[4];  // dictionary column index (chunk levels stored), or NO_DICT
  const ColTemplate ct = tmpl[c];
  const int tid = threadIdx.x;
  const uint64_t n = T.n;
  const uint64_t ch = row >> COL_CHUNK_LOG2;
  const uint64_t start = ch << COL_CHUNK_LOG2;
  const uint64_t cl = n < 1024 ? n : 1024;
  int logcl = 0;
  while ((1ULL << logcl) < cl) logcl++;
  // Opening record (proof.rs:44-66): value, index, chunk_index, index_in_chunk,
  // chunk_root, path_in_chunk (u64 len + siblings), path_to_chunk (u64 len + siblings)
  const uint32_t qi = q / P.open_per_q, s = q % P.open_per_q;
  uint32_t* qb = P.base + (8 + (uint64_t)qi * P.q_bytes) / 4;
  uint32_t* o = qb + (16 + (uint64_t)s * P.open_bytes) / 4;
  const uint64_t in = row - start;
  if (tid == 0) {
    o[2] = (uint32_t)row; o[3] = (uint32_t)(row >> 32);
    o[4] = (uint32_t)ch; o[5] = (uint32_t)(ch >> 32);
    o[6] = (uint32_t)in; o[7] = 0;
    o[16] = (uint32_t)logcl; o[17] = 0;
    o[18 + 8 * logcl] = (uint32_t)logChunks; o[19 + 8 * logcl] = 0;
    const uint64_t v = col_value(T, ct, row);
    o[0] = (uint32_t)v;
    o[1] = (uint32_t)(v >> 32);
  }
  const uint32_t* ob = outer + (uint64_t)c * outer_stride * 8;
  {  // path_to_chunk from the stored outer tree (all levels kept): thread
     // (level, word), one round of independent loads instead of a dependent
     // load / store per level on 8 lanes
    uint32_t* op = o + 20 + 8 * logcl;
    const int lvl = tid >> 3, w = tid & 7;
    if (lvl < logChunks) op[8 * lvl + w] = ob[8 * (tree_level_off(logChunks, 0, lvl) + ((ch >> lvl) ^ 1)) + w];
  }
  const bool pw = kind_piecewise(ct.kind) && ct.tab != NO_TAB;
  const bool dict = dsel != NO_DICT && logcl == COL_CHUNK_LOG2;
  const int K = dict ? plans[dsel].K : -1;
  if (pw) {
    if (tid < logcl) {
      uint32_t h[8];
      const uint64_t rs = start + (((in >> tid) ^ 1) << tid);
      if (pw_range_hash(T, ct.kind, tabs + 8 * (uint64_t)ct.tab, rs, tid,
                        reinterpret_cast<uint32_t(*)[8][64]>(&lds[0][0]), tid, h)) {
#pragma unroll
        for (int w = 0; w < 8; w++) o[18 + 8 * tid + w] = h[w];
      }
    }
    if (tid < 8) o[8 + tid] = ob[8 * ch + tid];  // chunk root = outer leaf
  } else if (dict && K >= 0) {
    const DictPlan Pl = plans[dsel];
    const uint32_t* tab = dtabs + 8 * dcols[dsel].tab;
    const int glog = DICT_LANE_LOG + (int)plans[dsel].a;
    const int D = glog - K;
    const uint64_t gstart = row & ~((1ULL << glog) - 1);
    for (int j = tid; j < (1 << D); j += TR_THREADS) {
      uint32_t h[8];
      dict_node_at(T, ct, Pl, tab, gstart + ((uint64_t)j << K), h);
#pragma unroll
      for (int w = 0; w < 8; w++) lds[w][j] = h[w];
    }
    if (tid < K) {  // siblings below the table level: T_l[code of the 2^l sibling rows]
      const int l = tid;
      const uint64_t rs = ((row >> l) ^ 1) << l;
      uint64_t idx = 0;
      for (int i = (1 << l) - 1; i >= 0; i--) idx = idx * Pl.R + (uint64_t)(dict_key_at(T, ct, rs + i) - Pl.min);
      const uint32_t* e = tab + 8 * ((uint64_t)l * DICT_CAP + idx);
#pragma unroll
      for (int w = 0; w < 8; w++) o[18 + 8 * l + w] = e[w];
    }
    __syncthreads();
    const uint64_t gin = (row - gstart) >> K;
    int cnt = 1 << D;
    // levels K+1 .. glog-1 of the group (its root, level glog, was stored by
    // the commitment): <= 32 parents, each on a quad of lanes (round 6: the
    // chain is latency-bound; b3_parent_quad)
    for (int lvl = K; lvl < glog; lvl++) {
      const int sib = (int)((gin >> (lvl - K)) ^ 1);
      if (tid < 8) o[18 + 8 * lvl + tid] = lds[tid][sib];
      if (lvl + 1 == glog) break;
      const int half = cnt >> 1;
      const int pq = tid >> 2, qq = tid & 3;
      uint32_t lo = 0, hi = 0;
      if (pq < half) lds_parent_quad(lds, pq, qq, lo, hi);
      __syncthreads();
      if (pq < half) {
        lds[qq][pq] = lo;
        lds[4 + qq][pq] = hi;
      }
      __syncthreads();
      cnt = half;
    }
    const uint32_t* lev = dlev + 8 * ((uint64_t)dsel * (T.n >> COL_CHUNK_LOG2) + ch) * DLEV_NODES;
    copy_dlev_siblings(lev, in, glog, o);
    if (tid < 8) o[8 + tid] = ob[8 * ch + tid];
  } else {
    // rebuild the chunk (or, for a K = -1 dictionary column, its 64-row group)
    const int glog = dict ? DICT_LANE_LOG + (int)plans[dsel].a : logcl;
    const uint64_t gstart = dict ? (row & ~((1ULL << glog) - 1)) : start;
    for (uint64_t i = tid; i < (1ULL << glog); i += TR_THREADS) {
      uint32_t h[8];
      leaf_labeled_rt(ct, col_value(T, ct, gstart + i), h);
#pragma unroll
      for (int w = 0; w < 8; w++) lds[w][i] = h[w];
    }
    __syncthreads();
    const uint64_t gin = row - gstart;
    int cnt = 1 << glog;
    for (int lvl = 0; lvl < glog; lvl++) {
      const int sib = (int)((gin >> lvl) ^ 1);
      if (tid < 8) o[18 + 8 * lvl + tid] = lds[tid][sib];
      const int half = cnt >> 1;
      uint32_t hh[2][8];
      int k = 0;
      for (int p = tid; p < half; p += TR_THREADS, k++) {
        uint32_t a[8], b[8];
#pragma unroll
        for (int w = 0; w < 8; w++) { a[w] = lds[w][2 * p]; b[w] = lds[w][2 * p + 1]; }
        b3_parent(a, b, hh[k]);
      }
      __syncthreads();
      k = 0;
      for (int p = tid; p < half; p += TR_THREADS, k++)
#pragma unroll
        for (int w = 0; w < 8; w++) lds[w][p] = hh[k][w];
      __syncthreads();
      cnt = half;
    }
    if (dict) {
      const uint32_t* lev = dlev + 8 * ((uint64_t)dsel * (T.n >> COL_CHUNK_LOG2) + ch) * DLEV_NODES;
      copy_dlev_siblings(lev, in, glog, o);
      if (tid < 8) o[8 + tid] = ob[8 * ch + tid];  // chunk root = outer leaf
    } else {
      if (tid < 8) o[8 + tid] = lds[tid][0];
    }
  }
}

constexpr int DICT_WG_ROWS = 64 << DICT_LANE_LOG;  // 4096: row0 / nrows alignment of a sliced commit
constexpr int DICT_RANGE_STEP = TR_THREADS * 16;                     // rows per WG sweep

// WG-wide min / max of one column's partial ranges (result valid on tid 0)
__device__ __forceinline__ void reduce_parts(const int64_t* pp, uint32_t nparts, int64_t& lo, int64_t& hi,
                                             int64_t* slo, int64_t* shi) {
  const int tid = threadIdx.x;
  lo = INT64_MAX;
  hi = INT64_MIN;
  for (uint32_t i = tid; i < nparts; i += TR_THREADS) {
    lo = pp[2 * i] < lo ? pp[2 * i] : lo;
    hi = pp[2 * i + 1] > hi ? pp[2 * i + 1] : hi;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t a = __shfl_xor(lo, o, 64), b = __shfl_xor(hi, o, 64);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  if ((tid & 63) == 0) { slo[tid >> 6] = lo; shi[tid >> 6] = hi; }
  __syncthreads();
  for (int w = 0; w < TR_THREADS / 64; w++) {
    lo = slo[w] < lo ? slo[w] : lo;
    hi = shi[w] > hi ? shi[w] : hi;
  }
  __syncthreads();
}

// Table level K by cost: table entries + n / 2^K gathered nodes (one hash
// each). Pricing gathers from tables of > 1 MB higher (they miss the reading
// XCD's L2) was measured slower in round 3: the extra compressions of the
// lower levels cost more than the misses save. (lo, hi): the column's range;
// (mlo, mhi): its tape's move range (head columns, has_mv), for the delta plan.
__device__ __forceinline__ DictPlan make_plan(int64_t lo, int64_t hi, bool has_mv, int64_t mlo, int64_t mhi,
                                              uint64_t n, uint64_t nrows, uint32_t tab_cap) {
  DictPlan P{};
  P.min = lo;
  P.K = -1;
  const uint64_t R = hi >= lo ? (uint64_t)hi - (uint64_t)lo + 1 : 1;
  if (R <= DICT_CAP) {
    P.R = (uint32_t)R;
    // cost of level K: the tables' entries + the nodes this device gathers
    // (nrows, not n: a sharded rank builds the same tables for 1/P of the rows)
    uint64_t best = 2 * nrows, tabcost = 0, sz = R;  // K = -1: nrows leaves + parents
    bool open = true;
    // unrolled: constant pw[] indices keep P in registers (a runtime index put
    // it in scratch memory, and the kernel took ~23 us for 33 tiny workgroups)
#pragma unroll
    for (int k = 0; k < DICT_LEVELS; k++) {
      open = open && (1ULL << k) <= n && sz <= (k ? tab_cap : DICT_CAP);
      if (open) {
        P.pw[k] = (uint32_t)sz;
        tabcost += sz;
        const uint64_t cost = tabcost + (nrows >> k);
        if (cost < best) { best = cost; P.K = k; }
        sz = sz * sz;
      }
    }
#pragma unroll
    for (int k = 0; k < DICT_LEVELS; k++)
      if (k > P.K) P.pw[k] = 0;
    // head delta plan (see DictPlan): 4-row groups from (head, 3 moves)
    const uint64_t dR = mhi >= mlo ? (uint64_t)mhi - (uint64_t)mlo + 1 : 0;
    if (has_mv && P.K <= 1 && n >= 4 && dR && R * R <= tab_cap && dR <= 256 && R * dR * dR * dR <= tab_cap) {
      P.K = 2;
      P.delta = 1;
      P.dmin = mlo;
      P.dR = (uint32_t)dR;
      P.pw[0] = (uint32_t)R;
      P.pw[1] = (uint32_t)(R * R);
      P.pw[2] = (uint32_t)(R * dR * dR * dR);
      for (int k = 3; k < DICT_LEVELS; k++) P.pw[k] = 0;
    }
  }
  // a lane's rows: 2^(6 + a), a = dict_extra(K) lowered one step per halving
  // of the device's rows below 2^22, so the commit has waves enough to fill
  // the chip (one wave per 64-lane WG, 4 per SIMD) on every shape: at 2^21
  // rows the K >= 3 columns take 128 rows per lane, the K = 2 ones 64
  // (round 5: k_col_commit_dict 314 -> 291 us per launch; a second step
  // 306 us, profiles/r05/ab/dict_rows_per_lane_ab{1,2}.txt)
  int a = dict_extra(P.K);
  for (uint64_t r = nrows; r < (1ULL << 22) && a > 0; r <<= 1) a--;
  P.a = (uint32_t)a;
  return P;
}

// per-(column, part) min / max of the raw integers: `sweeps` (1..8) sweeps of
// 16 rows per lane (one 16-byte-or-less load each); parts of 32768 rows keep
// the grid at ~2K workgroups for 2^21 rows, and a device with fewer rows (a
// sharded rank) takes smaller parts, so every column still has ~64 of them
__global__ void __launch_bounds__(TR_THREADS) k_dict_range(TraceDev T, const ColTemplate* __restrict__ tmpl,
                                                           const DictCol* __restrict__ dcols,
                                                           int64_t* __restrict__ part, uint32_t nparts,
                                                           uint64_t row0, uint64_t row_end, int sweeps) {
  __shared__ int64_t slo[TR_THREADS / 64], shi[TR_THREADS / 64];
  const ColTemplate ct = tmpl[dcols[blockIdx.y].col];
  const int tid = threadIdx.x;
  int64_t lo = INT64_MAX, hi = INT64_MIN;
  if (ct.kind == 6) {  // head: the per-block ranges of k_expand over the blocks meeting this part
    const uint64_t prow = (uint64_t)sweeps * DICT_RANGE_STEP;
    const uint64_t p0 = row0 + (uint64_t)blockIdx.x * prow;
    const uint64_t p1 = p0 + prow < row_end ? p0 + prow : row_end;
    const int64_t* hr = T.head_rng + 2 * ((uint64_t)ct.tape * T.nblk);
    for (uint32_t b = T.row_blk[p0] + tid; b <= T.row_blk[p1 - 1]; b += TR_THREADS) {
      lo = hr[2 * b] < lo ? hr[2 * b] : lo;
      hi = hr[2 * b + 1] > hi ? hr[2 * b + 1] : hi;
    }
  } else {  // narrow keys: 32-bit min / max
    int32_t l32 = INT32_MAX, h32 = INT32_MIN;
    for (int sw = 0; sw < sweeps; sw++) {
      const uint64_t r0 = row0 + (uint64_t)blockIdx.x * ((uint64_t)sweeps * DICT_RANGE_STEP) + (uint64_t)sw * DICT_RANGE_STEP +
                          (uint64_t)tid * 16;
      if (r0 >= row_end) break;
      int64_t k[16];
      switch (ct.kind) {
        case 0: case 3: load_keys<int8_t, 16>(dict_keys<int8_t>(T, ct) + r0, k); break;
        case 4: load_keys<uint8_t, 16>(dict_keys<uint8_t>(T, ct) + r0, k); break;
        default: load_keys<uint16_t, 16>(dict_keys<uint16_t>(T, ct) + r0, k); break;
      }
#pragma unroll
      for (int i = 0; i < 16; i++) {
        l32 = min(l32, (int32_t)k[i]);
        h32 = max(h32, (int32_t)k[i]);
      }
    }
    if (l32 <= h32) {
      lo = l32;
      hi = h32;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t a = __shfl_xor(lo, o, 64), b = __shfl_xor(hi, o, 64);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  if ((tid & 63) == 0) { slo[tid >> 6] = lo; shi[tid >> 6] = hi; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < TR_THREADS / 64; w++) {
      lo = slo[w] < lo ? slo[w] : lo;
      hi = shi[w] > hi ? shi[w] : hi;
    }
    int64_t* o = part + 2 * ((uint64_t)blockIdx.y * nparts + blockIdx.x);
    o[0] = lo;
    o[1] = hi;
  }
}

// one WG per dictionary column: reduce the partial ranges (and, for a head
// column, its tape's move ranges) and choose the plan. (Folding this into
// k_dict_range's last workgroup through agent-scope completion counters was
// measured 100 us slower per proof in round 5: the release / acquire cache
// maintenance of ~2000 workgroups disturbs the L2s the commit then gathers from.)
__global__ void __launch_bounds__(TR_THREADS) k_dict_plan(const int64_t* __restrict__ part, uint32_t nparts,
                                                          uint64_t n, uint64_t nrows, const DictCol* __restrict__ dcols,
                                                          DictPlan* __restrict__ plans, uint32_t tab_cap) {
  __shared__ int64_t slo[TR_THREADS / 64], shi[TR_THREADS / 64];
  int64_t lo, hi, mlo = 0, mhi = -1;
  reduce_parts(part + 2 * (uint64_t)blockIdx.x * nparts, nparts, lo, hi, slo, shi);
  const uint32_t mvc = dcols[blockIdx.x].mv;
  if (mvc != NO_DICT) reduce_parts(part + 2 * (uint64_t)mvc * nparts, nparts, mlo, mhi, slo, shi);
  if (threadIdx.x == 0) plans[blockIdx.x] = make_plan(lo, hi, mvc != NO_DICT, mlo, mhi, n, nrows, tab_cap);
}

// entry e of table level `lvl` of one dictionary column
__device__ __forceinline__ void dict_entry(const ColTemplate& ct, const DictCol& dc, const DictPlan& P, uint32_t S,
                                           uint32_t* __restrict__ tabs, int lvl, uint32_t e) {
  uint32_t* tl = tabs + 8 * (dc.tab + (uint64_t)lvl * DICT_CAP);
  uint32_t h[8];
  if (lvl == 2 && P.delta) {  // TD: (head code, 3 move codes) -> H(T_1, T_1)
    const uint32_t* t1 = tl - 8 * (uint64_t)DICT_CAP;
    const int64_t R = P.R, dR = P.dR;
    int64_t c[4];
    c[0] = e % R;
    int64_t rest = e / R;
    bool ok = true;
#pragma unroll
    for (int j = 1; j < 4; j++) {
      c[j] = c[j - 1] + P.dmin + rest % dR;
      rest /= dR;
      ok = ok && c[j] >= 0 && c[j] < R;
    }
    if (!ok) return;  // not a reachable group: never read
    uint32_t a[8], b[8];
    node_load(t1 + 8 * (uint64_t)(c[0] + R * c[1]), a);
    node_load(t1 + 8 * (uint64_t)(c[2] + R * c[3]), b);
    b3_parent(a, b, h);
  } else if (lvl == 0) {
    leaf_labeled_rt(ct, gl_from_i64(P.min + (int64_t)e), h);
  } else {
    const uint32_t* tp = tl - 8 * (uint64_t)DICT_CAP;
    uint32_t a[8], b[8];
    node_load(tp + 8 * (uint64_t)(e % S), a);
    node_load(tp + 8 * (uint64_t)(e / S), b);
    b3_parent(a, b, h);
  }
  node_store(tl + 8 * (uint64_t)e, h);
}

// Table level `lvl` of every dictionary column in one flat index space: each
// WG sizes the level per column from the plans (prefix sums in LDS) and
// grid-strides over all (column, entry) pairs, so a few hundred WGs share the
// big levels evenly and the empty ones cost one plan scan.
constexpr int DICT_FLAT_MAX = 1024;  // columns one WG can index
constexpr int DICT_FLAT_WGS = 2048;  // 8 waves per SIMD for the big levels
__global__ void __launch_bounds__(TR_THREADS) k_dict_level(const ColTemplate* __restrict__ tmpl,
                                                           const DictCol* __restrict__ dcols,
                                                           const DictPlan* __restrict__ plans,
                                                           uint32_t* __restrict__ tabs, int ndict, int lvl) {
  // columns [0, ndict) of the arrays passed (the host offsets them per chunk)
  __shared__ uint32_t off[DICT_FLAT_MAX + 1];
  const int tid = threadIdx.x;
  for (int c = tid; c < ndict; c += TR_THREADS) {
    const DictPlan& P = plans[c];
    uint32_t size = 0;
#pragma unroll
    for (int k = 0; k < DICT_LEVELS; k++)  // static indices only (no scratch copy of P)
      if (k == lvl && lvl <= P.K) size = P.pw[k];
    off[c + 1] = size;
  }
  __syncthreads();
  if (tid == 0) {
    off[0] = 0;
    for (int c = 0; c < ndict; c++) off[c + 1] += off[c];
  }
  __syncthreads();
  const uint32_t total = off[ndict];
  for (uint32_t g = blockIdx.x * TR_THREADS + tid; g < total; g += gridDim.x * TR_THREADS) {
    int lo = 0, hi = ndict;  // column c with off[c] <= g < off[c + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (off[mid] <= g) lo = mid;
      else hi = mid;
    }
    const DictPlan P = plans[lo];
    uint32_t S = 0;
#pragma unroll
    for (int k = 0; k + 1 < DICT_LEVELS; k++)
      if (k + 1 == lvl) S = P.pw[k];
    const DictCol dc = dcols[lo];
    dict_entry(tmpl[dc.col], dc, P, S, tabs, lvl, g - off[lo]);
  }
}

template <typename Key>
__device__ __forceinline__ void dict_lane(const Key* p, const DictPlan& P, const uint32_t* tab,
                                          const ColTemplate* ct, uint32_t (&h)[8]) {
  // a lane covers 2^(6 + a) rows: 2^(6+a-K) table nodes
  const uint32_t* tk = tab + 8 * (uint64_t)DICT_CAP * (P.K > 0 ? P.K : 0);
  switch (P.K * 4 + (int)P.a) {
    case 0 * 4 + 0: lane_tree_pf<6>(DictNodes<Key, 0>{p, tk, P.min, P.R}, h); break;
    case 1 * 4 + 0: lane_tree_pf<5>(DictNodes<Key, 1>{p, tk, P.min, P.R}, h); break;
    case 2 * 4 + 0: lane_tree_pf<4>(DictNodes<Key, 2>{p, tk, P.min, P.R}, h); break;
    case 2 * 4 + 1: lane_tree_pf<5>(DictNodes<Key, 2>{p, tk, P.min, P.R}, h); break;
    case 3 * 4 + 0: lane_tree_pf<3>(DictNodes<Key, 3>{p, tk, P.min, P.R}, h); break;
    case 3 * 4 + 1: lane_tree_pf<4>(DictNodes<Key, 3>{p, tk, P.min, P.R}, h); break;
    case 3 * 4 + 2: lane_tree_pf<5>(DictNodes<Key, 3>{p, tk, P.min, P.R}, h); break;
    case 4 * 4 + 0: lane_tree_pf<2>(DictNodes<Key, 4>{p, tk, P.min, P.R}, h); break;
    case 4 * 4 + 1: lane_tree_pf<3>(DictNodes<Key, 4>{p, tk, P.min, P.R}, h); break;
    case 4 * 4 + 2: lane_tree_pf<4>(DictNodes<Key, 4>{p, tk, P.min, P.R}, h); break;
    default: lane_tree<6>(RawLeaves<Key>{p, ct}, h); break;
  }
}

// 256-lane WG (4 waves) = 2^(llog + 8) rows of one dictionary column: each
// lane folds its 2^llog rows (llog = 6 + a) to one node in registers, and the
// levels llog+1..10 of the WG's chunks are computed from an LDS image by the
// first lanes of the WORKGROUP, so a level of 2^j parents keeps 2^j lanes of
// whole waves busy (128 parents: waves 0-1, the others wait at the barrier
// and leave their SIMD to other workgroups) instead of 32, 16, 8 of one
// wave's 64 lanes (round 5's one-wave workgroups: a third of a wave's issue
// slots at the upper levels went to idle lanes). Levels ping-pong between two
// LDS images: one barrier per level. The chunk roots are written as leaves of
// the column's outer tree. Requires n >= 1024; rows [row0, row_end) may end
// inside a workgroup (small sharded slices): lanes and parents past row_end
// are skipped (their LDS slots hold garbage that feeds only skipped parents).
// (__launch_bounds__(256, 5) for 5 waves per SIMD: 96 VGPRs with 97 spilled to
// scratch, 291-293 vs 280-284 us per launch, round 6: not kept)
constexpr int DICT_WG_LANES = 256;
__global__ void __launch_bounds__(DICT_WG_LANES) k_col_commit_dict(TraceDev T, const ColTemplate* __restrict__ tmpl,
                                                                   const DictCol* __restrict__ dcols,
                                                                   const DictPlan* __restrict__ plans,
                                                                   const uint32_t* __restrict__ tabs,
                                                                   uint32_t* __restrict__ outer, uint64_t outer_stride,
                                                                   uint64_t row0, uint64_t row_end,
                                                                   uint32_t* __restrict__ dlev, int kmin, int kmax) {
  __shared__ uint32_t lds[2][8][DICT_WG_LANES];
  // (XCD-interleaved column orders, so that one XCD's workgroups gather
  // from one column's tables at a time, measured slower in rounds 1 and 3)
  const uint32_t by = blockIdx.y, bx = blockIdx.x;
  const DictCol dc = dcols[by];
  const ColTemplate* ctp = tmpl + dc.col;
  const ColTemplate ct = *ctp;
  const DictPlan P = plans[by];
  if (P.K < kmin || P.K > kmax) return;  // the other launch's column (uniform per WG)
  const uint32_t* tab = tabs + 8 * dc.tab;
  const int lane = threadIdx.x;
  // high-K columns give each lane more rows (fewer LDS levels per row)
  const int a = (int)P.a;
  const int llog = DICT_LANE_LOG + a;  // rows per lane (log2)
  const uint64_t wg_row = row0 + ((uint64_t)bx << (llog + 8));
  if (wg_row >= row_end) return;  // grid is sized for a = 0 (uniform per WG: no barrier is skipped by half a WG)
  const uint64_t lrow = wg_row + ((uint64_t)lane << llog);
  const uint64_t nch_all = T.n >> COL_CHUNK_LOG2;
  uint32_t* dl = dlev + 8 * (uint64_t)by * nch_all * DLEV_NODES;
  if (lrow < row_end) {
    uint32_t h[8];
    switch (ct.kind) {
      case 0: case 3: dict_lane<int8_t>(dict_keys<int8_t>(T, ct) + lrow, P, tab, ctp, h); break;
      case 4: dict_lane<uint8_t>(dict_keys<uint8_t>(T, ct) + lrow, P, tab, ctp, h); break;
      case 5: dict_lane<uint16_t>(dict_keys<uint16_t>(T, ct) + lrow, P, tab, ctp, h); break;
      default:
        if (P.delta) {
          const uint64_t o = (uint64_t)ct.tape * T.n + lrow;
          const DeltaNodes dn{T.head + o, T.mv + o, T.row_flags + lrow, tab + 8 * (uint64_t)DICT_CAP,
                              tab + 16 * (uint64_t)DICT_CAP, P.min, P.dmin, P.R, P.dR};
          if (a == 1) lane_tree_pf<5>(dn, h);  // 4-row groups: 2^(4 + a) per lane
          else lane_tree_pf<4>(dn, h);
        } else {
          dict_lane<int32_t>(dict_keys<int32_t>(T, ct) + lrow, P, tab, ctp, h);
        }
        break;
    }
#pragma unroll
    for (int w = 0; w < 8; w++) lds[0][w][lane] = h[w];
    // chunk levels llog..9 are kept for the openings (DLEV_NODES per chunk)
    node_store(dl + 8 * ((lrow >> COL_CHUNK_LOG2) * DLEV_NODES + dlev_base(llog) +
                         ((lrow >> llog) & ((1u << (COL_CHUNK_LOG2 - llog)) - 1))),
               h);
  }
  __syncthreads();
  int cnt = DICT_WG_LANES, cur = 0;
  for (int lv = llog + 1; lv <= COL_CHUNK_LOG2; lv++) {
    const int half = cnt >> 1;
    // parent `lane` of this level covers rows from prow: skip it past row_end
    const uint64_t prow = wg_row + ((uint64_t)lane << lv);
    if (lane < half && prow < row_end) {
      uint32_t l[8], r[8], h[8];
#pragma unroll
      for (int w = 0; w < 8; w++) {
        const uint2 pr = *reinterpret_cast<const uint2*>(&lds[cur][w][2 * lane]);
        l[w] = pr.x;
        r[w] = pr.y;
      }
      b3_parent(l, r, h);
#pragma unroll
      for (int w = 0; w < 8; w++) lds[cur ^ 1][w][lane] = h[w];
      if (lv < COL_CHUNK_LOG2)
        node_store(dl + 8 * ((prow >> COL_CHUNK_LOG2) * DLEV_NODES + dlev_base(lv) +
                             ((prow >> lv) & ((1u << (COL_CHUNK_LOG2 - lv)) - 1))),
                   h);
    }
    __syncthreads();
    cur ^= 1;
    cnt = half;
  }
  // cnt chunk roots of this WG -> leaves of the column's outer tree
  for (int i = lane; i < cnt * 8; i += DICT_WG_LANES) {
    const uint64_t ch = (wg_row >> COL_CHUNK_LOG2) + (i >> 3);
    if (ch < nch_all && (ch << COL_CHUNK_LOG2) < row_end)
      outer[(uint64_t)dc.col * outer_stride * 8 + ch * 8 + (i & 7)] = lds[cur][i & 7][i >> 3];
  }
}

// ------------------------------------------------------------------ host
hipError_t launch_trace_image(hipStream_t st, const int8_t* raw_mv, const uint8_t* raw_hw, const uint16_t* raw_ws,
                              uint64_t n, int tau, int8_t* mv, uint8_t* wf, uint16_t* ws, uint64_t r0, uint64_t r1) {
  if (r1 > n) r1 = n;
  if (r0 >= r1 || tau <= 0) return hipSuccess;
  if (tau == 8) {
    r0 &= ~7ull;  // the rows in front of the slice are the raw buffer's other contents: never read
    const uint64_t g8 = ((r1 - r0 + 7) / 8 + TR_THREADS - 1) / TR_THREADS;
    if (g8 > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_trace_image8, dim3((unsigned)g8), dim3(TR_THREADS), 0, st, raw_mv, raw_hw, raw_ws, n, mv, wf,
                       ws, r0, r1);
    return hipGetLastError();
  }
  const uint64_t g = (r1 - r0 + TR_THREADS - 1) / TR_THREADS;
  if (g > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_trace_image, dim3((unsigned)g), dim3(TR_THREADS), 0, st, raw_mv, raw_hw, raw_ws, n, tau, mv,
                     wf, ws, r0, r1);
  return hipGetLastError();
}
hipError_t launch_expand(hipStream_t st, const TraceDev& T, uint32_t blk_lo, uint32_t blk_cnt, uint32_t* d_err) {
  if (blk_cnt == 0) return hipSuccess;
  if ((uint64_t)blk_lo + blk_cnt > T.nblk) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_expand, dim3(blk_cnt), dim3(TR_THREADS), 0, st, T, blk_lo, d_err);
  return hipGetLastError();
}
hipError_t launch_col_tables(hipStream_t st, const TraceDev& T, const ColTemplate* d_tmpl, const uint32_t* d_tab_cols,
                             int n_tab_cols, uint64_t max_units, uint32_t* tabs, uint32_t blk_lo, uint32_t blk_cnt) {
  if (n_tab_cols == 0) return hipSuccess;
  if ((uint64_t)blk_lo + blk_cnt > T.nblk) return hipErrorInvalidValue;
  const unsigned gx = (unsigned)((max_units + TR_THREADS - 1) / TR_THREADS);
  hipLaunchKernelGGL(k_col_tables, dim3(gx, n_tab_cols), dim3(TR_THREADS), 0, st, T, d_tmpl, d_tab_cols, tabs, blk_lo,
                     blk_cnt);
  return hipGetLastError();
}
static hipError_t dict_shape_ok(const TraceDev& T, uint64_t row0, uint64_t nrows) {
  if (T.n < (1ULL << COL_CHUNK_LOG2)) return hipErrorInvalidValue;
  if (row0 + nrows > T.n || (nrows != T.n && (row0 % DICT_WG_ROWS || nrows % DICT_WG_ROWS))) return hipErrorInvalidValue;
  return hipSuccess;
}
hipError_t launch_dict_prepare(hipStream_t st, const TraceDev& T, const ColTemplate* d_tmpl, const DictCol* d_dcols,
                               int ndict, int64_t* d_part, DictPlan* d_plans, uint64_t row0, uint64_t nrows,
                               uint32_t tab_cap) {
  if (ndict == 0) return hipSuccess;
  hipError_t e = dict_shape_ok(T, row0, nrows);
  if (e != hipSuccess) return e;
  if (tab_cap == 0 || tab_cap > DICT_CAP) return hipErrorInvalidValue;
  // parts of 1..8 sweeps: ~64 per column (the partial buffer holds n / 4096)
  const int sweeps = (int)std::max<uint64_t>(1, std::min<uint64_t>(8, nrows / (64ull * DICT_RANGE_STEP)));
  const uint64_t prow = (uint64_t)sweeps * DICT_RANGE_STEP;
  const uint32_t nparts = (uint32_t)((nrows + prow - 1) / prow);
  hipLaunchKernelGGL(k_dict_range, dim3(nparts, ndict), dim3(TR_THREADS), 0, st, T, d_tmpl, d_dcols, d_part, nparts,
                     row0, row0 + nrows, sweeps);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_dict_plan, dim3(ndict), dim3(TR_THREADS), 0, st, d_part, nparts, T.n, nrows, d_dcols, d_plans,
                     tab_cap);
  return hipGetLastError();
}
hipError_t launch_dict_levels(hipStream_t st, const ColTemplate* d_tmpl, const DictCol* d_dcols, int ndict,
                              const DictPlan* d_plans, uint32_t* d_dtabs, int lvl_lo, int lvl_hi) {
  if (lvl_lo < 0 || lvl_hi > DICT_LEVELS) return hipErrorInvalidValue;
  for (int l = lvl_lo; l < lvl_hi; l++) {
    // one flat launch per level (and per DICT_FLAT_MAX columns): all WGs
    // share every column's entries
    for (int c0 = 0; c0 < ndict; c0 += DICT_FLAT_MAX) {
      const int nc = ndict - c0 < DICT_FLAT_MAX ? ndict - c0 : DICT_FLAT_MAX;
      hipLaunchKernelGGL(k_dict_level, dim3(DICT_FLAT_WGS), dim3(TR_THREADS), 0, st, d_tmpl, d_dcols + c0,
                         d_plans + c0, d_dtabs, nc, l);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}
hipError_t launch_dict_commit_cols(hipStream_t st, const TraceDev& T, const ColTemplate* d_tmpl,
                                   const DictCol* d_dcols, int ndict, const DictPlan* d_plans,
                                   const uint32_t* d_dtabs, uint32_t* outer_nodes, uint64_t outer_stride_nodes,
                                   uint64_t row0, uint64_t nrows, uint32_t* d_dlev, int kmin, int kmax) {
  if (ndict == 0) return hipSuccess;
  hipError_t e = dict_shape_ok(T, row0, nrows);
  if (e != hipSuccess) return e;
  const uint64_t wg_rows = (uint64_t)DICT_WG_LANES << DICT_LANE_LOG;  // rows of a WG at a = 0
  const unsigned gx = (unsigned)((nrows + wg_rows - 1) / wg_rows);
  hipLaunchKernelGGL(k_col_commit_dict, dim3(gx, ndict), dim3(DICT_WG_LANES), 0, st, T, d_tmpl, d_dcols, d_plans, d_dtabs,
                     outer_nodes, outer_stride_nodes, row0, row0 + nrows, d_dlev, kmin, kmax);
  return hipGetLastError();
}
hipError_t launch_dict_commit(hipStream_t st, const TraceDev& T, const ColTemplate* d_tmpl, const DictCol* d_dcols,
                              int ndict, int64_t* d_part, DictPlan* d_plans, uint32_t* d_dtabs, uint32_t* outer_nodes,
                              uint64_t outer_stride_nodes, uint64_t row0, uint64_t nrows, uint32_t* d_dlev,
                              uint32_t tab_cap) {
  hipError_t e = launch_dict_prepare(st, T, d_tmpl, d_dcols, ndict, d_part, d_plans, row0, nrows, tab_cap);
  if (e == hipSuccess && ndict) e = launch_dict_levels(st, d_tmpl, d_dcols, ndict, d_plans, d_dtabs, 0, DICT_LEVELS);
  if (e == hipSuccess)
    e = launch_dict_commit_cols(st, T, d_tmpl, d_dcols, ndict, d_plans, d_dtabs, outer_nodes, outer_stride_nodes, row0,
                                nrows, d_dlev, -1, DICT_LEVELS);
  return e;
}

hipError_t launch_col_commit(hipStream_t st, const TraceDev& T, const ColTemplate* d_tmpl, const uint32_t* d_work,
                             int nwork, const uint32_t* tabs, uint32_t* outer_nodes, uint64_t outer_stride_nodes) {
  if (nwork == 0) return hipSuccess;
  hipLaunchKernelGGL(k_col_commit, dim3(nwork), dim3(TR_THREADS), 0, st, T, d_tmpl, d_work, tabs, outer_nodes,
                     outer_stride_nodes);
  return hipGetLastError();
}
hipError_t launch_col_commit_pw(hipStream_t st, const TraceDev& T, const ColTemplate* d_tmpl, const uint32_t* d_pw_cols,
                                int n_pw_cols, const uint32_t* d_chunks, int nchunks, const uint32_t* tabs,
                                uint32_t* outer_nodes, uint64_t outer_stride_nodes, uint32_t* d_err) {
  if (nchunks == 0 || n_pw_cols == 0) return hipSuccess;
  const uint64_t items = (uint64_t)n_pw_cols * nchunks;
  hipLaunchKernelGGL(k_col_commit_pw, dim3((unsigned)((items + PW_THREADS - 1) / PW_THREADS)), dim3(PW_THREADS), 0, st,
                     T, d_tmpl, d_pw_cols, n_pw_cols, d_chunks, nchunks, tabs, outer_nodes, outer_stride_nodes, d_err);
  return hipGetLastError();
}
hipError_t launch_compose_terms(hipStream_t st, const TraceDev& T, const ComposeTerms& Tm, uint64_t row0,
                                uint64_t nrows) {
  if (row0 + nrows > T.n) return hipErrorInvalidValue;
  if (nrows == 0) return hipSuccess;
  // two adjacent rows per lane (4 measured even in round 2); one row for n = 1
  // and odd row ranges. SEZKP_COMPOSE_ROWS=1|2|4 forces a form (read per
  // launch: the parity test switches it).
  const char* rw_s = getenv("SEZKP_COMPOSE_ROWS");
  int rw = rw_s ? atoi(rw_s) : 2;
  if (rw != 1 && rw != 2 && rw != 4) rw = 2;
  while (rw > 1 && (T.n < (uint64_t)rw || (row0 | nrows) % rw)) rw >>= 1;
  const unsigned g = (unsigned)((nrows / rw + TR_THREADS - 1) / TR_THREADS);
  if (rw == 4) hipLaunchKernelGGL(k_compose_terms<4>, dim3(g), dim3(TR_THREADS), 0, st, T, Tm, row0, row0 + nrows);
  else if (rw == 2) hipLaunchKernelGGL(k_compose_terms<2>, dim3(g), dim3(TR_THREADS), 0, st, T, Tm, row0, row0 + nrows);
  else hipLaunchKernelGGL(k_compose_terms<1>, dim3(g), dim3(TR_THREADS), 0, st, T, Tm, row0, row0 + nrows);
  return hipGetLastError();
}
hipError_t launch_compose_combine(hipStream_t st, const ComposeTerms& Tm, const DevChal* ch, const NttTables& tw,
                                  int logn, uint64_t* out, uint64_t row0, uint64_t nrows) {
  const unsigned grid = (unsigned)((nrows + TR_THREADS - 1) / TR_THREADS);
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(k_compose_combine, dim3(grid), dim3(TR_THREADS), 0, st, Tm, ch, tw, logn, out, row0,
                     row0 + nrows);
  return hipGetLastError();
}
hipError_t launch_col_open(hipStream_t st, const TraceDev& T, const ColTemplate* d_tmpl, const uint32_t* outer_nodes,
                           uint64_t outer_stride_nodes, int logChunks, const uint32_t* d_req, int nreq,
                           const ProofLayout& P, const uint32_t* tabs, const uint32_t* d_dlev,
                           const DictPlan* d_plans, const uint32_t* d_dtabs, const DictCol* d_dcols,
                           const uint32_t* d_count) {
  if (nreq == 0) return hipSuccess;
  if ((uint64_t)nreq > (uint64_t)P.nq * P.open_per_q) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_col_open, dim3(nreq), dim3(TR_THREADS), 0, st, T, d_tmpl, outer_nodes, outer_stride_nodes,
                     logChunks, d_req, P, tabs, d_dlev, d_plans, d_dtabs, d_dcols, d_count);
  return hipGetLastError();
}

}  // namespace sezkp

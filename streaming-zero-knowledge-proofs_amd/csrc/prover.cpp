// prover.cpp — host orchestration of the MI355X STARK v1 prover and the C ABI
// (include/sezkp_stark.h). Restates the schedule of
// crates/sezkp-stark/src/v1/prover.rs:61-462 in compute-once form: every hot
// loop runs as a HIP kernel on the context's stream; the host keeps the
// Fiat-Shamir transcript and assembles the bincode ProofV1 (proof.rs:80-98).
//
// Host<->device synchronisation points (each a few hundred bytes):
//   col roots -> [alphas, masks, z] -> layer-0 root -> [betas] -> FRI roots ->
//   [query indices] -> paths/openings.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sezkp_stark.h"
#include "codec.h"
#include "comm.h"
#include "host_crypto.h"
#include "sezkp_internal.h"

using namespace sezkp;

namespace {

constexpr int NUM_QUERIES = 30;  // params.rs:31
constexpr int BLOWUP_LOG2 = 3;   // params.rs:28
// ST_L0TREE brackets exactly one launch (k_layer16 over the LDE) so bench.py
// can quote that kernel's live duration; ST_L0UP holds its upper levels.
enum Stage { ST_EXPAND, ST_COMMIT, ST_OUTER, ST_COMPOSE, ST_INTT, ST_LDE, ST_DEEP, ST_L0TREE, ST_L0UP, ST_FRI,
             ST_OPEN, ST_PATHS, ST_NSTAGE };

struct Err {
  int32_t code;
  std::string msg;
};
#define HIP_OR_THROW(x)                                                                               \
  do {                                                                                                \
    hipError_t e_ = (x);                                                                              \
    if (e_ != hipSuccess) throw Err{SEZKP_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)}; \
  } while (0)

void set_err(char* err, size_t len, const std::string& m) {
  if (err && len) {
    snprintf(err, len, "%s", m.c_str());
  }
}

// --------------------------------------------------------------- twiddles
// w_{2^32}^e = hi[e>>16] * lo[e&0xffff]  and 3^e likewise (host-built once per device)
struct DevTables {
  uint64_t* d = nullptr;
  NttTables T{};
};
std::mutex g_tab_mu;
std::map<int, DevTables> g_tabs;

const NttTables& tables_for_device(int dev) {
  std::lock_guard<std::mutex> lk(g_tab_mu);
  auto it = g_tabs.find(dev);
  if (it != g_tabs.end()) return it->second.T;
  const int K = 32, S = 16;
  const size_t nl = 1u << S, nh = 1u << (K - S);
  std::vector<uint64_t> h(2 * (nl + nh));
  uint64_t* lo = h.data();
  uint64_t* hi = lo + nl;
  uint64_t* p3lo = hi + nh;
  uint64_t* p3hi = p3lo + nl;
  const uint64_t w = hgl_root_2exp(K);
  const uint64_t wS = hgl_pow(w, nl);
  const uint64_t t3S = hgl_pow(3, nl);
  uint64_t a = 1, b = 1, c = 1, d = 1;
  for (size_t i = 0; i < nl; i++) { lo[i] = a; a = hgl_mul(a, w); p3lo[i] = c; c = hgl_mul(c, 3); }
  for (size_t i = 0; i < nh; i++) { hi[i] = b; b = hgl_mul(b, wS); p3hi[i] = d; d = hgl_mul(d, t3S); }
  DevTables t;
  HIP_OR_THROW(hipSetDevice(dev));
  HIP_OR_THROW(hipMalloc(&t.d, h.size() * 8));
  HIP_OR_THROW(hipMemcpy(t.d, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  t.T.lo = t.d;
  t.T.hi = t.d + nl;
  t.T.p3_lo = t.d + nl + nh;
  t.T.p3_hi = t.d + 2 * nl + nh;
  t.T.K = K;
  t.T.S = S;
  return g_tabs.emplace(dev, t).first->second.T;
}

const char* KIND_NAME[7] = {"mv", "wflag", "wsym", "head", "winlen", "in_off", "out_off"};

std::string label_of(int c, uint32_t tau) {  // all_labels (openings.rs:89-116)
  if (c == 0) return "input_mv";
  if (c == 1) return "is_first";
  if (c == 2) return "is_last";
  return std::string(KIND_NAME[(c - 3) / tau]) + "_" + std::to_string((c - 3) % tau);
}

ColTemplate make_template(int c, uint32_t tau, const std::string& label) {
  ColTemplate t{};
  uint8_t b[64] = {0};
  memcpy(b, "col_leaf", 8);
  const uint32_t L = (uint32_t)label.size();
  for (int i = 0; i < 4; i++) b[8 + i] = (uint8_t)(L >> (8 * i));
  memcpy(b + 12, label.data(), L);
  for (int i = 0; i < 16; i++)
    t.words[i] = (uint32_t)b[4 * i] | (uint32_t)b[4 * i + 1] << 8 | (uint32_t)b[4 * i + 2] << 16 |
                 (uint32_t)b[4 * i + 3] << 24;
  t.off = 12 + L;
  t.block_len = 20 + L;
  if (c < 3) { t.kind = c; t.tape = 0; }
  else { t.kind = 3 + (c - 3) / tau; t.tape = (c - 3) % tau; }
  return t;
}

uint64_t rd64(const uint8_t* p) {
  uint64_t x = 0;
  for (int i = 7; i >= 0; i--) x = (x << 8) | p[i];
  return x;
}
int ilog2(uint64_t x) {
  int l = 0;
  while ((1ULL << l) < x) l++;
  return l;
}

}  // namespace

// ======================================================================== ctx
// Per-context executor (sezkp_ctx_prove_async / sezkp_ctx_wait): one worker
// thread runs the context's proofs, so a caller keeps several contexts in
// flight on one GPU and the VALU-bound trees of one proof overlap the
// memory- and latency-bound stages and host round trips of another.
struct AsyncSlot {
  enum State { IDLE, RUNNING, DONE };
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  State state = IDLE;
  bool stop = false;
  uint8_t root[32];
  int32_t rc = 0;
  std::string msg;
  size_t len = 0;
};

static int worker_delay_us() {
  static const int us = [] {
    const char* e = getenv("SEZKP_TEST_WORKER_DELAY_US");
    return e ? atoi(e) : 0;
  }();
  return us;
}

struct sezkp_ctx {
  int device = 0;
  std::unique_ptr<AsyncSlot> async;
  hipStream_t st = nullptr;
  hipStream_t st2 = nullptr;  // side stream: small FRI layers overlap the forest
  hipStream_t stc = nullptr;  // copy stream: staged uploads (sezkp_ctx_stage)
  hipEvent_t ev_fold = nullptr, ev_tail = nullptr, ev_expand = nullptr, ev_cols = nullptr;
  hipEvent_t ev_qin = nullptr, ev_qout = nullptr;  // the DEEP tables on the side stream, beside the INTT
  // Trace images, double-buffered: slot[active] feeds the proofs; stage()
  // fills slot[1 - active] on the copy stream while a proof runs, and the
  // next prove() switches to it (its kernels wait for the copy on the device).
  struct TraceSlot {
    int8_t* imv = nullptr;
    int8_t* mv = nullptr;
    uint8_t* wf = nullptr;
    uint16_t* ws = nullptr;
    uint64_t *bw = nullptr, *bi = nullptr, *bo = nullptr;
    uint8_t* raw = nullptr;     // step arrays as the view holds them (row-major), before k_trace_image
    uint64_t* h_tab = nullptr;  // pinned staging of bw | bi | bo
    hipEvent_t ready = nullptr;
    bool image_pending = false;  // staged: raw copied (copy stream), k_trace_image not yet run
  };
  TraceSlot slot[2];
  int active = 0;
  bool staged = false;       // slot[1 - active] holds a staged trace not yet proved
  std::mutex stage_mu;
  std::vector<uint64_t> cur_step_start;  // shape of the uploaded trace (block boundaries)
  NttTables tw{};
  // workspace of the current upload, and the previous upload's blocks kept
  // for reuse (keyed by byte size): re-uploading a trace of the same shape
  // allocates nothing. Spares left unclaimed are freed at the end of upload.
  std::vector<std::pair<void*, size_t>> dev_allocs, host_allocs, mapped_allocs;
  std::multimap<size_t, void*> spare_dev, spare_host, spare_mapped;
  // shape
  bool loaded = false;
  uint64_t n = 0, N = 0;
  int logn = 0, logN = 0, ncols = 0, logChunks = 0;
  uint32_t tau = 0, nblk = 0;
  TraceDev T{};
  std::vector<std::string> labels;
  ColTemplate* d_tmpl = nullptr;
  uint32_t* d_tabs = nullptr;       // leaf tables + uniform-subtree tables
  uint32_t* d_tab_cols = nullptr;
  int n_tab_cols = 0;
  uint64_t tab_units = 0;
  uint32_t* d_work = nullptr;       // dense (column, chunk) work items
  int n_work = 0;
  uint32_t* d_pw_cols = nullptr;    // piecewise-constant columns
  int n_pw_cols = 0;
  uint32_t* d_pw_chunks = nullptr;  // chunks committed by the piecewise kernel
  int n_pw_chunks = 0;
  DictCol* d_dcols = nullptr;       // dense small-range columns (dictionary commitment)
  int n_dict = 0;
  int64_t* d_dpart = nullptr;
  DictPlan* d_dplans = nullptr;
  uint32_t* d_dtabs = nullptr;
  uint32_t* d_dlev = nullptr;        // dictionary columns' chunk levels 6..9 (openings)
  std::vector<uint32_t> dict_of;     // column -> dictionary index or NO_DICT
  uint32_t* d_outer = nullptr;
  uint32_t* d_err = nullptr;  // device-side guard word: non-zero = a kernel saw an out-of-range index
  uint64_t outer_stride = 0;
  uint32_t* d_colroots = nullptr;
  uint64_t* d_base = nullptr;
  ComposeTerms Tm{};  // per-row composition sums (k_compose_terms, side stream)
  uint64_t *d_dq_part = nullptr, *d_dq_rlo = nullptr, *d_dq_rhi = nullptr, *d_dq_rhk = nullptr;  // DeepPoly
  uint64_t* d_lde = nullptr;
  uint64_t* d_fri = nullptr;
  uint32_t* d_roots = nullptr;
  // ---- Fiat-Shamir challenges (DevChal), written by the host transcript
  DevChal* d_chal = nullptr;        // read by every challenge-dependent kernel
  DevChal* h_chal = nullptr;        // pinned: the host transcript's copy source
  uint32_t* d_dict_of = nullptr;
  // ---- sharding: one proof over `world` GPUs (world == 1: the whole prover
  // on this device; every sharded quantity below degenerates to it)
  int rank = 0, world = 1, logP = 0;
  std::unique_ptr<Comm> comm;            // non-null: the sharded algorithm (also at P = 1, see ctx_create)
  bool sharded() const { return comm != nullptr; }
  // level the run-layer WGs reduce to: the run root (12) when run roots are
  // allgathered, else 6 so the upper jobs build levels 7.. with every lane busy
  int tree_stop() const { return sharded() ? L16_LOG : LSTORE_FRI; }
  // leaves per WG of the layer-0 tree and the forest: 4096, or 1024 when the
  // local LDE has at most 2^21 points (512 or fewer 4096-leaf WGs). Measured
  // (round 4, tools/r4i.sh): config 3 (N = 2^21) in flight 0.499 -> 0.479 ms per
  // proof, a P = 8 rank's trees even; at 2^22 points (a P = 4 rank) the
  // 4096-leaf WGs were faster (layer-0 tree 0.186 against 0.208 ms)
  int tree_wg_log = L16_LOG;
  int wg_stop() const { return std::min(tree_stop(), tree_wg_log); }
  uint64_t M = 0;                       // local LDE length N / P
  int logM = 0;
  int rR = -1;                          // run layers 0..rR (len >= 4096 P), the rest replicated
  uint64_t ch_lo = 0, ch_hi = 0;        // this rank's column chunks
  uint32_t blk_lo = 0, blk_cnt = 0;     // blocks overlapping this rank's rows (+ the next row)
  uint64_t* d_cyc = nullptr;            // P > 1: coset values f(3 w^(rank + P j)) (full_lde: all N values)
  // P = 2: every rank computes the whole N-point LDE (the single-device
  // schedule) and takes its own runs from it, instead of its coset and the
  // all-to-all: one link carries the all-to-all's N/4 values per rank at
  // 153 GB/s (~0.22 ms), more than the other half of the LDE costs (~0.09 ms)
  bool full_lde = false;
  uint64_t* d_xbuf = nullptr;           // P > 1: all-to-all send buffer
  uint64_t* d_rep = nullptr;            // replicated layers (P > 1: first the whole layer rR)
  std::vector<uint64_t*> lvals;         // per FRI layer: this rank's values
  std::vector<TreeDev> ltrees, caps;    // per FRI layer: local tree, cap (== local tree unless sharded)
  std::vector<uint32_t*> rr_gather;     // P > 1, per run layer: allgathered run roots [P][runs]
  std::vector<int> rep16;               // replicated layers with >= 4096 leaves (P > 1)
  int tail_first = 1;                   // first layer of the small-layer tail kernel
  FriLayerDev* d_layers = nullptr;
  ForestLayer* d_forest = nullptr;
  uint64_t* d_tailbuf = nullptr;   // single device: fold-replay scratch of the small-layer workgroups
  int n_forest = 0;
  uint32_t forest_wgs = 0;
  UpperJob* d_jobs = nullptr;  // upper-level passes: layer 0, then all fold layers
  std::vector<std::pair<size_t, int>> jobs0, jobsF;
  std::vector<std::pair<size_t, int>> jobsL0, jobsLR;  // sharded, 1024-leaf WGs: run trees' levels 11..12
  uint32_t* d_req = nullptr;
  uint32_t* h_req = nullptr;
  ProofLayout PL{};             // device proof body (after the column-root header)
  size_t hdr_bytes = 0;         // bincode header: domain_n, tau, col_roots
  std::vector<size_t> root_pos; // byte offset of each column root in the header
  uint8_t* h_proof = nullptr;   // pinned: header + body
  uint32_t* h_small = nullptr;  // col roots / fri roots staging
  size_t max_fri_req = 0, max_open_req = 0;
  hipEvent_t ev[ST_NSTAGE + 1]{};
  double stage_ms[ST_NSTAGE + 1]{};
  // SEZKP_KERNEL_EVENTS=1: an event pair around the FRI forest launch for its
  // live time (bench roofline)
  hipEvent_t kev[2]{};
  double kernel_ms = 0;
  // stage events: the openings kernel on the side stream (it overlaps
  // fri_paths on the prover stream, so it has its own pair)
  hipEvent_t oev[2]{};
  // host-side split of one prove(): wall, time blocked in stream syncs,
  // final D2H wait, proof serialization (after the last sync)
  double host_ms[4]{};
  bool have_times = false;
  // sharded: a failure after the first collective of a prove aborts the
  // communicator (peers blocked in an RCCL call then time out instead of
  // hanging) and leaves the context broken: every later call fails
  bool broken = false;
  bool coll_issued = false;
  // per-collective device time of the last sharded prove (HIP events around
  // each call on the prover stream) and the bytes this rank sends over links
  struct CollStat {
    const char* name;
    uint64_t bytes;
    hipEvent_t a, b;
  };
  std::vector<CollStat> coll_stats;
  std::vector<hipEvent_t> coll_ev;
  size_t coll_used = 0;
  // test hook (SEZKP_DEBUG_STALL_AFTER): a mapped word the stream waits on
  // after a collective, so that the collective looks stuck; set at destroy
  uint32_t* stall_word = nullptr;

  static void* take_spare(std::multimap<size_t, void*>& m, size_t bytes) {
    auto it = m.find(bytes);
    if (it == m.end()) return nullptr;
    void* p = it->second;
    m.erase(it);
    return p;
  }
  // contents are undefined (as hipMalloc's): a reused block holds the previous
  // upload's data, so every buffer is written before it is read
  template <class Tp>
  Tp* dalloc(size_t count) {
    const size_t bytes = count * sizeof(Tp) + 64;
    void* p = take_spare(spare_dev, bytes);
    if (!p) HIP_OR_THROW(hipMalloc(&p, bytes));
    dev_allocs.push_back({p, bytes});
    return static_cast<Tp*>(p);
  }
  template <class Tp>
  Tp* halloc(size_t count) {
    const size_t bytes = count * sizeof(Tp) + 64;
    void* p = take_spare(spare_host, bytes);
    if (!p) HIP_OR_THROW(hipHostMalloc(&p, bytes, hipHostMallocDefault));
    host_allocs.push_back({p, bytes});
    return static_cast<Tp*>(p);
  }
  // page-locked, coherent and mapped: kernels store into it over PCIe and the
  // host reads it after the stream sync (no copy launch). ROCm maps it at the
  // same address on the device.
  template <class Tp>
  Tp* hmapped(size_t count) {
    const size_t bytes = count * sizeof(Tp) + 64;
    void* p = take_spare(spare_mapped, bytes);
    if (!p) {
      HIP_OR_THROW(hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocCoherent));
      void* dp = nullptr;
      const hipError_t e = hipHostGetDevicePointer(&dp, p, 0);
      if (e != hipSuccess || dp != p) {
        (void)hipHostFree(p);
        throw Err{SEZKP_E_DEVICE, "mapped host memory is not addressable at its host address"};
      }
    }
    mapped_allocs.push_back({p, bytes});
    return static_cast<Tp*>(p);
  }
  // keep = true: the blocks become spares for the next upload
  void free_all(bool keep = false) {
    for (auto& a : dev_allocs) {
      if (keep) spare_dev.emplace(a.second, a.first);
      else (void)hipFree(a.first);
    }
    for (auto& a : host_allocs) {
      if (keep) spare_host.emplace(a.second, a.first);
      else (void)hipHostFree(a.first);
    }
    for (auto& a : mapped_allocs) {
      if (keep) spare_mapped.emplace(a.second, a.first);
      else (void)hipHostFree(a.first);
    }
    dev_allocs.clear();
    host_allocs.clear();
    mapped_allocs.clear();
    loaded = false;
  }
  void release_spares() {
    for (auto& s : spare_dev) (void)hipFree(s.second);
    for (auto& s : spare_host) (void)hipHostFree(s.second);
    for (auto& s : spare_mapped) (void)hipHostFree(s.second);
    spare_dev.clear();
    spare_host.clear();
    spare_mapped.clear();
  }
  bool busy() {
    if (!async) return false;
    std::lock_guard<std::mutex> lk(async->mu);
    return async->state != AsyncSlot::IDLE;
  }
  void worker() {
    AsyncSlot& a = *async;
    for (;;) {
      std::unique_lock<std::mutex> lk(a.mu);
      a.cv.wait(lk, [&] { return a.state == AsyncSlot::RUNNING || a.stop; });
      if (a.state != AsyncSlot::RUNNING) return;  // stop requested while idle
      uint8_t r[32];
      memcpy(r, a.root, 32);
      lk.unlock();
      // test hook: hold the worker back so that a stage() issued right after
      // prove_async runs before this proof starts (tests/test_gpu_parity.py)
      if (const int us = worker_delay_us()) std::this_thread::sleep_for(std::chrono::microseconds(us));
      int32_t rc = SEZKP_OK;
      std::string m;
      size_t len = 0;
      try {
        len = prove(r);
      } catch (const Err& e) {
        rc = e.code;
        m = e.msg;
      } catch (const std::exception& e) {
        rc = SEZKP_E_NOMEM;
        m = e.what();
      }
      lk.lock();
      a.rc = rc;
      a.msg = std::move(m);
      a.len = len;
      a.state = AsyncSlot::DONE;
      a.cv.notify_all();
    }
  }
  ~sezkp_ctx() {
    if (stall_word) __atomic_store_n(stall_word, 1u, __ATOMIC_SEQ_CST);  // release a stalled stream
    if (async) {  // let a proof in flight finish, then stop the worker
      {
        std::unique_lock<std::mutex> lk(async->mu);
        async->cv.wait(lk, [&] { return async->state != AsyncSlot::RUNNING; });
        async->stop = true;
      }
      async->cv.notify_all();
      if (async->th.joinable()) async->th.join();
    }
    if (st) (void)hipStreamSynchronize(st);
    if (st2) (void)hipStreamSynchronize(st2);
    if (stc) (void)hipStreamSynchronize(stc);
    free_all();
    release_spares();
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : coll_ev) (void)hipEventDestroy(e);
    for (auto& e : kev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : oev)
      if (e) (void)hipEventDestroy(e);
    if (st2) (void)hipStreamSynchronize(st2);
    if (ev_fold) (void)hipEventDestroy(ev_fold);
    if (ev_tail) (void)hipEventDestroy(ev_tail);
    if (ev_expand) (void)hipEventDestroy(ev_expand);
    if (ev_cols) (void)hipEventDestroy(ev_cols);
    if (ev_qin) (void)hipEventDestroy(ev_qin);
    if (ev_qout) (void)hipEventDestroy(ev_qout);
    if (stc) (void)hipStreamSynchronize(stc);
    for (auto& sl : slot)
      if (sl.ready) (void)hipEventDestroy(sl.ready);
    if (st) (void)hipStreamDestroy(st);
    if (st2 && st2 != st) (void)hipStreamDestroy(st2);
    if (stc) (void)hipStreamDestroy(stc);
    if (stall_word) (void)hipHostFree(stall_word);
  }

  // row0 / nrows: the view's step arrays hold only rows [row0, row0 + nrows)
  // (metadata and step_start still global): a sharded rank's slice
  void upload(const sezkp_block_view& v, uint64_t row0 = 0, uint64_t nrows = ~0ull);
  // stage the next trace (same shape) into the spare slot on the copy stream
  void stage(const sezkp_block_view& v);
  void alloc_slot(TraceSlot& t);
  // block tables + step arrays of `v` into slot t, async on stream s
  void write_trace(TraceSlot& t, const sezkp_block_view& v, hipStream_t s, uint64_t row0, uint64_t nrows,
                   bool staged_copy = false);
  void launch_image(TraceSlot& t, hipStream_t s, uint64_t row0, uint64_t nrows);
  void wait_copy_stream();
  void check_shape_same(const sezkp_block_view& v) const;
  void take_staged();
  // proves into the pinned staging buffer; returns its size (bytes at h_proof)
  size_t prove(const uint8_t root[32]);
  // the prover with the host transcript (three round trips: column roots,
  // layer-0 root, FRI roots)
  size_t prove_body(const uint8_t root[32]);
};

// SEZKP_COLL_TIMEOUT_S: how long a sharded rank waits for a stream holding
// collectives before it aborts the communicator (default 60 s; a T = 2^22
// proof takes ~10 ms once uploaded)
static double coll_timeout_s() {
  static const double t = getenv("SEZKP_COLL_TIMEOUT_S") ? atof(getenv("SEZKP_COLL_TIMEOUT_S")) : 60.0;
  return t > 0 ? t : 60.0;
}
static bool hook_match(const char* spec, int rank, const char* name) {
  if (!spec) return false;
  const char* colon = strchr(spec, ':');
  return colon && atoi(spec) == rank && strcmp(colon + 1, name) == 0;
}
// test hook: SEZKP_DEBUG_FAIL_AT=<rank>:<collective> makes that rank fail
// right before that collective of every sharded prove (tests/test_gpu_sharded.py)
static void fail_point(int rank, const char* name) {
  static const char* spec = getenv("SEZKP_DEBUG_FAIL_AT");
  if (!hook_match(spec, rank, name)) return;
  throw Err{SEZKP_E_DEVICE, std::string("injected failure before collective ") + name + " on rank " +
                                std::to_string(rank)};
}


// The column chunks [ch_lo, ch_hi) rank g of 2^logP commits (all of them on
// one device) and the blocks holding their rows [ch_lo * 1024, ch_hi * 1024]
// (the extra row: compose and the next_* openings read row i + 1; the last
// row's wrap to row 0 is never read: row n - 1 is a block's last row, where
// the head-update term vanishes, and its next_* openings belong to rank 0).
static void shard_range(const uint64_t* step_start, uint32_t nblk, int logn, int rank, int logP, uint64_t& ch_lo,
                        uint64_t& ch_hi, uint32_t& blk_lo, uint32_t& blk_cnt) {
  const uint64_t n = 1ULL << logn;
  const int logChunks = logn > COL_CHUNK_LOG2 ? logn - COL_CHUNK_LOG2 : 0;
  const uint64_t nchunks = 1ULL << logChunks, chunk_rows = n < 1024 ? n : 1024;
  ch_lo = (nchunks >> logP) * (uint64_t)rank;
  ch_hi = ch_lo + (nchunks >> logP);
  const uint64_t r0 = ch_lo * chunk_rows, r1 = std::min<uint64_t>(ch_hi * chunk_rows, n - 1);
  auto block_of = [&](uint64_t row) {
    return (uint32_t)(std::upper_bound(step_start, step_start + nblk + 1, row) - step_start - 1);
  };
  blk_lo = block_of(r0);
  blk_cnt = block_of(r1) - blk_lo + 1;
}

// Blocks of zero steps (step_hi = step_lo - 1, so step_hi - step_lo + 1 wraps
// to 0) contribute no rows: TraceColumns::build and RowIter skip them
// (columns.rs:254-257,281-284; openings.rs:209-238) and nothing else of
// prove_v1 reads a block (tau comes from the view). The device image is built
// from the view without them; the step arrays are shared, and every per-block
// field is copied here, on the host, before any asynchronous copy is issued
// (write_trace reads the per-block fields into its pinned table synchronously).
struct NonEmptyBlocks {
  sezkp_block_view v{};
  std::vector<uint16_t> version, ctrl_in, ctrl_out;
  std::vector<uint32_t> block_id, off_in, off_out;
  std::vector<uint64_t> step_lo, step_hi, step_start;
  std::vector<int64_t> in_head_in, in_head_out, win_left, win_right;
};
static const sezkp_block_view& drop_empty_blocks(const sezkp_block_view& in, NonEmptyBlocks& keep) {
  uint32_t empty = 0;
  for (uint32_t k = 0; k < in.n_blocks; k++) {
    if (in.step_hi[k] - in.step_lo[k] + 1 != 0) continue;  // wrapping, as the reference's usize cast
    if (in.step_start[k + 1] != in.step_start[k])
      throw Err{SEZKP_E_INVALID, "block " + std::to_string(k) + ": zero-step range [" + std::to_string(in.step_lo[k]) +
                                     ", " + std::to_string(in.step_hi[k]) + "] but movement_log has " +
                                     std::to_string(in.step_start[k + 1] - in.step_start[k]) + " steps"};
    empty++;
  }
  if (empty == 0) return in;
  const uint32_t tau = in.tau;
  keep = NonEmptyBlocks{};
  keep.step_start.push_back(in.step_start[0]);
  for (uint32_t k = 0; k < in.n_blocks; k++) {
    if (in.step_hi[k] - in.step_lo[k] + 1 == 0) continue;
    keep.version.push_back(in.version[k]);
    keep.block_id.push_back(in.block_id[k]);
    keep.step_lo.push_back(in.step_lo[k]);
    keep.step_hi.push_back(in.step_hi[k]);
    keep.ctrl_in.push_back(in.ctrl_in[k]);
    keep.ctrl_out.push_back(in.ctrl_out[k]);
    keep.in_head_in.push_back(in.in_head_in[k]);
    keep.in_head_out.push_back(in.in_head_out[k]);
    for (uint32_t r = 0; r < tau; r++) {
      const size_t i = (size_t)k * tau + r;
      keep.win_left.push_back(in.win_left[i]);
      keep.win_right.push_back(in.win_right[i]);
      keep.off_in.push_back(in.off_in[i]);
      keep.off_out.push_back(in.off_out[i]);
    }
    keep.step_start.push_back(in.step_start[k + 1]);
  }
  sezkp_block_view& v = keep.v;
  v = in;  // the step arrays stay the caller's
  v.n_blocks = in.n_blocks - empty;
  v.version = keep.version.data();
  v.block_id = keep.block_id.data();
  v.step_lo = keep.step_lo.data();
  v.step_hi = keep.step_hi.data();
  v.ctrl_in = keep.ctrl_in.data();
  v.ctrl_out = keep.ctrl_out.data();
  v.in_head_in = keep.in_head_in.data();
  v.in_head_out = keep.in_head_out.data();
  v.win_left = keep.win_left.data();
  v.win_right = keep.win_right.data();
  v.off_in = keep.off_in.data();
  v.off_out = keep.off_out.data();
  v.step_start = keep.step_start.data();
  return v;
}

void sezkp_ctx::upload(const sezkp_block_view& v_in, uint64_t row0, uint64_t nrows) {
  NonEmptyBlocks keep;
  const sezkp_block_view& v = drop_empty_blocks(v_in, keep);
  HIP_OR_THROW(hipSetDevice(device));
  // a stage() may still be copying into / transposing a slot on the copy
  // stream: it must finish before its buffers become spares for this upload
  std::lock_guard<std::mutex> lk(stage_mu);
  HIP_OR_THROW(hipStreamSynchronize(st));
  if (st2 != st) HIP_OR_THROW(hipStreamSynchronize(st2));
  if (stc) HIP_OR_THROW(hipStreamSynchronize(stc));
  free_all(true);
  tau = v.tau;
  nblk = v.n_blocks;
  // rows: sum over blocks of (step_hi - step_lo + 1) (columns.rs:254-257)
  uint64_t rows = 0;
  // the kernels index the step arrays through step_start: it must start at 0
  // and every block must hold step_hi - step_lo + 1 >= 1 steps (no wrap-around;
  // the blocks of zero steps, whose range wraps to 0, are gone already)
  if (nblk && v.step_start[0] != 0) throw Err{SEZKP_E_INVALID, "step_start[0] must be 0"};
  for (uint32_t k = 0; k < nblk; k++) {
    if (v.step_hi[k] < v.step_lo[k] || v.step_hi[k] - v.step_lo[k] >= (1ULL << 28))
      throw Err{SEZKP_E_INVALID, "block " + std::to_string(k) + ": step range [" + std::to_string(v.step_lo[k]) +
                                     ", " + std::to_string(v.step_hi[k]) + "] is empty or longer than 2^28"};
    const uint64_t len = v.step_hi[k] - v.step_lo[k] + 1;
    const uint64_t steps = v.step_start[k + 1] - v.step_start[k];
    if (len != steps)
      throw Err{SEZKP_E_INVALID, "block " + std::to_string(k) + ": step_hi-step_lo+1=" + std::to_string(len) +
                                     " but movement_log has " + std::to_string(steps) + " steps"};
    rows += len;
  }
  if (rows == 0 || (rows & (rows - 1)) != 0)
    throw Err{SEZKP_E_INVALID, "n_base must be a power of two (got " + std::to_string(rows) + ")"};  // lde.rs:51
  if (rows > (1ULL << 28)) throw Err{SEZKP_E_INVALID, "trace too long for one device (n > 2^28)"};
  n = rows;
  logn = ilog2(n);
  logN = logn + BLOWUP_LOG2;
  N = 1ULL << logN;
  ncols = 3 + 7 * (int)tau;
  logChunks = logn > COL_CHUNK_LOG2 ? logn - COL_CHUNK_LOG2 : 0;

  // ---- trace image (tape-major): the step arrays go over as the view holds
  // them (row-major [n][tau]) and are transposed on the device
  auto up = [&](auto* dst, const auto* src, size_t count) {
    if (count) HIP_OR_THROW(hipMemcpy(dst, src, count * sizeof(*src), hipMemcpyHostToDevice));
  };
  staged = false;
  active = 0;
  {
    hipEvent_t keep = slot[1].ready;
    slot[1] = TraceSlot{};
    slot[1].ready = keep;
  }
  alloc_slot(slot[0]);
  const uint64_t nchunks = 1ULL << logChunks, chunk_rows = n < 1024 ? n : 1024;
  // sharded: this rank commits chunks [ch_lo, ch_hi) of every column
  if (sharded()) {
    if (logn < 12 + logP || logP > 3)
      throw Err{SEZKP_E_INVALID, "sharded proving needs n >= 4096 * P rows and P <= 8 (n = " + std::to_string(n) +
                                     ", P = " + std::to_string(world) + ")"};
  }
  shard_range(v.step_start, nblk, logn, sharded() ? rank : 0, sharded() ? logP : 0, ch_lo, ch_hi, blk_lo, blk_cnt);
  uint64_t* d_bs = dalloc<uint64_t>(nblk + 1);
  up(d_bs, v.step_start, nblk + 1);
  cur_step_start.assign(v.step_start, v.step_start + nblk + 1);
  if (nrows == ~0ull) nrows = n - row0;
  {  // the rows this context reads: every row (one device) or the whole blocks over its chunks (+ the halo row)
    const uint64_t need0 = v.step_start[blk_lo], need1 = v.step_start[blk_lo + blk_cnt];
    if (row0 > need0 || row0 + nrows < need1 || row0 + nrows > n)
      throw Err{SEZKP_E_INVALID, "step arrays hold rows [" + std::to_string(row0) + ", " + std::to_string(row0 + nrows) +
                                     ") but this context needs rows [" + std::to_string(need0) + ", " +
                                     std::to_string(need1) + ")"};
  }
  write_trace(slot[0], v, st, row0, nrows);
  HIP_OR_THROW(hipStreamSynchronize(st));
  TraceSlot& t0 = slot[0];
  T.n = n;
  T.tau = (int)tau;
  T.nblk = nblk;
  T.input_mv = t0.imv;
  T.mv = t0.mv;
  T.wflag = t0.wf;
  T.wsym = t0.ws;
  T.blk_start = d_bs;
  T.blk_winlen = t0.bw;
  T.blk_offin = t0.bi;
  T.blk_offout = t0.bo;
  T.row_blk = dalloc<uint32_t>(n);
  T.row_flags = dalloc<uint8_t>(n);
  T.head = dalloc<int32_t>((size_t)tau * n + 2);
  T.head_rng = dalloc<int64_t>(2 * (size_t)tau * nblk + 2);

  // ---- column templates + outer trees (all levels kept)
  labels.clear();
  std::vector<ColTemplate> tm;
  for (int c = 0; c < ncols; c++) {
    labels.push_back(label_of(c, tau));
    if (labels.back().size() > 44) throw Err{SEZKP_E_INVALID, "column label too long"};
    tm.push_back(make_template(c, tau, labels.back()));
  }
  // per-column tables: leaf tables for small raw domains (i8/u8: 256, u16:
  // 65536 entries) and uniform-subtree tables U_0..U_10 for piecewise columns
  uint64_t tab_nodes = 0;
  std::vector<uint32_t> tab_cols, pw_cols;
  std::vector<DictCol> dcols;
  const bool use_dict = n >= (1ULL << COL_CHUNK_LOG2) && getenv("SEZKP_NO_DICT") == nullptr;
  tab_units = 0;
  for (int c = 0; c < ncols; c++) {
    ColTemplate& t = tm[c];
    t.tab = NO_TAB;
    t.tab_log = 0;
    if (use_dict && kind_dict(t.kind)) {
      dcols.push_back(DictCol{(uint32_t)c, NO_DICT, (uint64_t)dcols.size() * DICT_LEVELS * DICT_CAP});
    } else if (kind_has_leaf_table(t.kind)) {
      t.tab_log = t.kind == 5 ? 16 : 8;
      t.tab = tab_nodes;
      tab_nodes += 1ULL << t.tab_log;
      tab_units = std::max<uint64_t>(tab_units, 1ULL << t.tab_log);
      tab_cols.push_back(c);
    } else if (kind_piecewise(t.kind)) {
      const uint64_t units = (t.kind == 1 || t.kind == 2) ? 2 : nblk;
      t.tab = tab_nodes;
      tab_nodes += units * U_LEVELS;
      tab_units = std::max<uint64_t>(tab_units, units);
      tab_cols.push_back(c);
      pw_cols.push_back(c);
    }
  }
  // chunks whose rows cross few block boundaries go to the piecewise kernel;
  // the rest (many short blocks) are committed densely for every column
  std::vector<uint32_t> work, pw_chunks;
  std::vector<uint8_t> dense_chunk(nchunks, 0);
  {
    uint32_t k = 0;
    for (uint64_t ch = 0; ch < nchunks; ch++) {
      const uint64_t c0 = ch * chunk_rows, c1 = c0 + chunk_rows;
      while (k < nblk && v.step_start[k] <= c0) k++;
      int inside = 0;
      for (uint32_t j = k; j < nblk && v.step_start[j] < c1; j++)
        if (j == 0 || v.step_start[j] != v.step_start[j - 1]) inside++;
      if (ch < ch_lo || ch >= ch_hi) continue;
      if (inside <= 16) pw_chunks.push_back((uint32_t)ch);
      else dense_chunk[ch] = 1;
    }
  }
  for (int c = 0; c < ncols; c++) {
    if (use_dict && kind_dict(tm[c].kind)) continue;
    const bool pw = kind_piecewise(tm[c].kind);
    for (uint64_t ch = ch_lo; ch < ch_hi; ch++)
      if (!pw || dense_chunk[ch]) { work.push_back((uint32_t)c); work.push_back((uint32_t)ch); }
  }
  d_tmpl = dalloc<ColTemplate>(ncols);
  up(d_tmpl, tm.data(), tm.size());
  // column roots, then the guard words ([0] this rank's guard, [8 + r] rank
  // r's guard when sharded): one D2H copy
  d_colroots = dalloc<uint32_t>((size_t)ncols * 8 + 16);
  d_err = d_colroots + (size_t)ncols * 8;
  HIP_OR_THROW(hipMemset(d_err, 0, 64));
  d_tabs = dalloc<uint32_t>(tab_nodes * 8 + 8);
  n_tab_cols = (int)tab_cols.size();
  d_tab_cols = dalloc<uint32_t>(tab_cols.size() + 1);
  up(d_tab_cols, tab_cols.data(), tab_cols.size());
  for (DictCol& h : dcols)  // head columns: the same tape's mv column (delta plan)
    if (tm[h.col].kind == 6)
      for (size_t i = 0; i < dcols.size(); i++)
        if (tm[dcols[i].col].kind == 3 && tm[dcols[i].col].tape == tm[h.col].tape) h.mv = (uint32_t)i;
  n_dict = (int)dcols.size();
  d_dcols = dalloc<DictCol>(dcols.size() + 1);
  up(d_dcols, dcols.data(), dcols.size());
  d_dpart = dalloc<int64_t>(2 * dcols.size() * ((n + 4095) / 4096) + 2);
  d_dplans = dalloc<DictPlan>(dcols.size() + 1);
  d_dtabs = dalloc<uint32_t>(dcols.size() * DICT_LEVELS * DICT_CAP * 8 + 8);
  d_dlev = dalloc<uint32_t>(dcols.size() * (n >> COL_CHUNK_LOG2) * DLEV_NODES * 8 + 8);
  dict_of.assign(ncols, NO_DICT);
  for (size_t i = 0; i < dcols.size(); i++) dict_of[dcols[i].col] = (uint32_t)i;
  n_pw_cols = (int)pw_cols.size();
  d_pw_cols = dalloc<uint32_t>(pw_cols.size() + 1);
  up(d_pw_cols, pw_cols.data(), pw_cols.size());
  n_pw_chunks = (int)pw_chunks.size();
  d_pw_chunks = dalloc<uint32_t>(pw_chunks.size() + 1);
  up(d_pw_chunks, pw_chunks.data(), pw_chunks.size());
  n_work = (int)(work.size() / 2);
  d_work = dalloc<uint32_t>(work.size() + 2);
  up(d_work, work.data(), work.size());
  outer_stride = tree_stored_nodes(logChunks, 0);
  d_outer = dalloc<uint32_t>((size_t)ncols * outer_stride * 8);

  // ---- LDE / FRI workspace
  // Layer r has 2^(k-r) leaves. Run layers (r <= rR, >= 4096 P leaves) are
  // held as this rank's runs of 4096 (all of it when P = 1); the remaining
  // small layers are replicated on every rank.
  const int k = logN;
  const uint64_t S = 1ULL << L16_LOG;
  d_base = dalloc<uint64_t>(n);
  Tm.hr = dalloc<uint64_t>(n);
  Tm.sl = dalloc<uint64_t>(n);
  Tm.c3 = dalloc<int64_t>(n);
  Tm.c2 = dalloc<int32_t>(n + 2);
  Tm.sy = dalloc<int32_t>(n + 2);
  Tm.bf = dalloc<uint64_t>((size_t)nblk + 1);
  Tm.bl = dalloc<uint64_t>((size_t)nblk + 1);
  Tm.row_flags = T.row_flags;
  Tm.row_blk = T.row_blk;
  full_lde = sharded() && world == 2;
  {  // DEEP quotient tables (sized for this rank's M = N / P LDE points, or N)
    const uint64_t Ml = full_lde ? N : N >> logP;
    d_dq_part = dalloc<uint64_t>(n / 1024 + 1);  // partials of >= 1024 rows (dq_rows_per_part)
    d_dq_rlo = dalloc<uint64_t>(4096);
    d_dq_rhi = dalloc<uint64_t>(Ml > 4096 ? Ml >> 12 : 1);
    d_dq_rhk = dalloc<uint64_t>(n > 4096 ? n >> 12 : 1);
  }
  M = N >> logP;
  logM = logN - logP;
  // tree workgroups of 2048 leaves (1024 on small per-device LDEs): alone a
  // 4096-leaf workgroup is as fast, but with proofs in flight the half-size
  // ones let the concurrent proofs' kernels interleave (+5% in flight, round 5,
  // profiles/r05/ab/tree_wg2048_headline_ab.txt)
  tree_wg_log = M <= (1ULL << 21) ? L16S_LOG : L16M_LOG;
  rR = sharded() ? k - L16_LOG - logP : (k >= L16_LOG ? k - L16_LOG : -1);
  d_lde = dalloc<uint64_t>(M);
  if (sharded()) {
    d_cyc = dalloc<uint64_t>(full_lde ? N : M);
    if (!full_lde) d_xbuf = dalloc<uint64_t>(M);
  }
  lvals.assign(k + 1, nullptr);
  ltrees.assign(k + 1, TreeDev{});
  caps.assign(k + 1, TreeDev{});
  rr_gather.assign(k + 1, nullptr);
  uint64_t run_vals = 0, rep_vals = sharded() ? (S << logP) : 0;
  for (int r = 1; r <= k; r++) {
    if (r <= rR) run_vals += (N >> r) >> logP;
    else rep_vals += N >> r;
  }
  d_fri = dalloc<uint64_t>(run_vals + 1);
  d_rep = dalloc<uint64_t>(rep_vals + 1);
  d_roots = dalloc<uint32_t>((size_t)(k + 2) * 8);
  uint32_t* root_dummy = d_roots + 8 * (k + 1);
  uint64_t total_nodes = 0;
  for (int r = 0; r <= k; r++) {
    const int ll = r <= rR ? k - r - logP : k - r;
    total_nodes += tree_stored_nodes(ll, LSTORE_FRI);
    if (sharded() && r <= rR) total_nodes += tree_stored_nodes(k - r, L16_LOG) + ((N >> r) >> L16_LOG);
  }
  uint32_t* d_nodes = dalloc<uint32_t>(total_nodes * 8 + 8);
  uint64_t off = 0, voff = 0, roff = sharded() ? (S << logP) : 0;
  std::vector<FriLayerDev> ly(k + 1);
  for (int r = 0; r <= k; r++) {
    const bool run = r <= rR;
    if (r == 0) lvals[r] = d_lde;
    else if (run) { lvals[r] = d_fri + voff; voff += (N >> r) >> logP; }
    else { lvals[r] = d_rep + roff; roff += N >> r; }
    TreeDev& t = ltrees[r];
    t.nodes = d_nodes + off * 8;
    t.logLen = run ? k - r - logP : k - r;
    t.lstore = LSTORE_FRI;
    t.root = (run && sharded()) ? root_dummy : d_roots + 8 * r;
    off += tree_stored_nodes(t.logLen, LSTORE_FRI);
    caps[r] = t;
    if (run && sharded()) {
      TreeDev& c = caps[r];
      c.nodes = d_nodes + off * 8;
      c.logLen = k - r;
      c.lstore = L16_LOG;
      c.root = d_roots + 8 * r;
      off += tree_stored_nodes(k - r, L16_LOG);
      rr_gather[r] = d_nodes + off * 8;
      off += (N >> r) >> L16_LOG;
    }
    ly[r] = FriLayerDev{lvals[r], ltrees[r], caps[r], (uint32_t)(run && sharded()), (uint32_t)logP};
  }
  d_layers = dalloc<FriLayerDev>(k + 1);
  up(d_layers, ly.data(), ly.size());
  // replicated layers of >= 4096 leaves (P > 1), then the small-layer tail
  rep16.clear();
  tail_first = rR + 1 > 1 ? rR + 1 : 1;
  while (tail_first <= k && k - tail_first >= L16_LOG) rep16.push_back(tail_first++);
  // forest of the run layers 1..rR (local runs of 4096 leaves per WG) and,
  // sharded, of the replicated layers of >= 4096 leaves (whole subtrees of
  // 4096, level 12 and up from the upper jobs): their WGs run beside the run
  // layers' instead of as three serial few-WG launches after them, and come
  // first in the grid (each is one WG's 4096-leaf chain: started last, they
  // would set the launch's end)
  {
    std::vector<ForestLayer> fl;
    uint32_t wgs = 0;
    for (int r : rep16) {
      fl.push_back(ForestLayer{lvals[r], ltrees[r], wgs, (uint32_t)std::min(L16_LOG, tree_wg_log)});
      wgs += (uint32_t)(1ULL << (ltrees[r].logLen - tree_wg_log));
    }
    for (int r = 1; r <= rR; r++) {
      fl.push_back(ForestLayer{lvals[r], ltrees[r], wgs, (uint32_t)wg_stop()});
      wgs += (uint32_t)(1ULL << (ltrees[r].logLen - tree_wg_log));
    }
    n_forest = (int)fl.size();
    forest_wgs = wgs;
    d_forest = dalloc<ForestLayer>(fl.size() + 1);
    if (!fl.empty()) up(d_forest, fl.data(), fl.size());
    d_tailbuf = sharded() ? nullptr : dalloc<uint64_t>((size_t)TAIL_MAX << TAIL_MAX);
  }
  // upper levels (> 12): layer 0's cap, then every other cap / replicated tree
  {
    std::vector<std::vector<UpperJob>> p0, pF, pL0, pLR;
    // run layers start from the level their layer16 WGs stopped at
    const int from = tree_stop();
    // sharded: a run layer's cap starts from its allgathered run roots (the
    // first pass permutes them into cap order itself: no scatter launch)
    auto gath_of = [&](int r) -> const uint32_t* { return sharded() && r <= rR ? rr_gather[r] : nullptr; };
    auto nrun_of = [&](int r) -> uint64_t { return sharded() ? (N >> r) >> (L16_LOG + logP) : 0; };
    if (rR >= 0 && (caps[0].logLen > from || gath_of(0)))
      plan_upper_jobs(caps[0], from, p0, 0, gath_of(0), nrun_of(0), logP);
    const int rep_from = std::min(L16_LOG, tree_wg_log);
    for (int r = 1; r <= k; r++) {
      const bool runl = r <= rR;
      if ((runl || std::find(rep16.begin(), rep16.end(), r) != rep16.end()) &&
          (caps[r].logLen > (runl ? from : rep_from) || (runl && gath_of(r))))
        plan_upper_jobs(caps[r], runl ? from : rep_from, pF, 0, runl ? gath_of(r) : nullptr, nrun_of(r), logP);
    }
    // sharded with 1024-leaf WGs: the run trees' levels 11..12 (the run roots
    // the caps are gathered from) by upper jobs before each allgather
    if (sharded() && wg_stop() < L16_LOG && rR >= 0) {
      plan_upper_jobs(ltrees[0], wg_stop(), pL0, L16_LOG);
      for (int r = 1; r <= rR; r++) plan_upper_jobs(ltrees[r], wg_stop(), pLR, L16_LOG);
    }
    std::vector<UpperJob> all;
    jobs0.clear();
    jobsF.clear();
    jobsL0.clear();
    jobsLR.clear();
    auto add = [&](std::vector<std::vector<UpperJob>>& ps, std::vector<std::pair<size_t, int>>& out) {
      for (auto& v : ps) { out.push_back({all.size(), (int)v.size()}); all.insert(all.end(), v.begin(), v.end()); }
    };
    add(p0, jobs0);
    add(pF, jobsF);
    add(pL0, jobsL0);
    add(pLR, jobsLR);
    d_jobs = dalloc<UpperJob>(all.size() + 1);
    if (!all.empty()) up(d_jobs, all.data(), all.size());
  }
  max_fri_req = (size_t)NUM_QUERIES * 2 * k;
  max_open_req = (size_t)NUM_QUERIES * (3 + 9 * tau);
  // The query requests (a few KB per proof) live in mapped host memory that
  // the path / opening kernels read directly, so no small H2D copy queues
  // behind a staged trace upload on the copy engine (round 3,
  // tools/ab_req_mapped.sh: host -> proof 7.91 -> 7.97e9, mean of three)
  h_req = hmapped<uint32_t>(max_fri_req * 3 + max_open_req * OPEN_REQ_WORDS);
  d_req = h_req;
  // ---- proof layout (proof.rs:80-98, bincode fixint LE)
  {
    BinWriter w;
    w.u64(N);
    w.u64(tau);
    w.u64((uint64_t)ncols);
    root_pos.assign(ncols, 0);
    for (int c = 0; c < ncols; c++) {
      w.u64(labels[c].size());
      w.raw(labels[c].data(), labels[c].size());
      root_pos[c] = w.b.size();
      w.raw(std::string(32, '\0').data(), 32);
    }
    hdr_bytes = w.b.size();
    PL = ProofLayout{};
    PL.open_per_q = 9 * tau + 3;
    PL.nq = NUM_QUERIES;
    PL.k = k;
    PL.tau = tau;
    PL.open_bytes = 80 + 32 * (uint64_t)logn;  // path_in_chunk + path_to_chunk = log2(n) levels
    PL.q_bytes = 16 + PL.open_per_q * PL.open_bytes;
    PL.fr_off = 8 + NUM_QUERIES * PL.q_bytes;
    PL.fq_off = PL.fr_off + 8 + 32 * (uint64_t)(k + 1);
    PL.fq_bytes = 8 + 8 * (uint64_t)(k + 1) + 8;
    for (int r = 0; r < k; r++) PL.fq_bytes += 2 * (16 + 32 * (uint64_t)(k - r));
    PL.tail_off = PL.fq_off + 8 + NUM_QUERIES * PL.fq_bytes;
    PL.total = PL.tail_off + 8 + 32;
    PL.base = dalloc<uint32_t>(PL.total / 4 + 2);
    h_proof = halloc<uint8_t>(hdr_bytes + PL.total);
    memcpy(h_proof, w.b.data(), hdr_bytes);
  }
  h_small = halloc<uint32_t>((size_t)(ncols + k + 2) * 8);
  d_chal = dalloc<DevChal>(1);
  h_chal = halloc<DevChal>(1);
  d_dict_of = dalloc<uint32_t>((size_t)ncols);
  up(d_dict_of, dict_of.data(), dict_of.size());
  if (k > FS_MAX_BETAS) throw Err{SEZKP_E_INVALID, "LDE domain too large for the challenge record"};
  release_spares();
  loaded = true;
}

void sezkp_ctx::alloc_slot(TraceSlot& t) {
  const size_t cells = (size_t)tau * n, nt = (size_t)tau * nblk;
  t.imv = dalloc<int8_t>(n);
  t.mv = dalloc<int8_t>(cells);
  t.wf = dalloc<uint8_t>(cells);
  t.ws = dalloc<uint16_t>(cells);
  t.bw = dalloc<uint64_t>(3 * nt + 1);  // bw | bi | bo, one copy
  t.bi = t.bw + nt;
  t.bo = t.bi + nt;
  t.raw = dalloc<uint8_t>(4 * cells);  // wsym (2-byte aligned first), mv, has_write
  t.h_tab = halloc<uint64_t>(3 * nt + 1);
  if (!t.ready) HIP_OR_THROW(hipEventCreateWithFlags(&t.ready, hipEventDisableTiming));
}

// The copy stream holds only SDMA copies: no kernel and no event marker, so
// no packet waiting on a copy in flight sits in a hardware queue that other
// contexts' streams share (9 streams on the device's 4 queues at 3 contexts).
// Its copies finish long before the next proof of the context starts; this
// host-side poll is the completion check.
void sezkp_ctx::wait_copy_stream() {
  if (!stc) return;
  for (;;) {
    const hipError_t q = hipStreamQuery(stc);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) HIP_OR_THROW(q);
    std::this_thread::yield();
  }
}

// the row-major step arrays in t.raw -> the tape-major image, on `s`
void sezkp_ctx::launch_image(TraceSlot& t, hipStream_t s, uint64_t row0, uint64_t nrows) {
  const size_t cells = (size_t)tau * n;
  HIP_OR_THROW(launch_trace_image(s, reinterpret_cast<int8_t*>(t.raw + 2 * cells), t.raw + 3 * cells,
                                  reinterpret_cast<uint16_t*>(t.raw), n, tau, t.mv, t.wf, t.ws, row0, row0 + nrows));
  HIP_OR_THROW(hipEventRecord(t.ready, s));
  t.image_pending = false;
}

// Per-block tables on the host (window lengths, head offsets: tau * n_blocks
// values), then every array over PCIe asynchronously on `s` and the row-major
// step arrays transposed to the tape-major image on the device (staged_copy:
// the transposition is left to take_staged(), on the prover stream).
void sezkp_ctx::write_trace(TraceSlot& t, const sezkp_block_view& v, hipStream_t s, uint64_t row0, uint64_t nrows,
                            bool staged_copy) {
  const size_t cells = (size_t)tau * n, nt = (size_t)tau * nblk;
  // the previous copy out of h_tab (an earlier stage into this slot) and the
  // transposition of `raw` must be done
  wait_copy_stream();
  HIP_OR_THROW(hipEventSynchronize(t.ready));
  for (uint32_t k = 0; k < nblk; k++)
    for (uint32_t r = 0; r < tau; r++) {
      const size_t i = (size_t)k * tau + r, o = (size_t)r * nblk + k;
      const int64_t d = v.win_right[i] - v.win_left[i];
      const uint64_t wl = (d < 0 ? 0 - (uint64_t)d : (uint64_t)d) + 1;  // openings.rs:217
      t.h_tab[o] = wl % GL_P_HOST;
      t.h_tab[nt + o] = v.off_in[i];
      t.h_tab[2 * nt + o] = v.off_out[i];
    }
  // each array in copies of <= 4 MB, so a proof's D2H copy queued on the same
  // copy engine waits for one chunk, not for the rest of a 67 MB upload
  // (round 3, tools/ab_upload_chunk.sh: host -> proof 7.89 -> 7.94e9, within
  // the run-to-run spread)
  constexpr size_t chunk = (size_t)4 << 20;
  auto cp = [&](void* dst, const void* src, size_t bytes) {
    for (size_t o = 0; o < bytes;) {
      const size_t b = std::min(chunk, bytes - o);
      HIP_OR_THROW(hipMemcpyAsync((uint8_t*)dst + o, (const uint8_t*)src + o, b, hipMemcpyHostToDevice, s));
      o += b;
    }
  };
  uint16_t* raw_ws = reinterpret_cast<uint16_t*>(t.raw);
  int8_t* raw_mv = reinterpret_cast<int8_t*>(t.raw + 2 * cells);
  uint8_t* raw_hw = t.raw + 3 * cells;
  const size_t c0 = (size_t)row0 * tau, nc = (size_t)nrows * tau;
  cp(raw_ws + c0, v.wsym, nc * 2);
  cp(raw_mv + c0, v.mv, nc);
  cp(raw_hw + c0, v.has_write, nc);
  cp(t.imv + row0, v.input_mv, nrows);
  cp(t.bw, t.h_tab, 3 * nt * 8);
  if (staged_copy) t.image_pending = true;
  else launch_image(t, s, row0, nrows);
}

void sezkp_ctx::check_shape_same(const sezkp_block_view& v) const {
  if (v.tau != tau || v.n_blocks != nblk)
    throw Err{SEZKP_E_INVALID, "staged trace has another shape (tau / block count): call sezkp_ctx_upload"};
  if (nblk && memcmp(v.step_start, cur_step_start.data(), (size_t)(nblk + 1) * 8) != 0)
    throw Err{SEZKP_E_INVALID, "staged trace has other block boundaries: call sezkp_ctx_upload"};
  for (uint32_t k = 0; k < nblk; k++)  // the checks of upload()
    if (v.step_hi[k] < v.step_lo[k] || v.step_hi[k] - v.step_lo[k] + 1 != v.step_start[k + 1] - v.step_start[k])
      throw Err{SEZKP_E_INVALID, "block " + std::to_string(k) + ": step range does not match its steps"};
}

void sezkp_ctx::stage(const sezkp_block_view& v_in) {
  if (!loaded) throw Err{SEZKP_E_INVALID, "no trace uploaded: the first trace of a shape goes through upload"};
  NonEmptyBlocks keep;
  const sezkp_block_view& v = drop_empty_blocks(v_in, keep);
  check_shape_same(v);
  HIP_OR_THROW(hipSetDevice(device));
  std::lock_guard<std::mutex> lk(stage_mu);
  // the copy stream is created by the first stage(): streams map to the
  // device's hardware queues round-robin in creation order, so a context that
  // never stages keeps the (main, side) queue layout of the proofs in flight
  if (!stc) HIP_OR_THROW(hipStreamCreateWithFlags(&stc, hipStreamNonBlocking));
  TraceSlot& t = slot[1 - active];
  if (!t.imv) alloc_slot(t);  // first stage on this workspace: the spare image
  staged = false;             // (re)filling the spare slot
  write_trace(t, v, stc, 0, n, true);
  staged = true;
}

// Switch to a staged trace image (the device waits for its copy). Called by
// the thread that starts a proof (sezkp_ctx_prove_async calls it before
// handing the proof to the worker, so a stage() right after it fills the
// other slot, never the one this proof reads).
void sezkp_ctx::take_staged() {
  std::lock_guard<std::mutex> lk(stage_mu);
  if (staged) {
    active = 1 - active;
    staged = false;
    TraceSlot& t = slot[active];
    T.input_mv = t.imv;
    T.mv = t.mv;
    T.wflag = t.wf;
    T.wsym = t.ws;
    T.blk_winlen = t.bw;
    T.blk_offin = t.bi;
    T.blk_offout = t.bo;
    // the copies are done (host-side check, nothing queued on the copy
    // stream's hardware queue), then the transposition runs on the prover
    // stream ahead of this proof's kernels
    if (t.image_pending) {
      wait_copy_stream();
      launch_image(t, st, 0, n);
    } else {
      HIP_OR_THROW(hipStreamWaitEvent(st, t.ready, 0));
    }
  }
}

size_t sezkp_ctx::prove(const uint8_t mroot[32]) {
  if (broken)
    throw Err{SEZKP_E_DEVICE, "context unusable: an earlier prove aborted the communicator after a failure past "
                              "its first collective, or could not clear a tripped guard word (destroy the context "
                              "and create a new one)"};
  coll_issued = false;
  coll_used = 0;
  coll_stats.clear();
  try {
    return prove_body(mroot);
  } catch (...) {
    // peers may already be waiting in a collective this rank will never join
    // (or this rank in one they never join): abort so that every rank's
    // enqueued collectives stop and every rank returns an error
    if (sharded() && coll_issued) {
      // the stall test hook models a collective stuck on a dead peer; RCCL's
      // abort makes such a kernel exit, so the hook's wait ends here too
      // (ncclCommAbort would otherwise wait behind a stream nothing releases)
      if (stall_word) __atomic_store_n(stall_word, 1u, __ATOMIC_SEQ_CST);
      comm->abort();
      broken = true;
    }
    throw;
  }
}

size_t sezkp_ctx::prove_body(const uint8_t mroot[32]) {
  if (!loaded) throw Err{SEZKP_E_INVALID, "no trace uploaded"};
  // the trace image was fixed by take_staged() in the public entry point that
  // started this proof (for prove_async: before the worker runs, so a stage()
  // issued right after prove_async fills the other slot, never this one)
  using clk = std::chrono::steady_clock;
  const auto t_enter = clk::now();
  double t_sync = 0, t_last = 0;
  // SEZKP_HOST_TRACE=1: host-side marks (us from entry) printed per proof, to
  // split the Fiat-Shamir round trips into wake-up, host work and launch
  static const bool htrace = getenv("SEZKP_HOST_TRACE") != nullptr;
  std::vector<std::pair<const char*, double>> hmarks;
  auto mark = [&](const char* what) {
    if (htrace) hmarks.push_back({what, std::chrono::duration<double, std::micro>(clk::now() - t_enter).count()});
  };
  auto sync = [&]() {
    const auto t0 = clk::now();
    if (sharded() && coll_issued) {
      try {
        comm->wait(st, coll_timeout_s());
      } catch (const std::exception& e) {
        throw Err{SEZKP_E_DEVICE, std::string("rank ") + std::to_string(rank) + ": " + e.what()};
      }
    } else {
      // (polling hipStreamQuery instead measured 10-20 us slower per proof)
      HIP_OR_THROW(hipStreamSynchronize(st));
    }
    t_last = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    t_sync += t_last;
  };
  HIP_OR_THROW(hipSetDevice(device));
  const int k = logN;
  const char* kev_env = getenv("SEZKP_KERNEL_EVENTS");
  const bool kprobe = kev_env && atoi(kev_env) != 0;
  // Per-stage timed events only on request (SEZKP_STAGE_EVENTS=1, or with the
  // kernel events): each timed event record costs the stream ~3.5 us, so the
  // 13 of a proof added ~45 us to one proof at a time (round 4,
  // profiles/r04/stage_events_ab.txt); without them the device stage times
  // read 0
  const char* sev_env = getenv("SEZKP_STAGE_EVENTS");
  const bool stage_ev = kprobe || (sev_env && atoi(sev_env) != 0);
  auto rec = [&](int s) {
    if (stage_ev) HIP_OR_THROW(hipEventRecord(ev[s], st));
  };
  bool kdone = false;
  auto krec = [&](bool end) {
    if (!kprobe) return;
    HIP_OR_THROW(hipEventRecord(kev[end ? 1 : 0], st));
    if (end) kdone = true;
  };
  static const bool sync_debug = getenv("SEZKP_SYNC_DEBUG") != nullptr;  // name the failing kernel
  auto ok = [&](hipError_t e, const char* what) {
    if (e == hipSuccess && sync_debug) e = hipStreamSynchronize(st);
    if (e != hipSuccess) throw Err{SEZKP_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e)};
  };

  const bool sharded = this->sharded();
  const uint64_t S = 1ULL << L16_LOG;
  // every collective goes through coll(): the failure hook, the events of the
  // per-collective stats, and the mark that a failure from here on must abort
  // the communicator. `wire` = bytes this rank sends over the links.
  auto coll = [&](const char* name, uint64_t wire, auto&& issue) {
    fail_point(rank, name);
    while (coll_ev.size() < 2 * (coll_used + 1)) {
      hipEvent_t e;
      HIP_OR_THROW(hipEventCreate(&e));
      coll_ev.push_back(e);
    }
    hipEvent_t a = coll_ev[2 * coll_used], b = coll_ev[2 * coll_used + 1];
    coll_used++;
    HIP_OR_THROW(hipEventRecord(a, st));
    coll_issued = true;
    try {
      issue();
    } catch (const Err&) {
      throw;
    } catch (const std::exception& e) {
      throw Err{SEZKP_E_DEVICE, std::string(name) + ": " + e.what()};
    }
    HIP_OR_THROW(hipEventRecord(b, st));
    coll_stats.push_back(CollStat{name, wire, a, b});
    // test hook: SEZKP_DEBUG_STALL_AFTER=<rank>:<collective> holds that rank's
    // stream after the collective (a wait on a mapped word released only at
    // destroy), so the next wait must give up at SEZKP_COLL_TIMEOUT_S
    static const char* stall = getenv("SEZKP_DEBUG_STALL_AFTER");
    if (hook_match(stall, rank, name)) {
      if (!stall_word) {
        HIP_OR_THROW(hipHostMalloc(&stall_word, 64, hipHostMallocMapped | hipHostMallocCoherent));
        *stall_word = 0;
      }
      HIP_OR_THROW(hipStreamWaitValue32(st, stall_word, 1, hipStreamWaitValueGte, 0xFFFFFFFFu));
    }
  };
  const uint64_t P1 = (uint64_t)world - 1;
  const uint64_t row_lo = n >= 1024 ? ch_lo << COL_CHUNK_LOG2 : 0;
  const uint64_t row_hi = n >= 1024 ? ch_hi << COL_CHUNK_LOG2 : n;
  const bool no_deep_poly = getenv("SEZKP_NO_DEEP_POLY") != nullptr;
  // largest dictionary table above level 0 (entries; SEZKP_DICT_TAB_CAP, for A/Bs)
  uint32_t dict_tab_cap = DICT_CAP;
  if (const char* cap = getenv("SEZKP_DICT_TAB_CAP")) {
    const long v = atol(cap);
    if (v >= 1 && v <= (long)DICT_CAP) dict_tab_cap = (uint32_t)v;
  }
  const int nguard = sharded ? comm->world : 1;
  auto check_guards = [&](const uint32_t* g_h, int ng) {
    for (int r = 0; r < ng; r++) {
      const uint32_t g = g_h[r];
      // the guard carries a data-dependent flag (GUARD_HEAD_RANGE from
      // k_expand): clear it, stream-ordered, so one bad trace does not fail
      // the later proofs of good ones on this context
      if (g) {
        // a failed clear would leave the guard set and fail every later proof
        // with this one's error: mark the context unusable instead
        const hipError_t me = hipMemsetAsync(d_err, 0, 64, st);
        if (me != hipSuccess) {
          broken = true;
          throw Err{SEZKP_E_DEVICE, std::string("guard word tripped (code ") + std::to_string(g) +
                                        ") and clearing it failed: " + hipGetErrorString(me) +
                                        "; the context is unusable"};
        }
      }
      const std::string who = " on rank " + std::to_string(sharded ? r : rank);
      if (g & GUARD_HEAD_RANGE)
        throw Err{SEZKP_E_INVALID, "a block's head position leaves the i32 range" + who +
                                       " (block too long for its moves: block length x max |mv| must stay below 2^31)"};
      if (g) throw Err{SEZKP_E_DEVICE, "column commitment guard tripped" + who + " (code " + std::to_string(g) + ")"};
    }
  };
  // ---- transcript prelude + column roots (prover.rs:67-81) -> alphas,
  // masks, z: the roots come back and the host's transcript writes the
  // challenge record that the kernels read. (A device transcript that
  // derived every challenge on the stream was built in round 4 and measured
  // slower: one workgroup's chain of dependent BLAKE3 compressions took
  // 40 / 23 / 54 us per point against ~25 / 17 / 21 us of host round trip; it
  // was removed in round 5.)
  Transcript tr("sezkp-stark/v1");
  const uint64_t shift_inv = hgl_inv(3);
  uint64_t z = 0, zn = 0;
  bool dq = false;
  const size_t gofs = sharded ? 8 : 0;
  // sharded: each rank turns its own rows into D_j (DeepPoly) and one
  // allgather (with the partial sums of f(z)) gives every rank the n values
  // for the n-point INTT its coset needs; without the quotient the
  // composition values are allgathered as they are. SEZKP_DIST_INTT=1 runs
  // the distributed INTT instead (block rows in, all n coefficients out: one
  // all-to-all, P-point DFTs + twiddle, one all-to-all, a local (n/P)-point
  // INTT, then the allgather every rank's coset needs anyway; rank g's rows
  // are [g n/P, (g+1) n/P), n >= 4096 P). Round 5's per-rank cost model
  // prefers the replicated INTT at every P (profiles/r05/ab/intt_{replicated,
  // distributed}_detail.json: two
  // collectives fewer outweigh (P - 1)/P of a 2^21-point INTT; P = 8 1.204
  // -> 1.132 ms predicted), so it is the default.
  const bool dist_intt = sharded && world > 1 && getenv("SEZKP_DIST_INTT") && atoi(getenv("SEZKP_DIST_INTT")) != 0;
  DeepPoly dpoly{d_dq_rlo, d_dq_rhi, d_dq_rhk};
  std::vector<uint8_t> roots((size_t)(k + 1) * 32);
  uint64_t rows[NUM_QUERIES], frows[NUM_QUERIES];
  std::vector<uint64_t> pos((size_t)NUM_QUERIES * (k + 1));
  size_t nf = 0, no = 0;

  // ---- the proof as four device phases and three host phases (the
  // Fiat-Shamir round trips). Each enqueue_* issues one phase's work on the
  // streams; each host_* reads what the previous phase copied back, runs the
  // transcript and fills what the next phase copies in. (Round 6 measured
  // the phases enqueued ahead behind stream wait-value gates that the host
  // opened: a P = 8 rank's device stages took 0.94 against 0.90 ms, the
  // kernels after each gate running slower; the round trips stay
  // synchronous.)
  auto enqueue_A = [&]() {
    rec(0);
    // ---- column commitments (openings.rs:306-398): this rank's chunks, then
    // every rank gathers all chunk roots and builds the outer trees
    ok(launch_expand(st, T, blk_lo, blk_cnt, d_err), "expand");
    rec(1);
    // piecewise / table / dense columns on the side stream, concurrent with the
    // (VALU-bound) dictionary columns; disjoint outer-tree leaves. (Starting
    // them later, beside part of the dictionary chain only, or on a CU-masked
    // stream, measured even or slower in round 3.)
    HIP_OR_THROW(hipEventRecord(ev_expand, st));
    HIP_OR_THROW(hipStreamWaitEvent(st2, ev_expand, 0));
    ok(launch_col_tables(st2, T, d_tmpl, d_tab_cols, n_tab_cols, tab_units, d_tabs, blk_lo, blk_cnt), "col_tables");
    ok(launch_col_commit(st2, T, d_tmpl, d_work, n_work, d_tabs, d_outer, outer_stride), "col_commit");
    ok(launch_col_commit_pw(st2, T, d_tmpl, d_pw_cols, n_pw_cols, d_pw_chunks, n_pw_chunks, d_tabs, d_outer,
                            outer_stride, d_err), "col_commit_pw");
    // the composition's transcript-independent half (the row sums), also
    // beside the dictionary commitments: only its combine with the alphas is
    // left after the transcript's first round trip
    ok(launch_compose_terms(st2, T, Tm, row_lo, row_hi - row_lo), "compose_terms");
    HIP_OR_THROW(hipEventRecord(ev_cols, st2));
    // (the commit of the K <= 2 columns on a third stream beside table levels
    // 3..4 measured slower, round 6: profiles/r06/ab/dict_split_streams_ab.txt)
    ok(launch_dict_commit(st, T, d_tmpl, d_dcols, n_dict, d_dpart, d_dplans, d_dtabs, d_outer, outer_stride, row_lo,
                          row_hi - row_lo, d_dlev, dict_tab_cap),
       "col_commit_dict");
    HIP_OR_THROW(hipStreamWaitEvent(st, ev_cols, 0));
    // test hook: SEZKP_DEBUG_TRIP_GUARD=<rank> sets that rank's guard word, to
    // check that the failure is collective (tests/test_gpu_sharded.py)
    static const char* trip = getenv("SEZKP_DEBUG_TRIP_GUARD");
    if (trip && atoi(trip) == rank) HIP_OR_THROW(hipMemsetAsync(d_err, 0x7f, 1, st));
    if (sharded) {
      // the chunk roots of every column and every rank's guard word in one
      // group: sharded ranks see all guard words, so a trip on any rank makes
      // ALL ranks fail at the first check, before the next collective (no rank
      // is left blocked in an RCCL call its peers never reach)
      const size_t bytes = (size_t)(ch_hi - ch_lo) * 32;
      coll("col_chunk_roots", P1 * (bytes * ncols + 4), [&] {
        comm->group_start();
        for (int c = 0; c < ncols; c++) {
          uint32_t* lvl0 = d_outer + (size_t)c * outer_stride * 8;
          comm->allgather(lvl0 + ch_lo * 8, lvl0, bytes, st);
        }
        comm->allgather(d_err, d_err + 8, 4, st);
        comm->group_end();
      });
    }
    rec(2);
    TreeDev outer0{d_outer, d_colroots, logChunks, 0};
    ok(launch_tree_upper(st, &outer0, ncols, outer_stride, 8, 0), "col_outer");
    rec(3);
    // one copy: the column roots and the guard words stored right behind them
    // (d_err = d_colroots + 8 ncols; sharded, every rank's word at d_err + 8)
    HIP_OR_THROW(hipMemcpyAsync(h_small, d_colroots, (size_t)ncols * 32 + 4 * (gofs + nguard), hipMemcpyDeviceToHost,
                                st));
  };
  auto host_1 = [&]() {
    const uint32_t* colroots_h = h_small;
    check_guards(h_small + 8 * ncols + gofs, nguard);
    std::vector<uint8_t> colroots((const uint8_t*)colroots_h, (const uint8_t*)colroots_h + (size_t)ncols * 32);
    for (int c = 0; c < ncols; c++) memcpy(h_proof + root_pos[c], colroots.data() + 32 * c, 32);

    // ---- transcript prelude + column roots (prover.rs:67-81); every rank
    // replays the same transcript, so challenges need no broadcast
    tr.absorb("manifest_root", mroot, 32);
    tr.absorb_u64("n", n);
    tr.absorb_u64("tau", tau);
    tr.absorb_u64("n_cols", (uint64_t)ncols);
    for (int c = 0; c < ncols; c++) tr.absorb("col_root", colroots.data() + 32 * c, 32);
    // alphas (params.rs:82-92) with the reuse of prover.rs:86-98
    mark("tr_roots");
    auto ab = tr.challenge("alphas", 64);
    uint64_t a[8];
    for (int i = 0; i < 8; i++) a[i] = rd64(ab.data() + 8 * i) % GL_P_HOST;
    // masks (masking.rs:56-79): one cubic
    tr.absorb("masks", "masks", 5);
    tr.absorb_u64("n_masks", 1);
    tr.absorb_u64("deg", 4);
    uint64_t mask[4];
    for (int j = 0; j < 4; j++) mask[j] = rd64(tr.challenge("mask_coeff", 8).data()) % GL_P_HOST;
    // OOD point + coset nudge (prover.rs:119-135)
    z = rd64(tr.challenge("ood_point", 8).data()) % GL_P_HOST;
    for (;;) {
      uint64_t t = hgl_mul(z, shift_inv);
      for (int i = 0; i < k; i++) t = hgl_mul(t, t);
      if (t != 1) break;
      z = hgl_add(z, 1);
    }
    for (int i = 0; i < 8; i++) h_chal->alpha[i] = a[i];
    for (int j = 0; j < 4; j++) h_chal->mask[j] = mask[j];
    zn = hgl_pow(z, n);
    // ---- composition (this rank's rows), DEEP quotient, INTT
    mark("z_done");
    // single device: DEEP as the LDE of H = q + c S (DeepPoly); the base
    // evaluations become q(w^j) before the INTT. Not when z^n = 1 (z on the
    // base domain) or z = 0, nor below 16 rows: the per-point DEEP below.
    mark("compose_issued");
    dq = logn >= 4 && z != 0 && zn != 1 && !no_deep_poly;
    if (dq) {
      const uint64_t K1 = hgl_mul(hgl_sub(1, zn), hgl_inv(n % GL_P_HOST));             // f(z) = K1 S
      const uint64_t zN = hgl_pow(zn, N / n);
      uint64_t K2 = hgl_mul(hgl_pow(z, N - 1), hgl_inv(hgl_sub(hgl_pow(3, N), zN)));  // c' = f(z) K2
      // rank g evaluates the coset 3 w_N^g <w_M>: H's N coefficients fold to M
      // (M >= n): h'_k = [k < n] q_k (3 w_N^g)^k + c' G rho^k, rho = (3/z) w_N^g,
      // G = sum_{t<P} rho^(tM); single device: rho = 3/z, G = 1
      // (full_lde: the whole domain, as on one device)
      const int cP = full_lde ? 0 : logP;
      const uint64_t cg = full_lde ? 0 : (uint64_t)rank;
      const uint64_t M_ = N >> cP;
      const uint64_t rho = hgl_mul(hgl_mul(3, hgl_inv(z)), hgl_pow(hgl_root_2exp((uint32_t)logN), cg));
      const uint64_t rhoM = hgl_pow(rho, M_);
      uint64_t G = 0, pw = 1;
      for (int t = 0; t < (1 << cP); t++) {
        G = hgl_add(G, pw);
        pw = hgl_mul(pw, rhoM);
      }
      K2 = hgl_mul(K2, G);
      h_chal->z = z;
      h_chal->zn = zn;
      h_chal->K1 = K1;
      h_chal->K2 = K2;
      h_chal->rho = rho;
      h_chal->rho4096 = hgl_pow(rho, 4096);
      h_chal->K3 = hgl_mul(hgl_mul(zn, hgl_inv(z)), hgl_inv(n % GL_P_HOST));  // z^(n-1) / n: kappa = K3 S
    }
  };
  auto enqueue_B = [&]() {
    // alphas, masks and the DEEP constants for the kernels below
    HIP_OR_THROW(hipMemcpyAsync(d_chal, h_chal, offsetof(DevChal, beta), hipMemcpyHostToDevice, st));
    const uint64_t dq_per = dq_rows_per_part(row_hi - row_lo);  // base rows per partial sum (k_inv_base WG)
    if (dq) {
      // the composition's combine (alphas, mask) fused with the DEEP quotient:
      // D_j = C_j / (w^j - z) and the partial sums of f(z) (DeepPoly); the
      // INTT runs on D, f(z) is needed by the tables only
      ok(launch_inv_base(st, Tm, d_base, d_dq_part, logn, d_chal, tw, row_lo, row_hi - row_lo, dq_per), "inv_base");
    } else {
      ok(launch_compose_combine(st, Tm, d_chal, tw, logn, d_base, row_lo, row_hi - row_lo), "compose");
      if (sharded && !dist_intt)
        coll("base_values", P1 * (row_hi - row_lo) * 8,
             [&] { comm->allgather(d_base + row_lo, d_base, (size_t)(row_hi - row_lo) * 8, st); });
    }
    rec(4);
    // sharded: this rank's partial sums of f(z) travel with the INTT exchange
    // that gathers every rank's values (one collective)
    auto gather_fz = [&](uint64_t nrows) {
      if (dq) comm->allgather(d_dq_part + row_lo / dq_per, d_dq_part, (size_t)(nrows / dq_per) * 8, st);
    };
    if (dist_intt) {
      const uint64_t m = n >> logP, Q = m >> logP;
      if (row_lo != (uint64_t)rank * m || row_hi - row_lo != m) throw Err{SEZKP_E_INVALID, "sharded INTT: row split"};
      uint64_t* blk = d_base + row_lo;
      // d_lde: r[g Q + t] = x[g m + rank Q + t]
      coll("intt_alltoall1", P1 * Q * 8, [&] { comm->alltoall(blk, d_lde, Q * 8, st); });
      ok(bintt_dft_twiddle(st, d_lde, world, Q, (uint32_t)rank, logn, tw), "intt_dft");
      coll("intt_alltoall2", P1 * Q * 8, [&] { comm->alltoall(d_lde, blk, Q * 8, st); });  // blk[j] = y_rank[j]
      ok(ntt_dif(st, blk, logn - logP, true, tw), "intt_local");  // slot p: n a_(rank + P bitrev(p))
      coll("intt_coeffs", P1 * (m * 8 + (dq ? m / dq_per * 8 : 0)), [&] {
        comm->group_start();
        comm->allgather(blk, d_base, m * 8, st);
        gather_fz(m);
        comm->group_end();
      });
    } else {
      if (sharded && dq) {
        const uint64_t nrows = row_hi - row_lo;
        coll("d_values", P1 * (nrows * 8 + nrows / dq_per * 8), [&] {
          comm->group_start();
          comm->allgather(d_base + row_lo, d_base, (size_t)nrows * 8, st);
          gather_fz(nrows);
          comm->group_end();
        });
      }
      // the DEEP tables (f(z) from the partial sums, the r^t / c' r^(4096t) /
      // kappa r^(4096t) power tables: a latency-bound ~10 us) on the side
      // stream beside the INTT, which does not read them
      if (dq) {
        HIP_OR_THROW(hipEventRecord(ev_qin, st));
        HIP_OR_THROW(hipStreamWaitEvent(st2, ev_qin, 0));
        ok(launch_q_tables(st2, d_dq_part, logn, full_lde ? logN : logM, d_chal, d_dq_rlo, d_dq_rhi, d_dq_rhk, dq_per),
           "q_tables");
        HIP_OR_THROW(hipEventRecord(ev_qout, st2));
      }
      ok(ntt_dif(st, d_base, logn, true, tw), "intt");  // -> n * coeffs, bit-reversed
      if (dq) HIP_OR_THROW(hipStreamWaitEvent(st, ev_qout, 0));
    }
    if (dq && dist_intt)
      ok(launch_q_tables(st, d_dq_part, logn, full_lde ? logN : logM, d_chal, d_dq_rlo, d_dq_rhi, d_dq_rhk, dq_per),
         "q_tables");
    rec(5);
    // ---- coset LDE (prover.rs:137-189, lde.rs:42-97): rank g evaluates on
    // 3 w_N^g <w_M> (M = N/P), no communication
    const uint64_t inv_n = hgl_inv(n % GL_P_HOST);
    uint64_t* lde_out = sharded ? d_cyc : d_lde;
    // the evaluated coset: 3 w_N^g <w_M> (rank g of P), or the whole domain
    const int eP = full_lde ? 0 : logP;
    const uint32_t eg = full_lde ? 0u : (uint32_t)rank;
    const int logE = logN - eP;
    const uint64_t coset_e = sharded && !full_lde ? ((uint64_t)rank << (tw.K - logN)) : 0;
    const DeepFuse dfuse{z, logN, eP, eg};
    bool deep_fused = dq;
    const int src_logP = dist_intt ? logP : 0;
    if (dq)
      ok(ntt_dit(st, lde_out, logE, false, tw, d_base, logn, inv_n, coset_e, nullptr, nullptr, &dpoly, src_logP),
         "lde_ntt");
    else
      ok(ntt_dit(st, lde_out, logE, false, tw, d_base, logn, inv_n, coset_e, &dfuse, &deep_fused, nullptr, src_logP),
         "lde_ntt");
    rec(6);
    if (!deep_fused) ok(launch_deep(st, lde_out, logN, z, tw, eP, eg), "deep");
    if (full_lde) {  // this rank's runs of 4096 out of the whole LDE
      ok(launch_runs_extract(st, d_cyc, d_lde, M, logP, (uint32_t)rank), "runs_extract");
    } else if (sharded) {  // cyclic coset -> runs of 4096: one all-to-all over xGMI
      ok(launch_cyc_pack(st, d_cyc, d_xbuf, M, logP), "cyc_pack");
      coll("lde_alltoall", P1 * (M >> logP) * 8, [&] { comm->alltoall(d_xbuf, d_cyc, (size_t)(M >> logP) * 8, st); });
      ok(launch_cyc_unpack(st, d_cyc, d_lde, M, logP), "cyc_unpack");
    }
    rec(7);
    // ---- layer-0 tree: local runs, then the cap from allgathered run roots
    if (rR >= 0) {
      ok(launch_layer16(st, d_lde, nullptr, ltrees[0].logLen, 0, 0, ltrees[0], wg_stop(), nullptr, tree_wg_log),
         "layer0_tree");
      rec(ST_L0TREE + 1);
      for (auto& p : jobsL0) ok(launch_upper_jobs(st, d_jobs + p.first, p.second), "layer0_runroots");
      if (sharded) {
        const uint64_t nrun = M >> L16_LOG;
        const uint32_t* lv12 = ltrees[0].nodes + 8 * tree_level_off(ltrees[0].logLen, LSTORE_FRI, L16_LOG);
        coll("layer0_run_roots", P1 * nrun * 32, [&] { comm->allgather(lv12, rr_gather[0], (size_t)nrun * 32, st); });
      }
      for (auto& p : jobs0) ok(launch_upper_jobs(st, d_jobs + p.first, p.second), "layer0_upper");
    } else {
      ok(launch_leaf_subtree(st, d_lde, nullptr, logN, 0, 0, ltrees[0]), "layer0_tree");
      rec(ST_L0TREE + 1);
    }
    rec(ST_L0UP + 1);
    // ---- layer-0 root -> all betas at once (prover.rs:184-198)
    HIP_OR_THROW(hipMemcpyAsync(h_small, d_roots, 32, hipMemcpyDeviceToHost, st));
  };
  auto host_2 = [&]() {
    memcpy(roots.data(), h_small, 32);
    tr.absorb("fri_layer_root", roots.data(), 32);
    auto bb = tr.challenge("fri_betas", 8 * (size_t)k);
    for (int r = 0; r < k; r++) h_chal->beta[r] = rd64(bb.data() + 8 * r) % GL_P_HOST;
  };
  auto enqueue_C = [&]() {
    HIP_OR_THROW(hipMemcpyAsync(d_chal->beta, h_chal->beta, 8 * (size_t)k, hipMemcpyHostToDevice, st));

    // ---- FRI folds + layer trees (prover.rs:192-239). Folds of run layers are
    // rank-local (i and i + len/2 share i mod 4096P). The kernels read the
    // betas from the challenge record: beta r folds layer r into layer r + 1.
    const uint64_t* dbeta = d_chal->beta;
    // layers of <= 2^11 leaves: one launch on the side stream, overlapping the
    // forest / upper levels (its source is the last fold-chain output)
    auto tail_args = [&](const uint64_t* src_vals) {
      TailArgs ta{};
      ta.src = src_vals;
      ta.Ls = k - tail_first;
      ta.beta = dbeta + (tail_first - 1);
      for (int j = 0; j <= ta.Ls; j++) {
        ta.vals[j] = lvals[tail_first + j];
        ta.tree[j] = ltrees[tail_first + j];
      }
      return ta;
    };
    auto launch_tail = [&](const uint64_t* src_vals) {
      if (tail_first > k) return;
      const TailArgs ta = tail_args(src_vals);
      HIP_OR_THROW(hipEventRecord(ev_fold, st));
      HIP_OR_THROW(hipStreamWaitEvent(st2, ev_fold, 0));
      ok(launch_fri_tail(st2, ta), "fri_tail");
      HIP_OR_THROW(hipEventRecord(ev_tail, st2));
    };
    mark("folds");
    const bool tail_merged = !sharded && tail_first <= k && n_forest > 0 && d_tailbuf;
    // fold chain, up to FOLD_MAX layers per pass (2 measured even); the forest
    // follows the whole chain (hashing the first pass's layers beside the later
    // folds measured slower in round 3: the forest starves the folds)
    for (int r = 0; r < rR;) {
      const int F = std::min(FOLD_MAX, rR - r);
      if (F >= 2) {
        FoldOuts fo{};
        fo.beta = dbeta + r;
        for (int m = 1; m <= F; m++) fo.out[m - 1] = lvals[r + m];
        ok(launch_foldm(st, lvals[r], fo, F, ltrees[r + F].logLen), "fri_foldm");
        r += F;
      } else {
        ok(launch_fold(st, lvals[r], lvals[r + 1], ltrees[r + 1].logLen, 0, dbeta + r), "fri_fold");
        r += 1;
      }
    }
    const uint64_t* rep_src = rR >= 0 ? lvals[rR] : d_lde;  // full values of the layer above the replicated ones
    // single device: the small layers ride in the forest launch's first
    // workgroups (sharded: their own kernel on the side stream)
    if (tail_merged) {
      const TailArgs ta = tail_args(rep_src);
      krec(false);
      ok(launch_forest16(st, d_forest, n_forest, forest_wgs, &ta, d_tailbuf, 0, tree_wg_log), "fri_forest");
      krec(true);
    } else if (!sharded) {
      launch_tail(rep_src);
      ok(launch_forest16(st, d_forest, n_forest, forest_wgs, nullptr, nullptr, 0, tree_wg_log), "fri_forest");
    } else {
      // the whole of layer rR, then the replicated layers folded from it in one
      // pass, the tail (side stream) and one forest of run + replicated layers
      coll("fri_rep_values", P1 * S * 8, [&] { comm->allgather(lvals[rR], d_rep, (size_t)S * 8, st); });
      rep_src = d_rep;
      const int last = rR + (int)rep16.size();
      for (int r = rR; r < last;) {
        const int F = std::min(FOLD_MAX, last - r);
        const uint64_t* src = r == rR ? d_rep : lvals[r];
        if (F >= 2) {
          FoldOuts fo{};
          fo.beta = dbeta + r;
          for (int m = 1; m <= F; m++) fo.out[m - 1] = lvals[r + m];
          ok(launch_foldm(st, src, fo, F, ltrees[r + F].logLen), "fri_rep_folds");
        } else {
          ok(launch_fold(st, src, lvals[r + 1], ltrees[r + 1].logLen, 0, dbeta + r), "fri_rep_fold");
        }
        r += F;
      }
      if (!rep16.empty()) rep_src = lvals[rep16.back()];
      // (the tail launched after the forest instead measured even, round 6)
      launch_tail(rep_src);
      ok(launch_forest16(st, d_forest, n_forest, forest_wgs, nullptr, nullptr, 0, tree_wg_log), "fri_forest");
      for (auto& p : jobsLR) ok(launch_upper_jobs(st, d_jobs + p.first, p.second), "fri_runroots");
      uint64_t wire = 0;
      for (int r = 1; r <= rR; r++) wire += P1 * ((N >> r) >> (L16_LOG + logP)) * 32;
      coll("fri_run_roots", wire, [&] {
        comm->group_start();
        for (int r = 1; r <= rR; r++) {
          const uint64_t nrun = (N >> r) >> (L16_LOG + logP);
          const uint32_t* lv12 = ltrees[r].nodes + 8 * tree_level_off(ltrees[r].logLen, LSTORE_FRI, L16_LOG);
          comm->allgather(lv12, rr_gather[r], (size_t)nrun * 32, st);
        }
        comm->group_end();
      });
      // (the caps' first upper-level pass reads the gathered roots in place)
    }
    for (auto& p : jobsF) ok(launch_upper_jobs(st, d_jobs + p.first, p.second), "fri_upper");
    if (tail_first <= k && !tail_merged) HIP_OR_THROW(hipStreamWaitEvent(st, ev_tail, 0));
    rec(ST_FRI + 1);
    // ---- FRI roots -> query rows mod n and mod N (prover.rs:248, 297), the
    // path / opening requests each rank owns and (device mode) the body fields
    if (sharded) HIP_OR_THROW(hipMemsetAsync(PL.base, 0, PL.total, st));  // one writer per byte
    HIP_OR_THROW(hipMemcpyAsync(h_small, d_roots, (size_t)(k + 1) * 32, hipMemcpyDeviceToHost, st));
  };
  auto host_3 = [&]() {
    memcpy(roots.data(), h_small, (size_t)(k + 1) * 32);
    for (int r = 1; r <= k; r++) tr.absorb("fri_layer_root", roots.data() + 32 * r, 32);

    // ---- queries (prover.rs:248, 297)
    mark("tr_fri");
    auto qb = tr.challenge("row_queries", 8 * NUM_QUERIES);
    for (int i = 0; i < NUM_QUERIES; i++) rows[i] = rd64(qb.data() + 8 * i) % n;
    auto fb = tr.challenge("row_queries", 8 * NUM_QUERIES);
    for (int i = 0; i < NUM_QUERIES; i++) frows[i] = rd64(fb.data() + 8 * i) % N;

    mark("queries");
    // FRI path requests (layer, index, ordinal) for the records this rank owns:
    // run layers by run owner, replicated layers on rank 0
    for (int q = 0; q < NUM_QUERIES; q++) {
      uint64_t* p = &pos[(size_t)q * (k + 1)];
      p[0] = frows[q];
      uint64_t len = N;
      for (int r = 0; r < k; r++) {
        const uint64_t half = len / 2;
        for (int side = 0; side < 2; side++) {
          const uint64_t idx = side ? (p[r] ^ half) : p[r];
          const int owner = (sharded && r <= rR) ? (int)((idx >> L16_LOG) & (uint64_t)(world - 1)) : 0;
          if (owner != rank) continue;
          h_req[3 * nf] = (uint32_t)r;
          h_req[3 * nf + 1] = (uint32_t)idx;
          h_req[3 * nf + 2] = (uint32_t)(q * 2 * k + 2 * r + side);
          nf++;
        }
        p[r + 1] = p[r] % half;
        len = half;
      }
    }
    // column opening requests in proof order (prover.rs:252-292, proof.rs:44-66),
    // each by the rank owning the row's chunk
    uint32_t* oreq = h_req + 3 * max_fri_req;
    size_t ord = 0;
    auto push_open = [&](int c, uint64_t row) {
      const uint64_t ch = n >= 1024 ? row >> COL_CHUNK_LOG2 : 0;
      if (ch >= ch_lo && ch < ch_hi) {
        uint32_t* rq = oreq + (size_t)OPEN_REQ_WORDS * no;
        rq[0] = (uint32_t)c;
        rq[1] = (uint32_t)row;
        rq[2] = (uint32_t)(row >> 32);
        rq[3] = (uint32_t)ord;
        rq[4] = dict_of[c];
        no++;
      }
      ord++;
    };
    for (int q = 0; q < NUM_QUERIES; q++) {
      const uint64_t row = rows[q], ip1 = row + 1 < n ? row + 1 : 0;  // next_wrap
      for (uint32_t r = 0; r < tau; r++) {
        push_open(3 + 0 * tau + r, row);   // mv
        push_open(3 + 0 * tau + r, ip1);   // next_mv
        push_open(3 + 1 * tau + r, row);   // write_flag
        push_open(3 + 2 * tau + r, row);   // write_sym
        push_open(3 + 3 * tau + r, row);   // head
        push_open(3 + 3 * tau + r, ip1);   // next_head
        push_open(3 + 4 * tau + r, row);   // win_len
        push_open(3 + 5 * tau + r, row);   // in_off
        push_open(3 + 6 * tau + r, row);   // out_off
      }
      push_open(1, row);  // is_first
      push_open(2, row);  // is_last
      push_open(0, row);  // input_mv
    }
  };
  auto enqueue_D = [&](size_t nf_grid, size_t no_grid, const uint32_t* cnt_f, const uint32_t* cnt_o) {
    mark("req_copy");
    const uint32_t* req = d_req;
    // the openings and the FRI paths write disjoint sections of the proof image
    // and are both latency-bound small grids: the openings run on the side
    // stream beside the path kernel, and (single device) their section (~70% of
    // the proof) goes back over PCIe from there while the paths still run
    mark("col_open");
    HIP_OR_THROW(hipEventRecord(ev_fold, st));
    HIP_OR_THROW(hipStreamWaitEvent(st2, ev_fold, 0));
    if (stage_ev) HIP_OR_THROW(hipEventRecord(oev[0], st2));
    ok(launch_col_open(st2, T, d_tmpl, d_outer, outer_stride, logChunks, req + 3 * max_fri_req, (int)no_grid, PL,
                       d_tabs, d_dlev, d_dplans, d_dtabs, d_dcols, cnt_o),
       "col_open");
    if (stage_ev) HIP_OR_THROW(hipEventRecord(oev[1], st2));
    rec(ST_OPEN + 1);
    mark("col_open_issued");
    if (!sharded) HIP_OR_THROW(hipMemcpyAsync(h_proof + hdr_bytes, PL.base, PL.fr_off, hipMemcpyDeviceToHost, st2));
    HIP_OR_THROW(hipEventRecord(ev_tail, st2));
    mark("open_d2h_issued");
    ok(launch_fri_paths(st, d_layers, req, (int)nf_grid, PL, cnt_f), "fri_paths");
    mark("fri_paths_issued");
    if (sharded) {
      HIP_OR_THROW(hipStreamWaitEvent(st, ev_tail, 0));  // the openings are part of the byte-sum
      coll("proof_allreduce", 2 * P1 * PL.total / (uint64_t)world, [&] { comm->allreduce_sum_u8(PL.base, PL.total, st); });
    }
    rec(ST_PATHS + 1);
    const uint64_t d2h_from = sharded ? 0 : PL.fr_off;
    HIP_OR_THROW(hipMemcpyAsync(h_proof + hdr_bytes + d2h_from, (const uint8_t*)PL.base + d2h_from,
                                PL.total - d2h_from, hipMemcpyDeviceToHost, st));
    mark("proof_d2h_issued");
    HIP_OR_THROW(hipMemcpyAsync(h_small + 8 * (k + 1), lvals[k], 8, hipMemcpyDeviceToHost, st));
    if (!sharded) HIP_OR_THROW(hipStreamWaitEvent(st, ev_tail, 0));
    mark("issued");
  };

  enqueue_A();
  sync();
  mark("sync1");
  host_1();
  enqueue_B();
  sync();
  mark("sync2");
  host_2();
  enqueue_C();
  sync();
  mark("sync3");
  host_3();
  enqueue_D(nf, no, nullptr, nullptr);
  sync();
  mark("sync4");
  if (htrace) {
    for (auto& m : hmarks) fprintf(stderr, "%s %.1f ", m.first, m.second);
    fprintf(stderr, "\n");
  }
  for (int s = 0; s <= ST_NSTAGE; s++) stage_ms[s] = 0;
  if (stage_ev) {
    for (int s = 0; s < ST_NSTAGE; s++) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, ev[s], ev[s + 1]) == hipSuccess) stage_ms[s] = ms;
    }
    // col_openings = the openings kernel's own time on the side stream (it
    // overlaps fri_paths); the host's query round trip before it (roots D2H,
    // transcript, requests) falls in no stage, only in `total`
    float oms = 0;
    stage_ms[ST_OPEN] = hipEventElapsedTime(&oms, oev[0], oev[1]) == hipSuccess ? oms : 0.0;
    float tot = 0;
    (void)hipEventElapsedTime(&tot, ev[0], ev[ST_NSTAGE]);
    stage_ms[ST_NSTAGE] = tot;
  }
  {
    float ms = 0;
    kernel_ms = kdone && hipEventElapsedTime(&ms, kev[0], kev[1]) == hipSuccess ? ms : 0.0;
  }
  have_times = true;
  // an event pair not recorded on this path fails above; that error must not
  // surface as the next launch's hipGetLastError()
  (void)hipGetLastError();
  // ---- host-known parts of the body: counts, query headers, FRI roots,
  // positions, final value (prover.rs:242-243), manifest root
  const auto t_ser = clk::now();
  uint8_t* body = h_proof + hdr_bytes;
  auto put64 = [&](uint64_t at, uint64_t v) { memcpy(body + at, &v, 8); };
  put64(0, NUM_QUERIES);
  for (int q = 0; q < NUM_QUERIES; q++) {
    put64(8 + q * PL.q_bytes, rows[q]);
    put64(8 + q * PL.q_bytes + 8, tau);
  }
  put64(PL.fr_off, (uint64_t)k + 1);
  memcpy(body + PL.fr_off + 8, roots.data(), roots.size());
  put64(PL.fq_off, NUM_QUERIES);
  for (int q = 0; q < NUM_QUERIES; q++) {
    const uint64_t at = PL.fq_off + 8 + q * PL.fq_bytes;
    put64(at, (uint64_t)k + 1);
    for (int r = 0; r <= k; r++) put64(at + 8 + 8 * r, pos[(size_t)q * (k + 1) + r]);
    put64(at + 8 + 8 * (uint64_t)(k + 1), (uint64_t)k);
  }
  memcpy(body + PL.tail_off, h_small + 8 * (k + 1), 8);
  memcpy(body + PL.tail_off + 8, mroot, 32);
  const size_t out = hdr_bytes + PL.total;
  const auto t_end = clk::now();
  host_ms[0] = std::chrono::duration<double, std::milli>(t_end - t_enter).count();
  host_ms[1] = t_sync;
  host_ms[2] = t_last;
  host_ms[3] = std::chrono::duration<double, std::milli>(t_end - t_ser).count();
  return out;
}

// ==================================================================== C ABI
extern "C" {

uint32_t sezkp_abi_version(void) { return SEZKP_ABI_VERSION; }
const char* sezkp_version(void) { return "sezkp-mi355x 0.1.0 (stark-v1, gfx950)"; }

void sezkp_buf_free(sezkp_buf* b) {
  if (b && b->data) {
    free(b->data);
    b->data = nullptr;
    b->len = 0;
  }
}

static void to_buf(const std::vector<uint8_t>& v, sezkp_buf* out) {
  out->data = (uint8_t*)malloc(v.size() ? v.size() : 1);
  if (!out->data) throw Err{SEZKP_E_NOMEM, "out of host memory"};
  memcpy(out->data, v.data(), v.size());
  out->len = v.size();
}
static void to_buf(const std::string& s, sezkp_buf* out) { to_buf(std::vector<uint8_t>(s.begin(), s.end()), out); }

static sezkp_ctx* ctx_create(int32_t device, int32_t rank, int32_t world, const uint8_t* uid,
                             const sezkp_host_comm* hc, char* err, size_t err_len, bool solo = false) {
  try {
    if (world < 1 || world > 8 || (world & (world - 1)) || rank < 0 || rank >= world)
      throw Err{SEZKP_E_INVALID, "world must be a power of two <= 8 and 0 <= rank < world"};
    std::unique_ptr<sezkp_ctx> c(new sezkp_ctx());
    c->device = device;
    c->rank = rank;
    c->world = world;
    c->logP = ilog2((uint64_t)world);
    int cnt = 0;
    HIP_OR_THROW(hipGetDeviceCount(&cnt));
    if (device < 0 || device >= cnt) throw Err{SEZKP_E_DEVICE, "no such HIP device " + std::to_string(device)};
    HIP_OR_THROW(hipSetDevice(device));
    HIP_OR_THROW(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
    for (auto& e : c->ev) HIP_OR_THROW(hipEventCreate(&e));
    for (auto& e : c->kev) HIP_OR_THROW(hipEventCreate(&e));
    for (auto& e : c->oev) HIP_OR_THROW(hipEventCreate(&e));
    HIP_OR_THROW(hipStreamCreateWithFlags(&c->st2, hipStreamNonBlocking));
    HIP_OR_THROW(hipEventCreateWithFlags(&c->ev_fold, hipEventDisableTiming));
    HIP_OR_THROW(hipEventCreateWithFlags(&c->ev_tail, hipEventDisableTiming));
    HIP_OR_THROW(hipEventCreateWithFlags(&c->ev_expand, hipEventDisableTiming));
    HIP_OR_THROW(hipEventCreateWithFlags(&c->ev_cols, hipEventDisableTiming));
    HIP_OR_THROW(hipEventCreateWithFlags(&c->ev_qin, hipEventDisableTiming));
    HIP_OR_THROW(hipEventCreateWithFlags(&c->ev_qout, hipEventDisableTiming));
    c->tw = tables_for_device(device);
    // SEZKP_FORCE_SHARDED=1 runs the sharded algorithm (and its RCCL calls)
    // with a one-rank communicator: tests it on a single GPU
    const bool force = uid && getenv("SEZKP_FORCE_SHARDED") != nullptr;
    if (world > 1 || force || solo) {
      try {
        c->comm.reset(solo ? make_solo_comm(rank, world)
                           : hc ? make_host_comm(rank, world, *hc) : make_rccl_comm(rank, world, uid));
      } catch (const std::exception& e) {
        throw Err{SEZKP_E_DEVICE, e.what()};
      }
    }
    return c.release();
  } catch (const Err& e) {
    set_err(err, err_len, e.msg);
  } catch (const std::exception& e) {
    set_err(err, err_len, e.what());
  }
  return nullptr;
}

sezkp_ctx* sezkp_ctx_create(int32_t device, char* err, size_t err_len) {
  return ctx_create(device, 0, 1, nullptr, nullptr, err, err_len);
}
sezkp_ctx* sezkp_ctx_create_sharded(int32_t device, int32_t rank, int32_t world, const uint8_t unique_id[128],
                                    char* err, size_t err_len) {
  if (!unique_id && world > 1) {
    set_err(err, err_len, "null unique id");
    return nullptr;
  }
  return ctx_create(device, rank, world, unique_id, nullptr, err, err_len);
}
sezkp_ctx* sezkp_ctx_create_sharded_host(int32_t device, int32_t rank, int32_t world, const sezkp_host_comm* comm,
                                         char* err, size_t err_len) {
  if (!comm) {
    set_err(err, err_len, "null host comm");
    return nullptr;
  }
  return ctx_create(device, rank, world, nullptr, comm, err, err_len);
}
sezkp_ctx* sezkp_ctx_create_sharded_solo(int32_t device, int32_t rank, int32_t world, char* err, size_t err_len) {
  return ctx_create(device, rank, world, nullptr, nullptr, err, err_len, true);
}
int32_t sezkp_comm_unique_id(uint8_t out[128], char* err, size_t err_len) {
  try {
    rccl_unique_id(out);
    return SEZKP_OK;
  } catch (const std::exception& e) {
    set_err(err, err_len, e.what());
    return SEZKP_E_DEVICE;
  }
}
void sezkp_ctx_destroy(sezkp_ctx* ctx) { delete ctx; }

int32_t sezkp_ctx_stage(sezkp_ctx* ctx, const sezkp_block_view* blocks, char* err, size_t err_len) {
  try {
    if (!ctx || !blocks) throw Err{SEZKP_E_INVALID, "null argument"};
    ctx->stage(*blocks);
    return SEZKP_OK;
  } catch (const Err& e) {
    set_err(err, err_len, e.msg);
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, err_len, e.what());
    return SEZKP_E_NOMEM;
  }
}
int32_t sezkp_host_register(void* p, size_t bytes) {
  if (!p || !bytes) return SEZKP_E_INVALID;
  return hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess ? SEZKP_OK : SEZKP_E_DEVICE;
}
int32_t sezkp_host_unregister(void* p) {
  if (!p) return SEZKP_E_INVALID;
  return hipHostUnregister(p) == hipSuccess ? SEZKP_OK : SEZKP_E_DEVICE;
}

int32_t sezkp_ctx_upload(sezkp_ctx* ctx, const sezkp_block_view* blocks, char* err, size_t err_len) {
  try {
    if (!ctx || !blocks) throw Err{SEZKP_E_INVALID, "null argument"};
    if (ctx->busy()) throw Err{SEZKP_E_INVALID, "a proof is in flight on this context (call sezkp_ctx_wait)"};
    ctx->upload(*blocks);
    return SEZKP_OK;
  } catch (const Err& e) {
    set_err(err, err_len, e.msg);
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, err_len, e.what());
    return SEZKP_E_NOMEM;
  }
}

int32_t sezkp_ctx_upload_rows(sezkp_ctx* ctx, const sezkp_block_view* blocks, uint64_t row0, uint64_t nrows,
                              char* err, size_t err_len) {
  try {
    if (!ctx || !blocks) throw Err{SEZKP_E_INVALID, "null argument"};
    if (ctx->busy()) throw Err{SEZKP_E_INVALID, "a proof is in flight on this context (call sezkp_ctx_wait)"};
    ctx->upload(*blocks, row0, nrows);
    return SEZKP_OK;
  } catch (const Err& e) {
    set_err(err, err_len, e.msg);
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, err_len, e.what());
    return SEZKP_E_NOMEM;
  }
}
int32_t sezkp_shard_rows(const uint64_t* step_start, uint32_t n_blocks, int32_t rank, int32_t world, uint64_t* row0,
                         uint64_t* nrows) {
  if (!step_start || !row0 || !nrows || !n_blocks || world < 1 || world > 8 || (world & (world - 1)) || rank < 0 ||
      rank >= world)
    return SEZKP_E_INVALID;
  const uint64_t n = step_start[n_blocks];
  if (!n || (n & (n - 1))) return SEZKP_E_INVALID;
  const int logn = ilog2(n), logP = ilog2((uint64_t)world);
  if (world > 1 && logn < 12 + logP) return SEZKP_E_INVALID;
  uint64_t ch_lo, ch_hi;
  uint32_t blk_lo, blk_cnt;
  shard_range(step_start, n_blocks, logn, rank, logP, ch_lo, ch_hi, blk_lo, blk_cnt);
  *row0 = step_start[blk_lo];
  *nrows = step_start[blk_lo + blk_cnt] - *row0;
  return SEZKP_OK;
}

int32_t sezkp_ctx_prove(sezkp_ctx* ctx, const uint8_t manifest_root[32], uint32_t flags, sezkp_buf* proof_bytes,
                        char* err, size_t err_len) {
  (void)flags;
  try {
    if (!ctx || !manifest_root || !proof_bytes) throw Err{SEZKP_E_INVALID, "null argument"};
    if (ctx->busy()) throw Err{SEZKP_E_INVALID, "a proof is in flight on this context (call sezkp_ctx_wait)"};
    ctx->take_staged();
    const size_t len = ctx->prove(manifest_root);
    proof_bytes->data = (uint8_t*)malloc(len ? len : 1);
    if (!proof_bytes->data) throw Err{SEZKP_E_NOMEM, "out of host memory"};
    memcpy(proof_bytes->data, ctx->h_proof, len);
    proof_bytes->len = len;
    return SEZKP_OK;
  } catch (const Err& e) {
    set_err(err, err_len, e.msg);
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, err_len, e.what());
    return SEZKP_E_NOMEM;
  }
}

int32_t sezkp_ctx_prove_borrow(sezkp_ctx* ctx, const uint8_t manifest_root[32], uint32_t flags, const uint8_t** data,
                               size_t* len, char* err, size_t err_len) {
  (void)flags;
  try {
    if (!ctx || !manifest_root || !data || !len) throw Err{SEZKP_E_INVALID, "null argument"};
    if (ctx->busy()) throw Err{SEZKP_E_INVALID, "a proof is in flight on this context (call sezkp_ctx_wait)"};
    ctx->take_staged();
    *len = ctx->prove(manifest_root);
    *data = ctx->h_proof;
    return SEZKP_OK;
  } catch (const Err& e) {
    set_err(err, err_len, e.msg);
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, err_len, e.what());
    return SEZKP_E_NOMEM;
  }
}

int32_t sezkp_ctx_prove_async(sezkp_ctx* ctx, const uint8_t manifest_root[32], uint32_t flags, char* err,
                              size_t err_len) {
  (void)flags;
  try {
    if (!ctx || !manifest_root) throw Err{SEZKP_E_INVALID, "null argument"};
    if (!ctx->loaded) throw Err{SEZKP_E_INVALID, "context has no trace: call sezkp_ctx_upload first"};
    if (!ctx->async) {
      ctx->async.reset(new AsyncSlot());
      ctx->async->th = std::thread([ctx] { ctx->worker(); });
    }
    AsyncSlot& a = *ctx->async;
    {
      std::lock_guard<std::mutex> lk(a.mu);
      if (a.state != AsyncSlot::IDLE)
        throw Err{SEZKP_E_INVALID, "a proof is already in flight on this context (call sezkp_ctx_wait)"};
      HIP_OR_THROW(hipSetDevice(ctx->device));
      ctx->take_staged();  // this proof's trace image is fixed before the call returns
      memcpy(a.root, manifest_root, 32);
      a.state = AsyncSlot::RUNNING;
    }
    a.cv.notify_all();
    return SEZKP_OK;
  } catch (const Err& e) {
    set_err(err, err_len, e.msg);
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, err_len, e.what());
    return SEZKP_E_NOMEM;
  }
}

int32_t sezkp_ctx_wait(sezkp_ctx* ctx, const uint8_t** data, size_t* len, char* err, size_t err_len) {
  if (!ctx || !data || !len) {
    set_err(err, err_len, "null argument");
    return SEZKP_E_INVALID;
  }
  if (!ctx->async) {
    set_err(err, err_len, "no proof in flight on this context");
    return SEZKP_E_INVALID;
  }
  AsyncSlot& a = *ctx->async;
  std::unique_lock<std::mutex> lk(a.mu);
  if (a.state == AsyncSlot::IDLE) {
    set_err(err, err_len, "no proof in flight on this context");
    return SEZKP_E_INVALID;
  }
  a.cv.wait(lk, [&] { return a.state == AsyncSlot::DONE; });
  a.state = AsyncSlot::IDLE;
  if (a.rc != SEZKP_OK) {
    set_err(err, err_len, a.msg);
    return a.rc;
  }
  *data = ctx->h_proof;
  *len = a.len;
  return SEZKP_OK;
}

int32_t sezkp_ctx_stage_times(const sezkp_ctx* ctx, double* out_ms, int32_t max) {
  if (!ctx || !ctx->have_times) return 0;
  int cnt = 0;
  for (int s = 0; s <= ST_NSTAGE && cnt < max; s++) out_ms[cnt++] = ctx->stage_ms[s];
  for (int s = 0; s < 4 && cnt < max; s++) out_ms[cnt++] = ctx->host_ms[s];
  if (cnt < max) out_ms[cnt++] = ctx->kernel_ms;
  return cnt;
}
void* sezkp_ctx_stream(const sezkp_ctx* ctx) { return ctx ? (void*)ctx->st : nullptr; }
int32_t sezkp_ctx_comm_stats(const sezkp_ctx* ctx, sezkp_comm_stat* out, int32_t max) {
  if (!ctx || !out || max <= 0) return 0;
  int32_t cnt = 0;
  for (const auto& c : ctx->coll_stats) {
    if (cnt >= max) break;
    sezkp_comm_stat& o = out[cnt++];
    memset(o.name, 0, sizeof o.name);
    strncpy(o.name, c.name, sizeof o.name - 1);
    o.bytes = c.bytes;
    float ms = 0;
    o.ms = hipEventElapsedTime(&ms, c.a, c.b) == hipSuccess ? ms : -1.0;
  }
  (void)hipGetLastError();
  return cnt;
}

// Distributed four-step NTT over the context's ranks (BASELINE
// config 4). Forward: local M-point NTT (DIF) -> bit-reverse + w_N^(g k2)
// twiddle into the send image -> one all-to-all -> in-place P-point DFTs.
// Inverse: the same pipeline backwards, so the two round-trip in place. One
// rank needs no send image: the transform is bit-reversed in place.
int32_t sezkp_ctx_dist_ntt(sezkp_ctx* ctx, uint64_t* local, uint64_t* scratch, uint32_t log_n, int32_t dir,
                           char* err, size_t err_len) {
  try {
    if (!ctx || !local || !scratch) throw Err{SEZKP_E_INVALID, "null argument"};
    if (ctx->busy()) throw Err{SEZKP_E_INVALID, "a proof is in flight on this context (call sezkp_ctx_wait)"};
    if (ctx->broken) throw Err{SEZKP_E_DEVICE, "context unusable after an aborted collective"};
    if (dir != 1 && dir != -1) throw Err{SEZKP_E_INVALID, "dir must be +1 or -1"};
    const int P = ctx->world, logP = ctx->logP;
    if (log_n > 32 || (int)log_n < 8 + logP)
      throw Err{SEZKP_E_INVALID, "dist_ntt needs 2^(8 + log P) <= n <= 2^32"};
    HIP_OR_THROW(hipSetDevice(ctx->device));
    hipStream_t st = ctx->st;
    const int logM = (int)log_n - logP;
    const uint64_t M = 1ULL << logM, Q = M >> logP;
    const uint64_t e_step = (uint64_t)ctx->rank << (32 - log_n);  // w_N^(g k) = w_{2^32}^(g k 2^(32 - log n))
    const bool inv = dir < 0;
    auto ok = [](hipError_t e, const char* what) {
      if (e != hipSuccess) throw Err{SEZKP_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e)};
    };
    const uint64_t inv_n = inv ? hgl_inv((1ULL << log_n) % GL_P_HOST) : 1;
    hipError_t nat_err = hipSuccess;
    if (P == 1 && ntt_dif_natural(st, local, scratch, logM, inv, ctx->tw, inv_n, &nat_err)) {
      // no exchange: natural order in and out (2^19..2^26 without a bit-reversal pass)
      ok(nat_err, "dist_ntt local");
    } else if (P == 1) {  // no exchange: the twiddle is 1 and the permutation swaps tile pairs in place
      if (!inv) {
        ok(ntt_dif(st, local, logM, false, ctx->tw), "dist_ntt local");
        ok(bitrev_inplace(st, local, logM, 1, false), "dist_ntt bitrev");
      } else {
        ok(bitrev_inplace(st, local, logM, inv_n, true), "dist_ntt bitrev");
        ok(ntt_dit(st, local, logM, true, ctx->tw, nullptr, 0, 1), "dist_ntt local");
      }
    } else if (!inv) {
      ok(ntt_dif(st, local, logM, false, ctx->tw), "dist_ntt local");
      ok(dntt_permute_twiddle(st, local, scratch, logM, ctx->tw, e_step, false, false, 1), "dist_ntt twiddle");
      ctx->comm->alltoall(scratch, local, Q * 8, st);
      ok(dntt_dft(st, local, P, Q, false), "dist_ntt dft");
    } else {
      ok(dntt_dft(st, local, P, Q, true), "dist_ntt dft");
      ctx->comm->alltoall(local, scratch, Q * 8, st);
      ok(dntt_permute_twiddle(st, scratch, local, logM, ctx->tw, e_step, true, true, inv_n), "dist_ntt twiddle");
      ok(ntt_dit(st, local, logM, true, ctx->tw, nullptr, 0, 1), "dist_ntt local");
    }
    return SEZKP_OK;
  } catch (const Err& e) {
    set_err(err, err_len, e.msg);
    return e.code;
  } catch (const std::exception& e) {
    set_err(err, err_len, e.what());
    return SEZKP_E_DEVICE;
  }
}

static std::vector<MetaEntry> meta_for(uint64_t domain_n, uint32_t tau, uint32_t flags) {
  std::vector<MetaEntry> m = {{"proto", true, "stark-v1", 0}, {"domain_n", false, "", domain_n}, {"tau", false, "", tau}};
  if (flags & SEZKP_FLAG_STREAMING) m.push_back({"mode", true, "streaming", 0});
  return m;
}

int32_t sezkp_stark_v1_prove(const sezkp_block_view* blocks, const uint8_t manifest_root[32], uint32_t flags,
                             sezkp_buf* proof_bytes, sezkp_buf* meta_json, char* err, size_t err_len) {
  sezkp_ctx* ctx = sezkp_ctx_create(0, err, err_len);
  if (!ctx) return SEZKP_E_DEVICE;
  int32_t rc = sezkp_ctx_upload(ctx, blocks, err, err_len);
  if (rc == SEZKP_OK) rc = sezkp_ctx_prove(ctx, manifest_root, flags, proof_bytes, err, err_len);
  if (rc == SEZKP_OK && meta_json) {
    try {
      to_buf(meta_to_json(meta_for(ctx->N, ctx->tau, flags)), meta_json);
    } catch (const Err& e) {
      set_err(err, err_len, e.msg);
      rc = e.code;
    }
  }
  sezkp_ctx_destroy(ctx);
  return rc;
}

int32_t sezkp_stark_v1_prove_artifact_cbor(const sezkp_block_view* blocks, const uint8_t manifest_root[32],
                                           uint32_t flags, sezkp_buf* artifact_cbor, char* err, size_t err_len) {
  sezkp_buf pb{};
  int32_t rc = sezkp_stark_v1_prove(blocks, manifest_root, flags, &pb, nullptr, err, err_len);
  if (rc != SEZKP_OK) return rc;
  try {
    std::vector<uint8_t> proof(pb.data, pb.data + pb.len);
    sezkp_buf_free(&pb);
    const uint64_t domain_n = rd64(proof.data());
    const uint32_t tau = blocks->tau;
    to_buf(encode_artifact_cbor("stark", manifest_root, proof, meta_for(domain_n, tau, flags)), artifact_cbor);
    return SEZKP_OK;
  } catch (const Err& e) {
    set_err(err, err_len, e.msg);
    return e.code;
  }
}

// ---------------------------------------------------------- kernel level
int32_t sezkp_gl_ntt(uint64_t* d, uint64_t* scratch, uint32_t log_n, int32_t dir, void* stream) {
  try {
    int dev = 0;
    HIP_OR_THROW(hipGetDevice(&dev));
    const NttTables& T = tables_for_device(dev);
    hipStream_t st = (hipStream_t)stream;
    if (log_n > 28 || (dir != 1 && dir != -1) || !d || (log_n < 8 && !scratch)) return SEZKP_E_INVALID;
    if (log_n == 0) return SEZKP_OK;
    const bool inv = dir < 0;
    const uint64_t scale = inv ? hgl_inv((1ULL << log_n) % GL_P_HOST) : 1;
    hipError_t e = hipSuccess;  // 2^19..2^22: the last pass stores in natural order (scratch is clobbered)
    if (ntt_dif_natural(st, d, scratch, (int)log_n, inv, T, scale, &e)) return e == hipSuccess ? SEZKP_OK : SEZKP_E_DEVICE;
    if (ntt_dif(st, d, (int)log_n, inv, T) != hipSuccess) return SEZKP_E_DEVICE;
    if (log_n >= 8) {
      if (bitrev_inplace(st, d, (int)log_n, scale, inv) != hipSuccess) return SEZKP_E_DEVICE;
    } else {
      if (bitrev_permute(st, d, scratch, (int)log_n, scale, inv) != hipSuccess) return SEZKP_E_DEVICE;
      if (hipMemcpyAsync(d, scratch, 8ULL << log_n, hipMemcpyDeviceToDevice, st) != hipSuccess) return SEZKP_E_DEVICE;
    }
    return SEZKP_OK;
  } catch (const Err& e) {
    return e.code;
  }
}

// kernel-level ABI: one lane per digest / element, so grids stay below 2^31 workgroups
constexpr uint64_t KABI_MAX_N = 1ULL << 38;

int32_t sezkp_gl_coset_lde_deep(uint64_t* evals, uint32_t log_n, uint32_t log_blowup, uint64_t shift, uint64_t z,
                                uint64_t* out, uint8_t* leaves32, void* stream) {
  try {
    int dev = 0;
    HIP_OR_THROW(hipGetDevice(&dev));
    const NttTables& T = tables_for_device(dev);
    hipStream_t st = (hipStream_t)stream;
    shift %= GL_P_HOST;
    z %= GL_P_HOST;
    // N = 1 (log_n + log_blowup = 0) is rejected: the prover never asks for it
    // (n = 1 still has N = 8) and the NTT/DEEP launches assume N >= 2
    if (log_blowup > 3 || log_n + log_blowup == 0 || log_n + log_blowup > 28 || shift == 0 || !evals || !out)
      return SEZKP_E_INVALID;
    if (leaves32 && (reinterpret_cast<uintptr_t>(leaves32) & 15)) return SEZKP_E_INVALID;
    const int logN = (int)(log_n + log_blowup);
    // every denominator shift w^i - z must be nonzero: (z / shift)^N != 1
    {
      uint64_t t = hgl_mul(z, hgl_inv(shift));
      for (int i = 0; i < logN; i++) t = hgl_mul(t, t);
      if (t == 1) return SEZKP_E_INVALID;
    }
    if (ntt_dif(st, evals, (int)log_n, true, T) != hipSuccess) return SEZKP_E_DEVICE;
    uint64_t* scratch = nullptr;
    bool ok = true;
    if (shift != 3) {  // the LDE load applies 3^j n^-1: pre-scale the coefficients by (shift / 3)^j
      const size_t cnt = 2048 + (log_n > 11 ? (1ULL << (log_n - 11)) : 1);
      HIP_OR_THROW(hipMallocAsync(reinterpret_cast<void**>(&scratch), cnt * 8, st));
      ok = launch_scale_pow_bitrev(st, evals, (int)log_n, hgl_mul(shift, hgl_inv(3)), scratch) == hipSuccess;
    }
    const uint64_t inv_n = hgl_inv((1ULL << log_n) % GL_P_HOST);
    const DeepFuse dfuse{z, logN, 0, 0};
    bool deep_fused = false;
    ok = ok && ntt_dit(st, out, logN, false, T, evals, (int)log_n, inv_n, 0, shift == 3 ? &dfuse : nullptr,
                       &deep_fused) == hipSuccess;
    ok = ok && (deep_fused || launch_deep(st, out, logN, z, T, 0, 0, shift) == hipSuccess);
    ok = ok && (!leaves32 ||
                launch_leaves_u64(st, out, 1ULL << logN, reinterpret_cast<uint32_t*>(leaves32)) == hipSuccess);
    if (scratch) (void)hipFreeAsync(scratch, st);  // stream-ordered: after the launches above
    return ok ? SEZKP_OK : SEZKP_E_DEVICE;
  } catch (const Err& e) {
    return e.code;
  }
}

int32_t sezkp_fri_fold(const uint64_t* in, uint64_t n_out, uint64_t beta, uint64_t* out, void* stream) {
  if (n_out == 0 || (n_out & (n_out - 1)) || n_out > KABI_MAX_N || !in || !out) return SEZKP_E_INVALID;
  if (launch_fold_any((hipStream_t)stream, in, out, n_out, beta % GL_P_HOST) != hipSuccess)
    return SEZKP_E_DEVICE;
  return SEZKP_OK;
}

int32_t sezkp_fs_xof(const uint8_t* stream_bytes, size_t stream_len, const uint32_t* pos, const uint8_t* suffixes,
                     const uint32_t* sfx_len, const uint32_t* out_len, uint32_t nchal, uint8_t* out, void* stream) {
  (void)stream;  // ABI 3 signature; the transcript runs on the host since round 5
  if (!nchal || !pos || !sfx_len || !out_len || !out || (stream_len && !stream_bytes)) return SEZKP_E_INVALID;
  std::vector<uint8_t> msg;
  for (uint32_t i = 0; i < nchal; i++) {
    if (pos[i] > stream_len || (sfx_len[i] && !suffixes)) return SEZKP_E_INVALID;
    msg.assign(stream_bytes, stream_bytes + pos[i]);
    msg.insert(msg.end(), suffixes, suffixes + sfx_len[i]);
    suffixes += sfx_len[i];
    sezkp_blake3(msg.data(), msg.size(), out, out_len[i]);
    out += out_len[i];
  }
  return SEZKP_OK;
}

int32_t sezkp_blake3_leaves_u64(const uint64_t* vals, uint64_t n, uint8_t* leaves32, void* stream) {
  if (n > KABI_MAX_N || (reinterpret_cast<uintptr_t>(leaves32) & 15) || (n && (!vals || !leaves32)))
    return SEZKP_E_INVALID;
  if (launch_leaves_u64((hipStream_t)stream, vals, n, reinterpret_cast<uint32_t*>(leaves32)) != hipSuccess)
    return SEZKP_E_DEVICE;
  return SEZKP_OK;
}

int32_t sezkp_blake3_leaves_labeled(const uint64_t* vals, uint64_t n, const char* label, uint32_t label_len,
                                    uint8_t* leaves32, void* stream) {
  if (n > KABI_MAX_N || label_len > 44 || (label_len && !label) || (reinterpret_cast<uintptr_t>(leaves32) & 15) ||
      (n && (!vals || !leaves32)))
    return SEZKP_E_INVALID;
  const ColTemplate ct = make_template(0, 1, std::string(label ? label : "", label_len));
  if (launch_leaves_labeled((hipStream_t)stream, vals, n, ct, reinterpret_cast<uint32_t*>(leaves32)) != hipSuccess)
    return SEZKP_E_DEVICE;
  return SEZKP_OK;
}

// MerkleTree level table (merkle.rs:46-71): n = 0 is one zero leaf
static MerkleLevels merkle_levels(uint64_t n) {
  MerkleLevels L{};
  uint64_t len = n ? n : 1, off = 0;
  int l = 0;
  for (;;) {
    L.off[l] = off;
    L.len[l] = len;
    if (len == 1) break;
    off += len;
    len = (len + 1) / 2;
    l++;
  }
  L.depth = l;
  return L;
}

uint64_t sezkp_merkle_node_count(uint64_t n) {
  if (n > KABI_MAX_N) return 0;
  const MerkleLevels L = merkle_levels(n);
  return L.off[L.depth] + 1;
}

int32_t sezkp_merkle_build(const uint8_t* leaves32, uint64_t n, uint8_t* nodes32, void* stream) {
  if (n > KABI_MAX_N || !nodes32 || (reinterpret_cast<uintptr_t>(nodes32) & 15) ||
      (n && (!leaves32 || (reinterpret_cast<uintptr_t>(leaves32) & 15))))
    return SEZKP_E_INVALID;
  hipStream_t st = (hipStream_t)stream;
  const MerkleLevels L = merkle_levels(n);
  uint32_t* nodes = reinterpret_cast<uint32_t*>(nodes32);
  if (n == 0) return hipMemsetAsync(nodes32, 0, 32, st) == hipSuccess ? SEZKP_OK : SEZKP_E_DEVICE;
  if (nodes32 != leaves32 && hipMemcpyAsync(nodes32, leaves32, 32 * n, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return SEZKP_E_DEVICE;
  for (int l = 1; l <= L.depth; l++)
    if (launch_merkle_level(st, nodes + 8 * L.off[l - 1], L.len[l - 1], nodes + 8 * L.off[l]) != hipSuccess)
      return SEZKP_E_DEVICE;
  return SEZKP_OK;
}

int32_t sezkp_merkle_paths(const uint8_t* nodes32, uint64_t n, const uint64_t* idx, uint32_t q, uint8_t* out32,
                           void* stream) {
  if (n > KABI_MAX_N || (uint64_t)q * 64 > KABI_MAX_N || (reinterpret_cast<uintptr_t>(nodes32) & 15) ||
      (reinterpret_cast<uintptr_t>(out32) & 15) || (q && (!nodes32 || !idx || !out32)))
    return SEZKP_E_INVALID;
  const MerkleLevels L = merkle_levels(n);
  if (launch_merkle_paths((hipStream_t)stream, reinterpret_cast<const uint32_t*>(nodes32), L, idx, q,
                          reinterpret_cast<uint32_t*>(out32)) != hipSuccess)
    return SEZKP_E_DEVICE;
  return SEZKP_OK;
}

int32_t sezkp_fri_fold_commit(const uint64_t* in, uint64_t n_out, uint64_t beta, uint64_t* out, uint8_t* root32,
                              void* stream) {
  if (n_out == 0 || (n_out & (n_out - 1)) || n_out > KABI_MAX_N || !in || !out || !root32) return SEZKP_E_INVALID;
  const int L = ilog2(n_out);
  hipStream_t st = (hipStream_t)stream;
  uint32_t* nodes = nullptr;
  const uint64_t cnt = tree_stored_nodes(L, LSTORE_FRI) + 1;
  if (hipMalloc(&nodes, cnt * 32 + 32) != hipSuccess) return SEZKP_E_DEVICE;
  TreeDev t{nodes, nodes + cnt * 8, L, LSTORE_FRI};
  int32_t rc = SEZKP_OK;
  if (launch_leaf_subtree(st, in, out, L, 1, beta % GL_P_HOST, t) != hipSuccess) rc = SEZKP_E_DEVICE;
  if (rc == SEZKP_OK && hipMemcpyAsync(root32, t.root, 32, hipMemcpyDeviceToHost, st) != hipSuccess) rc = SEZKP_E_DEVICE;
  if (rc == SEZKP_OK && hipStreamSynchronize(st) != hipSuccess) rc = SEZKP_E_DEVICE;
  (void)hipFree(nodes);
  return rc;
}

int32_t sezkp_merkle_root_u64(const uint64_t* vals, uint64_t n, uint8_t* root32, void* stream) {
  if (n == 0 || (n & (n - 1)) || n > KABI_MAX_N || !vals || !root32) return SEZKP_E_INVALID;
  const int L = ilog2(n);
  hipStream_t st = (hipStream_t)stream;
  uint32_t* nodes = nullptr;
  const uint64_t cnt = tree_stored_nodes(L, LSTORE_FRI) + 1;
  if (hipMalloc(&nodes, cnt * 32 + 32) != hipSuccess) return SEZKP_E_DEVICE;
  TreeDev t{nodes, nodes + cnt * 8, L, LSTORE_FRI};
  int32_t rc = SEZKP_OK;
  if (launch_leaf_subtree(st, vals, nullptr, L, 0, 0, t) != hipSuccess) rc = SEZKP_E_DEVICE;
  if (rc == SEZKP_OK && hipMemcpyAsync(root32, t.root, 32, hipMemcpyDeviceToHost, st) != hipSuccess) rc = SEZKP_E_DEVICE;
  if (rc == SEZKP_OK && hipStreamSynchronize(st) != hipSuccess) rc = SEZKP_E_DEVICE;
  (void)hipFree(nodes);
  return rc;
}

// ---------------------------------------------------------- host helpers
int32_t sezkp_manifest_root(const sezkp_block_view* blocks, uint8_t out[32]) {
  if (!blocks || !out) return SEZKP_E_INVALID;
  manifest_root(*blocks, out);
  return SEZKP_OK;
}
int32_t sezkp_manifest_frontier_root(const sezkp_block_view* blocks, uint8_t out[32]) {
  if (!blocks || !out) return SEZKP_E_INVALID;
  manifest_frontier_root(*blocks, out);
  return SEZKP_OK;
}

struct sezkp_blocks {
  BlockStore s;
  std::vector<uint64_t> line_off;  // sezkp_blocks_decode_jsonl_meta: each line's byte offset
};
int32_t sezkp_blocks_decode_jsonl_meta(const uint8_t* data, size_t len, uint64_t lo, uint64_t hi, sezkp_blocks** out,
                                       char* err, size_t err_len) {
  return sezkp_blocks_decode_jsonl_lines(data, len, lo, hi, 0, out, err, err_len);
}
int32_t sezkp_blocks_decode_jsonl_lines(const uint8_t* data, size_t len, uint64_t lo, uint64_t hi, int32_t steps,
                                        sezkp_blocks** out, char* err, size_t err_len) {
  if (!out || (!data && len) || lo > hi) return SEZKP_E_INVALID;
  std::unique_ptr<sezkp_blocks> b(new sezkp_blocks());
  std::string e;
  if (!decode_blocks_jsonl_meta(reinterpret_cast<const char*>(data), len, lo, hi, b->s, b->line_off, e, steps != 0)) {
    set_err(err, err_len, e);
    return SEZKP_E_DECODE;
  }
  *out = b.release();
  return SEZKP_OK;
}
int32_t sezkp_blocks_line_offsets(const sezkp_blocks* b, const uint64_t** offsets, size_t* n) {
  if (!b || !offsets || !n) return SEZKP_E_INVALID;
  *offsets = b->line_off.data();
  *n = b->line_off.size();
  return SEZKP_OK;
}
int32_t sezkp_manifest_leaf_hashes(const sezkp_block_view* blocks, uint8_t* out) {
  if (!blocks || (!out && blocks->n_blocks)) return SEZKP_E_INVALID;
  for (uint32_t k = 0; k < blocks->n_blocks; k++) manifest_leaf_hash(*blocks, k, out + 32ull * k);
  return SEZKP_OK;
}
int32_t sezkp_merkle_root_of_leaves(const uint8_t* leaves, size_t n, int32_t frontier, uint8_t out[32]) {
  if (!out || (!leaves && n)) return SEZKP_E_INVALID;
  merkle_root_of_leaves(leaves, n, frontier != 0, out);
  return SEZKP_OK;
}
int32_t sezkp_blocks_decode_cbor(const uint8_t* data, size_t len, sezkp_blocks** out, char* err, size_t err_len) {
  if (!out || (!data && len)) return SEZKP_E_INVALID;
  std::unique_ptr<sezkp_blocks> b(new sezkp_blocks());
  std::string e;
  if (!decode_blocks_cbor(data, len, b->s, e)) {
    set_err(err, err_len, e);
    return SEZKP_E_DECODE;
  }
  *out = b.release();
  return SEZKP_OK;
}
int32_t sezkp_blocks_decode_jsonl(const uint8_t* data, size_t len, sezkp_blocks** out, char* err, size_t err_len) {
  if (!out || (!data && len)) return SEZKP_E_INVALID;
  std::unique_ptr<sezkp_blocks> b(new sezkp_blocks());
  std::string e;
  if (!decode_blocks_jsonl(reinterpret_cast<const char*>(data), len, b->s, e)) {
    set_err(err, err_len, e);
    return SEZKP_E_DECODE;
  }
  *out = b.release();
  return SEZKP_OK;
}
// `sezkp-cli simulate --t T --b b --tau tau` (main.rs:317-350): generate_trace
// (tracegen.cpp, rand 0.9 StdRng bit-exact; the reference fixes seed 42) +
// partition_trace into blocks of b steps.
int32_t sezkp_simulate_blocks(uint64_t t, uint32_t b, uint32_t tau, uint64_t seed, sezkp_blocks** out, char* err,
                              size_t err_len) {
  try {
    if (!out || b == 0 || tau > 255 || t == 0 || t > (1ULL << 32)) {
      set_err(err, err_len, "simulate: need 0 < t <= 2^32, b > 0, tau <= 255");
      return SEZKP_E_INVALID;
    }
    std::vector<int8_t> imv(t), mv(t * tau);
    std::vector<uint8_t> hw(t * tau);
    std::vector<uint16_t> ws(t * tau);
    int32_t rc = sezkp_simulate_trace(t, tau, seed, imv.data(), mv.data(), hw.data(), ws.data());
    if (rc != SEZKP_OK) return rc;
    std::unique_ptr<sezkp_blocks> bl(new sezkp_blocks());
    partition_trace(bl->s, t, tau, b, imv.data(), mv.data(), hw.data(), ws.data());
    *out = bl.release();
    return SEZKP_OK;
  } catch (const std::bad_alloc&) {
    set_err(err, err_len, "simulate: out of host memory");
    return SEZKP_E_NOMEM;
  }
}
int32_t sezkp_blocks_encode_cbor(const sezkp_block_view* blocks, sezkp_buf* out) {
  try {
    if (!blocks || !out) return SEZKP_E_INVALID;
    to_buf(encode_blocks_cbor(*blocks), out);
    return SEZKP_OK;
  } catch (const std::exception&) {
    return SEZKP_E_NOMEM;
  }
}
int32_t sezkp_blocks_encode_jsonl(const sezkp_block_view* blocks, sezkp_buf* out) {
  try {
    if (!blocks || !out) return SEZKP_E_INVALID;
    to_buf(encode_blocks_jsonl(*blocks), out);
    return SEZKP_OK;
  } catch (const Err& e) {
    return e.code;
  } catch (const std::exception&) {
    return SEZKP_E_NOMEM;
  }
}
int32_t sezkp_manifest_decode(const uint8_t* data, size_t len, int32_t is_json, uint8_t root[32],
                              uint32_t* n_leaves, char* err, size_t err_len) {
  if (!data || !root) return SEZKP_E_INVALID;
  std::string e;
  const bool ok = is_json ? decode_manifest_json(reinterpret_cast<const char*>(data), len, root, n_leaves, e)
                          : decode_manifest_cbor(data, len, root, n_leaves, e);
  if (!ok) {
    set_err(err, err_len, e);
    return SEZKP_E_DECODE;
  }
  return SEZKP_OK;
}
const sezkp_block_view* sezkp_blocks_view(const sezkp_blocks* b) { return b ? &b->s.view : nullptr; }
void sezkp_blocks_free(sezkp_blocks* b) { delete b; }
void sezkp_blake3(const uint8_t* data, size_t len, uint8_t* out, size_t out_len) {
  Blake3 h;
  h.update(data, len);
  h.finalize(out, out_len);
}

}  // extern "C"

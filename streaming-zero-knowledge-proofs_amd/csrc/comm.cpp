// comm.cpp — RCCL and host-callback implementations of sezkp::Comm.
//
// RCCL: one communicator per process (one process per GPU), collectives on
// the prover's stream; with xGMI point-to-point links the exchanges are
// ring/direct per-link bound, so the prover sends few, large messages
// (one all-to-all of the LDE, one allgather per commitment step).
#include "comm.h"

#include <rccl/rccl.h>
#include <string.h>

#include <chrono>
#include <stdexcept>
#include <thread>

namespace sezkp {

// Poll the stream against the deadline (every transport: a peer that failed
// never joins a collective this rank has enqueued, and a plain stream sync
// would then block forever). Short proofs finish in a few ms: spin first,
// then back off.
void Comm::wait(hipStream_t st, double timeout_s) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  // spin on the stream for the first 10 ms (a proof's host round trips wait
  // 50-500 us; sleeping 50 us per poll added ~100 us to each of them, round
  // 4 kernel trace of a sharded rank), then poll with sleeps up to the deadline
  for (int spin = 0;; spin++) {
    const hipError_t q = hipStreamQuery(st);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) throw std::runtime_error(std::string("stream: ") + hipGetErrorString(q));
    if ((spin & 63) != 0) continue;
    const std::string ae = async_error();
    if (!ae.empty()) throw std::runtime_error("collective failed: " + ae);
    const double el = std::chrono::duration<double>(clk::now() - t0).count();
    if (el > timeout_s)
      throw std::runtime_error("collective timeout: no progress within " + std::to_string(timeout_s) +
                               " s (SEZKP_COLL_TIMEOUT_S); a peer rank failed or stalled");
    if (el > 0.01) std::this_thread::sleep_for(std::chrono::microseconds(el > 0.2 ? 1000 : 50));
  }
}

namespace {

void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}
void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

struct RcclComm final : Comm {
  ncclComm_t c = nullptr;
  RcclComm(int r, int w, const uint8_t uid[128]) {
    rank = r;
    world = w;
    ncclUniqueId id;
    static_assert(sizeof(id.internal) == 128, "ncclUniqueId size");
    memcpy(id.internal, uid, 128);
    nccl_check(ncclCommInitRank(&c, w, id, r), "ncclCommInitRank");
  }
  ~RcclComm() override {
    if (c) (void)ncclCommDestroy(c);
  }
  std::string async_error() override {
    ncclResult_t ae = ncclSuccess;
    if (c && ncclCommGetAsyncError(c, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
      return ncclGetErrorString(ae);
    return {};
  }
  void abort() override {
    if (c) (void)ncclCommAbort(c);
    c = nullptr;
  }
  void live() const {
    if (!c) throw std::runtime_error("communicator aborted after an earlier failure");
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t st) override {
    live();
    nccl_check(ncclAllGather(send, recv, bytes, ncclUint8, c, st), "ncclAllGather");
  }
  void alltoall(const void* send, void* recv, size_t bytes, hipStream_t st) override {
    live();
    nccl_check(ncclAllToAll(send, recv, bytes, ncclUint8, c, st), "ncclAllToAll");
  }
  void allreduce_sum_u8(void* buf, size_t bytes, hipStream_t st) override {
    live();
    nccl_check(ncclAllReduce(buf, buf, bytes, ncclUint8, ncclSum, c, st), "ncclAllReduce");
  }
  void group_start() override {
    live();
    nccl_check(ncclGroupStart(), "ncclGroupStart");
  }
  void group_end() override { nccl_check(ncclGroupEnd(), "ncclGroupEnd"); }
  std::string name() const override { return "rccl"; }
};

// Device buffers are staged through host memory around each callback.
struct HostComm final : Comm {
  sezkp_host_comm cb;
  std::vector<uint8_t> hs, hr;
  HostComm(int r, int w, const sezkp_host_comm& c) : cb(c) {
    rank = r;
    world = w;
    if (!cb.allgather || !cb.alltoall || !cb.allreduce_sum_u8) throw std::runtime_error("host comm: null callback");
  }
  void d2h(void* h, const void* d, size_t b, hipStream_t st) {
    hip_check(hipMemcpyAsync(h, d, b, hipMemcpyDeviceToHost, st), "comm D2H");
    hip_check(hipStreamSynchronize(st), "comm sync");
  }
  void h2d(void* d, const void* h, size_t b, hipStream_t st) {
    hip_check(hipMemcpyAsync(d, h, b, hipMemcpyHostToDevice, st), "comm H2D");
    hip_check(hipStreamSynchronize(st), "comm sync");
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t st) override {
    hs.resize(bytes);
    hr.resize(bytes * world);
    d2h(hs.data(), send, bytes, st);
    if (cb.allgather(cb.user, hs.data(), hr.data(), bytes) != 0) throw std::runtime_error("host comm allgather failed");
    h2d(recv, hr.data(), bytes * world, st);
  }
  void alltoall(const void* send, void* recv, size_t bytes, hipStream_t st) override {
    hs.resize(bytes * world);
    hr.resize(bytes * world);
    d2h(hs.data(), send, bytes * world, st);
    if (cb.alltoall(cb.user, hs.data(), hr.data(), bytes) != 0) throw std::runtime_error("host comm alltoall failed");
    h2d(recv, hr.data(), bytes * world, st);
  }
  void allreduce_sum_u8(void* buf, size_t bytes, hipStream_t st) override {
    hs.resize(bytes);
    d2h(hs.data(), buf, bytes, st);
    if (cb.allreduce_sum_u8(cb.user, hs.data(), bytes) != 0) throw std::runtime_error("host comm allreduce failed");
    h2d(buf, hs.data(), bytes, st);
  }
  std::string name() const override { return "host"; }
};

// One rank of a P-rank sharded prove alone on one GPU (the per-rank cost
// model): every collective keeps only this rank's own contribution (a local
// copy into its slot; the peers' slots hold whatever was there), so the
// rank's kernels run with their real shapes and the bytes each collective
// would put on the links are recorded by the caller. The proof bytes are
// meaningless; the timings are the rank's.
struct SoloComm final : Comm {
  SoloComm(int r, int w) {
    rank = r;
    world = w;
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t st) override {
    uint8_t* dst = static_cast<uint8_t*>(recv) + (size_t)rank * bytes;
    if (dst != send) hip_check(hipMemcpyAsync(dst, send, bytes, hipMemcpyDeviceToDevice, st), "solo allgather");
  }
  void alltoall(const void* send, void* recv, size_t bytes, hipStream_t st) override {
    const size_t o = (size_t)rank * bytes;
    hip_check(hipMemcpyAsync(static_cast<uint8_t*>(recv) + o, static_cast<const uint8_t*>(send) + o, bytes,
                             hipMemcpyDeviceToDevice, st),
              "solo alltoall");
  }
  void allreduce_sum_u8(void*, size_t, hipStream_t) override {}
  std::string name() const override { return "solo"; }
};

}  // namespace

Comm* make_solo_comm(int rank, int world) { return new SoloComm(rank, world); }
Comm* make_rccl_comm(int rank, int world, const uint8_t unique_id[128]) { return new RcclComm(rank, world, unique_id); }
Comm* make_host_comm(int rank, int world, const sezkp_host_comm& cb) { return new HostComm(rank, world, cb); }
void rccl_unique_id(uint8_t out[128]) {
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  memcpy(out, id.internal, 128);
}

}  // namespace sezkp

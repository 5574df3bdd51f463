// comm.h — the three exchange steps of the sharded prover, over RCCL (xGMI)
// in production or over caller-supplied host callbacks (tests, or any
// transport the embedding application owns).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/sezkp_stark.h"

namespace sezkp {

struct Comm {
  int rank = 0, world = 1;
  virtual ~Comm() = default;
  // recv[r * bytes .. (r+1) * bytes) = rank r's send (device buffers, stream-ordered)
  virtual void allgather(const void* send, void* recv, size_t bytes, hipStream_t st) = 0;
  // recv segment r = rank r's send segment for this rank (bytes per peer)
  virtual void alltoall(const void* send, void* recv, size_t bytes, hipStream_t st) = 0;
  // byte-wise sum over ranks, result on every rank (proof bodies: each byte has one writer)
  virtual void allreduce_sum_u8(void* buf, size_t bytes, hipStream_t st) = 0;
  virtual void group_start() {}
  virtual void group_end() {}
  virtual std::string name() const = 0;
  // Wait for `st` (which may hold collectives): polls the stream and
  // async_error(), and throws once `timeout_s` passes or the communicator
  // reports an error (a peer that failed never joins a collective this rank
  // has enqueued, so a plain stream sync would block forever). The same
  // policy for every transport (host collectives are tested with it).
  void wait(hipStream_t st, double timeout_s);
  // non-empty: the transport saw an asynchronous failure (RCCL: ncclCommGetAsyncError)
  virtual std::string async_error() { return {}; }
  // Tear the communicator down so that enqueued collectives stop waiting for
  // peers (ncclCommAbort); the owner is unusable afterwards.
  virtual void abort() {}
};

// throws std::runtime_error on failure
Comm* make_rccl_comm(int rank, int world, const uint8_t unique_id[128]);
Comm* make_host_comm(int rank, int world, const sezkp_host_comm& cb);
// one rank alone on one GPU: own contributions only (the per-rank cost model)
Comm* make_solo_comm(int rank, int world);
void rccl_unique_id(uint8_t out[128]);

}  // namespace sezkp

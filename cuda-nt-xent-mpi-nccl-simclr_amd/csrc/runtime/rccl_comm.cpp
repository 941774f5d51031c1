// RCCL implementation of ntxent::Comm (see include/ntxent/comm.h).
#include "ntxent/comm.h"

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

#include "ntxent/ntxent.h"
#include "ntxent/trace.h"

namespace ntxent {
void LocalComm::all_gather(const void* send, void* recv, size_t bytes, hipStream_t stream) {
  if (send != recv && bytes) NTXENT_HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, stream));
}

void LocalComm::reduce_scatter_sum(const float* send, float* recv, size_t count, hipStream_t stream) {
  if (send != recv && count)
    NTXENT_HIP_CHECK(hipMemcpyAsync(recv, send, count * sizeof(float), hipMemcpyDeviceToDevice, stream));
}

void LocalComm::send_recv(const std::vector<P2POp>& ops, hipStream_t stream) {
  // world 1: the only peer is this rank; the k-th send feeds the k-th receive
  std::vector<const P2POp*> sends, recvs;
  for (const auto& o : ops) {
    NTXENT_CHECK(o.peer == 0, "LocalComm::send_recv: peer out of range");
    (o.send ? sends : recvs).push_back(&o);
  }
  NTXENT_CHECK(sends.size() == recvs.size(), "LocalComm::send_recv: unmatched send/receive");
  for (size_t k = 0; k < sends.size(); ++k) {
    NTXENT_CHECK(sends[k]->bytes == recvs[k]->bytes, "LocalComm::send_recv: size mismatch");
    if (sends[k]->bytes && sends[k]->buf != recvs[k]->buf)
      NTXENT_HIP_CHECK(hipMemcpyAsync(recvs[k]->buf, sends[k]->buf, sends[k]->bytes, hipMemcpyDeviceToDevice, stream));
  }
}

// ---- ThreadComm ---------------------------------------------------------------------------
struct ThreadComm::Call {
  const void* send = nullptr;
  void* recv = nullptr;
  size_t bytes = 0;
  const std::vector<P2POp>* ops = nullptr;
  hipEvent_t ready = nullptr, done = nullptr;
};

class ThreadCommGroup {
 public:
  explicit ThreadCommGroup(int world) : world_(world), calls_(world) {}
  int world() const { return world_; }
  // host rendezvous of the W callers (generation counted, reusable)
  void barrier() {
    std::unique_lock<std::mutex> l(m_);
    const long gen = gen_;
    if (++arrived_ == world_) {
      arrived_ = 0;
      ++gen_;
      cv_.notify_all();
    } else {
      cv_.wait(l, [&] { return gen != gen_; });
    }
  }
  std::vector<ThreadComm::Call*>& calls() { return calls_; }

 private:
  int world_;
  std::mutex m_;
  std::condition_variable cv_;
  int arrived_ = 0;
  long gen_ = 0;
  std::vector<ThreadComm::Call*> calls_;
};

std::shared_ptr<ThreadCommGroup> make_thread_comm_group(int world) {
  NTXENT_CHECK(world >= 1, "thread comm: world must be >= 1");
  return std::make_shared<ThreadCommGroup>(world);
}

ThreadComm::ThreadComm(std::shared_ptr<ThreadCommGroup> group, int rank) : group_(std::move(group)), rank_(rank) {
  NTXENT_CHECK(group_ && rank >= 0 && rank < group_->world(), "ThreadComm: bad rank");
  NTXENT_HIP_CHECK(hipEventCreateWithFlags(&ready_, hipEventDisableTiming));
  NTXENT_HIP_CHECK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
}

ThreadComm::~ThreadComm() {
  if (ready_) hipEventDestroy(ready_);
  if (done_) hipEventDestroy(done_);
  if (scratch_) hipFree(scratch_);
}

int ThreadComm::world() const { return group_->world(); }

float* ThreadComm::scratch(size_t floats) {
  if (floats > scratch_floats_) {
    // (the device is idle for this rank's buffers: a reduction's scratch is only read by its own
    // stream after the rendezvous)
    if (scratch_) NTXENT_HIP_CHECK(hipFree(scratch_));
    NTXENT_HIP_CHECK(hipMalloc(&scratch_, floats * sizeof(float)));
    scratch_floats_ = floats;
  }
  return scratch_;
}

// 1. mark this rank's enqueued work (ready), publish the call; rendezvous
// 2. enqueue the copies out of the peers' buffers (each after that peer's ready event); mark done
// 3. rendezvous; wait for every peer's copies (done) -> the peers' buffers may change again
// 4. `after` (the reduction, once every copy has landed); rendezvous so that no rank re-records
//    its events before every peer has enqueued its waits on them
template <typename Copies, typename After>
void ThreadComm::collective(Call& c, hipStream_t stream, Copies&& copies, After&& after) {
  auto& calls = group_->calls();
  NTXENT_HIP_CHECK(hipEventRecord(ready_, stream));
  c.ready = ready_;
  c.done = done_;
  calls[rank_] = &c;
  group_->barrier();
  copies(calls);
  NTXENT_HIP_CHECK(hipEventRecord(done_, stream));
  group_->barrier();
  for (int q = 0; q < world(); ++q)
    if (q != rank_) NTXENT_HIP_CHECK(hipStreamWaitEvent(stream, calls[q]->done, 0));
  after();
  group_->barrier();
}

void ThreadComm::all_gather(const void* send, void* recv, size_t bytes, hipStream_t stream) {
  Call c;
  c.send = send;
  collective(c, stream, [&](std::vector<Call*>& calls) {
    char* out = static_cast<char*>(recv);
    for (int q = 0; q < world(); ++q) {
      char* dst = out + (size_t)q * bytes;
      if (calls[q]->send == dst || bytes == 0) continue;
      if (q != rank_) NTXENT_HIP_CHECK(hipStreamWaitEvent(stream, calls[q]->ready, 0));
      NTXENT_HIP_CHECK(hipMemcpyAsync(dst, calls[q]->send, bytes, hipMemcpyDeviceToDevice, stream));
    }
  }, [] {});
}

void ThreadComm::all_reduce_sum(float* buf, size_t count, hipStream_t stream) {
  Call c;
  c.send = buf;
  const int W = world();
  float* tmp = scratch((size_t)W * count);
  collective(c, stream, [&](std::vector<Call*>& calls) {
    for (int q = 0; q < W; ++q) {
      if (q != rank_) NTXENT_HIP_CHECK(hipStreamWaitEvent(stream, calls[q]->ready, 0));
      NTXENT_HIP_CHECK(hipMemcpyAsync(tmp + (size_t)q * count, calls[q]->send, count * sizeof(float),
                                      hipMemcpyDeviceToDevice, stream));
    }
  }, [&] { launch_sum_slabs(tmp, W, count, buf, stream); });
}

void ThreadComm::reduce_scatter_sum(const float* send, float* recv, size_t count, hipStream_t stream) {
  Call c;
  c.send = send;
  const int W = world();
  float* tmp = scratch((size_t)W * count);
  collective(c, stream, [&](std::vector<Call*>& calls) {
    for (int q = 0; q < W; ++q) {
      if (q != rank_) NTXENT_HIP_CHECK(hipStreamWaitEvent(stream, calls[q]->ready, 0));
      NTXENT_HIP_CHECK(hipMemcpyAsync(tmp + (size_t)q * count,
                                      static_cast<const float*>(calls[q]->send) + (size_t)rank_ * count,
                                      count * sizeof(float), hipMemcpyDeviceToDevice, stream));
    }
  }, [&] { launch_sum_slabs(tmp, W, count, recv, stream); });
}

void ThreadComm::send_recv(const std::vector<P2POp>& ops, hipStream_t stream) {
  Call c;
  c.ops = &ops;
  collective(c, stream, [&](std::vector<Call*>& calls) {
    // the k-th receive from q matches q's k-th send to this rank
    std::vector<int> seen(world(), 0);
    for (const auto& o : ops) {
      NTXENT_CHECK(o.peer >= 0 && o.peer < world(), "ThreadComm::send_recv: peer out of range");
      if (o.send) continue;
      const int q = o.peer, k = seen[q]++;
      const P2POp* match = nullptr;
      int n = 0;
      for (const auto& so : *calls[q]->ops)
        if (so.send && so.peer == rank_ && n++ == k) { match = &so; break; }
      NTXENT_CHECK(match != nullptr && match->bytes == o.bytes, "ThreadComm::send_recv: unmatched transfer");
      if (o.bytes == 0) continue;
      if (q != rank_) NTXENT_HIP_CHECK(hipStreamWaitEvent(stream, calls[q]->ready, 0));
      NTXENT_HIP_CHECK(hipMemcpyAsync(o.buf, match->buf, o.bytes, hipMemcpyDeviceToDevice, stream));
    }
  }, [] {});
}

void Comm::all_gather_chunks(const void* send, void* recv, size_t bytes, int nchunks, hipStream_t stream,
                             hipEvent_t* events) {
  NTXENT_CHECK(nchunks >= 1, "all_gather_chunks: nchunks must be >= 1");
  const int W = world(), r = rank();
  char* out = static_cast<char*>(recv);
  const char* in = static_cast<const char*>(send);
  char* own = out + (size_t)r * bytes;
  const size_t unit = 256;
  const size_t units = (bytes + unit - 1) / unit;
  for (int c = 0; c < nchunks; ++c) {
    const size_t b0 = std::min(bytes, units * c / nchunks * unit), b1 = std::min(bytes, units * (c + 1) / nchunks * unit);
    if (b1 > b0) {
      if (in != own) NTXENT_HIP_CHECK(hipMemcpyAsync(own + b0, in + b0, b1 - b0, hipMemcpyDeviceToDevice, stream));
      std::vector<P2POp> ops;
      for (int k = 1; k < W; ++k) {  // mesh: one link per peer, all in one group
        const int to = (r + k) % W, from = (r - k + W) % W;
        ops.push_back({true, own + b0, b1 - b0, to});
        ops.push_back({false, out + (size_t)from * bytes + b0, b1 - b0, from});
      }
      if (!ops.empty()) send_recv(ops, stream);
    }
    if (events) NTXENT_HIP_CHECK(hipEventRecord(events[c], stream));
  }
}
}  // namespace ntxent

#ifdef NTXENT_NO_RCCL
namespace ntxent {
namespace {
[[noreturn]] void no_rccl() { throw std::runtime_error("ntxent: built without RCCL (ENABLE_RCCL=OFF)"); }
}  // namespace
std::string RcclComm::unique_id() { no_rccl(); }
std::string RcclComm::version() { return "none"; }
RcclComm::RcclComm(int, int, const std::string&, int, AllGatherAlgo algo) : algo_(algo) { no_rccl(); }
RcclComm::~RcclComm() = default;
void RcclComm::all_gather(const void*, void*, size_t, hipStream_t) { no_rccl(); }
void RcclComm::all_reduce_sum(float*, size_t, hipStream_t) { no_rccl(); }
void RcclComm::reduce_scatter_sum(const float*, float*, size_t, hipStream_t) { no_rccl(); }
void RcclComm::send_recv(const std::vector<P2POp>&, hipStream_t) { no_rccl(); }
void RcclComm::check() {}
void RcclComm::abort() {}
}  // namespace ntxent
#else
#include <rccl/rccl.h>

#define NTXENT_RCCL_CHECK(expr)                                                               \
  do {                                                                                        \
    ncclResult_t _r = (expr);                                                                 \
    if (_r != ncclSuccess) {                                                                  \
      throw std::runtime_error(std::string("RCCL error ") + ncclGetErrorString(_r) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + " in " #expr);     \
    }                                                                                         \
  } while (0)

namespace ntxent {

static_assert(sizeof(ncclUniqueId) == RcclComm::kIdBytes, "ncclUniqueId size");

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  NTXENT_RCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

std::string RcclComm::version() {
  int v = 0;
  NTXENT_RCCL_CHECK(ncclGetVersion(&v));
  return std::to_string(v);
}

RcclComm::RcclComm(int rank, int world, const std::string& id, int device, AllGatherAlgo algo)
    : rank_(rank), world_(world), algo_(algo) {
  NTXENT_CHECK(world >= 1 && rank >= 0 && rank < world, "RcclComm: bad rank/world");
  NTXENT_CHECK(id.size() == kIdBytes, "RcclComm: unique id must be 128 bytes");
  if (device >= 0) NTXENT_HIP_CHECK(hipSetDevice(device));
  NTXENT_HIP_CHECK(hipGetDevice(&device_));
  ncclUniqueId uid;
  std::memcpy(&uid, id.data(), sizeof(uid));
  ncclComm_t c = nullptr;
  NTXENT_TRACE("ntxent.rccl.init");
  NTXENT_RCCL_CHECK(ncclCommInitRank(&c, world, uid, rank));
  comm_ = c;
}

RcclComm::~RcclComm() {
  if (comm_ && !aborted_) ncclCommDestroy(static_cast<ncclComm_t>(comm_));
}

void RcclComm::all_gather(const void* send, void* recv, size_t bytes, hipStream_t stream) {
  NTXENT_TRACE("ntxent.allgather");
  fault_point("allgather");
  NTXENT_CHECK(!aborted_, "RcclComm: communicator aborted");
  auto c = static_cast<ncclComm_t>(comm_);
  if (world_ == 1) {
    if (send != recv) NTXENT_HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, stream));
    return;
  }
  if (algo_ == AllGatherAlgo::kRccl) {
    NTXENT_RCCL_CHECK(ncclAllGather(send, recv, bytes, ncclChar, c, stream));
    return;
  }
  // Mesh: own shard to every peer and every peer's shard straight into its slot, all in one
  // group so the 7 xGMI links run concurrently (a ring would use one link per step).
  char* out = static_cast<char*>(recv);
  char* own = out + (size_t)rank_ * bytes;
  if (send != own) NTXENT_HIP_CHECK(hipMemcpyAsync(own, send, bytes, hipMemcpyDeviceToDevice, stream));
  NTXENT_RCCL_CHECK(ncclGroupStart());
  for (int k = 1; k < world_; ++k) {
    const int to = (rank_ + k) % world_, from = (rank_ - k + world_) % world_;
    NTXENT_RCCL_CHECK(ncclSend(own, bytes, ncclChar, to, c, stream));
    NTXENT_RCCL_CHECK(ncclRecv(out + (size_t)from * bytes, bytes, ncclChar, from, c, stream));
  }
  NTXENT_RCCL_CHECK(ncclGroupEnd());
}

void RcclComm::all_reduce_sum(float* buf, size_t count, hipStream_t stream) {
  NTXENT_TRACE("ntxent.allreduce");
  fault_point("allreduce");
  NTXENT_CHECK(!aborted_, "RcclComm: communicator aborted");
  if (world_ == 1) return;
  NTXENT_RCCL_CHECK(ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, static_cast<ncclComm_t>(comm_), stream));
}

void RcclComm::reduce_scatter_sum(const float* send, float* recv, size_t count, hipStream_t stream) {
  NTXENT_TRACE("ntxent.reducescatter");
  fault_point("reducescatter");
  NTXENT_CHECK(!aborted_, "RcclComm: communicator aborted");
  if (world_ == 1) {
    if (send != recv && count)
      NTXENT_HIP_CHECK(hipMemcpyAsync(recv, send, count * sizeof(float), hipMemcpyDeviceToDevice, stream));
    return;
  }
  NTXENT_RCCL_CHECK(ncclReduceScatter(send, recv, count, ncclFloat32, ncclSum, static_cast<ncclComm_t>(comm_), stream));
}

void RcclComm::send_recv(const std::vector<P2POp>& ops, hipStream_t stream) {
  NTXENT_TRACE("ntxent.sendrecv");
  fault_point("sendrecv");
  NTXENT_CHECK(!aborted_, "RcclComm: communicator aborted");
  auto c = static_cast<ncclComm_t>(comm_);
  NTXENT_RCCL_CHECK(ncclGroupStart());
  for (const auto& o : ops) {
    NTXENT_CHECK(o.peer >= 0 && o.peer < world_, "RcclComm::send_recv: peer out of range");
    if (o.send) NTXENT_RCCL_CHECK(ncclSend(o.buf, o.bytes, ncclChar, o.peer, c, stream));
    else NTXENT_RCCL_CHECK(ncclRecv(o.buf, o.bytes, ncclChar, o.peer, c, stream));
  }
  NTXENT_RCCL_CHECK(ncclGroupEnd());
}

void RcclComm::check() {
  if (!comm_ || aborted_) return;
  ncclResult_t async = ncclSuccess;
  NTXENT_RCCL_CHECK(ncclCommGetAsyncError(static_cast<ncclComm_t>(comm_), &async));
  if (async != ncclSuccess && async != ncclInProgress)
    throw std::runtime_error(std::string("RCCL async error: ") + ncclGetErrorString(async));
}

void RcclComm::abort() {
  if (comm_ && !aborted_) {
    ncclCommAbort(static_cast<ncclComm_t>(comm_));
    aborted_ = true;
  }
}

}  // namespace ntxent
#endif  // NTXENT_NO_RCCL

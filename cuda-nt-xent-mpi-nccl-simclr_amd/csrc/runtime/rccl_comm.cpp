// RCCL implementation of ntxent::Comm (see include/ntxent/comm.h).
#include "ntxent/comm.h"

#include <algorithm>
#include <cstring>
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

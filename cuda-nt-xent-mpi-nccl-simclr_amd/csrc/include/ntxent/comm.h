// ntxent-mi355x — collective layer of the native runtime (RCCL over xGMI).
//
// The reference links MPI and NCCL in CMake (CMakeLists.txt:13-14,41-47,115-121) but never
// calls either. Here the collectives the data-parallel NT-Xent needs are
// a small interface with an RCCL implementation:
//
//   all_gather   normalised rows Zq / ZqT (32 MiB per rank at B=4096, d=2048, fp16) and the
//                per-row LSE (fp32, Rpad floats per rank);
//   all_reduce   the scalar loss.
//
// MI355X nodes are a full xGMI mesh (7 links x ~153 GB/s per GPU), so besides RCCL's own
// all-gather (kRccl) there is a direct mesh variant (kMesh: every rank sends its shard to
// all peers at once with grouped ncclSend/ncclRecv, one link per peer) — pick by measurement.
// Bootstrap: rank 0 calls RcclComm::unique_id(), the bytes are broadcast by any side channel
// (torch.distributed store, file, MPI if present), every rank constructs RcclComm.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <memory>
#include <string>

namespace ntxent {

enum class AllGatherAlgo : int { kRccl = 0, kMesh = 1 };

// Collectives enqueued on a caller-provided stream (graph-capturable).
class Comm {
 public:
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // recv = concat over ranks of `bytes` from each rank's send. In place when
  // send == recv + rank * bytes.
  virtual void all_gather(const void* send, void* recv, size_t bytes, hipStream_t stream) = 0;
  virtual void all_reduce_sum(float* buf, size_t count, hipStream_t stream) = 0;
  // Throws if an asynchronous communicator error was reported (RCCL: ncclCommGetAsyncError).
  virtual void check() {}
};

// world = 1: every collective is a (possibly no-op) local copy.
class LocalComm final : public Comm {
 public:
  int rank() const override { return 0; }
  int world() const override { return 1; }
  void all_gather(const void* send, void* recv, size_t bytes, hipStream_t stream) override;
  void all_reduce_sum(float*, size_t, hipStream_t) override {}
};

// RCCL communicator (one per process / GPU).
class RcclComm final : public Comm {
 public:
  static constexpr size_t kIdBytes = 128;  // sizeof(ncclUniqueId)
  static std::string unique_id();          // call on one rank, broadcast the bytes
  RcclComm(int rank, int world, const std::string& id, int device = -1,
           AllGatherAlgo algo = AllGatherAlgo::kRccl);
  ~RcclComm() override;
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  int rank() const override { return rank_; }
  int world() const override { return world_; }
  void all_gather(const void* send, void* recv, size_t bytes, hipStream_t stream) override;
  void all_reduce_sum(float* buf, size_t count, hipStream_t stream) override;
  void check() override;
  void abort();  // tear the communicator down after an error (pending collectives fail)
  AllGatherAlgo algo() const { return algo_; }
  void set_algo(AllGatherAlgo a) { algo_ = a; }
  static std::string version();

 private:
  void* comm_ = nullptr;  // ncclComm_t
  int rank_ = 0, world_ = 1, device_ = 0;
  AllGatherAlgo algo_;
  bool aborted_ = false;
};

}  // namespace ntxent

// ntxent-mi355x — collective layer of the native runtime (RCCL over xGMI).
//
// The reference links MPI and NCCL in CMake (CMakeLists.txt:13-14,41-47,115-121) but never
// calls either. Here the collectives the data-parallel NT-Xent needs are
// a small interface with an RCCL implementation:
//
//   all_gather   normalised rows Zq / ZqT (32 MiB per rank at B=4096, d=2048, fp16) and the
//                per-row LSE (fp32, Rpad floats per rank);
//   all_reduce   the scalar loss;
//   reduce_scatter / send_recv / all_gather_chunks   the gradient reduce-scatter, the grouped
//                point-to-point exchanges of the symmetric data-parallel mode and chunked row
//                gathers (consumers start on the chunks that have arrived).
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
#include <vector>

namespace ntxent {

enum class AllGatherAlgo : int { kRccl = 0, kMesh = 1 };

// One side of a point-to-point transfer (see Comm::send_recv).
struct P2POp {
  bool send = true;     // true: send `bytes` from buf to peer; false: receive into buf from peer
  void* buf = nullptr;
  size_t bytes = 0;
  int peer = 0;
};

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
  // recv[count] = sum over ranks of send[rank * count .. (rank + 1) * count) (the backward
  // "reduce-scatter of embedding grads" of the data-parallel NT-Xent).
  virtual void reduce_scatter_sum(const float* send, float* recv, size_t count, hipStream_t stream) = 0;
  // One grouped batch of point-to-point transfers: every peer's transfers run concurrently on its
  // own xGMI link (RCCL: ncclGroupStart/End). Sends and receives between a pair match in order.
  virtual void send_recv(const std::vector<P2POp>& ops, hipStream_t stream) = 0;
  // all_gather in `nchunks` pieces of every rank's shard: piece c of all ranks (one grouped
  // batch) lands before piece c + 1, and events[c] (optional, nchunks of them) is recorded on
  // `stream` after piece c, so consumers can start on the rows that have arrived. In place as
  // all_gather. Bytes are split on 256-byte boundaries.
  void all_gather_chunks(const void* send, void* recv, size_t bytes, int nchunks, hipStream_t stream,
                         hipEvent_t* events = nullptr);
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
  void reduce_scatter_sum(const float* send, float* recv, size_t count, hipStream_t stream) override;
  void send_recv(const std::vector<P2POp>& ops, hipStream_t stream) override;  // peer 0 only: copies
};

// In-process W-rank communicator: rank r is driven by its own host thread, all ranks in one
// process (one GPU or several). Every collective is a host rendezvous of the W callers plus
// device copies between their buffers, ordered on each caller's stream by events (a rank's copy
// of a peer's buffer waits for the peer's enqueued work up to the call; every rank then waits
// for all copies before its stream moves on), so stream semantics match RCCL's. Reductions sum
// in rank order (deterministic). For single-GPU rehearsals of the multi-rank Engine paths and
// their tests; RCCL refuses two ranks on one device.
class ThreadCommGroup;
std::shared_ptr<ThreadCommGroup> make_thread_comm_group(int world);
class ThreadComm final : public Comm {
 public:
  ThreadComm(std::shared_ptr<ThreadCommGroup> group, int rank);
  ~ThreadComm() override;
  ThreadComm(const ThreadComm&) = delete;
  ThreadComm& operator=(const ThreadComm&) = delete;

  int rank() const override { return rank_; }
  int world() const override;
  void all_gather(const void* send, void* recv, size_t bytes, hipStream_t stream) override;
  void all_reduce_sum(float* buf, size_t count, hipStream_t stream) override;
  void reduce_scatter_sum(const float* send, float* recv, size_t count, hipStream_t stream) override;
  void send_recv(const std::vector<P2POp>& ops, hipStream_t stream) override;
  struct Call;  // one rank's posted collective (rccl_comm.cpp)

 private:
  template <typename Copies, typename After>
  void collective(Call& c, hipStream_t stream, Copies&& copies, After&& after);
  float* scratch(size_t floats);
  std::shared_ptr<ThreadCommGroup> group_;
  int rank_ = 0;
  hipEvent_t ready_ = nullptr, done_ = nullptr;
  float* scratch_ = nullptr;
  size_t scratch_floats_ = 0;
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
  void reduce_scatter_sum(const float* send, float* recv, size_t count, hipStream_t stream) override;
  void send_recv(const std::vector<P2POp>& ops, hipStream_t stream) override;
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

// ntxent-mi355x — native (libtorch-free) NT-Xent runtime.
//
// The reference's C++ surface is a pair of ATen functions that allocate O((2N)^2) buffers per
// call (src/ntxent_kernel.cu:138-239). Engine is the MI355X-native replacement for C++
// users, the native benchmark and the C++ tests:
//
//   * one arena allocation per (shape, dtype, world) sized up front — no allocation, host
//     sync or host decision inside a step, so a whole fwd+bwd step is hipGraph-capturable
//     (capture()/replay()) and replays with no per-kernel launch overhead;
//   * data parallel through a Comm (RCCL over xGMI): prep writes this rank's normalised rows
//     straight into its slot of the gathered buffer, the all-gathers run on a high-priority
//     comm stream while the own-rank (upper-triangular) tiles are computed, and only the
//     remote tiles wait for them; the ZqT gather is waited for only by the backward;
//   * roctx ranges per stage (NTXENT_ROCTX=1) and fault-injection sites (NTXENT_FAULT).
//
// Usage:
//   ntxent::Engine e({/*rows=*/8192, /*dim=*/2048, 0.07f, DType::BF16, DType::F16});
//   e.forward(h, stream); e.backward(nullptr, dh, stream);  float l = e.loss(stream);
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <utility>
#include <vector>

#include "ntxent/comm.h"
#include "ntxent/ntxent.h"

namespace ntxent {

// Global-batch negatives at world > 1 (parallel/ has the same two modes on torch.distributed):
//   kAllGather: every rank gathers all rows and computes its full row block S_{r,:};
//   kSymmetric: every rank pair's similarity block is computed ONCE (sym_jobs): rows travel
//     point to point in chunks (half an all-gather's bytes), the computing rank keeps row and
//     column partials and produces the partner's gradient contribution, sent back point to point
//     (Comm::send_recv: one grouped batch, a peer per xGMI link) while its own dZ GEMMs run.
enum class Negatives : int { kAllGather = 0, kSymmetric = 1 };

struct EngineConfig {
  int rows = 0;               // local rows R = 2 x per-view batch ([view1; view2] stacked)
  int dim = 0;
  float temperature = 0.07f;
  DType input = DType::BF16;  // dtype of h / dh
  // MFMA operand dtype (fp32 = exact path; FP8 = e4m3 forward GEMM, fp16 backward, cosines
  // always kept). Default: fp16, or bf16 in a CMake -DUSE_FP16=OFF build.
#ifdef NTXENT_DEFAULT_COMPUTE_BF16
  DType compute = DType::BF16;
#else
  DType compute = DType::F16;
#endif
  bool keep_cos = true;       // keep cosine tiles for the backward (else recompute them)
  // FP8 compute: the backward's coefficient matrix and Z^T in e4m3 too (Q8Stats; world 1).
  // -1: the process default (set_fp8_backward), 0 / 1: off / on.
  int fp8_backward = -1;
  bool check_finite = false;  // loss() throws on a non-finite loss
  bool small_path = true;     // single-rank small problems: the one-launch fwd / bwd kernels
  int small_splits = 0;       // small path: backward column splits (0: small_bwd_splits)
  // world > 1: CUs the similarity GEMMs leave free while an overlapped all-gather is in flight
  // (the persistent GEMM would otherwise hold every CU and the RCCL kernels could not start)
  int comm_reserve_cus = 8;
  Negatives negatives = Negatives::kSymmetric;  // world > 1 (kSymmetric keeps cosines)
  int device = -1;            // -1: current device
};

class Engine {
 public:
  explicit Engine(const EngineConfig& cfg, Comm* comm = nullptr);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  // Asynchronous on `stream`. h: device [rows][dim] (input dtype). The loss lands in
  // loss_device() (global mean over all ranks).
  void forward(const void* h, hipStream_t stream);
  // grad_out: device fp32 scalar, or nullptr for 1. dh: device [rows][dim] (input dtype).
  // Requires the preceding forward() of the same h.
  void backward(const float* grad_out, void* dh, hipStream_t stream);
  void step(const void* h, void* dh, hipStream_t stream) {
    forward(h, stream);
    backward(nullptr, dh, stream);
  }

  // hipGraph of one step() for fixed h / dh pointers; replay() launches it.
  void capture(const void* h, void* dh, hipStream_t stream);
  void replay(hipStream_t stream);
  bool captured() const { return exec_ != nullptr; }

  float loss(hipStream_t stream);  // synchronises `stream`
  const float* loss_device() const { return loss_; }
  const float* lse2_device() const { return lse2_all_; }  // [W*Rpad], log2 units
  const float* inv_norm_device() const { return inv_; }
  const Geometry& geometry() const { return g_; }
  const EngineConfig& config() const { return cfg_; }
  size_t device_bytes() const { return arena_bytes_; }
  int fwd_tiles() const { return n_fwd_; }
  int own_tiles() const { return n_own_; }
  int dz_tiles() const { return n_dz_; }
  bool small() const { return small_; }
  bool symmetric() const { return symm_; }
  Comm* comm() const { return comm_; }

 private:
  EngineConfig cfg_;
  Geometry g_;
  Comm* comm_ = nullptr;
  const void* h_ = nullptr;  // input of the last forward (read by the backward)
  int rank_ = 0, world_ = 1, device_ = 0;
  int n_fwd_ = 0, n_own_ = 0, n_dz_ = 0;
  size_t cs_ = 2;             // bytes per element of the backward dtype (zq, ZqT, cosines, C)
  bool f8_ = false;           // fp8 forward GEMM (e4m3 copy zq8_all_), fp16 backward
  bool fuse_ = false;          // normalisation backward in the dZ epilogue (NormFuse)
  int* dot_cnt_ = nullptr;     // dot fold counters (NormFuse::dot_cnt)
  float* dotp_ = nullptr;      // dot partials [Rpad][dot_slots] (fuse_)
  float* dot_ = nullptr;       // dot [Rpad]
  // symmetric data-parallel mode (Negatives::kSymmetric, engine_sym.cpp)
  bool symm_ = false;
  std::vector<SymJob> jobs_, inc_;
  int nch_ = 1, nfull_ = 0;
  std::vector<std::pair<int, int>> segs_;  // (first, count) of each row chunk's cross tiles
  float2* part_x_ = nullptr;               // column partials of the cross tiles
  float2* fold_pre_ = nullptr;             // folded LSE scratch (RawRows::fold_pre / fold_cnt)
  int* fold_cnt_ = nullptr;
  float2* xsend_ = nullptr;                // packed column partials of the k-split block (one run per row tile
  float2* xrecv_ = nullptr;                // otherwise: one send/recv per partner instead of one per row tile)
  char* mbuf_ = nullptr;                   // partners' mirrored coefficient blocks
  char* contrib_ = nullptr;                // partners' gradient contributions (nfull + split blocks)
  char* recv_ = nullptr;                   // received contributions [inc][Rpad][dim_n]
  size_t ccs_ = 2;                         // bytes per contribution element (fp16, fp32 plans: 4)
  int4* dz_rows_ = nullptr;                // dz_view tile lists: see init_sym
  std::vector<std::pair<int, int>> dz_ranges_;
  std::vector<hipEvent_t> ev_chunk_;
  hipEvent_t ev_f16_ = nullptr, ev_x_ = nullptr, ev_xdone_ = nullptr, ev_c_ = nullptr, ev_cdone_ = nullptr;
  void init_sym();
  void forward_sym(const void* h, hipStream_t s);
  void backward_sym(const float* grad_out, void* dh, hipStream_t s);
  const int4* dz_rows(int m0, int m1) const;
  void dz_view(const char* abuf, long a_tile0, long a_panel_tiles, const char* bbuf, int b_block0, long b_col0,
               int k_tiles, int m0, int m1, void* out, bool accum, bool out_f16, hipStream_t s,
               const GemmWorkspace& ws);
  bool q8_ = false;            // fp8 backward (e4m3 C and Z^T, EngineConfig::fp8_backward)
  float* q8_mneg_ = nullptr;   // Q8Stats: negatives-only row max [Rpad], min LSE [1]
  float* q8_lmin_ = nullptr;
  char* zq8t_ = nullptr;       // e4m3(256 Zq^T) [dim_n][q8_ldt]
  bool small_ = false;        // small-problem path (small_kernels.hip)
  void* small_scratch_ = nullptr;
  DType bwd_ = DType::F16;
  void* arena_ = nullptr;
  size_t arena_bytes_ = 0;
  char* zq_all_ = nullptr;
  char* zq8_all_ = nullptr;
  char* zqt_all_ = nullptr;
  float* inv_ = nullptr;
  float* ypos_ = nullptr;
  float2* part_ = nullptr;
  char* sbuf_ = nullptr;
  char* cbuf_ = nullptr;
  float* lse2_all_ = nullptr;
  float* cpos_ = nullptr;
  float* block_loss_ = nullptr;
  float* loss_ = nullptr;
  float* one_ = nullptr;
  float* slabs_ = nullptr;
  int4* fwd_tiles_ = nullptr;
  int4* dz_tiles_ = nullptr;
  GemmWorkspace ws_;
  hipStream_t comm_stream_ = nullptr;
  hipEvent_t ev_prep_ = nullptr, ev_zq_ = nullptr, ev_zqt_ = nullptr;

  bool zqt_pending_ = false;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
};

}  // namespace ntxent

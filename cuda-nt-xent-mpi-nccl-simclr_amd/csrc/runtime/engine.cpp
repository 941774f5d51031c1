// Native NT-Xent runtime (see include/ntxent/engine.h).
//
// Replaces the reference host launchers ntxent_forward_cuda / ntxent_backward_cuda
// (src/ntxent_kernel.cu:138-203, 205-239): those allocate the 2N x 2N logits, softmax and
// grad_logits per call and run cuBLAS on the legacy stream; here every buffer lives in one
// arena sized once, all work is stream-ordered (graph-capturable) and collectives overlap
// the own-rank tiles.
#include "ntxent/engine.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <stdexcept>
#include <vector>

#include "ntxent/trace.h"

namespace ntxent {

// float2 elements of the packed column-partial runs of the jobs whose partner row range is not a
// whole block (k0 > 0 or k1 < row_tiles: the runs of consecutive row tiles are Rpad apart, not
// adjacent), see Engine::forward_sym
static size_t sym_xpack_floats2(const std::vector<SymJob>& jobs, int row_tiles) {
  size_t n = 0;
  for (const SymJob& j : jobs)
    if (j.k1 - j.k0 != row_tiles) n += (size_t)(j.m1 - j.m0) * (j.k1 - j.k0) * kTile;
  return n;
}
namespace {

constexpr size_t kAlign = 256;

size_t align_up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

}  // namespace

Engine::Engine(const EngineConfig& cfg, Comm* comm) : cfg_(cfg), comm_(comm) {
  NTXENT_TRACE("ntxent.engine.init");
  if (cfg.device >= 0) NTXENT_HIP_CHECK(hipSetDevice(cfg.device));
  NTXENT_HIP_CHECK(hipGetDevice(&device_));
  rank_ = comm ? comm->rank() : 0;
  world_ = comm ? comm->world() : 1;
  g_ = make_geometry(cfg.rows, cfg.dim, world_, rank_, cfg.temperature);
  f8_ = cfg.compute == DType::FP8;
#ifdef NTXENT_NO_FP8
  if (f8_) throw std::runtime_error("ntxent::Engine: fp8 compute requested but this build has ENABLE_FP8=OFF");
#endif
  if (f8_) cfg_.keep_cos = true;  // fp8: the fp16 backward uses the forward's own cosines
  bwd_ = backward_dtype(cfg.compute);
  cs_ = dtype_size(bwd_);
  small_ = cfg.small_path && world_ == 1 && small_path_eligible(g_, cfg.compute);
  symm_ = world_ > 1 && cfg.negatives == Negatives::kSymmetric;
  if (symm_) {
    cfg_.keep_cos = true;  // the coefficient pass reads both blocks' cosines from the forward
    jobs_ = sym_jobs(world_, rank_, g_.row_tiles);
    inc_ = sym_incoming(world_, rank_, g_.row_tiles);
    nch_ = sym_num_chunks(g_.row_tiles);
    ccs_ = bwd_ == DType::F32 ? 4 : 2;
  }
  q8_ = !small_ && fp8_backward_eligible(g_, cfg.compute) &&
        (cfg.fp8_backward < 0 ? fp8_backward_enabled() : cfg.fp8_backward != 0);
  // normalisation backward fused into the dZ epilogue (the coefficient pass emits dot partials;
  // the symmetric mode sums received contributions in launch_norm_bwd instead)
  // (not on fp8 plans: dot_i = sum_j C_ij cos_ij would use the e4m3 forward's cosines, ~1e-2 off)
  fuse_ = !small_ && !symm_ && !f8_ && bwd_ != DType::F32 && g_.dim % 8 == 0;

  const auto ft = symm_ ? build_sym_fwd_tiles(g_, jobs_, nch_) : build_fwd_tiles(g_);
  const auto dt = build_dz_tiles(g_);
  n_fwd_ = (int)ft.size();
  n_own_ = count_own_fwd_tiles(g_);
  n_dz_ = (int)dt.size();
  ws_.num_cus = device_info(device_).num_cus;
  ws_.bytes = gemm_workspace_bytes(std::max(n_fwd_, n_dz_), ws_.num_cus);

  const size_t W = world_, Rp = g_.rows_pad, R = g_.rows;
  struct Slot { void** p; size_t bytes; };
  const std::vector<Slot> slots = {
      {(void**)&zq_all_, W * Rp * g_.ld_k * cs_},
      {(void**)&zq8_all_, f8_ ? W * Rp * g_.ld_k8 : 0},
      {(void**)&zqt_all_, q8_ ? 0 : W * g_.dim_n * g_.ld_t * cs_},
      {(void**)&zq8t_, q8_ ? (size_t)g_.dim_n * (size_t)q8_ldt(g_) : 0},
      {(void**)&q8_mneg_, q8_ ? Rp * 4 : 0},
      {(void**)&q8_lmin_, q8_ ? (size_t)4 : (size_t)0},
      {(void**)&inv_, R * 4},
      {(void**)&ypos_, R * 4},
      {(void**)&part_, (size_t)g_.col_tiles * Rp * sizeof(float2)},
      {(void**)&sbuf_, cfg_.keep_cos ? (size_t)n_fwd_ * kTileElems * cs_ : 0},
      {(void**)&cbuf_, (size_t)g_.row_tiles * (symm_ ? sym_c_ld(g_) : g_.col_tiles) * kTileElems * cs_},
      {(void**)&lse2_all_, W * Rp * 4},
      {(void**)&cpos_, Rp * 4},
      {(void**)&block_loss_, (size_t)lse_scratch_floats(g_) * 4},
      {(void**)&loss_, 4},
      {(void**)&one_, 4},
      // symmetric mode, fp32 plans: the received contributions follow the own slab (one stack)
      {(void**)&slabs_, Rp * g_.dim_n * 4 * (symm_ && ccs_ == 4 ? 1 + inc_.size() : 1)},
      {(void**)&fold_pre_, world_ == 1 ? Rp * sizeof(float2) : 0},
      {(void**)&fold_cnt_, world_ == 1 ? (Rp / 64 + 1) * sizeof(int) : 0},
      {(void**)&part_x_, symm_ ? (size_t)g_.col_tiles * Rp * sizeof(float2) : 0},
      {(void**)&xsend_, symm_ ? sym_xpack_floats2(jobs_, g_.row_tiles) * sizeof(float2) : 0},
      {(void**)&xrecv_, symm_ ? sym_xpack_floats2(inc_, g_.row_tiles) * sizeof(float2) : 0},
      {(void**)&mbuf_, symm_ ? (size_t)std::max(1, world_ / 2) * g_.row_tiles * g_.row_tiles * kTileElems * cs_ : 0},
      {(void**)&contrib_, symm_ ? (jobs_.size() + 1) * Rp * g_.dim_n * ccs_ : 0},
      {(void**)&recv_, symm_ && ccs_ == 2 ? inc_.size() * Rp * g_.dim_n * ccs_ : 0},
      {(void**)&dz_rows_, symm_ ? (size_t)4 * (world_ + 1) * g_.row_tiles * (g_.dim_n / kTile) * sizeof(int4) : 0},
      {(void**)&dotp_, fuse_ ? Rp * (size_t)dot_slots(g_) * 4 : 0},
      {(void**)&dot_, fuse_ ? Rp * 4 : 0},
      {(void**)&dot_cnt_, fuse_ ? 2 * sizeof(int) : 0},
      {(void**)&fwd_tiles_, ft.size() * sizeof(int4)},
      {(void**)&dz_tiles_, dt.size() * sizeof(int4)},
      {&ws_.ptr, ws_.bytes},
      {&small_scratch_, small_ ? small_scratch_bytes(g_, std::max(small_bwd_splits(g_), cfg.small_splits)) : 0},
  };
  size_t total = 0;
  for (const auto& s : slots) total += align_up(s.bytes);
  arena_bytes_ = total;
  NTXENT_HIP_CHECK(hipMalloc(&arena_, total));
  char* base = static_cast<char*>(arena_);
  for (const auto& s : slots) {
    *s.p = s.bytes ? base : nullptr;
    base += align_up(s.bytes);
  }
  // zero once: the stream-K and LSE arrival counters are self-cleaning afterwards
  NTXENT_HIP_CHECK(hipMemset(arena_, 0, total));
  NTXENT_HIP_CHECK(hipMemcpy(fwd_tiles_, ft.data(), ft.size() * sizeof(int4), hipMemcpyHostToDevice));
  NTXENT_HIP_CHECK(hipMemcpy(dz_tiles_, dt.data(), dt.size() * sizeof(int4), hipMemcpyHostToDevice));
  const float one = 1.0f;
  NTXENT_HIP_CHECK(hipMemcpy(one_, &one, 4, hipMemcpyHostToDevice));
  if (world_ > 1) {
    int lo = 0, hi = 0;
    NTXENT_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    NTXENT_HIP_CHECK(hipStreamCreateWithPriority(&comm_stream_, hipStreamNonBlocking, hi));
    NTXENT_HIP_CHECK(hipEventCreateWithFlags(&ev_prep_, hipEventDisableTiming));
    NTXENT_HIP_CHECK(hipEventCreateWithFlags(&ev_zq_, hipEventDisableTiming));
    NTXENT_HIP_CHECK(hipEventCreateWithFlags(&ev_zqt_, hipEventDisableTiming));
  }
  if (symm_) init_sym();
}

Engine::~Engine() {
  for (hipEvent_t e : ev_chunk_) hipEventDestroy(e);
  for (hipEvent_t e : {ev_f16_, ev_x_, ev_xdone_, ev_c_, ev_cdone_})
    if (e) hipEventDestroy(e);
  if (exec_) hipGraphExecDestroy(exec_);
  if (graph_) hipGraphDestroy(graph_);
  if (ev_prep_) hipEventDestroy(ev_prep_);
  if (ev_zq_) hipEventDestroy(ev_zq_);
  if (ev_zqt_) hipEventDestroy(ev_zqt_);
  if (comm_stream_) hipStreamDestroy(comm_stream_);
  if (arena_) hipFree(arena_);
}

void Engine::forward(const void* h, hipStream_t s) {
  NTXENT_TRACE("ntxent.forward");
  h_ = h;
  if (symm_) {
    forward_sym(h, s);
    return;
  }
  const size_t Rp = g_.rows_pad;
  char* zq_local = zq_all_ + (size_t)rank_ * Rp * g_.ld_k * cs_;
  char* zqt_local = zqt_all_ + (size_t)rank_ * g_.dim_n * g_.ld_t * cs_;
  const bool raw = world_ == 1 && !small_ && !f8_ && cfg_.keep_cos && raw_forward_enabled() &&
                   raw_forward_eligible(g_, cfg_.input, cfg_.compute);
  RawRows rr;
  rr.h = h;
  rr.in = cfg_.input;
  rr.inv = inv_;
  rr.zqt = zqt_local;
  rr.zt = bwd_;
  // the LSE launch's outputs: the diagonal remainder's launch may compute them (rr.lse_folded)
  rr.ypos = ypos_;
  rr.lse2 = lse2_all_;
  rr.cpos = cpos_;
  rr.block_loss = block_loss_;
  rr.loss = loss_;
  rr.fold_pre = fold_pre_;
  rr.fold_cnt = fold_cnt_;
  // forward GEMM operand: the e4m3 rows for fp8 plans, else zq itself (or the input rows: raw)
  char* op_all = f8_ ? zq8_all_ : zq_all_;
  const size_t op_bytes = f8_ ? Rp * g_.ld_k8 : Rp * g_.ld_k * cs_;
  char* op_local = op_all + (size_t)rank_ * op_bytes;
  {
    NTXENT_TRACE("ntxent.prep");
    fault_point("prep");
    if (small_) {  // one launch (row prologue fused up to kSmallFuseMaxRows): tiles + LSE merge + loss
      // (lse2 -> lse2_all_, a_i -> cpos_)
      if (!small_fwd_fused(g_)) launch_prep(cfg_.input, bwd_, h, zq_local, inv_, ypos_, g_, s);
      NTXENT_TRACE("ntxent.small_fwd");
      fault_point("fwd");
      launch_small_fwd(cfg_.input, cfg_.compute, h, zq_local, inv_, ypos_, lse2_all_, cpos_, loss_, small_scratch_,
                       g_, s);
      if (fault_armed("nonfinite")) NTXENT_HIP_CHECK(hipMemsetAsync(loss_, 0xFF, 4, s));  // NaN
      return;
    }
    // raw-operand forward (RawRows): no unit rows at all, the prologue computes inv and ypos only
    launch_prep(cfg_.input, bwd_, h, raw ? nullptr : zq_local, inv_, ypos_, g_, s, f8_ ? op_local : nullptr);
    // world 1: the transpose is written by the LSE launch (beside the merge, see below)
    if (world_ > 1) launch_transpose(bwd_, zq_local, zqt_local, g_, s);
  }
  if (world_ > 1) {
    // Gathers on the comm stream; the own-rank tiles only need this rank's slot.
    NTXENT_HIP_CHECK(hipEventRecord(ev_prep_, s));
    NTXENT_HIP_CHECK(hipStreamWaitEvent(comm_stream_, ev_prep_, 0));
    comm_->all_gather(op_local, op_all, op_bytes, comm_stream_);
    NTXENT_HIP_CHECK(hipEventRecord(ev_zq_, comm_stream_));
    // the backward's B operand: the ZqT blocks
    comm_->all_gather(zqt_local, zqt_all_, (size_t)g_.dim_n * g_.ld_t * cs_, comm_stream_);
    NTXENT_HIP_CHECK(hipEventRecord(ev_zqt_, comm_stream_));
    zqt_pending_ = true;
  }
  // both forward launches overlap a gather (rows, then ZqT): leave CUs for the RCCL kernels
  bool zt_fwd = false;  // Z^T written by the forward launch (raw, beside the diagonal remainder)
  GemmWorkspace ws_ovl = ws_;
  if (world_ > 1) ws_ovl.sched_cus = std::max(1, ws_.num_cus - std::min(cfg_.comm_reserve_cus, ws_.num_cus / 2));
  {
    NTXENT_TRACE("ntxent.fwd_gemm.own");
    fault_point("fwd");
    zt_fwd = launch_fwd_stats(cfg_.compute, op_local, op_all, fwd_tiles_, n_own_, part_, sbuf_, ws_ovl, g_, s,
                              BlockView{}, nullptr, own_diag_tail(g_), nullptr, raw ? &rr : nullptr);
  }
  if (n_fwd_ > n_own_) {
    NTXENT_TRACE("ntxent.fwd_gemm.remote");
    if (world_ > 1) NTXENT_HIP_CHECK(hipStreamWaitEvent(s, ev_zq_, 0));
    launch_fwd_stats(cfg_.compute, op_local, op_all, fwd_tiles_ + n_own_, n_fwd_ - n_own_, part_,
                     sbuf_ ? sbuf_ + (size_t)n_own_ * kTileElems * cs_ : nullptr, ws_ovl, g_, s);
  }
  fault_point("lse");
  if (!(raw && rr.lse_folded)) {
    NTXENT_TRACE("ntxent.lse");
    if (q8_) {
      Q8Stats q8;
      q8.mneg2 = q8_mneg_;
      q8.lmin = q8_lmin_;
      q8.zq8t = zq8t_;
      launch_lse(part_, ypos_, lse2_all_, cpos_, block_loss_, loss_, g_, s, bwd_, zq_local, nullptr, &q8);
    } else if (world_ == 1)
      launch_lse(part_, ypos_, lse2_all_, cpos_, block_loss_, loss_, g_, s, bwd_, raw ? nullptr : zq_local,
                 zt_fwd ? nullptr : zqt_local, nullptr, raw && !zt_fwd ? &rr : nullptr);
    else
      launch_lse(part_, ypos_, lse2_all_, cpos_, block_loss_, loss_, g_, s);
  }
  if (world_ > 1) {
    NTXENT_TRACE("ntxent.lse_gather");
    comm_->all_gather(lse2_all_ + (size_t)rank_ * Rp, lse2_all_, Rp * 4, s);
    comm_->all_reduce_sum(loss_, 1, s);
  }
  if (fault_armed("nonfinite")) NTXENT_HIP_CHECK(hipMemsetAsync(loss_, 0xFF, 4, s));  // NaN
}

void Engine::backward(const float* grad_out, void* dh, hipStream_t s) {
  NTXENT_TRACE("ntxent.backward");
  NTXENT_CHECK(h_ != nullptr, "backward() before forward()");
  if (symm_) {
    backward_sym(grad_out, dh, s);
    return;
  }
  const size_t Rp = g_.rows_pad;
  const char* zq_local = zq_all_ + (size_t)rank_ * Rp * g_.ld_k * cs_;
  Q8Stats q8;  // fp8 backward (q8_)
  q8.mneg2 = q8_mneg_;
  q8.lmin = q8_lmin_;
  q8.zq = zq_local;
  if (small_) {
    NTXENT_TRACE("ntxent.small_bwd");
    fault_point("dz");
    launch_small_bwd(cfg_.input, cfg_.compute, zq_local, h_, inv_, lse2_all_, cpos_, grad_out ? grad_out : one_, dh,
                     small_scratch_, g_, s, std::min(cfg_.small_splits, small_rows_pad(g_) / 64));
    return;
  }
  // half C: upper coefficient tiles only, the dZ reads the lower ones transposed
  const bool half_c = cfg_.keep_cos && !q8_ && half_c_enabled() && dz_half_c_eligible(bwd_, g_, n_dz_, ws_);
  // the dot reduce folded into the dZ (NormFuse::dot_cnt)
  const bool dfold = fuse_ && !q8_ && dz_dot_fold_eligible(bwd_, g_, n_dz_, ws_);
  {
    NTXENT_TRACE("ntxent.coef");
    fault_point("coef");
    if (cfg_.keep_cos)
      launch_coef(bwd_, sbuf_, cbuf_, lse2_all_, cpos_, fwd_tiles_, n_fwd_, g_, s, nullptr, dotp_, q8_ ? &q8 : nullptr,
                  half_c);
    else
      launch_coef_gemm(cfg_.compute, zq_local, zq_all_, cbuf_, lse2_all_, cpos_, fwd_tiles_, n_fwd_, ws_, g_, s,
                       BlockView{}, dotp_);
    if (fuse_ && !dfold) launch_dot_reduce(dotp_, dot_, g_, s);
  }
  if (zqt_pending_) {
    NTXENT_HIP_CHECK(hipStreamWaitEvent(s, ev_zqt_, 0));
    zqt_pending_ = false;
  }
  {
    NTXENT_TRACE("ntxent.dz_gemm");
    fault_point("dz");
    NormFuse nf;
    nf.h = h_;
    nf.in = cfg_.input;
    nf.inv = inv_;
    nf.dot = dot_;
    nf.grad_out = grad_out ? grad_out : one_;
    nf.dh = dh;
    if (dfold) {
      nf.dotp = dotp_;
      nf.dot_cnt = dot_cnt_;
    }
    const bool fused =
        q8_ ? launch_dz(DType::FP8, cbuf_, zq8t_, dz_tiles_, n_dz_, slabs_, ws_, g_, s, /*out_f16=*/true,
                        fuse_ ? &nf : nullptr, &q8, cpos_)
            : launch_dz(bwd_, cbuf_, zqt_all_, dz_tiles_, n_dz_, slabs_, ws_, g_, s, /*out_f16=*/bwd_ != DType::F32,
                        fuse_ ? &nf : nullptr, nullptr, nullptr, half_c);
    if (fused) return;  // dh written by the dZ epilogue
  }
  {
    NTXENT_TRACE("ntxent.norm_bwd");
    fault_point("norm_bwd");
    if (bwd_ != DType::F32)  // fp16 dZ slab (reduced-precision plans)
      launch_norm_bwd(cfg_.input, nullptr, 0, h_, inv_, grad_out ? grad_out : one_, dh, g_, s, slabs_, 1);
    else
      launch_norm_bwd(cfg_.input, slabs_, 1, h_, inv_, grad_out ? grad_out : one_, dh, g_, s);
  }
}

void Engine::capture(const void* h, void* dh, hipStream_t s) {
  NTXENT_TRACE("ntxent.graph.capture");
  fault_point("graph");
  NTXENT_CHECK(s != nullptr, "graph capture needs a non-default stream");
  if (exec_) { hipGraphExecDestroy(exec_); exec_ = nullptr; }
  if (graph_) { hipGraphDestroy(graph_); graph_ = nullptr; }
  NTXENT_HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  try {
    step(h, dh, s);
  } catch (...) {
    hipGraph_t g = nullptr;
    hipStreamEndCapture(s, &g);
    if (g) hipGraphDestroy(g);
    throw;
  }
  NTXENT_HIP_CHECK(hipStreamEndCapture(s, &graph_));
  NTXENT_HIP_CHECK(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0));
}

void Engine::replay(hipStream_t s) {
  NTXENT_CHECK(exec_ != nullptr, "replay() before capture()");
  NTXENT_HIP_CHECK(hipGraphLaunch(exec_, s));
}

float Engine::loss(hipStream_t s) {
  float l = 0.f;
  NTXENT_HIP_CHECK(hipMemcpyAsync(&l, loss_, 4, hipMemcpyDeviceToHost, s));
  NTXENT_HIP_CHECK(hipStreamSynchronize(s));
  if (comm_) comm_->check();
  if (cfg_.check_finite && !std::isfinite(l)) throw std::runtime_error("ntxent: non-finite loss");
  return l;
}

}  // namespace ntxent

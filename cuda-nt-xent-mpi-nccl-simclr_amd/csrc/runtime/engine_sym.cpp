// Engine: symmetric data-parallel mode (EngineConfig::negatives = Negatives::kSymmetric).
//
// The native counterpart of parallel/symmetric.py (same block assignment sym_jobs, same tile
// lists and stage launchers, same exchanges), over ntxent::Comm instead of torch.distributed:
// every unordered rank pair's similarity block is computed once across the group.
//
//   forward : prep (+ own ZqT) -> rows point to point in sym_num_chunks chunks on the comm
//             stream (Comm::send_recv, a peer per xGMI link) while the own upper-triangular
//             tiles run -> each chunk's cross tiles as it lands -> cross tiles' column partials
//             to their rows' owners -> LSE -> LSE all-gather + loss all-reduce.
//   backward: partners' ZqT blocks transposed locally -> coefficient pass (own tiles mirrored,
//             cross tiles mirrored per partner) -> partners' gradient contributions C_{q,r} Z_r
//             (one stacked GEMM for the full blocks) sent point to point while this rank's own
//             dZ GEMMs run -> normalisation backward summing the received contributions.
// No reference counterpart (the reference has no multi-GPU code).
#include <algorithm>

#include "ntxent/engine.h"
#include "ntxent/trace.h"

namespace ntxent {

void Engine::init_sym() {
  const int rt = g_.row_tiles, ct = g_.col_tiles;
  // chunk segments of the cross tiles (build_sym_fwd_tiles order)
  int first = n_own_;
  for (int c = 0; c < nch_; ++c) {
    const int c0 = rt * c / nch_, c1 = rt * (c + 1) / nch_;
    int n = 0;
    for (const SymJob& j : jobs_) n += (j.m1 - j.m0) * std::max(0, std::min(j.k1, c1) - std::max(j.k0, c0));
    segs_.push_back({first, n});
    first += n;
  }
  NTXENT_CHECK(first == n_fwd_, "symmetric engine: tile segments do not cover the tile list");
  for (const SymJob& j : jobs_) nfull_ += (j.m0 == 0 && j.m1 == rt && j.k0 == 0 && j.k1 == rt) ? 1 : 0;
  for (int i = 0; i < nfull_; ++i)
    NTXENT_CHECK(jobs_[i].m0 == 0 && jobs_[i].m1 == rt && jobs_[i].k0 == 0 && jobs_[i].k1 == rt,
                 "symmetric engine: full blocks must precede the split block");
  // dz_view tile lists (row tiles [m0, m1) x every dim_n tile): partners' full blocks stacked,
  // the split block's partner rows, the own rows, the split block's own rows
  const int tn = g_.dim_n / kTile;
  dz_ranges_ = {{0, std::max(1, nfull_) * rt}, {0, rt}};
  if ((int)jobs_.size() > nfull_) {
    const SymJob& sp = jobs_.back();
    dz_ranges_.push_back({sp.k0, sp.k1});
    dz_ranges_.push_back({sp.m0, sp.m1});
  }
  std::vector<int4> v;
  for (const auto& r : dz_ranges_)
    for (int ti = r.first; ti < r.second; ++ti)
      for (int n = 0; n < tn; ++n) v.push_back(make_int4(ti, n, 0, 0));
  NTXENT_CHECK(v.size() <= (size_t)4 * (world_ + 1) * rt * tn, "symmetric engine: tile-list slot too small");
  NTXENT_HIP_CHECK(hipMemcpy(dz_rows_, v.data(), v.size() * sizeof(int4), hipMemcpyHostToDevice));
  (void)ct;
  ev_chunk_.resize(nch_);
  for (auto& e : ev_chunk_) NTXENT_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (hipEvent_t* e : {&ev_f16_, &ev_x_, &ev_xdone_, &ev_c_, &ev_cdone_})
    NTXENT_HIP_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
}

const int4* Engine::dz_rows(int m0, int m1) const {
  size_t off = 0;
  const int tn = g_.dim_n / kTile;
  for (const auto& r : dz_ranges_) {
    if (r.first == m0 && r.second == m1) return dz_rows_ + off;
    off += (size_t)(r.second - r.first) * tn;
  }
  NTXENT_CHECK(false, "symmetric engine: no tile list for this row range");
  return nullptr;
}

// out[row tiles m0..m1) (+)= A * B (the torch op dz_view, ntxent_torch.cpp): A = coefficient
// tiles from tile a_tile0 (row panels a_panel_tiles tiles apart), K = k_tiles * 256 columns of
// the ZqT blocks from block b_block0, column b_col0 (a K range past one block covers whole blocks).
void Engine::dz_view(const char* abuf, long a_tile0, long a_panel_tiles, const char* bbuf, int b_block0, long b_col0,
                     int k_tiles, int m0, int m1, void* out, bool accum, bool out_f16, hipStream_t s,
                     const GemmWorkspace& ws) {
  if (m1 <= m0 || k_tiles == 0) return;
  const long blk = (long)g_.dim_n * g_.ld_t;
  const long kcols = (long)k_tiles * kTile;
  long kblk_cols = kcols;
  if (b_col0 + kcols > g_.rows_pad) {
    NTXENT_CHECK(b_col0 == 0 && kcols % g_.rows_pad == 0, "symmetric engine: multi-block K must cover whole blocks");
    kblk_cols = g_.rows_pad;
  }
  const char* a = abuf + (size_t)a_tile0 * kTileElems * cs_;
  const char* b = bbuf + ((size_t)b_block0 * blk + b_col0) * cs_;
  launch_dz_view(bwd_, a, a_panel_tiles, b, kblk_cols, blk, k_tiles, dz_rows(m0, m1), (m1 - m0) * (g_.dim_n / kTile),
                 out, accum, ws, g_, s, out_f16);
}

void Engine::forward_sym(const void* h, hipStream_t s) {
  const size_t Rp = g_.rows_pad;
  const int rt = g_.row_tiles, r = rank_;
  char* zq_local = zq_all_ + (size_t)r * Rp * g_.ld_k * cs_;
  char* zqt_local = zqt_all_ + (size_t)r * g_.dim_n * g_.ld_t * cs_;
  char* op_all = f8_ ? zq8_all_ : zq_all_;
  const size_t op_row = f8_ ? g_.ld_k8 : g_.ld_k * cs_;  // bytes per forward-operand row
  char* op_local = op_all + (size_t)r * Rp * op_row;
  {
    NTXENT_TRACE("ntxent.prep");
    fault_point("prep");
    launch_prep(cfg_.input, bwd_, h, zq_local, inv_, ypos_, g_, s, f8_ ? op_local : nullptr);
    launch_transpose(bwd_, zq_local, zqt_local, g_, s);  // own B operand of the backward
  }
  // rows point to point, chunk c of the row tiles per grouped batch (the cross tiles of chunk c
  // run while chunk c + 1 is on the wire)
  NTXENT_HIP_CHECK(hipEventRecord(ev_prep_, s));
  NTXENT_HIP_CHECK(hipStreamWaitEvent(comm_stream_, ev_prep_, 0));
  for (int c = 0; c < nch_; ++c) {
    const int c0 = rt * c / nch_, c1 = rt * (c + 1) / nch_;
    std::vector<P2POp> ops;
    for (const SymJob& p : inc_) {  // p.q uses my row tiles [k0, k1)
      const int a0 = std::max(p.k0, c0), a1 = std::min(p.k1, c1);
      if (a0 < a1) ops.push_back({true, op_local + (size_t)a0 * kTile * op_row, (size_t)(a1 - a0) * kTile * op_row, p.q});
    }
    for (const SymJob& j : jobs_) {  // I use q's row tiles [k0, k1)
      const int a0 = std::max(j.k0, c0), a1 = std::min(j.k1, c1);
      if (a0 < a1)
        ops.push_back({false, op_all + ((size_t)j.q * Rp + (size_t)a0 * kTile) * op_row, (size_t)(a1 - a0) * kTile * op_row,
                       j.q});
    }
    if (!ops.empty()) comm_->send_recv(ops, comm_stream_);
    NTXENT_HIP_CHECK(hipEventRecord(ev_chunk_[c], comm_stream_));
  }
  if (f8_) {  // the backward runs on the fp16 rows
    std::vector<P2POp> ops;
    const size_t row = g_.ld_k * cs_;
    for (const SymJob& p : inc_)
      ops.push_back({true, zq_local + (size_t)p.k0 * kTile * row, (size_t)(p.k1 - p.k0) * kTile * row, p.q});
    for (const SymJob& j : jobs_)
      ops.push_back({false, zq_all_ + ((size_t)j.q * Rp + (size_t)j.k0 * kTile) * row, (size_t)(j.k1 - j.k0) * kTile * row,
                     j.q});
    comm_->send_recv(ops, comm_stream_);
    NTXENT_HIP_CHECK(hipEventRecord(ev_f16_, comm_stream_));
  }
  GemmWorkspace ws_ovl = ws_;
  ws_ovl.sched_cus = std::max(1, ws_.num_cus - std::min(cfg_.comm_reserve_cus, ws_.num_cus / 2));
  const size_t sc_tile = (size_t)kTileElems * cs_;
  {
    NTXENT_TRACE("ntxent.fwd_gemm.own");
    fault_point("fwd");
    launch_fwd_stats(cfg_.compute, op_local, op_all, fwd_tiles_, n_own_, part_, sbuf_, ws_ovl, g_, s, BlockView{},
                     part_x_, own_diag_tail(g_));
  }
  for (int c = 0; c < nch_; ++c) {
    NTXENT_TRACE("ntxent.fwd_gemm.cross");
    NTXENT_HIP_CHECK(hipStreamWaitEvent(s, ev_chunk_[c], 0));
    const bool more = c + 1 < nch_ || f8_;
    launch_fwd_stats(cfg_.compute, op_local, op_all, fwd_tiles_ + segs_[c].first, segs_[c].second, part_,
                     sbuf_ + (size_t)segs_[c].first * sc_tile, more ? ws_ovl : ws_, g_, s, BlockView{}, part_x_, 0);
  }
  if (f8_) NTXENT_HIP_CHECK(hipStreamWaitEvent(s, ev_f16_, 0));
  {
    // column partials of the cross tiles -> their rows' owners: rank q's part slots
    // [r * rt + m] for its rows [k0, k1), one run per row tile m, Rpad apart. A whole-block job
    // (k0 = 0, k1 = rt) has its runs back to back: ONE send / recv. The k-split block's runs are
    // packed into xsend_ (one 2-D copy) and unpacked from xrecv_ after the exchange: one op per
    // partner instead of one per row tile (W = 8: 224 -> 8 RCCL ops per step; each op costs the
    // host several microseconds inside the group call).
    NTXENT_TRACE("ntxent.fwd_col_partials");
    std::vector<P2POp> ops;
    const size_t f2 = sizeof(float2);
    struct Unpack { float2* dst; const float2* src; size_t run; int rows; };
    std::vector<Unpack> unpack;
    size_t so = 0, ro = 0;
    for (const SymJob& j : jobs_) {
      const size_t run = (size_t)(j.k1 - j.k0) * kTile;  // float2 per row tile
      float2* first = part_x_ + ((size_t)(j.q * rt + j.m0) * Rp + (size_t)j.k0 * kTile);
      const int nm = j.m1 - j.m0;
      if (run == Rp) {
        ops.push_back({true, first, (size_t)nm * Rp * f2, j.q});
      } else {
        NTXENT_HIP_CHECK(hipMemcpy2DAsync(xsend_ + so, run * f2, first, Rp * f2, run * f2, nm, hipMemcpyDeviceToDevice, s));
        ops.push_back({true, xsend_ + so, (size_t)nm * run * f2, j.q});
        so += (size_t)nm * run;
      }
    }
    for (const SymJob& p : inc_) {
      const size_t run = (size_t)(p.k1 - p.k0) * kTile;
      float2* first = part_ + ((size_t)(p.q * rt + p.m0) * Rp + (size_t)p.k0 * kTile);
      const int nm = p.m1 - p.m0;
      if (run == Rp) {
        ops.push_back({false, first, (size_t)nm * Rp * f2, p.q});
      } else {
        ops.push_back({false, xrecv_ + ro, (size_t)nm * run * f2, p.q});
        unpack.push_back({first, xrecv_ + ro, run, nm});
        ro += (size_t)nm * run;
      }
    }
    NTXENT_HIP_CHECK(hipEventRecord(ev_x_, s));
    NTXENT_HIP_CHECK(hipStreamWaitEvent(comm_stream_, ev_x_, 0));
    comm_->send_recv(ops, comm_stream_);
    NTXENT_HIP_CHECK(hipEventRecord(ev_xdone_, comm_stream_));
    NTXENT_HIP_CHECK(hipStreamWaitEvent(s, ev_xdone_, 0));
    for (const Unpack& u : unpack)
      NTXENT_HIP_CHECK(hipMemcpy2DAsync(u.dst, Rp * f2, u.src, u.run * f2, u.run * f2, u.rows, hipMemcpyDeviceToDevice, s));
  }
  {
    NTXENT_TRACE("ntxent.lse");
    fault_point("lse");
    launch_lse(part_, ypos_, lse2_all_, cpos_, block_loss_, loss_, g_, s);
  }
  {
    NTXENT_TRACE("ntxent.lse_gather");
    comm_->all_gather(lse2_all_ + (size_t)r * Rp, lse2_all_, Rp * 4, s);
    comm_->all_reduce_sum(loss_, 1, s);
  }
  if (fault_armed("nonfinite")) NTXENT_HIP_CHECK(hipMemsetAsync(loss_, 0xFF, 4, s));  // NaN
}

void Engine::backward_sym(const float* grad_out, void* dh, hipStream_t s) {
  const size_t Rp = g_.rows_pad;
  const int rt = g_.row_tiles, r = rank_, W = world_;
  const size_t blk_t = (size_t)g_.dim_n * g_.ld_t * cs_;
  const size_t slab = Rp * g_.dim_n;  // elements of one contribution slab
  {
    NTXENT_TRACE("ntxent.transpose_partners");
    for (const SymJob& j : jobs_)  // partners' B operands of the own dZ GEMMs
      launch_transpose(bwd_, zq_all_ + (size_t)j.q * Rp * g_.ld_k * cs_, zqt_all_ + (size_t)j.q * blk_t, g_, s);
  }
  {
    NTXENT_TRACE("ntxent.coef");
    fault_point("coef");
    launch_coef(bwd_, sbuf_, cbuf_, lse2_all_, cpos_, fwd_tiles_, n_fwd_, g_, s, mbuf_);
  }
  const bool f16c = ccs_ == 2;
  // the partners' contributions: full blocks in ONE stacked GEMM (slots 0 .. nfull-1), the split
  // block's rows after them
  {
    NTXENT_TRACE("ntxent.dz_partners");
    fault_point("dz");
    if (nfull_ > 0) dz_view(mbuf_, 0, rt, zqt_all_, r, 0, rt, 0, nfull_ * rt, contrib_, false, f16c, s, ws_);
    if ((int)jobs_.size() > nfull_) {
      const SymJob& sp = jobs_.back();
      const int slot = ((sp.q - r - 1) % W + W) % W;
      dz_view(mbuf_, (long)slot * rt * rt + sp.m0, rt, zqt_all_, r, (long)sp.m0 * kTile, sp.m1 - sp.m0, sp.k0, sp.k1,
              contrib_ + (size_t)nfull_ * slab * ccs_, false, f16c, s, ws_);
    }
  }
  // point to point: contributions out, the partners' contributions to my rows in (fp32 plans:
  // into the slab stack after the own slab)
  char* recv = f16c ? recv_ : reinterpret_cast<char*>(slabs_) + slab * 4;
  std::vector<P2POp> ops;
  for (size_t i = 0; i < jobs_.size(); ++i) {
    const SymJob& j = jobs_[i];
    const size_t row = (size_t)g_.dim_n * ccs_;
    ops.push_back({true, contrib_ + i * slab * ccs_ + (size_t)j.k0 * kTile * row, (size_t)(j.k1 - j.k0) * kTile * row, j.q});
  }
  for (size_t i = 0; i < inc_.size(); ++i) {
    const SymJob& p = inc_[i];
    const size_t row = (size_t)g_.dim_n * ccs_;
    ops.push_back({false, recv + i * slab * ccs_ + (size_t)p.k0 * kTile * row, (size_t)(p.k1 - p.k0) * kTile * row, p.q});
  }
  NTXENT_HIP_CHECK(hipEventRecord(ev_c_, s));
  NTXENT_HIP_CHECK(hipStreamWaitEvent(comm_stream_, ev_c_, 0));
  comm_->send_recv(ops, comm_stream_);
  NTXENT_HIP_CHECK(hipEventRecord(ev_cdone_, comm_stream_));
  {
    // own contributions while the partners' travel: C_{r,r} Z_r + the full blocks (consecutive
    // rank blocks r .. r+nfull, two GEMMs if they wrap) + the split block's rows. The compact
    // cbuf holds column block r + d at column slots [d * rt, (d + 1) * rt) (sym_c_ld).
    NTXENT_TRACE("ntxent.dz_own");
    // (a local workspace view: the member stays untouched whatever these launches throw)
    GemmWorkspace ws_ovl = ws_;
    ws_ovl.sched_cus = std::max(1, ws_.num_cus - std::min(cfg_.comm_reserve_cus, ws_.num_cus / 2));
    const int nb = 1 + nfull_, first = std::min(nb, W - r), cld = sym_c_ld(g_);
    dz_view(cbuf_, 0, cld, zqt_all_, r, 0, first * rt, 0, rt, slabs_, false, false, s, ws_ovl);
    if (nb > first)
      dz_view(cbuf_, (long)first * rt, cld, zqt_all_, 0, 0, (nb - first) * rt, 0, rt, slabs_, true, false, s, ws_ovl);
    if ((int)jobs_.size() > nfull_) {
      const SymJob& sp = jobs_.back();
      const int d = ((sp.q - r) % W + W) % W;
      dz_view(cbuf_, (long)d * rt + sp.k0, cld, zqt_all_, sp.q, (long)sp.k0 * kTile, sp.k1 - sp.k0, sp.m0, sp.m1, slabs_,
              true, false, s, ws_ovl);
    }
  }
  NTXENT_HIP_CHECK(hipStreamWaitEvent(s, ev_cdone_, 0));
  {
    NTXENT_TRACE("ntxent.norm_bwd");
    fault_point("norm_bwd");
    const float* go = grad_out ? grad_out : one_;
    if (f16c)
      launch_norm_bwd(cfg_.input, slabs_, 1, h_, inv_, go, dh, g_, s, recv_, (int)inc_.size());
    else
      launch_norm_bwd(cfg_.input, slabs_, 1 + (int)inc_.size(), h_, inv_, go, dh, g_, s);
  }
}

}  // namespace ntxent

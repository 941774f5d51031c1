// PyTorch (ROCm) op layer + Python binding of the MI355X NT-Xent kernels.
//
// Replaces the reference's host launchers (src/ntxent_kernel.cu:138-239) and its pybind11
// bindings (src/binding_new.cpp:4-21): same Python names and kwargs (`forward`, `backward`,
// `check_tensor_core_support`), plus
//   * TORCH_LIBRARY registration under `ntxent_cuda` (what python/test.py:137 expects) and
//     under `ntxent`;
//   * stage-level ops (prep / fwd_stats / lse / coef / dz / norm_bwd) over a cached `Plan`
//     (geometry + XCD-ordered tile lists resident on the device), which the Python autograd
//     Function and the RCCL data-parallel path compose.
//
// No host synchronisation anywhere in these ops: they only enqueue on the current HIP stream.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPCachingAllocatorMasqueradingAsCUDA.h>

#include <algorithm>
#include <map>
#include <memory>
#include <atomic>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "ntxent/engine.h"
#include "ntxent/ntxent.h"

namespace ntxent {
namespace th {

DType to_dtype(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return DType::F32;
    case at::kHalf: return DType::F16;
    case at::kBFloat16: return DType::BF16;
    default: NTXENT_CHECK(false, std::string("unsupported dtype ") + c10::toString(t));
  }
  return DType::F32;
}

at::ScalarType to_scalar(DType t) {
  return t == DType::F32 ? at::kFloat : (t == DType::F16 ? at::kHalf : (t == DType::BF16 ? at::kBFloat16 : at::kByte));
}

// Compute-dtype policy. Normalised rows live in [-1, 1], where fp16's 10-bit mantissa beats
// bf16's 7 bits at equal MFMA rate, so reduced precision means fp16 unless asked otherwise.
DType choose_compute(at::ScalarType in, bool use_mixed_precision, const std::string& override_) {
  if (override_ == "fp32" || override_ == "float32") return DType::F32;
  if (override_ == "fp16" || override_ == "float16") return DType::F16;
  if (override_ == "bf16" || override_ == "bfloat16") return DType::BF16;
  if (override_ == "fp8" || override_ == "float8") return DType::FP8;
  NTXENT_CHECK(override_.empty() || override_ == "auto", "compute_dtype must be auto|fp32|fp16|bf16|fp8");
  if (in == at::kFloat && !use_mixed_precision) return DType::F32;
  return DType::F16;
}

struct Plan {
  Geometry g;
  DType comp = DType::F16;
  int device = 0;
  at::Tensor fwd_tiles;  // int32 [n, 4] on device
  int n_fwd = 0;
  int n_own = 0;  // own-rank tiles at the head of fwd_tiles
  at::Tensor dz_tiles;
  int n_dz = 0;
  int num_cus = 256;
  bool small = false;  // single-rank small-problem path (kernels/small_kernels.hip)

  int rows() const { return g.rows; }
  int rows_pad() const { return g.rows_pad; }
  int dim() const { return g.dim; }
  int dim_k() const { return g.dim_k; }
  int ld_k() const { return g.ld_k; }
  int ld_t() const { return g.ld_t; }
  int dim_n() const { return g.dim_n; }
  int world() const { return g.world; }
  int rank() const { return g.rank; }
  int row_tiles() const { return g.row_tiles; }
  int col_tiles() const { return g.col_tiles; }
  double temperature() const { return g.temperature; }
  std::string compute_dtype() const { return dtype_name(comp); }
  DType bwd() const { return backward_dtype(comp); }                  // zq / sc / C / ZqT dtype
  long op_ld() const { return comp == DType::FP8 ? g.ld_k8 : g.ld_k; }  // forward operand row stride
  std::string backward_dtype_name() const { return dtype_name(bwd()); }
};

static at::Tensor upload_tiles(const std::vector<int4>& v, int device) {
  auto cpu = torch::empty({(long)v.size(), 4}, torch::dtype(torch::kInt32));
  std::memcpy(cpu.data_ptr<int>(), v.data(), v.size() * sizeof(int4));
  return cpu.to(torch::Device(torch::kCUDA, device), /*non_blocking=*/false);
}

std::shared_ptr<Plan> get_plan(int rows, int dim, int world, int rank, double temperature,
                               const std::string& compute, int device) {
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, int, float, int, int>, std::shared_ptr<Plan>> cache;
  const DType comp = choose_compute(at::kFloat, compute != "fp32" && compute != "float32", compute);
  auto key = std::make_tuple(rows, dim, world, rank, (float)temperature, (int)comp, device);
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  auto p = std::make_shared<Plan>();
  p->g = make_geometry(rows, dim, world, rank, (float)temperature);
  p->comp = comp;
  p->device = device;
  const DeviceInfo& di = device_info(device);
  p->num_cus = di.num_cus;
  auto ft = build_fwd_tiles(p->g);
  p->n_fwd = (int)ft.size();
  p->n_own = count_own_fwd_tiles(p->g);
  p->fwd_tiles = upload_tiles(ft, device);
  auto dt = build_dz_tiles(p->g);
  p->n_dz = (int)dt.size();
  p->dz_tiles = upload_tiles(dt, device);
  p->small = small_path_eligible(p->g, comp);
  cache.emplace(key, p);
  return p;
}

static hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

static void check_input(const at::Tensor& h, const char* name) {
  NTXENT_CHECK(h.is_cuda(), std::string(name) + " must be a GPU (HIP) tensor");
  NTXENT_CHECK(h.is_contiguous(), std::string(name) + " must be contiguous");
}

static at::TensorOptions opts(const at::Tensor& like, at::ScalarType t) {
  return at::TensorOptions().dtype(t).device(like.device());
}

// Zero-initialised scratch for the kernels' self-cleaning arrival counters (stream-K tile
// arrivals, LSE and small-path last-block-done tickets) and their partials. Every launch returns
// its counters to zero, so a buffer is zeroed only when it is (re)allocated and no memset runs
// per launch. The cache is keyed by (device, slot, STREAM): launches sharing one buffer are then
// always stream-ordered, and losses evaluated concurrently on different streams never race on
// one ticket (a counter reset in the middle of another stream's launch would leave it non-zero
// and starve every later last-arriver). A grown buffer replaces the old one; the caching
// allocator keeps the old block alive until its stream is done.
static at::Tensor device_scratch(const at::Tensor& like, size_t bytes, int slot) {
  static std::mutex mu;
  static std::map<std::tuple<int, int, hipStream_t>, at::Tensor> cache;
  std::lock_guard<std::mutex> lock(mu);
  auto& t = cache[{(int)like.device().index(), slot, cur_stream(like)}];
  if (!t.defined() || (size_t)t.numel() < bytes) t = at::zeros({(long)bytes}, opts(like, at::kByte));
  return t;
}


// reserve_cus: CUs this launch leaves free for communication kernels that overlap it (a
// per-launch argument: parallel/commstats.py:comm_reserve_cus), at most half the chip.
static GemmWorkspace gemm_ws(const at::Tensor& like, int ntiles, const Plan& P, int reserve_cus = 0) {
  NTXENT_CHECK(reserve_cus >= 0, "reserve_cus must be >= 0");
  GemmWorkspace ws;
  ws.num_cus = P.num_cus;
  ws.sched_cus = std::max(1, P.num_cus - std::min(reserve_cus, P.num_cus / 2));
  ws.bytes = gemm_workspace_bytes(ntiles, P.num_cus);
  ws.ptr = device_scratch(like, ws.bytes, 0).data_ptr();
  return ws;
}

// ---- stage ops ----------------------------------------------------------------------
// `zq_out` (optional): write the normalised rows into this [rows_pad, ld_k] buffer — e.g. this
// rank's slot of the all-gather destination, so the gather runs in place.
// Returns {zq, inv, ypos, zq8}: zq in the backward dtype; zq8 (uint8 e4m3 rows [rows_pad, ld_k8])
// only for fp8 plans (undefined otherwise), written into `zq8_out` when given.
std::vector<at::Tensor> prep(const at::Tensor& h, const Plan& P, const c10::optional<at::Tensor>& zq_out,
                             const c10::optional<at::Tensor>& zq8_out) {
  check_input(h, "h");
  NTXENT_CHECK(h.dim() == 2 && h.size(0) == P.g.rows && h.size(1) == P.g.dim, "h shape does not match plan");
  const at::DeviceGuard guard(h.device());
  at::Tensor zq;
  if (zq_out.has_value() && zq_out->defined()) {
    zq = *zq_out;
    check_input(zq, "zq_out");
    NTXENT_CHECK(zq.numel() == (long)P.g.rows_pad * P.g.ld_k && zq.scalar_type() == to_scalar(P.bwd()),
                 "zq_out must be [rows_pad, ld_k] in the backward dtype");
  } else {
    zq = at::empty({P.g.rows_pad, P.g.ld_k}, opts(h, to_scalar(P.bwd())));
  }
  at::Tensor zq8;
  if (P.comp == DType::FP8) {
    if (zq8_out.has_value() && zq8_out->defined()) {
      zq8 = *zq8_out;
      check_input(zq8, "zq8_out");
      NTXENT_CHECK(zq8.numel() == (long)P.g.rows_pad * P.g.ld_k8 && zq8.scalar_type() == at::kByte,
                   "zq8_out must be uint8 [rows_pad, ld_k8]");
    } else {
      zq8 = at::empty({P.g.rows_pad, P.g.ld_k8}, opts(h, at::kByte));
    }
  }
  auto inv = at::empty({P.g.rows}, opts(h, at::kFloat));
  auto ypos = at::empty({P.g.rows}, opts(h, at::kFloat));
  launch_prep(to_dtype(h.scalar_type()), P.bwd(), h.data_ptr(), zq.data_ptr(), inv.data_ptr<float>(),
              ypos.data_ptr<float>(), P.g, cur_stream(h), zq8.defined() ? zq8.data_ptr() : nullptr);
  return {zq, inv, ypos, zq8};
}

at::Tensor transpose(const at::Tensor& zq, const Plan& P, const c10::optional<at::Tensor>& zqt_out) {
  check_input(zq, "zq");
  const at::DeviceGuard guard(zq.device());
  at::Tensor zqt;
  if (zqt_out.has_value() && zqt_out->defined()) {
    zqt = *zqt_out;
    check_input(zqt, "zqt_out");
    NTXENT_CHECK(zqt.numel() == (long)P.g.dim_n * P.g.ld_t && zqt.scalar_type() == zq.scalar_type(),
                 "zqt_out must be [dim_n, ld_t]");
  } else {
    zqt = at::empty({P.g.dim_n, P.g.ld_t}, zq.options());
  }
  launch_transpose(P.bwd(), zq.data_ptr(), zqt.data_ptr(), P.g, cur_stream(zq));
  return zqt;
}

// zero_cos: the raw op (Python fwd_stats) returns zeros in the lower 64x64 regions of diagonal
// tiles, which the forward may leave unwritten (the coefficient pass mirrors them from the upper
// ones, diag_up_kernel); the training path keeps the buffer uninitialised (a 66 MiB memset per
// step at the headline otherwise)
std::vector<at::Tensor> fwd_stats(const at::Tensor& zq_local, const at::Tensor& zq_all, const Plan& P,
                                  bool keep_cos, bool zero_cos = false) {
  check_input(zq_local, "zq_local");
  check_input(zq_all, "zq_all");
  NTXENT_CHECK(zq_all.size(0) == (long)P.g.world * P.g.rows_pad && zq_all.size(1) == P.op_ld(),
               "zq_all must be [world*rows_pad, ld] in the forward operand dtype (ld_k, or ld_k8 for fp8)");
  const at::DeviceGuard guard(zq_local.device());
  auto part = at::empty({P.g.col_tiles, P.g.rows_pad, 2}, opts(zq_local, at::kFloat));
  at::Tensor sc;
  if (keep_cos)
    sc = zero_cos ? at::zeros({(long)P.n_fwd * kTileElems}, opts(zq_local, to_scalar(P.bwd())))
                  : at::empty({(long)P.n_fwd * kTileElems}, opts(zq_local, to_scalar(P.bwd())));
  auto ws = gemm_ws(zq_local, P.n_fwd, P);
  launch_fwd_stats(P.comp, zq_local.data_ptr(), zq_all.data_ptr(),
                   reinterpret_cast<const int4*>(P.fwd_tiles.data_ptr<int>()), P.n_fwd,
                   reinterpret_cast<float2*>(part.data_ptr<float>()), sc.defined() ? sc.data_ptr() : nullptr,
                   ws, P.g, cur_stream(zq_local), BlockView{}, nullptr,
                   P.n_fwd == P.n_own ? own_diag_tail(P.g) : 0);
  return {part, sc};
}

// Forward tiles [first, first + count) of the plan's list into caller-owned `part` / `sc`
// (sc may be undefined). The own-rank tiles come first (P.n_own of them) and read only this
// rank's slot of zq_all, so they can run while the rest of zq_all is being gathered.
void fwd_stats_range(const at::Tensor& zq_local, const at::Tensor& zq_all, const Plan& P, at::Tensor& part,
                     const c10::optional<at::Tensor>& sc, int first, int count, int reserve_cus) {
  check_input(zq_local, "zq_local");
  check_input(zq_all, "zq_all");
  check_input(part, "part");
  NTXENT_CHECK(first >= 0 && count >= 0 && first + count <= P.n_fwd, "tile range out of bounds");
  NTXENT_CHECK(part.numel() == (long)P.g.col_tiles * P.g.rows_pad * 2 && part.scalar_type() == at::kFloat,
               "part must be float32 [col_tiles, rows_pad, 2]");
  NTXENT_CHECK(zq_all.numel() == (long)P.g.world * P.g.rows_pad * P.op_ld(),
               "zq_all must be [world*rows_pad, ld] in the forward operand dtype");
  const bool keep = sc.has_value() && sc->defined();
  if (keep) NTXENT_CHECK(sc->numel() == (long)P.n_fwd * kTileElems, "sc must hold n_fwd tiles");
  if (count == 0) return;
  const at::DeviceGuard guard(zq_local.device());
  auto ws = gemm_ws(zq_local, count, P, reserve_cus);
  char* scp = keep ? static_cast<char*>(sc->data_ptr()) + (size_t)first * kTileElems * dtype_size(P.bwd()) : nullptr;
  launch_fwd_stats(P.comp, zq_local.data_ptr(), zq_all.data_ptr(),
                   reinterpret_cast<const int4*>(P.fwd_tiles.data_ptr<int>()) + first, count,
                   reinterpret_cast<float2*>(part.data_ptr<float>()), scp, ws, P.g, cur_stream(zq_local), BlockView{},
                   nullptr, first + count == P.n_own ? std::min(count, own_diag_tail(P.g)) : 0);
}

// Writes this rank's slice of lse2_all (log2 units) and cpos (the positive coefficient
// -(a_i + a_p) of the local rows); returns the local loss contribution.
at::Tensor lse(const at::Tensor& part, const at::Tensor& ypos, at::Tensor& lse2_all, at::Tensor& cpos,
               const Plan& P, const c10::optional<at::Tensor>& zq = c10::nullopt,
               const c10::optional<at::Tensor>& zqt = c10::nullopt) {
  check_input(part, "part");
  NTXENT_CHECK(lse2_all.numel() == (long)P.g.world * P.g.rows_pad && lse2_all.scalar_type() == at::kFloat,
               "lse2_all must be float32 [world*rows_pad]");
  NTXENT_CHECK(cpos.numel() >= P.g.rows_pad && cpos.scalar_type() == at::kFloat, "cpos must be float32 [>= rows_pad]");
  const at::DeviceGuard guard(part.device());
  auto block_loss = device_scratch(part, (size_t)lse_scratch_floats(P.g) * 4, 1);
  auto loss = at::empty({}, opts(part, at::kFloat));
  const bool tr = zq.has_value() && zq->defined();
  if (tr) {  // also write zqt = zq^T (the rank-local rows) from the same launch
    NTXENT_CHECK(zqt.has_value() && zqt->defined(), "lse: zqt missing");
    check_input(*zq, "zq");
    check_input(*zqt, "zqt");
    NTXENT_CHECK(zq->numel() == (long)P.g.rows_pad * P.g.ld_k && zq->scalar_type() == to_scalar(P.bwd()),
                 "lse: zq must be [rows_pad, ld_k] in the backward dtype");
    NTXENT_CHECK(zqt->numel() == (long)P.g.dim_n * P.g.ld_t && zqt->scalar_type() == zq->scalar_type(),
                 "lse: zqt must be [dim_n, ld_t]");
  }
  launch_lse(reinterpret_cast<const float2*>(part.data_ptr<float>()), ypos.data_ptr<float>(),
             lse2_all.data_ptr<float>(), cpos.data_ptr<float>(), static_cast<float*>(block_loss.data_ptr()),
             loss.data_ptr<float>(), P.g, cur_stream(part), P.bwd(), tr ? zq->data_ptr() : nullptr,
             tr ? zqt->data_ptr() : nullptr);
  return loss;
}

// Kept cosines (compact, one slot per forward tile) -> coefficient buffer (all tiles).
at::Tensor coef(const at::Tensor& sbuf, const at::Tensor& lse2_all, const at::Tensor& cpos, const Plan& P,
                float* dotp = nullptr, bool half_c = false) {
  check_input(sbuf, "sbuf");
  NTXENT_CHECK(sbuf.numel() == (long)P.n_fwd * kTileElems, "sbuf does not match the plan's forward tiles");
  const at::DeviceGuard guard(sbuf.device());
  auto cbuf = at::empty({(long)P.g.row_tiles * P.g.col_tiles * kTileElems}, sbuf.options());
  launch_coef(P.bwd(), sbuf.data_ptr(), cbuf.data_ptr(), lse2_all.data_ptr<float>(), cpos.data_ptr<float>(),
              reinterpret_cast<const int4*>(P.fwd_tiles.data_ptr<int>()), P.n_fwd, P.g, cur_stream(sbuf), nullptr,
              dotp, nullptr, half_c);
  return cbuf;
}

at::Tensor coef_gemm(const at::Tensor& zq_local, const at::Tensor& zq_all, const at::Tensor& lse2_all,
                     const at::Tensor& cpos, const Plan& P, float* dotp = nullptr) {
  check_input(zq_local, "zq_local");
  const at::DeviceGuard guard(zq_local.device());
  auto cbuf = at::empty({(long)P.g.row_tiles * P.g.col_tiles * kTileElems}, opts(zq_local, to_scalar(P.bwd())));
  auto ws = gemm_ws(zq_local, P.n_fwd, P);
  launch_coef_gemm(P.comp, zq_local.data_ptr(), zq_all.data_ptr(), cbuf.data_ptr(), lse2_all.data_ptr<float>(),
                   cpos.data_ptr<float>(), reinterpret_cast<const int4*>(P.fwd_tiles.data_ptr<int>()), P.n_fwd,
                   ws, P.g, cur_stream(zq_local), BlockView{}, dotp);
  return cbuf;
}

at::Tensor dz(const at::Tensor& sc, const at::Tensor& zqt_all, const Plan& P, const NormFuse* nf = nullptr,
              bool* fused = nullptr, bool half_c = false) {
  check_input(sc, "sc");
  check_input(zqt_all, "zqt_all");
  NTXENT_CHECK(zqt_all.numel() == (long)P.g.world * P.g.dim_n * P.g.ld_t, "zqt_all must be [world, dim_n, ld_t]");
  const at::DeviceGuard guard(sc.device());
  // reduced-precision plans keep dZ in fp16 (half the store and the normalisation backward's read)
  const bool f16 = P.bwd() != DType::F32;
  auto slabs = at::empty({1, P.g.rows_pad, P.g.dim_n}, opts(sc, f16 ? at::kHalf : at::kFloat));
  auto ws = gemm_ws(sc, P.n_dz, P);
  const bool f = launch_dz(P.bwd(), sc.data_ptr(), zqt_all.data_ptr(),
                           reinterpret_cast<const int4*>(P.dz_tiles.data_ptr<int>()), P.n_dz, slabs.data_ptr(), ws, P.g,
                           cur_stream(sc), f16, nf, nullptr, nullptr, half_c);
  if (fused) *fused = f;
  return slabs;
}

at::Tensor norm_bwd(const at::Tensor& slabs, const at::Tensor& h, const at::Tensor& inv, const at::Tensor& grad_out,
                    const Plan& P) {
  check_input(h, "h");
  const at::DeviceGuard guard(h.device());
  auto go = grad_out.to(at::kFloat).contiguous();
  auto dh = at::empty_like(h);
  if (slabs.scalar_type() == at::kHalf)  // one fp16 dZ slab (dz() of a reduced-precision plan)
    launch_norm_bwd(to_dtype(h.scalar_type()), nullptr, 0, h.data_ptr(), inv.data_ptr<float>(), go.data_ptr<float>(),
                    dh.data_ptr(), P.g, cur_stream(h), slabs.data_ptr(), 1);
  else
    launch_norm_bwd(to_dtype(h.scalar_type()), slabs.data_ptr<float>(), 1, h.data_ptr(), inv.data_ptr<float>(),
                    go.data_ptr<float>(), dh.data_ptr(), P.g, cur_stream(h));
  return dh;
}

// ---- ring-negatives stage ops (O(local) memory; parallel/ring.py) --------------------------
// `zq_chunk` holds the normalised rows of ONE rank (rows_pad x op_ld): the rank whose global
// column tiles start at `b_tile0`. `tiles` is an explicit int32 [n, 4] tile list (a subset of
// the plan's forward tiles).
static const int4* tile_ptr(const at::Tensor& tiles, int& n) {
  check_input(tiles, "tiles");
  NTXENT_CHECK(tiles.dim() == 2 && tiles.size(1) == 4 && tiles.scalar_type() == at::kInt, "tiles must be int32 [n, 4]");
  n = (int)tiles.size(0);
  return reinterpret_cast<const int4*>(tiles.data_ptr<int>());
}

void fwd_stats_tiles(const at::Tensor& zq_local, const at::Tensor& zq_chunk, int b_tile0, const at::Tensor& tiles,
                     const Plan& P, at::Tensor& part, int reserve_cus) {
  check_input(zq_local, "zq_local");
  check_input(zq_chunk, "zq_chunk");
  check_input(part, "part");
  NTXENT_CHECK(zq_chunk.numel() == (long)P.g.rows_pad * P.op_ld(), "zq_chunk must be one rank's [rows_pad, ld] rows");
  NTXENT_CHECK(part.numel() == (long)P.g.col_tiles * P.g.rows_pad * 2 && part.scalar_type() == at::kFloat,
               "part must be float32 [col_tiles, rows_pad, 2]");
  int n = 0;
  const int4* tp = tile_ptr(tiles, n);
  if (n == 0) return;
  const at::DeviceGuard guard(zq_local.device());
  auto ws = gemm_ws(zq_local, n, P, reserve_cus);
  BlockView bv;
  bv.b_tile0 = b_tile0;
  launch_fwd_stats(P.comp, zq_local.data_ptr(), zq_chunk.data_ptr(), tp, n,
                   reinterpret_cast<float2*>(part.data_ptr<float>()), nullptr, ws, P.g, cur_stream(zq_local), bv);
}

// Coefficient tiles of one column block (recomputed S) into a compact [row_tiles][c_ld] tile
// buffer whose first column tile is global tile c_tile0.
at::Tensor coef_gemm_tiles(const at::Tensor& zq_local, const at::Tensor& zq_chunk, int b_tile0, const at::Tensor& tiles,
                           const at::Tensor& lse2_all, const at::Tensor& cpos, const Plan& P, int c_ld, int c_tile0,
                           int reserve_cus) {
  check_input(zq_local, "zq_local");
  check_input(zq_chunk, "zq_chunk");
  NTXENT_CHECK(c_ld > 0, "c_ld must be positive");
  int n = 0;
  const int4* tp = tile_ptr(tiles, n);
  const at::DeviceGuard guard(zq_local.device());
  auto cbuf = at::empty({(long)P.g.row_tiles * c_ld * kTileElems}, opts(zq_local, to_scalar(P.bwd())));
  if (n == 0) return cbuf;
  auto ws = gemm_ws(zq_local, n, P, reserve_cus);
  BlockView bv;
  bv.b_tile0 = b_tile0;
  bv.c_ld = c_ld;
  bv.c_tile0 = c_tile0;
  launch_coef_gemm(P.comp, zq_local.data_ptr(), zq_chunk.data_ptr(), cbuf.data_ptr(), lse2_all.data_ptr<float>(),
                   cpos.data_ptr<float>(), tp, n, ws, P.g, cur_stream(zq_local), bv);
  return cbuf;
}

// dZ contribution of one column block: slabs = C_block [rows_pad x rows_pad] * Z_chunk, with
// zqt_chunk = that rank's [dim_n, ld_t] transposed rows (a one-block, world-1 geometry).
at::Tensor dz_block(const at::Tensor& cbuf_block, const at::Tensor& zqt_chunk, const Plan& P, int reserve_cus) {
  check_input(cbuf_block, "cbuf_block");
  check_input(zqt_chunk, "zqt_chunk");
  NTXENT_CHECK(zqt_chunk.numel() == (long)P.g.dim_n * P.g.ld_t, "zqt_chunk must be [dim_n, ld_t]");
  NTXENT_CHECK(cbuf_block.numel() == (long)P.g.row_tiles * P.g.row_tiles * kTileElems, "cbuf_block must be row_tiles^2 tiles");
  const at::DeviceGuard guard(cbuf_block.device());
  Geometry g1 = P.g;
  g1.world = 1;
  g1.rank = 0;
  g1.col_tiles = g1.row_tiles;
  auto slabs = at::empty({1, P.g.rows_pad, P.g.dim_n}, opts(cbuf_block, at::kFloat));
  auto ws = gemm_ws(cbuf_block, P.n_dz, P, reserve_cus);
  launch_dz(P.bwd(), cbuf_block.data_ptr(), zqt_chunk.data_ptr(), reinterpret_cast<const int4*>(P.dz_tiles.data_ptr<int>()),
            P.n_dz, slabs.data_ptr<float>(), ws, g1, cur_stream(cbuf_block));
  return slabs;
}

// ---- symmetric data-parallel stage ops (parallel/symmetric.py) -----------------------------
// Every unordered rank pair's similarity block is computed once across the group: the
// computing rank keeps row AND column partials (kTileCross tiles), forms both coefficient
// blocks C_{r,q} and C_{q,r} = C_{r,q}^T from its kept cosines, and produces the partner's
// gradient contribution C_{q,r} Z_r, which the caller sends to q.
static std::vector<SymJob> to_jobs(const std::vector<std::tuple<int, int, int, int, int>>& jobs) {
  std::vector<SymJob> v;
  for (const auto& j : jobs) v.push_back(SymJob{std::get<0>(j), std::get<1>(j), std::get<2>(j), std::get<3>(j), std::get<4>(j)});
  return v;
}

at::Tensor sym_fwd_tiles(const Plan& P, const std::vector<std::tuple<int, int, int, int, int>>& jobs, int nchunks) {
  return upload_tiles(build_sym_fwd_tiles(P.g, to_jobs(jobs), nchunks), P.device);
}

// Forward tiles `tiles` (own block + kTileCross) over the gathered rows: row partials -> part,
// column partials of cross tiles -> part_x ([col_tiles, rows_pad, 2], see launch_fwd_stats).
void fwd_stats_sym(const at::Tensor& zq_local, const at::Tensor& zq_all, const at::Tensor& tiles, const Plan& P,
                   at::Tensor& part, at::Tensor& part_x, const c10::optional<at::Tensor>& sc, int first, int count,
                   int reserve_cus) {
  check_input(zq_local, "zq_local");
  check_input(zq_all, "zq_all");
  check_input(part, "part");
  check_input(part_x, "part_x");
  int n = 0;
  const int4* tp = tile_ptr(tiles, n);
  NTXENT_CHECK(first >= 0 && count >= 0 && first + count <= n, "tile range out of bounds");
  const long pn = (long)P.g.col_tiles * P.g.rows_pad * 2;
  NTXENT_CHECK(part.numel() == pn && part.scalar_type() == at::kFloat, "part must be float32 [col_tiles, rows_pad, 2]");
  NTXENT_CHECK(part_x.numel() == pn && part_x.scalar_type() == at::kFloat, "part_x must be float32 [col_tiles, rows_pad, 2]");
  NTXENT_CHECK(zq_all.numel() == (long)P.g.world * P.g.rows_pad * P.op_ld(),
               "zq_all must be [world*rows_pad, ld] in the forward operand dtype");
  const bool keep = sc.has_value() && sc->defined();
  if (keep) NTXENT_CHECK(sc->numel() == (long)n * kTileElems && sc->scalar_type() == to_scalar(P.bwd()),
                         "sc must hold one tile per entry of `tiles` in the backward dtype");
  if (count == 0) return;
  const at::DeviceGuard guard(zq_local.device());
  auto ws = gemm_ws(zq_local, count, P, reserve_cus);
  char* scp = keep ? static_cast<char*>(sc->data_ptr()) + (size_t)first * kTileElems * dtype_size(P.bwd()) : nullptr;
  launch_fwd_stats(P.comp, zq_local.data_ptr(), zq_all.data_ptr(), tp + first, count,
                   reinterpret_cast<float2*>(part.data_ptr<float>()), scp, ws, P.g, cur_stream(zq_local), BlockView{},
                   reinterpret_cast<float2*>(part_x.data_ptr<float>()),
                   first + count == P.n_own ? std::min(count, own_diag_tail(P.g)) : 0);
}

// Kept cosines of `tiles` -> own coefficient tiles in cbuf ([row_tiles][col_tiles] tiles) and the
// partners' mirrored blocks in mbuf ([max(1, world/2)][row_tiles][row_tiles] tiles, one slot per partner).
void coef_sym(const at::Tensor& sbuf, const at::Tensor& tiles, const at::Tensor& lse2_all, const at::Tensor& cpos,
              const Plan& P, at::Tensor& cbuf, at::Tensor& mbuf) {
  check_input(sbuf, "sbuf");
  check_input(cbuf, "cbuf");
  check_input(mbuf, "mbuf");
  int n = 0;
  const int4* tp = tile_ptr(tiles, n);
  const auto st = to_scalar(P.bwd());
  NTXENT_CHECK(sbuf.numel() == (long)n * kTileElems && sbuf.scalar_type() == st, "sbuf must hold one tile per entry");
  NTXENT_CHECK(cbuf.numel() == (long)P.g.row_tiles * sym_c_ld(P.g) * kTileElems && cbuf.scalar_type() == st,
               "cbuf must be [row_tiles * sym_c_ld] tiles (compact symmetric layout)");
  // partner slots (q - rank - 1) mod W of the cross tiles run 0 .. W/2 - 1 (parallel/symmetric.py)
  NTXENT_CHECK(mbuf.numel() == (long)std::max(1, P.g.world / 2) * P.g.row_tiles * P.g.row_tiles * kTileElems &&
                   mbuf.scalar_type() == st, "mbuf must be [max(1, world/2) * row_tiles * row_tiles] tiles");
  NTXENT_CHECK(lse2_all.numel() == (long)P.g.world * P.g.rows_pad, "lse2_all must be [world*rows_pad]");
  if (n == 0) return;
  const at::DeviceGuard guard(sbuf.device());
  launch_coef(P.bwd(), sbuf.data_ptr(), cbuf.data_ptr(), lse2_all.data_ptr<float>(), cpos.data_ptr<float>(), tp, n, P.g,
              cur_stream(sbuf), mbuf.data_ptr());
}

// out[row tiles m0..m1) (+)= A * B with A = tiles of `abuf` starting at tile index a_tile0 (row
// panels a_panel_tiles tiles apart; row tile mt at a_tile0 + mt * a_panel_tiles), K = k_tiles * 256
// columns of B = `bbuf` (ZqT blocks [nblk, dim_n, ld_t], or one [dim_n, ld_t]) starting at block
// b_block0, column b_col0; a K range longer than one block runs over consecutive whole blocks.
// `out` is float32 [>= m1 * 256, dim_n] (row tiles may exceed row_tiles: stacked outputs).
void dz_view(const at::Tensor& abuf, long a_tile0, long a_panel_tiles, const at::Tensor& bbuf, int b_block0, long b_col0,
             int k_tiles, int m0, int m1, at::Tensor& out, bool accum, const Plan& P, int reserve_cus) {
  check_input(abuf, "abuf");
  check_input(bbuf, "bbuf");
  check_input(out, "out");
  const auto st = to_scalar(P.bwd());
  NTXENT_CHECK(abuf.scalar_type() == st && bbuf.scalar_type() == st, "operands must be in the backward dtype");
  NTXENT_CHECK(0 <= m0 && m0 <= m1, "bad row tile range");
  NTXENT_CHECK(k_tiles >= 0 && a_panel_tiles >= k_tiles && a_tile0 >= 0, "bad A view");
  if (m1 > m0)
    NTXENT_CHECK(a_tile0 + (long)(m1 - 1) * a_panel_tiles + k_tiles <= abuf.numel() / kTileElems, "A view out of bounds");
  const long blk = (long)P.g.dim_n * P.g.ld_t;
  NTXENT_CHECK(bbuf.numel() % blk == 0, "bbuf must be [nblk, dim_n, ld_t]");
  const long nblk = bbuf.numel() / blk;
  const long kcols = (long)k_tiles * kTile;
  long kblk_cols = kcols;
  if (b_col0 + kcols > P.g.rows_pad) {  // spans whole rank blocks
    NTXENT_CHECK(b_col0 == 0 && kcols % P.g.rows_pad == 0, "multi-block K ranges must cover whole blocks");
    kblk_cols = P.g.rows_pad;
  }
  const long nspan = (kcols + kblk_cols - 1) / kblk_cols;
  NTXENT_CHECK(b_block0 >= 0 && b_block0 + nspan <= nblk && b_col0 >= 0, "B view out of bounds");
  const bool out_f16 = out.scalar_type() == at::kHalf;
  NTXENT_CHECK((out.scalar_type() == at::kFloat || out_f16) && out.dim() == 2 && out.size(1) == P.g.dim_n &&
                   out.size(0) >= (long)m1 * kTile, "out must be float32 or float16 [>= m1*256, dim_n]");
  NTXENT_CHECK(!(out_f16 && accum), "fp16 output cannot accumulate");
  if (m1 == m0 || k_tiles == 0) return;
  const at::DeviceGuard guard(abuf.device());
  at::Tensor sub;
  {
    static std::mutex mu;
    static std::map<std::tuple<int, int, int, int>, at::Tensor> cache;
    std::lock_guard<std::mutex> lock(mu);
    auto& c = cache[{P.device, P.g.dim_n, m0, m1}];
    if (!c.defined()) {
      std::vector<int4> v;
      for (int ti = m0; ti < m1; ++ti)
        for (int tn = 0; tn < P.g.dim_n / kTile; ++tn) v.push_back(make_int4(ti, tn, 0, 0));
      c = upload_tiles(v, P.device);
    }
    sub = c;
  }
  const long cs = (long)dtype_size(P.bwd());
  const char* a = static_cast<const char*>(abuf.data_ptr()) + a_tile0 * kTileElems * cs;
  const char* b = static_cast<const char*>(bbuf.data_ptr()) + ((long)b_block0 * blk + b_col0) * cs;
  auto ws = gemm_ws(abuf, (int)sub.size(0), P, reserve_cus);
  launch_dz_view(P.bwd(), a, a_panel_tiles, b, kblk_cols, blk, k_tiles, reinterpret_cast<const int4*>(sub.data_ptr<int>()),
                 (int)sub.size(0), out.data_ptr(), accum, ws, P.g, cur_stream(abuf), out_f16);
}

// norm_bwd over a stack of partial dZ slabs [nslabs, rows_pad, dim_n] fp32, plus optional
// fp16 slabs `xslabs` [nx, rows_pad, dim_n] (received partner contributions), summed in order.
at::Tensor norm_bwd_slabs(const at::Tensor& slabs, const at::Tensor& h, const at::Tensor& inv, const at::Tensor& grad_out,
                          const Plan& P, const c10::optional<at::Tensor>& xslabs) {
  check_input(h, "h");
  check_input(slabs, "slabs");
  NTXENT_CHECK(slabs.dim() == 3 && slabs.size(1) == P.g.rows_pad && slabs.size(2) == P.g.dim_n &&
                   slabs.scalar_type() == at::kFloat, "slabs must be float32 [n, rows_pad, dim_n]");
  const void* xp = nullptr;
  int nx = 0;
  if (xslabs.has_value() && xslabs->defined() && xslabs->numel() > 0) {
    check_input(*xslabs, "xslabs");
    NTXENT_CHECK(xslabs->dim() == 3 && xslabs->size(1) == P.g.rows_pad && xslabs->size(2) == P.g.dim_n &&
                     xslabs->scalar_type() == at::kHalf, "xslabs must be float16 [n, rows_pad, dim_n]");
    xp = xslabs->data_ptr();
    nx = (int)xslabs->size(0);
  }
  const at::DeviceGuard guard(h.device());
  auto go = grad_out.to(at::kFloat).contiguous();
  auto dh = at::empty_like(h);
  launch_norm_bwd(to_dtype(h.scalar_type()), slabs.data_ptr<float>(), (int)slabs.size(0), h.data_ptr(),
                  inv.data_ptr<float>(), go.data_ptr<float>(), dh.data_ptr(), P.g, cur_stream(h), xp, nx);
  return dh;
}

// ---- single-process fused flows ------------------------------------------------------
// Small-problem path (set_small_path, default on): the one-launch forward / backward of
// small_kernels.hip for plans with Plan::small.

static int small_splits(const Plan& P) {
  const int nt = small_rows_pad(P.g) / 64;
  const int o = small_splits_override();
  return o > 0 ? std::min(o, nt) : small_bwd_splits(P.g);
}
static at::Tensor small_scratch(const at::Tensor& like, const Plan& P) {
  return device_scratch(like, small_scratch_bytes(P.g, std::max(small_splits(P), small_bwd_splits(P.g))), 2);
}

// Returns {loss, zq, zqt, inv, lse2, sc, cpos}; `sc` holds the kept cosines (keep_cos) or is
// undefined.
std::vector<at::Tensor> fused_forward(const at::Tensor& h, double T, const std::string& compute, bool keep_cos) {
  check_input(h, "h");
  NTXENT_CHECK(h.dim() == 2, "z must be 2-D [2N, d]");
  const at::DeviceGuard guard(h.device());
  // "auto" = the input-dtype policy (fp32 stays exact); mixed precision is requested by the
  // callers as an explicit "fp16".
  const DType comp = choose_compute(h.scalar_type(), false, compute);
  auto P = get_plan((int)h.size(0), (int)h.size(1), 1, 0, T, dtype_name(comp), h.device().index());
  if (P->small && small_path_enabled()) {
    // {loss, zq, -, inv, lse2, -, a}: the backward recomputes S from zq (small_bwd). One launch:
    // the forward kernel normalises the rows itself (small_fwd_fused) and writes zq / inv.
    const int rp = small_rows_pad(P->g);
    auto lse2 = at::empty({rp}, opts(h, at::kFloat));
    auto arow = at::empty({rp}, opts(h, at::kFloat));
    auto loss = at::empty({}, opts(h, at::kFloat));
    at::Tensor zq, inv;
    float* ypos = nullptr;
    if (small_fwd_fused(P->g)) {
      zq = at::empty({rp, P->g.ld_k}, opts(h, to_scalar(P->comp)));
      inv = at::empty({P->g.rows}, opts(h, at::kFloat));
    } else {
      auto pr = prep(h, *P, c10::nullopt, c10::nullopt);
      zq = pr[0];
      inv = pr[1];
      ypos = pr[2].data_ptr<float>();
    }
    launch_small_fwd(to_dtype(h.scalar_type()), P->comp, h.data_ptr(), zq.data_ptr(), inv.data_ptr<float>(), ypos,
                     lse2.data_ptr<float>(), arow.data_ptr<float>(), loss.data_ptr<float>(),
                     small_scratch(h, *P).data_ptr(), P->g, cur_stream(h));
    return {loss, zq, at::Tensor(), inv, lse2, at::Tensor(), arow};
  }
  const DType in = to_dtype(h.scalar_type());
  if (keep_cos && comp != DType::FP8 && raw_forward_enabled() && raw_forward_eligible(P->g, in, comp)) {
    // raw-operand forward (RawRows): the GEMM reads h itself and normalises in its epilogue; the
    // prologue only computes inv and the positive logits, the LSE launch writes Z^T = (h inv)^T.
    // zq is returned empty (0 elements, the backward dtype): nothing reads unit rows
    auto inv = at::empty({P->g.rows}, opts(h, at::kFloat));
    auto ypos = at::empty({P->g.rows}, opts(h, at::kFloat));
    auto s = cur_stream(h);
    launch_prep(in, P->bwd(), h.data_ptr(), nullptr, inv.data_ptr<float>(), ypos.data_ptr<float>(), P->g, s);
    RawRows raw;
    raw.h = h.data_ptr();
    raw.in = in;
    raw.inv = inv.data_ptr<float>();
    auto zqt = at::empty({P->g.dim_n, P->g.ld_t}, opts(h, to_scalar(P->bwd())));
    raw.zqt = zqt.data_ptr();
    raw.zt = P->bwd();
    auto part = at::empty({P->g.col_tiles, P->g.rows_pad, 2}, opts(h, at::kFloat));
    auto sc = at::empty({(long)P->n_fwd * kTileElems}, opts(h, to_scalar(P->bwd())));
    auto ws = gemm_ws(h, P->n_fwd, *P);
    auto lse2 = at::empty({P->g.rows_pad}, opts(h, at::kFloat));
    auto cpos = at::empty({P->g.rows_pad}, opts(h, at::kFloat));
    auto block_loss = device_scratch(h, (size_t)lse_scratch_floats(P->g) * 4, 1);
    auto loss = at::empty({}, opts(h, at::kFloat));
    // the LSE outputs: the diagonal remainder's launch may compute them itself (RawRows::lse_folded)
    raw.ypos = ypos.data_ptr<float>();
    raw.lse2 = lse2.data_ptr<float>();
    raw.cpos = cpos.data_ptr<float>();
    raw.block_loss = static_cast<float*>(block_loss.data_ptr());
    raw.loss = loss.data_ptr<float>();
    auto fold_pre = at::empty({P->g.rows_pad, 2}, opts(h, at::kFloat));
    raw.fold_pre = reinterpret_cast<float2*>(fold_pre.data_ptr<float>());
    raw.fold_cnt = static_cast<int*>(device_scratch(h, (size_t)(P->g.rows_pad / 64 + 1) * 4, 3).data_ptr());
    const bool zt_fwd = launch_fwd_stats(P->comp, nullptr, nullptr, reinterpret_cast<const int4*>(P->fwd_tiles.data_ptr<int>()), P->n_fwd,
                     reinterpret_cast<float2*>(part.data_ptr<float>()), sc.data_ptr(), ws, P->g, s, BlockView{}, nullptr,
                     P->n_fwd == P->n_own ? own_diag_tail(P->g) : 0, nullptr, &raw);
    if (!raw.lse_folded)
      launch_lse(reinterpret_cast<const float2*>(part.data_ptr<float>()), ypos.data_ptr<float>(), lse2.data_ptr<float>(),
                 cpos.data_ptr<float>(), static_cast<float*>(block_loss.data_ptr()), loss.data_ptr<float>(), P->g, s,
                 P->bwd(), nullptr, zt_fwd ? nullptr : zqt.data_ptr(), nullptr, zt_fwd ? nullptr : &raw);
    return {loss, at::empty({0}, opts(h, to_scalar(P->bwd()))), zqt, inv, lse2, sc, cpos};
  }
  auto pr = prep(h, *P, c10::nullopt, c10::nullopt);
  // ZqT (the dZ GEMM's B operand) is first read in the backward: the LSE launch writes it from
  // extra blocks beside the merge (one stream: a side-stream transpose cost an event record and
  // a join of ~5-7 us each, or stretched the forward GEMM when launched beside it).
  auto zqt = at::empty({P->g.dim_n, P->g.ld_t}, pr[0].options());
  // fp8 plans: the forward GEMM reads the e4m3 copy and always keeps its cosines (fp16), so
  // the fp16 backward uses exactly the forward's logits
  const bool f8 = comp == DType::FP8;
  auto fs = f8 ? fwd_stats(pr[3], pr[3], *P, true) : fwd_stats(pr[0], pr[0], *P, keep_cos);
  auto lse2 = at::empty({P->g.rows_pad}, opts(h, at::kFloat));
  if (f8 && fp8_backward_enabled() && fp8_backward_eligible(P->g, comp)) {
    // fp8 backward: zqt = e4m3(256 Zq^T) (uint8: the backward's marker); cpos carries the LSE
    // pass's Q8Stats after its Rpad entries: [cpos | mneg2 (Rpad) | lmin]
    const long Rp = P->g.rows_pad;
    auto cpos = at::empty({2 * Rp + 64}, opts(h, at::kFloat));
    auto zq8t = at::empty({P->g.dim_n, q8_ldt(P->g)}, opts(h, at::kByte));
    Q8Stats q8;
    q8.mneg2 = cpos.data_ptr<float>() + Rp;
    q8.lmin = cpos.data_ptr<float>() + 2 * Rp;
    q8.zq8t = zq8t.data_ptr();
    auto block_loss = device_scratch(h, (size_t)lse_scratch_floats(P->g) * 4, 1);
    auto loss = at::empty({}, opts(h, at::kFloat));
    launch_lse(reinterpret_cast<const float2*>(fs[0].data_ptr<float>()), pr[2].data_ptr<float>(), lse2.data_ptr<float>(),
               cpos.data_ptr<float>(), static_cast<float*>(block_loss.data_ptr()), loss.data_ptr<float>(), P->g,
               cur_stream(h), DType::F16, pr[0].data_ptr(), nullptr, &q8);
    return {loss, pr[0], zq8t, pr[1], lse2, fs[1], cpos};
  }
  // (fp8 plans: 64 spare entries mark the e4m3 forward for the backward, which sees the fp16 rows)
  auto cpos = at::empty({P->g.rows_pad + (f8 ? 64 : 0)}, opts(h, at::kFloat));
  auto loss = lse(fs[0], pr[2], lse2, cpos, *P, pr[0], zqt);
  return {loss, pr[0], zqt, pr[1], lse2, fs[1], cpos};
}

at::Tensor fused_backward(const at::Tensor& h, const at::Tensor& zq, const c10::optional<at::Tensor>& zqt_in,
                          const at::Tensor& inv,
                          const at::Tensor& lse2, const c10::optional<at::Tensor>& sc_in, const at::Tensor& cpos,
                          const at::Tensor& grad_out, double T) {
  const at::DeviceGuard guard(h.device());
  const DType comp = to_dtype(zq.scalar_type());
  auto P = get_plan((int)h.size(0), (int)h.size(1), 1, 0, T, dtype_name(comp), h.device().index());
  const at::Tensor zqt = zqt_in.has_value() ? *zqt_in : at::Tensor();
  if (!zqt.defined()) {  // small-problem forward (see fused_forward): `cpos` holds a_i
    NTXENT_CHECK(P->small, "fused_backward: missing ZqT for a large-problem plan");
    auto go = grad_out.to(at::kFloat).reshape({-1}).narrow(0, 0, 1).contiguous();
    auto dh = at::empty_like(h);
    launch_small_bwd(to_dtype(h.scalar_type()), P->comp, zq.data_ptr(), h.data_ptr(), inv.data_ptr<float>(),
                     lse2.data_ptr<float>(), cpos.data_ptr<float>(), go.data_ptr<float>(), dh.data_ptr(),
                     small_scratch(h, *P).data_ptr(), P->g, cur_stream(h), small_splits(*P));
    return dh;
  }
  if (zqt.scalar_type() == at::kByte) {  // fp8 backward (see fused_forward)
    const long Rp = P->g.rows_pad;
    Q8Stats q8;
    q8.mneg2 = const_cast<float*>(cpos.data_ptr<float>()) + Rp;
    q8.lmin = const_cast<float*>(cpos.data_ptr<float>()) + 2 * Rp;
    q8.zq = zq.data_ptr();
    NTXENT_CHECK(sc_in.has_value() && sc_in->defined() && cpos.numel() == 2 * Rp + 64,
                 "fused_backward (fp8): kept cosines and the forward's Q8Stats required");
    // (no fused normalisation backward on fp8 plans: its dot_i = sum_j C_ij cos_ij would use the
    // e4m3 forward's cosines instead of z_i . g_i, a ~1e-2 radial error in dh)
    const bool fuse = false;
    at::Tensor dotp, dot, dh, go;
    if (fuse) {
      dotp = at::empty({Rp * dot_slots(P->g)}, opts(h, at::kFloat));
      dot = at::empty({Rp}, opts(h, at::kFloat));
    }
    auto cb = at::empty({(long)P->g.row_tiles * P->g.col_tiles * kTileElems}, opts(h, at::kByte));
    launch_coef(DType::F16, sc_in->data_ptr(), cb.data_ptr(), lse2.data_ptr<float>(), cpos.data_ptr<float>(),
                reinterpret_cast<const int4*>(P->fwd_tiles.data_ptr<int>()), P->n_fwd, P->g, cur_stream(h), nullptr,
                fuse ? dotp.data_ptr<float>() : nullptr, &q8);
    NormFuse nf;
    if (fuse) {
      launch_dot_reduce(dotp.data_ptr<float>(), dot.data_ptr<float>(), P->g, cur_stream(h));
      go = grad_out.to(at::kFloat).reshape({-1}).narrow(0, 0, 1).contiguous();
      dh = at::empty_like(h);
      nf.h = h.data_ptr();
      nf.in = to_dtype(h.scalar_type());
      nf.inv = inv.data_ptr<float>();
      nf.dot = dot.data_ptr<float>();
      nf.grad_out = go.data_ptr<float>();
      nf.dh = dh.data_ptr();
    }
    auto slabs = at::empty({1, P->g.rows_pad, P->g.dim_n}, opts(h, at::kHalf));
    auto ws = gemm_ws(h, P->n_dz, *P);
    const bool fused = launch_dz(DType::FP8, cb.data_ptr(), zqt.data_ptr(),
                                 reinterpret_cast<const int4*>(P->dz_tiles.data_ptr<int>()), P->n_dz, slabs.data_ptr(),
                                 ws, P->g, cur_stream(h), /*out_f16=*/true, fuse ? &nf : nullptr, &q8,
                                 cpos.data_ptr<float>());
    return fused ? dh : norm_bwd(slabs, h, inv, grad_out, *P);
  }
  // 16-bit plans finish the normalisation backward in the dZ epilogue with dot_i = z_i . g_i =
  // sum_j C_ij cos_ij from partials the coefficient pass emits (not on fp8-forward plans: that sum
  // would use the e4m3 forward's cosines)
  const bool f8_fwd = cpos.numel() != P->g.rows_pad;  // see fused_forward
  const bool fuse = P->bwd() != DType::F32 && P->g.dim % 8 == 0 && !f8_fwd;
  at::Tensor dotp, dot;
  if (fuse) {
    dotp = at::empty({(long)P->g.rows_pad * dot_slots(P->g)}, opts(h, at::kFloat));
    dot = at::empty({P->g.rows_pad}, opts(h, at::kFloat));
  }
  float* dp = fuse ? dotp.data_ptr<float>() : nullptr;
  at::Tensor cb;
  // half C: upper coefficient tiles only, the dZ reads the lower ones transposed (whole-tile dZ)
  const bool half_c = sc_in.has_value() && sc_in->defined() && half_c_enabled() &&
                      dz_half_c_eligible(P->bwd(), P->g, P->n_dz, gemm_ws(h, P->n_dz, *P));
  if (sc_in.has_value() && sc_in->defined()) {
    cb = coef(*sc_in, lse2, cpos, *P, dp, half_c);
  } else {
    // (a raw-operand forward returns no unit rows: a second backward rebuilds them to recompute S)
    const at::Tensor zr = zq.numel() > 0 ? zq : prep(h, *P, c10::nullopt, c10::nullopt)[0];
    cb = coef_gemm(zr, zr, lse2, cpos, *P, dp);
  }
  at::Tensor dh, go;
  NormFuse nf;
  // the dot reduce folded into the dZ (NormFuse::dot_cnt): per-stream counters (device_scratch)
  const bool dfold = fuse && dz_dot_fold_eligible(P->bwd(), P->g, P->n_dz, gemm_ws(h, P->n_dz, *P));
  if (fuse) {
    if (dfold) {
      nf.dotp = dp;
      nf.dot_cnt = static_cast<int*>(device_scratch(h, 2 * sizeof(int), 4).data_ptr());
    } else {
      launch_dot_reduce(dp, dot.data_ptr<float>(), P->g, cur_stream(h));
    }
    go = grad_out.to(at::kFloat).reshape({-1}).narrow(0, 0, 1).contiguous();
    dh = at::empty_like(h);
    nf.h = h.data_ptr();
    nf.in = to_dtype(h.scalar_type());
    nf.inv = inv.data_ptr<float>();
    nf.dot = dot.data_ptr<float>();
    nf.grad_out = go.data_ptr<float>();
    nf.dh = dh.data_ptr();
  }
  bool fused = false;
  auto slabs = dz(cb, zqt, *P, fuse ? &nf : nullptr, &fused, half_c);
  return fused ? dh : norm_bwd(slabs, h, inv, grad_out, *P);
}

// ---- reference-compatible API (src/binding_new.cpp:5-20) -------------------------------
at::Tensor forward_op(const at::Tensor& z, double T, bool use_mixed_precision) {
  auto out = fused_forward(z.contiguous(), T, use_mixed_precision ? "fp16" : "auto", /*keep_cos=*/false);
  return out[0];
}

// Row statistics handed from forward_with_stats to backward. The backward trusts a caller's LSE
// only when it is exactly a tensor forward_with_stats returned, unmodified since, for the SAME z
// tensor (same TensorImpl, same version counter: no in-place update in between), the same T and
// the same precision; anything else (the reference's softmax, an empty tensor, a stale LSE from
// an earlier step or another temperature) makes the backward recompute the statistics, so a
// result never silently depends on stale caller-provided stats.
namespace {
struct StatsTag {
  c10::weak_intrusive_ptr<c10::TensorImpl> stats, z;
  int64_t stats_ver = 0, z_ver = 0;
  double T = 0.0;
  bool mp = false;
};
std::mutex g_tag_mu;
std::vector<StatsTag> g_tags;  // most recent last; bounded
constexpr size_t kMaxTags = 32;

void tag_stats(const at::Tensor& stats, const at::Tensor& z, double T, bool mp) {
  std::lock_guard<std::mutex> lock(g_tag_mu);
  g_tags.erase(std::remove_if(g_tags.begin(), g_tags.end(), [](const StatsTag& t) { return t.stats.expired(); }),
               g_tags.end());
  if (g_tags.size() >= kMaxTags) g_tags.erase(g_tags.begin());
  g_tags.push_back(StatsTag{c10::weak_intrusive_ptr<c10::TensorImpl>(stats.getIntrusivePtr()),
                            c10::weak_intrusive_ptr<c10::TensorImpl>(z.getIntrusivePtr()), stats._version(),
                            z._version(), T, mp});
}

bool stats_match(const at::Tensor& stats, const at::Tensor& z, double T, bool mp) {
  if (!stats.defined() || !z.defined()) return false;
  std::lock_guard<std::mutex> lock(g_tag_mu);
  for (auto it = g_tags.rbegin(); it != g_tags.rend(); ++it) {
    auto sp = it->stats.lock();
    if (!sp || sp.get() != stats.unsafeGetTensorImpl()) continue;
    auto zp = it->z.lock();
    return zp && zp.get() == z.unsafeGetTensorImpl() && it->z_ver == z._version() &&
           it->stats_ver == stats._version() && it->T == T && it->mp == mp;
  }
  return false;
}
}  // namespace

std::vector<at::Tensor> forward_with_stats(const at::Tensor& z, double T, bool use_mixed_precision) {
  auto out = fused_forward(z.contiguous(), T, use_mixed_precision ? "fp16" : "auto", false);
  const int R = (int)z.size(0);
  auto lse_nat = out[4].narrow(0, 0, R) * (float)0.6931471805599453;
  tag_stats(lse_nat, z, T, use_mixed_precision);
  return {out[0], lse_nat};
}

// backward(z, stats, grad_out, T): the reference passes a softmax matrix here that its own
// forward never returns (src/ntxent_kernel.cu:202). Here `stats` may be the per-row LSE that
// forward_with_stats returned for this z (see StatsTag): the backward then costs ONE similarity
// GEMM (the cosines are recomputed inside the coefficient GEMM; a stateless op keeps none).
// Anything else in that slot is ignored and the row statistics are recomputed (one more
// similarity GEMM).
// Returns (grad_z, grad_logits). grad_logits = dL/dS [2N, 2N] (fp32) is a debug/parity output
// built only when want_grad_logits is set; otherwise it is an empty tensor, so the default call
// runs no extra GEMM and allocates nothing quadratic.
std::tuple<at::Tensor, at::Tensor> backward_op(const at::Tensor& z_in, const at::Tensor& stats,
                                               const at::Tensor& grad_out, double T, bool use_mixed_precision,
                                               bool want_grad_logits) {
  auto z = z_in.contiguous();
  const at::DeviceGuard guard(z.device());
  const DType comp = choose_compute(z.scalar_type(), use_mixed_precision, "");
  auto P = get_plan((int)z.size(0), (int)z.size(1), 1, 0, T, dtype_name(comp), z.device().index());
  auto pr = prep(z, *P, c10::nullopt, c10::nullopt);
  auto zqt = transpose(pr[0], *P, c10::nullopt);
  const long R = z.size(0), n = R / 2, Rp = P->g.rows_pad;
  at::Tensor lse2, cpos;
  const bool have_lse = stats.defined() && stats.dim() == 1 && stats.size(0) == R && stats.is_floating_point() &&
                        stats.device() == z.device() && stats_match(stats, z_in, T, use_mixed_precision);
  if (have_lse) {
    // lse2 in log2 units; C_i,p(i) = -(a_i + a_p(i)), a_i = 1 - P_ip = -expm1(y_ip - lse_i)
    // (expm1 keeps a_i accurate when P_ip -> 1)
    auto lse_nat = stats.to(at::kFloat);
    lse2 = at::zeros({Rp}, opts(z, at::kFloat));
    lse2.narrow(0, 0, R).copy_(lse_nat * (float)1.4426950408889634);
    auto y_nat = pr[2].narrow(0, 0, R) * (float)0.6931471805599453;
    auto a = -at::expm1(y_nat - lse_nat);
    cpos = at::zeros({Rp}, opts(z, at::kFloat));
    cpos.narrow(0, 0, R).copy_(-(a + at::roll(a, {n})));
  } else {
    lse2 = at::empty({Rp}, opts(z, at::kFloat));
    cpos = at::empty({Rp}, opts(z, at::kFloat));
    auto fs = fwd_stats(pr[0], pr[0], *P, false);
    lse(fs[0], pr[2], lse2, cpos, *P);
  }
  auto sc = coef_gemm(pr[0], pr[0], lse2, cpos, *P);
  auto slabs = dz(sc, zqt, *P);
  auto go = grad_out.to(at::kFloat).reshape({-1}).narrow(0, 0, 1).contiguous();
  auto dh = norm_bwd(slabs, z, pr[1], go, *P);
  at::Tensor grad_logits;
  if (want_grad_logits) {
    // dL/dS_ij = grad_out * (P_ij - [j == p(i)]) / 2N  (debug/parity output)
    auto zf = z.to(at::kFloat);
    auto zn = zf / zf.norm(2, {1}, true).clamp_min(1e-12);
    auto S = at::matmul(zn, zn.t()) / T;
    S.fill_diagonal_(-std::numeric_limits<float>::infinity());
    auto lse_nat = lse2.narrow(0, 0, R) * (float)0.6931471805599453;
    auto G = at::exp(S - lse_nat.unsqueeze(1));
    auto idx = at::arange(R, opts(z, at::kLong));
    auto pos = (idx + n) % R;
    G.index_put_({idx, pos}, G.index({idx, pos}) - 1.0);
    grad_logits = G * (go / (double)R);
  } else {
    grad_logits = at::empty({0}, opts(z, at::kFloat));
  }
  return {dh, grad_logits};
}

bool check_tensor_core_support() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  return check_matrix_core_support(dev);
}


// ---- the native Engine from Python (ntxent_amd.native) ------------------------------------
// The libtorch-free runtime (engine.h: one arena, fixed launch sequence, hipGraph capture,
// RcclComm data parallelism) driven from torch tensors on the current stream. The RCCL unique
// id is produced by rccl_unique_id() on one rank and handed to the others by the caller
// (ntxent_amd.native bootstraps it through the torch.distributed store).
namespace {
DType parse_dtype_name(const std::string& s) {
  if (s == "float32" || s == "fp32") return DType::F32;
  if (s == "float16" || s == "fp16") return DType::F16;
  if (s == "bfloat16" || s == "bf16") return DType::BF16;
  if (s == "fp8" || s == "e4m3") return DType::FP8;
  throw std::invalid_argument("unknown dtype '" + s + "' (fp32|fp16|bf16|fp8)");
}
at::ScalarType scalar_of(DType t) {
  return t == DType::F32 ? at::kFloat : (t == DType::F16 ? at::kHalf : at::kBFloat16);
}

class NativeEngine {
 public:
  NativeEngine(int rows, int dim, double T, const std::string& input, const std::string& compute,
               const std::string& negatives, int rank, int world, const std::string& uid, int device, bool keep_cos,
               int comm_reserve_cus, std::shared_ptr<RcclComm> comm = nullptr)
      : device_(device) {
    NTXENT_CHECK(world >= 1 && rank >= 0 && rank < world, "NativeEngine: bad rank/world");
    NTXENT_CHECK(negatives == "symmetric" || negatives == "allgather", "negatives must be symmetric|allgather");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(device);
    if (comm) {  // a communicator shared by every engine of this process group (one RCCL init)
      NTXENT_CHECK(comm->rank() == rank && comm->world() == world, "NativeEngine: communicator rank/world mismatch");
      comm_ = std::move(comm);
    } else if (world > 1) {
      comm_ = std::make_shared<RcclComm>(rank, world, uid, device);
    }
    EngineConfig cfg;
    cfg.rows = rows;
    cfg.dim = dim;
    cfg.temperature = (float)T;
    cfg.input = parse_dtype_name(input);
    NTXENT_CHECK(cfg.input != DType::FP8, "NativeEngine: input must be fp32|fp16|bf16");
    cfg.compute = compute == "auto" ? (cfg.input == DType::F32 ? DType::F32 : DType::F16) : parse_dtype_name(compute);
    cfg.keep_cos = keep_cos;
    cfg.comm_reserve_cus = comm_reserve_cus;
    cfg.negatives = negatives == "symmetric" ? Negatives::kSymmetric : Negatives::kAllGather;
    cfg.device = device;
    in_ = scalar_of(cfg.input);
    eng_ = std::make_unique<Engine>(cfg, comm_.get());
  }

  void forward(const at::Tensor& h) {
    check_h(h);
    c10::hip::HIPGuardMasqueradingAsCUDA guard(device_);
    h_ = h;  // the backward reads the forward's h
    eng_->forward(h.data_ptr(), cur_stream(h));
  }
  at::Tensor backward(const c10::optional<at::Tensor>& grad_out) {
    NTXENT_CHECK(h_.defined(), "NativeEngine.backward needs a preceding forward");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(device_);
    at::Tensor go;
    if (grad_out && grad_out->defined()) {
      go = grad_out->to(h_.device(), at::kFloat).reshape({1}).contiguous();
    }
    at::Tensor dh = at::empty_like(h_);
    eng_->backward(go.defined() ? go.data_ptr<float>() : nullptr, dh.data_ptr(), cur_stream(h_));
    return dh;
  }
  // the global mean loss as a 0-d fp32 tensor (stream-ordered copy of the engine's slot)
  at::Tensor loss_tensor() const {
    NTXENT_CHECK(h_.defined(), "no forward yet");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(device_);
    at::Tensor out = at::empty({}, h_.options().dtype(at::kFloat));
    NTXENT_HIP_CHECK(hipMemcpyAsync(out.data_ptr(), eng_->loss_device(), sizeof(float), hipMemcpyDeviceToDevice,
                                    cur_stream(h_)));
    return out;
  }
  std::tuple<at::Tensor, at::Tensor> step(const at::Tensor& h) {
    forward(h);
    at::Tensor dh = backward(c10::nullopt);
    return {loss_tensor(), dh};
  }
  // hipGraph of one step for fixed h (dh is returned and reused by every replay). The graph
  // holds h's and dh's device pointers, so both are kept alive in their own members (gh_, gdh_)
  // for as long as the graph exists, whatever forward()/step() do with h_ in between.
  // Single process only: a captured step of a multi-rank engine would bake RCCL calls into the
  // graph.
  at::Tensor capture(const at::Tensor& h) {
    check_h(h);
    NTXENT_CHECK(world() == 1, "NativeEngine.capture: single-process engines only (world == 1)");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(device_);
    at::Tensor dh = at::empty_like(h);
    eng_->capture(h.data_ptr(), dh.data_ptr(), cur_stream(h));
    gh_ = h;
    gdh_ = dh;
    h_ = h;  // loss_tensor() after a replay reads the graph's forward
    return gdh_;
  }
  void replay() {
    NTXENT_CHECK(eng_->captured() && gh_.defined(), "NativeEngine.replay needs capture()");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(device_);
    // the engine's backward reads the forward input: point it back at the captured one
    h_ = gh_;
    eng_->replay(cur_stream(gh_));
  }
  size_t device_bytes() const { return eng_->device_bytes(); }
  bool symmetric() const { return eng_->symmetric(); }
  bool small() const { return eng_->small(); }
  int rank() const { return comm_ ? comm_->rank() : 0; }
  int world() const { return comm_ ? comm_->world() : 1; }

 private:
  void check_h(const at::Tensor& h) const {
    const auto& c = eng_->config();
    NTXENT_CHECK(h.is_cuda() && h.device().index() == device_, "h must be on the engine's device");
    NTXENT_CHECK(h.scalar_type() == in_, "h dtype does not match the engine's input dtype");
    NTXENT_CHECK(h.dim() == 2 && h.size(0) == c.rows && h.size(1) == c.dim && h.is_contiguous(),
                 "h must be a contiguous [rows, dim] tensor");
  }
  int device_ = 0;
  at::ScalarType in_ = at::kBFloat16;
  std::shared_ptr<RcclComm> comm_;  // declared before eng_: destroyed after it
  std::unique_ptr<Engine> eng_;
  at::Tensor h_;         // input of the last forward (read by backward)
  at::Tensor gh_, gdh_;  // the captured graph's input and output (alive while the graph exists)
};
}  // namespace

}  // namespace th
}  // namespace ntxent

// ---- torch.ops registration (python/test.py:137 resolves `torch.ops.ntxent_cuda`) -------
TORCH_LIBRARY(ntxent_cuda, m) {
  m.def("forward(Tensor z, float T, bool use_mixed_precision=False) -> Tensor");
  m.def("backward(Tensor z, Tensor softmax, Tensor grad_out, float T, bool use_mixed_precision=False, bool want_grad_logits=False) -> (Tensor, Tensor)");
  m.def("check_tensor_core_support() -> bool", &ntxent::th::check_tensor_core_support);
}
TORCH_LIBRARY_IMPL(ntxent_cuda, CUDA, m) {
  m.impl("forward", &ntxent::th::forward_op);
  m.impl("backward", &ntxent::th::backward_op);
}
TORCH_LIBRARY(ntxent, m) {
  m.def("forward(Tensor z, float T, bool use_mixed_precision=False) -> Tensor");
  m.def("forward_with_stats(Tensor z, float T, bool use_mixed_precision=False) -> Tensor[]");
  m.def("backward(Tensor z, Tensor softmax, Tensor grad_out, float T, bool use_mixed_precision=False, bool want_grad_logits=False) -> (Tensor, Tensor)");
}
TORCH_LIBRARY_IMPL(ntxent, CUDA, m) {
  m.impl("forward", &ntxent::th::forward_op);
  m.impl("forward_with_stats", &ntxent::th::forward_with_stats);
  m.impl("backward", &ntxent::th::backward_op);
}

// ---- pybind11 module ---------------------------------------------------------------------
PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  namespace py = pybind11;
  using namespace ntxent::th;
  m.doc() = "MI355X (gfx950) NT-Xent loss: MFMA/LDS HIP kernels";
  py::class_<Plan, std::shared_ptr<Plan>>(m, "Plan")
      .def_property_readonly("rows", &Plan::rows)
      .def_property_readonly("rows_pad", &Plan::rows_pad)
      .def_property_readonly("dim", &Plan::dim)
      .def_property_readonly("dim_k", &Plan::dim_k)
      .def_property_readonly("ld_k", &Plan::ld_k)
      .def_property_readonly("ld_t", &Plan::ld_t)
      .def_property_readonly("dim_n", &Plan::dim_n)
      .def_property_readonly("world", &Plan::world)
      .def_property_readonly("rank", &Plan::rank)
      .def_property_readonly("row_tiles", &Plan::row_tiles)
      .def_property_readonly("col_tiles", &Plan::col_tiles)
      .def_property_readonly("temperature", &Plan::temperature)
      .def_property_readonly("compute_dtype", &Plan::compute_dtype)
      .def_property_readonly("backward_dtype", &Plan::backward_dtype_name)
      .def_property_readonly("ld_k8", [](const Plan& p) { return p.g.ld_k8; })
      .def_property_readonly("sym_c_ld", [](const Plan& p) { return sym_c_ld(p.g); })
      .def_readonly("n_fwd_tiles", &Plan::n_fwd)
      .def_readonly("n_own_tiles", &Plan::n_own)
      .def_readonly("n_dz_tiles", &Plan::n_dz)
      .def_readonly("small", &Plan::small)
      .def_readonly("fwd_tiles", &Plan::fwd_tiles)
      .def_readonly("dz_tiles", &Plan::dz_tiles);
  // one RCCL communicator per (process group, device), shared by the engines of every shape
  py::class_<ntxent::RcclComm, std::shared_ptr<ntxent::RcclComm>>(m, "RcclCommunicator")
      .def(py::init([](int rank, int world, const py::bytes& uid, int device) {
             return std::make_shared<ntxent::RcclComm>(rank, world, std::string(uid), device);
           }),
           py::arg("rank"), py::arg("world"), py::arg("uid"), py::arg("device"))
      .def_property_readonly("rank", &ntxent::RcclComm::rank)
      .def_property_readonly("world", &ntxent::RcclComm::world)
      .def("check", &ntxent::RcclComm::check)
      .def("abort", &ntxent::RcclComm::abort);
  py::class_<NativeEngine>(m, "NativeEngine")
      .def(py::init<int, int, double, const std::string&, const std::string&, const std::string&, int, int,
                    const std::string&, int, bool, int, std::shared_ptr<ntxent::RcclComm>>(),
           py::arg("rows"), py::arg("dim"), py::arg("temperature"), py::arg("input") = "bf16",
           py::arg("compute") = "auto", py::arg("negatives") = "symmetric", py::arg("rank") = 0, py::arg("world") = 1,
           py::arg("uid") = std::string(), py::arg("device") = 0, py::arg("keep_cos") = true,
           py::arg("comm_reserve_cus") = 8, py::arg("comm") = py::none())
      .def("forward", &NativeEngine::forward, py::arg("h"))
      .def("backward", &NativeEngine::backward, py::arg("grad_out") = py::none())
      .def("loss_tensor", &NativeEngine::loss_tensor)
      .def("step", &NativeEngine::step, py::arg("h"))
      .def("capture", &NativeEngine::capture, py::arg("h"))
      .def("replay", &NativeEngine::replay)
      .def_property_readonly("device_bytes", &NativeEngine::device_bytes)
      .def_property_readonly("symmetric", &NativeEngine::symmetric)
      .def_property_readonly("small", &NativeEngine::small)
      .def_property_readonly("rank", &NativeEngine::rank)
      .def_property_readonly("world", &NativeEngine::world);
  m.def("rccl_unique_id", []() { return py::bytes(ntxent::RcclComm::unique_id()); });
  m.def("get_plan", &get_plan, py::arg("rows"), py::arg("dim"), py::arg("world"), py::arg("rank"),
        py::arg("temperature"), py::arg("compute"), py::arg("device"));
  m.def("choose_compute", [](const std::string& in_dtype, bool mp, const std::string& ov) {
    at::ScalarType t = in_dtype == "float32" ? at::kFloat : (in_dtype == "float16" ? at::kHalf : at::kBFloat16);
    return std::string(ntxent::dtype_name(choose_compute(t, mp, ov)));
  });
  m.def("prep", &prep, py::arg("h"), py::arg("plan"), py::arg("zq_out") = py::none(), py::arg("zq8_out") = py::none());
  m.def("transpose", &transpose, py::arg("zq"), py::arg("plan"), py::arg("zqt_out") = py::none());
  m.def("fwd_stats_range", &fwd_stats_range, py::arg("zq_local"), py::arg("zq_all"), py::arg("plan"), py::arg("part"),
        py::arg("sc"), py::arg("first"), py::arg("count"), py::arg("reserve_cus") = 0);
  m.def("fwd_stats", [](const at::Tensor& zl, const at::Tensor& za, const Plan& P, bool keep) {
    return fwd_stats(zl, za, P, keep, true);
  }, py::arg("zq_local"), py::arg("zq_all"), py::arg("plan"), py::arg("keep_cos"));
  m.def("lse", &lse, py::arg("part"), py::arg("ypos"), py::arg("lse2_all"), py::arg("cpos"), py::arg("plan"),
        py::arg("zq") = py::none(), py::arg("zqt") = py::none());
  m.def("coef", [](const at::Tensor& sbuf, const at::Tensor& lse2_all, const at::Tensor& cpos, const Plan& P) {
    return coef(sbuf, lse2_all, cpos, P);
  }, py::arg("sbuf"), py::arg("lse2_all"), py::arg("cpos"), py::arg("plan"));
  m.def("coef_gemm", [](const at::Tensor& zl, const at::Tensor& za, const at::Tensor& lse2_all, const at::Tensor& cpos,
                        const Plan& P) { return coef_gemm(zl, za, lse2_all, cpos, P); });
  m.def("dz", [](const at::Tensor& sc, const at::Tensor& zqt_all, const Plan& P) { return dz(sc, zqt_all, P); });
  m.def("set_fp8_backward", &ntxent::set_fp8_backward, py::arg("on"));
  m.def("set_raw_forward", &ntxent::set_raw_forward, py::arg("on"));
  m.def("raw_forward_enabled", &ntxent::raw_forward_enabled);
  m.def("set_lse_fold", &ntxent::set_lse_fold, py::arg("on"));
  m.def("lse_fold_enabled", &ntxent::lse_fold_enabled);
  m.def("set_half_c", &ntxent::set_half_c, py::arg("on"));
  m.def("half_c_enabled", &ntxent::half_c_enabled);
  m.def("set_dot_fold", &ntxent::set_dot_fold, py::arg("on"));
  m.def("dot_fold_enabled", &ntxent::dot_fold_enabled);
  m.def("set_dot_fold_spin", &ntxent::set_dot_fold_spin, py::arg("polls"));
  m.def("dot_fold_spin", &ntxent::dot_fold_spin);
  m.def("fp8_backward_enabled", &ntxent::fp8_backward_enabled);
  m.def("fwd_splitk_pieces", &ntxent::fwd_splitk_pieces, py::arg("ntiles"), py::arg("nk"), py::arg("cus"),
        py::arg("diag_tail"));
  m.def("fwd_diag_remainder", &ntxent::fwd_diag_remainder, py::arg("ntiles"), py::arg("nk"), py::arg("cus"),
        py::arg("diag_tail"), py::arg("f8") = false);
  m.def("norm_bwd", &norm_bwd, py::arg("slabs"), py::arg("h"), py::arg("inv"), py::arg("grad_out"), py::arg("plan"));
  m.def("fwd_stats_tiles", &fwd_stats_tiles, py::arg("zq_local"), py::arg("zq_chunk"), py::arg("b_tile0"),
        py::arg("tiles"), py::arg("plan"), py::arg("part"), py::arg("reserve_cus") = 0);
  m.def("coef_gemm_tiles", &coef_gemm_tiles, py::arg("zq_local"), py::arg("zq_chunk"), py::arg("b_tile0"),
        py::arg("tiles"), py::arg("lse2_all"), py::arg("cpos"), py::arg("plan"), py::arg("c_ld"), py::arg("c_tile0"),
        py::arg("reserve_cus") = 0);
  m.def("dz_block", &dz_block, py::arg("cbuf_block"), py::arg("zqt_chunk"), py::arg("plan"), py::arg("reserve_cus") = 0);
  m.def("sym_fwd_tiles", &sym_fwd_tiles, py::arg("plan"), py::arg("jobs"), py::arg("nchunks") = 1);
  m.def("fwd_stats_sym", &fwd_stats_sym, py::arg("zq_local"), py::arg("zq_all"), py::arg("tiles"), py::arg("plan"),
        py::arg("part"), py::arg("part_x"), py::arg("sc"), py::arg("first"), py::arg("count"), py::arg("reserve_cus") = 0);
  m.def("coef_sym", &coef_sym, py::arg("sbuf"), py::arg("tiles"), py::arg("lse2_all"), py::arg("cpos"), py::arg("plan"),
        py::arg("cbuf"), py::arg("mbuf"));
  m.def("dz_view", &dz_view, py::arg("abuf"), py::arg("a_tile0"), py::arg("a_panel_tiles"), py::arg("bbuf"),
        py::arg("b_block0"), py::arg("b_col0"), py::arg("k_tiles"), py::arg("m0"), py::arg("m1"), py::arg("out"),
        py::arg("accum"), py::arg("plan"), py::arg("reserve_cus") = 0);
  m.def("norm_bwd_slabs", &norm_bwd_slabs, py::arg("slabs"), py::arg("h"), py::arg("inv"), py::arg("grad_out"),
        py::arg("plan"), py::arg("xslabs") = py::none());
  m.def("fused_forward", &fused_forward, py::arg("h"), py::arg("T"), py::arg("compute") = "auto",
        py::arg("keep_cos") = true);
  m.def("fused_backward", &fused_backward);
  m.def("set_small_path", &ntxent::set_small_path, py::arg("on"));
  m.def("small_path_enabled", &ntxent::small_path_enabled);
  m.def("set_small_splits", &ntxent::set_small_splits, py::arg("n"));
  m.def("set_small_fuse_rows", &ntxent::set_small_fuse_rows, py::arg("rows"));
  m.def("small_fwd_fused", [](const Plan& P) { return ntxent::small_fwd_fused(P.g); });
  // reference API names and kwargs
  m.def("forward", &forward_op, py::arg("z"), py::arg("T"), py::arg("use_mixed_precision") = false);
  m.def("forward_with_stats", &forward_with_stats, py::arg("z"), py::arg("T"), py::arg("use_mixed_precision") = false);
  m.def("backward", &backward_op, py::arg("z"), py::arg("softmax"), py::arg("grad_out"), py::arg("T"),
        py::arg("use_mixed_precision") = false, py::arg("want_grad_logits") = false);
  m.def("check_tensor_core_support", &check_tensor_core_support);
  m.def("check_matrix_core_support", &check_tensor_core_support);
  m.def("get_optimal_block_size", &ntxent::get_optimal_block_size);
  m.def("device_info", [](int dev) {
    const auto& d = ntxent::device_info(dev);
    py::dict r;
    r["device"] = d.device;
    r["num_cus"] = d.num_cus;
    r["lds_per_block"] = d.lds_per_block;
    r["warp_size"] = d.warp_size;
    r["arch"] = d.arch;
    r["is_gfx950"] = d.is_gfx950;
    return r;
  });
  // host-only planning helpers (no device needed: unit-tested on CPU)
  m.def("geometry", [](int rows, int dim, int world, int rank, double T) {
    const auto g = ntxent::make_geometry(rows, dim, world, rank, (float)T);
    py::dict r;
    r["rows"] = g.rows; r["rows_pad"] = g.rows_pad; r["dim"] = g.dim; r["dim_k"] = g.dim_k;
    r["dim_n"] = g.dim_n; r["ld_k"] = g.ld_k; r["ld_t"] = g.ld_t; r["world"] = g.world;
    r["rank"] = g.rank; r["row_tiles"] = g.row_tiles; r["col_tiles"] = g.col_tiles;
    r["global_rows"] = g.global_rows;
    return r;
  }, py::arg("rows"), py::arg("dim"), py::arg("world") = 1, py::arg("rank") = 0, py::arg("T") = 0.07);
  auto tiles_to_list = [](const std::vector<int4>& v) {
    py::list l;
    for (const auto& t : v) l.append(py::make_tuple(t.x, t.y, t.z));
    return l;
  };
  m.def("fwd_tile_list", [tiles_to_list](int rows, int dim, int world, int rank) {
    return tiles_to_list(ntxent::build_fwd_tiles(ntxent::make_geometry(rows, dim, world, rank, 0.07f)));
  }, py::arg("rows"), py::arg("dim"), py::arg("world") = 1, py::arg("rank") = 0);
  m.def("dz_tile_list", [tiles_to_list](int rows, int dim, int world, int rank) {
    return tiles_to_list(ntxent::build_dz_tiles(ntxent::make_geometry(rows, dim, world, rank, 0.07f)));
  }, py::arg("rows"), py::arg("dim"), py::arg("world") = 1, py::arg("rank") = 0);
  m.def("sym_fwd_tile_list", [tiles_to_list](int rows, int dim, int world, int rank,
                                             const std::vector<std::tuple<int, int, int, int, int>>& jobs, int nchunks) {
    return tiles_to_list(
        ntxent::build_sym_fwd_tiles(ntxent::make_geometry(rows, dim, world, rank, 0.07f), to_jobs(jobs), nchunks));
  }, py::arg("rows"), py::arg("dim"), py::arg("world"), py::arg("rank"), py::arg("jobs"), py::arg("nchunks") = 1);
  m.def("schedule", [](int ntiles, int nk, int num_cus) {
    const auto s = ntxent::make_schedule(ntiles, nk, num_cus);
    py::dict r;
    r["grid"] = s.grid; r["nk"] = s.nk; r["dp_tiles"] = s.dp_tiles; r["sk_tiles"] = s.sk_tiles;
    r["ipb"] = s.ipb;
    return r;
  }, py::arg("ntiles"), py::arg("nk"), py::arg("num_cus"));
  m.def("gemm_workspace_bytes", &ntxent::gemm_workspace_bytes);
  m.attr("TILE") = ntxent::kTile;
  m.attr("K_STEP_BYTES") = ntxent::kKStepBytes;
}

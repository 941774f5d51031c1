// ntxent_bench — native C++ benchmark of the MI355X NT-Xent kernels (no libtorch).
//
// Counterpart of the reference's forward-only latency sweep (src/benchmark.cpp:16-97:
// B in {32..1024} x D in {64,128,256}, T=0.07, 1 warmup + 100 timed runs, mean/std/min/max).
// Differences by design: hipEvent timing on the stream (not host chrono around a device
// sync), forward, backward and fwd+bwd are all timed, and the BASELINE configs are included.
//
//   ntxent_bench                       # reference sweep (fwd, bwd, fwd+bwd)
//   ntxent_bench --batch 4096 --dim 2048 --dtype bf16 --iters 50
//   ntxent_bench --check               # also compare loss against a host fp64 evaluation
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "ntxent/ntxent.h"

using namespace ntxent;

namespace {

uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFF + ((u >> 16) & 1);  // round to nearest even
  return (uint16_t)(u >> 16);
}

uint16_t f32_to_f16(float f) {
  _Float16 h = (_Float16)f;
  uint16_t u;
  std::memcpy(&u, &h, 2);
  return u;
}

struct Buffers {
  void* h = nullptr;
  void* dh = nullptr;
  void* zq = nullptr;
  void* zqt = nullptr;
  float* inv = nullptr;
  float* ypos = nullptr;
  float2* part = nullptr;
  void* sbuf = nullptr;
  void* cbuf = nullptr;
  float* lse2 = nullptr;
  float* cpos = nullptr;
  float* block_loss = nullptr;
  float* loss = nullptr;
  float* grad_out = nullptr;
  float* slabs = nullptr;
  int4* fwd_tiles = nullptr;
  int4* dz_tiles = nullptr;
  int n_fwd = 0, n_dz = 0, ksplit = 1;
};

struct Result {
  double mean = 0, stdev = 0, mn = 0, mx = 0;
};

Result stats(std::vector<float> v) {
  Result r;
  double s = 0;
  for (float x : v) s += x;
  r.mean = s / v.size();
  double q = 0;
  for (float x : v) q += (x - r.mean) * (x - r.mean);
  r.stdev = std::sqrt(q / v.size());  // population std (as the reference, src/benchmark.cpp:42-53)
  r.mn = *std::min_element(v.begin(), v.end());
  r.mx = *std::max_element(v.begin(), v.end());
  return r;
}

class Bench {
 public:
  Bench(int batch, int dim, DType in, DType comp, float T, int ncus)
      : in_(in), comp_(comp), g_(make_geometry(2 * batch, dim, 1, 0, T)) {
    const size_t is = dtype_size(in), cs = dtype_size(comp);
    const size_t R = g_.rows, Rp = g_.rows_pad;
    auto ft = build_fwd_tiles(g_);
    b_.ksplit = choose_dz_ksplit(g_, ncus);
    auto dt = build_dz_tiles(g_, b_.ksplit);
    b_.n_fwd = (int)ft.size();
    b_.n_dz = (int)dt.size();
    NTXENT_HIP_CHECK(hipMalloc(&b_.h, R * dim * is));
    NTXENT_HIP_CHECK(hipMalloc(&b_.dh, R * dim * is));
    NTXENT_HIP_CHECK(hipMalloc(&b_.zq, Rp * g_.ld_k * cs));
    NTXENT_HIP_CHECK(hipMalloc(&b_.zqt, (size_t)g_.dim_n * g_.ld_t * cs));
    NTXENT_HIP_CHECK(hipMalloc(&b_.inv, R * 4));
    NTXENT_HIP_CHECK(hipMalloc(&b_.ypos, R * 4));
    NTXENT_HIP_CHECK(hipMalloc(&b_.part, (size_t)g_.col_tiles * Rp * 8));
    NTXENT_HIP_CHECK(hipMalloc(&b_.sbuf, (size_t)b_.n_fwd * kTileElems * cs));
    NTXENT_HIP_CHECK(hipMalloc(&b_.cbuf, (size_t)g_.row_tiles * g_.col_tiles * kTileElems * cs));
    NTXENT_HIP_CHECK(hipMalloc(&b_.lse2, Rp * 4));
    NTXENT_HIP_CHECK(hipMalloc(&b_.cpos, Rp * 4));
    NTXENT_HIP_CHECK(hipMalloc(&b_.block_loss, Rp / 256 * 4 + 64));
    NTXENT_HIP_CHECK(hipMalloc(&b_.loss, 4));
    NTXENT_HIP_CHECK(hipMalloc(&b_.grad_out, 4));
    NTXENT_HIP_CHECK(hipMalloc(&b_.slabs, (size_t)b_.ksplit * Rp * g_.dim_n * 4));
    NTXENT_HIP_CHECK(hipMalloc(&b_.fwd_tiles, ft.size() * sizeof(int4)));
    NTXENT_HIP_CHECK(hipMalloc(&b_.dz_tiles, dt.size() * sizeof(int4)));
    NTXENT_HIP_CHECK(hipMemcpy(b_.fwd_tiles, ft.data(), ft.size() * sizeof(int4), hipMemcpyHostToDevice));
    NTXENT_HIP_CHECK(hipMemcpy(b_.dz_tiles, dt.data(), dt.size() * sizeof(int4), hipMemcpyHostToDevice));
    const float one = 1.0f;
    NTXENT_HIP_CHECK(hipMemcpy(b_.grad_out, &one, 4, hipMemcpyHostToDevice));
    // synthetic random-normal embeddings (two noisy views of shared bases)
    std::mt19937 rng(1234);
    std::normal_distribution<float> nd;
    host_.resize(R * dim);
    const size_t n = R / 2;
    for (size_t i = 0; i < n; ++i)
      for (int e = 0; e < dim; ++e) {
        const float b = nd(rng);
        host_[i * dim + e] = b + 0.5f * nd(rng);
        host_[(i + n) * dim + e] = b + 0.5f * nd(rng);
      }
    std::vector<uint16_t> h16(R * dim);
    if (in == DType::F32) {
      NTXENT_HIP_CHECK(hipMemcpy(b_.h, host_.data(), R * dim * 4, hipMemcpyHostToDevice));
    } else {
      for (size_t k = 0; k < h16.size(); ++k) {
        h16[k] = in == DType::BF16 ? f32_to_bf16(host_[k]) : f32_to_f16(host_[k]);
        // keep the host copy equal to what the device sees
        if (in == DType::BF16) {
          uint32_t u = (uint32_t)h16[k] << 16;
          std::memcpy(&host_[k], &u, 4);
        } else {
          _Float16 hh;
          std::memcpy(&hh, &h16[k], 2);
          host_[k] = (float)hh;
        }
      }
      NTXENT_HIP_CHECK(hipMemcpy(b_.h, h16.data(), R * dim * 2, hipMemcpyHostToDevice));
    }
    NTXENT_HIP_CHECK(hipStreamCreate(&s_));
    ws_.num_cus = ncus;
    ws_.bytes = gemm_workspace_bytes(std::max(b_.n_fwd, b_.n_dz), ncus);
    NTXENT_HIP_CHECK(hipMalloc(&ws_.ptr, ws_.bytes));
  }
  ~Bench() {
    hipFree(b_.h); hipFree(b_.dh); hipFree(b_.zq); hipFree(b_.zqt); hipFree(b_.inv); hipFree(b_.ypos);
    hipFree(b_.part); hipFree(b_.sbuf); hipFree(b_.cbuf); hipFree(b_.lse2); hipFree(b_.cpos);
    hipFree(b_.block_loss); hipFree(b_.loss); hipFree(b_.grad_out); hipFree(b_.slabs);
    hipFree(b_.fwd_tiles); hipFree(b_.dz_tiles); hipFree(ws_.ptr);
    hipStreamDestroy(s_);
  }

  void fwd() {
    launch_prep(in_, comp_, b_.h, b_.zq, b_.inv, b_.ypos, g_, s_);
    launch_transpose(comp_, b_.zq, b_.zqt, g_, s_);
    launch_fwd_stats(comp_, b_.zq, b_.zq, b_.fwd_tiles, b_.n_fwd, b_.part, b_.sbuf, ws_, g_, s_);
    launch_lse(b_.part, b_.ypos, b_.lse2, b_.cpos, b_.block_loss, b_.loss, g_, s_);
  }
  void bwd() {
    launch_coef(comp_, b_.sbuf, b_.cbuf, b_.lse2, b_.cpos, b_.fwd_tiles, b_.n_fwd, g_, s_);
    launch_dz(comp_, b_.cbuf, b_.zqt, b_.dz_tiles, b_.n_dz, b_.slabs, ws_, g_, s_);
    launch_norm_bwd(in_, b_.slabs, b_.ksplit, b_.h, b_.inv, b_.grad_out, b_.dh, g_, s_);
  }

  // times `which` (0 fwd, 1 bwd, 2 fwd+bwd) with hipEvents; returns per-run ms
  std::vector<float> time(int which, int warmup, int iters) {
    hipEvent_t a, b;
    NTXENT_HIP_CHECK(hipEventCreate(&a));
    NTXENT_HIP_CHECK(hipEventCreate(&b));
    auto run = [&]() {
      if (which == 0) fwd();
      else if (which == 1) bwd();
      else { fwd(); bwd(); }
    };
    if (which == 1) fwd();
    for (int i = 0; i < warmup; ++i) run();
    std::vector<float> out;
    for (int i = 0; i < iters; ++i) {
      if (which == 1) fwd();  // the backward consumes forward state; untimed refresh
      NTXENT_HIP_CHECK(hipEventRecord(a, s_));
      run();
      NTXENT_HIP_CHECK(hipEventRecord(b, s_));
      NTXENT_HIP_CHECK(hipEventSynchronize(b));
      float ms = 0;
      NTXENT_HIP_CHECK(hipEventElapsedTime(&ms, a, b));
      out.push_back(ms);
    }
    hipEventDestroy(a);
    hipEventDestroy(b);
    return out;
  }

  float loss() {
    float l = 0;
    NTXENT_HIP_CHECK(hipStreamSynchronize(s_));
    NTXENT_HIP_CHECK(hipMemcpy(&l, b_.loss, 4, hipMemcpyDeviceToHost));
    return l;
  }

  // host fp64 NT-Xent of the same inputs (small shapes only)
  double host_loss() const {
    const int R = g_.rows, d = g_.dim, n = R / 2;
    std::vector<double> z((size_t)R * d);
    for (int i = 0; i < R; ++i) {
      double ss = 0;
      for (int e = 0; e < d; ++e) ss += (double)host_[(size_t)i * d + e] * host_[(size_t)i * d + e];
      const double iv = 1.0 / std::max(std::sqrt(ss), 1e-12);
      for (int e = 0; e < d; ++e) z[(size_t)i * d + e] = host_[(size_t)i * d + e] * iv;
    }
    double tot = 0;
    std::vector<double> row(R);
    for (int i = 0; i < R; ++i) {
      double mx = -1e300;
      for (int j = 0; j < R; ++j) {
        double s = 0;
        for (int e = 0; e < d; ++e) s += z[(size_t)i * d + e] * z[(size_t)j * d + e];
        row[j] = s / g_.temperature;
        if (j != i) mx = std::max(mx, row[j]);
      }
      double se = 0;
      for (int j = 0; j < R; ++j)
        if (j != i) se += std::exp(row[j] - mx);
      tot += mx + std::log(se) - row[(i + n) % R];
    }
    return tot / R;
  }

  const Geometry& geom() const { return g_; }
  int n_fwd() const { return b_.n_fwd; }

 private:
  DType in_, comp_;
  Geometry g_;
  Buffers b_;
  GemmWorkspace ws_;
  hipStream_t s_ = nullptr;
  std::vector<float> host_;
};

DType parse_dtype(const std::string& s) {
  if (s == "fp32") return DType::F32;
  if (s == "fp16") return DType::F16;
  return DType::BF16;
}

double fwd_flops(const Geometry& g) {
  const double R = g.rows, d = g.dim;
  return R * R * d;  // upper-triangular S (2 R^2 d / 2)
}
double bwd_flops(const Geometry& g) { return 2.0 * g.rows * (double)g.rows * g.dim; }

}  // namespace

int main(int argc, char** argv) {
  int batch = 0, dim = 0, iters = 100, warmup = 1;
  std::string dtype = "bf16", compute = "auto";
  float T = 0.07f;
  bool check = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() { return std::string(i + 1 < argc ? argv[++i] : ""); };
    if (a == "--batch") batch = std::stoi(next());
    else if (a == "--dim") dim = std::stoi(next());
    else if (a == "--iters") iters = std::stoi(next());
    else if (a == "--warmup") warmup = std::stoi(next());
    else if (a == "--dtype") dtype = next();
    else if (a == "--compute") compute = next();
    else if (a == "--temperature") T = std::stof(next());
    else if (a == "--check") check = true;
    else if (a == "-h" || a == "--help") {
      std::printf("usage: ntxent_bench [--batch B --dim D] [--dtype bf16|fp16|fp32] [--compute auto|fp16|bf16|fp32]\n"
                  "                    [--iters N] [--warmup W] [--temperature T] [--check]\n");
      return 0;
    }
  }
  int dev = 0;
  NTXENT_HIP_CHECK(hipSetDevice(dev));
  const DeviceInfo& di = device_info(dev);
  std::printf("Device: %s, %d CUs, matrix cores: %s\n", di.arch.c_str(), di.num_cus,
              check_matrix_core_support(dev) ? "yes (gfx950 MFMA)" : "no");
  const DType in = parse_dtype(dtype);
  const DType comp = compute == "auto" ? (in == DType::F32 ? DType::F32 : DType::F16) : parse_dtype(compute);

  std::vector<std::pair<int, int>> shapes;
  if (batch > 0) {
    shapes.push_back({batch, dim > 0 ? dim : 2048});
  } else {  // the reference sweep (src/benchmark.cpp:68-71)
    for (int b : {32, 64, 128, 256, 512, 1024})
      for (int d : {64, 128, 256}) shapes.push_back({b, d});
  }
  std::printf("%6s %6s %5s | %-38s | %-38s | %-38s | %12s %9s\n", "B", "D", "dtype",
              "fwd ms: mean / std / min / max", "bwd ms: mean / std / min / max",
              "fwd+bwd ms: mean / std / min / max", "samples/s", "TFLOP/s");
  for (auto [b, d] : shapes) {
    Bench bench(b, d, in, comp, T, di.num_cus);
    const Result f = stats(bench.time(0, warmup, iters));
    const Result bw = stats(bench.time(1, warmup, iters));
    const Result fb = stats(bench.time(2, warmup, iters));
    const double tf = (fwd_flops(bench.geom()) + bwd_flops(bench.geom())) / (fb.mean * 1e-3) / 1e12;
    std::printf("%6d %6d %5s | %8.4f %8.4f %8.4f %8.4f   | %8.4f %8.4f %8.4f %8.4f   | %8.4f %8.4f %8.4f %8.4f   | %12.1f %9.1f\n",
                b, d, dtype.c_str(), f.mean, f.stdev, f.mn, f.mx, bw.mean, bw.stdev, bw.mn, bw.mx, fb.mean,
                fb.stdev, fb.mn, fb.mx, b / (fb.mean * 1e-3), tf);
    if (check && b <= 1024 && d <= 512) {
      bench.fwd();
      const double ref = bench.host_loss();
      const double got = bench.loss();
      std::printf("       check: loss %.6f host-fp64 %.6f |diff| %.2e\n", got, ref, std::fabs(got - ref));
      if (std::fabs(got - ref) > 2e-2 * std::max(1.0, std::fabs(ref))) {
        std::fprintf(stderr, "loss mismatch\n");
        return 1;
      }
    }
  }
  return 0;
}

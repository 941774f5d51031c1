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
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <random>
#include <string>
#include <vector>

#include "ntxent/engine.h"

using namespace ntxent;

namespace {

uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFF + ((u >> 16) & 1);  // round to nearest even
  return (uint16_t)(u >> 16);
}

// IEEE binary16 conversions in plain C++ (round to nearest even; host compilers without
// _Float16 build this too).
uint16_t f32_to_f16(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const int32_t exp = (int32_t)((x >> 23) & 0xFF) - 127 + 15;
  uint32_t man = x & 0x7FFFFFu;
  if (((x >> 23) & 0xFF) == 0xFF) return (uint16_t)(sign | 0x7C00u | (man ? 0x200u : 0u));  // inf / nan
  if (exp >= 31) return (uint16_t)(sign | 0x7C00u);                                          // overflow
  if (exp <= 0) {                                                                            // subnormal / zero
    if (exp < -10) return (uint16_t)sign;
    man |= 0x800000u;
    const int shift = 14 - exp;
    uint32_t h = man >> shift;
    const uint32_t rem = man & ((1u << shift) - 1), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (h & 1u))) ++h;
    return (uint16_t)(sign | h);
  }
  uint32_t h = ((uint32_t)exp << 10) | (man >> 13);
  const uint32_t rem = man & 0x1FFFu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;  // may carry into the exponent: correct
  return (uint16_t)(sign | h);
}

float f16_to_f32(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1Fu, man = h & 0x3FFu, x;
  if (exp == 0) {
    if (man == 0) {
      x = sign;
    } else {  // normalise the subnormal
      exp = 1;
      while (!(man & 0x400u)) { man <<= 1; --exp; }
      man &= 0x3FFu;
      x = sign | ((exp + 127 - 15) << 23) | (man << 13);
    }
  } else if (exp == 31) {
    x = sign | 0x7F800000u | (man << 13);
  } else {
    x = sign | ((exp + 127 - 15) << 23) | (man << 13);
  }
  float f;
  std::memcpy(&f, &x, 4);
  return f;
}

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

// Synthetic two-view embeddings: view2 = shared basis + noise, like positives of a trained
// encoder, so the loss is well inside (0, log(2N-1)).
std::vector<float> synthetic_views(int rows, int dim, unsigned seed) {
  std::mt19937 rng(seed);
  std::normal_distribution<float> nd;
  std::vector<float> h((size_t)rows * dim);
  const size_t n = rows / 2;
  for (size_t i = 0; i < n; ++i)
    for (int e = 0; e < dim; ++e) {
      const float b = nd(rng);
      h[i * dim + e] = b + 0.5f * nd(rng);
      h[(i + n) * dim + e] = b + 0.5f * nd(rng);
    }
  return h;
}

// Uploads `host` in dtype `in`; rounds `host` to what the device sees.
void* upload(std::vector<float>& host, DType in) {
  void* d = nullptr;
  const size_t n = host.size();
  NTXENT_HIP_CHECK(hipMalloc(&d, n * dtype_size(in)));
  if (in == DType::F32) {
    NTXENT_HIP_CHECK(hipMemcpy(d, host.data(), n * 4, hipMemcpyHostToDevice));
    return d;
  }
  std::vector<uint16_t> h16(n);
  for (size_t k = 0; k < n; ++k) {
    h16[k] = in == DType::BF16 ? f32_to_bf16(host[k]) : f32_to_f16(host[k]);
    if (in == DType::BF16) {
      uint32_t u = (uint32_t)h16[k] << 16;
      std::memcpy(&host[k], &u, 4);
    } else {
      host[k] = f16_to_f32(h16[k]);
    }
  }
  NTXENT_HIP_CHECK(hipMemcpy(d, h16.data(), n * 2, hipMemcpyHostToDevice));
  return d;
}


class Bench {
 public:
  Bench(int batch, int dim, DType in, DType comp, float T, bool keep_cos, Comm* comm, unsigned seed,
        bool small_path = true, int small_splits = 0, Negatives neg = Negatives::kSymmetric)
      : in_(in) {
    EngineConfig c;
    c.negatives = neg;
    c.rows = 2 * batch;
    c.dim = dim;
    c.temperature = T;
    c.input = in;
    c.compute = comp;
    c.keep_cos = keep_cos;
    c.small_path = small_path;
    c.small_splits = small_splits;
    host_ = synthetic_views(c.rows, dim, seed);
    h_ = upload(host_, in);
    NTXENT_HIP_CHECK(hipMalloc(&dh_, host_.size() * dtype_size(in)));
    NTXENT_HIP_CHECK(hipStreamCreateWithFlags(&s_, hipStreamNonBlocking));
    e_ = std::make_unique<Engine>(c, comm);
  }
  ~Bench() {
    e_.reset();
    hipFree(h_);
    hipFree(dh_);
    hipStreamDestroy(s_);
  }

  void fwd() { e_->forward(h_, s_); }
  void bwd() { e_->backward(nullptr, dh_, s_); }
  // Bit pattern checksum of dh after one fwd + bwd (FNV-1a over the raw bytes) plus its L1 norm:
  // two builds whose kernels differ only in data layout or prefetching must print the same hash.
  std::pair<unsigned long long, double> grad_digest() {
    fwd();
    bwd();
    NTXENT_HIP_CHECK(hipStreamSynchronize(s_));
    const size_t n = host_.size(), es = dtype_size(in_);
    std::vector<unsigned char> raw(n * es);
    NTXENT_HIP_CHECK(hipMemcpy(raw.data(), dh_, raw.size(), hipMemcpyDeviceToHost));
    unsigned long long hsh = 1469598103934665603ull;
    for (unsigned char c : raw) hsh = (hsh ^ c) * 1099511628211ull;
    double l1 = 0.0;
    for (size_t i = 0; i < n; ++i) {
      float v;
      if (es == 4) std::memcpy(&v, &raw[4 * i], 4);
      else {
        unsigned short u;
        std::memcpy(&u, &raw[2 * i], 2);
        if (in_ == DType::BF16) {
          const unsigned w = (unsigned)u << 16;
          std::memcpy(&v, &w, 4);
        } else {
          v = (float)*reinterpret_cast<const _Float16*>(&u);
        }
      }
      l1 += std::fabs((double)v);
    }
    return {hsh, l1};
  }

  // times `which` (0 fwd, 1 bwd, 2 fwd+bwd, 3 fwd+bwd as one hipGraph) with hipEvents
  std::vector<float> time(int which, int warmup, int iters) {
    hipEvent_t a, b;
    NTXENT_HIP_CHECK(hipEventCreate(&a));
    NTXENT_HIP_CHECK(hipEventCreate(&b));
    if (which == 3 && !e_->captured()) e_->capture(h_, dh_, s_);
    auto run = [&]() {
      if (which == 0) fwd();
      else if (which == 1) bwd();
      else if (which == 2) { fwd(); bwd(); }
      else e_->replay(s_);
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

  float loss() { return e_->loss(s_); }

  // host fp64 NT-Xent of the same inputs (small shapes, world 1 only)
  double host_loss() const {
    const Geometry& g = e_->geometry();
    const int R = g.rows, d = g.dim, n = R / 2;
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
        row[j] = s / g.temperature;
        if (j != i) mx = std::max(mx, row[j]);
      }
      double se = 0;
      for (int j = 0; j < R; ++j)
        if (j != i) se += std::exp(row[j] - mx);
      tot += mx + std::log(se) - row[(i + n) % R];
    }
    return tot / R;
  }

  const Geometry& geom() const { return e_->geometry(); }
  const Engine& engine() const { return *e_; }

 private:
  DType in_;
  std::vector<float> host_;
  void* h_ = nullptr;
  void* dh_ = nullptr;
  hipStream_t s_ = nullptr;
  std::unique_ptr<Engine> e_;
};

DType parse_dtype(const std::string& s) {
  if (s == "fp32") return DType::F32;
  if (s == "fp16") return DType::F16;
  if (s == "fp8") return DType::FP8;
  return DType::BF16;
}

// Useful MFMA FLOPs of one rank's fwd+bwd: upper-triangular own block + remote blocks (fwd),
// full dZ GEMM over all global columns (bwd).
double step_flops(const Geometry& g) {
  const double R = g.rows, d = g.dim, RG = (double)g.global_rows;
  return R * R * d + 2.0 * R * (RG - R) * d + 2.0 * R * RG * d;
}

struct Options {
  int batch = 0, dim = 0, iters = 100, warmup = 1, gpus = 1;
  std::string dtype = "bf16", compute = "auto", json;
  float T = 0.07f;
  bool check = false, graph = false, recompute = false, small = true, grad_digest = false;
  int small_splits = 0;
  Negatives negatives = Negatives::kSymmetric;
  bool emulate = false;  // --gpus N as N emulated ranks on GPU 0 (ThreadComm), not N GPUs over RCCL
  // one rank per PROCESS (--proc-rank r of --gpus N): the RCCL unique id goes through uid_file;
  // --shared-gpu puts every rank on GPU 0 (launch each with its own NCCL_HOSTID: RCCL then
  // connects them over its socket transport, tools/cpp_rccl_procs.py)
  int proc_rank = -1;
  std::string uid_file;
  bool shared_gpu = false;
};

// Minimal reusable thread barrier (C++17).
class ThreadBarrier {
 public:
  explicit ThreadBarrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> l(m_);
    const int gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
    } else {
      cv_.wait(l, [&] { return gen != gen_; });
    }
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  int n_, count_ = 0, gen_ = 0;
};

// Data-parallel run: one thread per GPU, one RCCL communicator per thread (no MPI needed);
// every rank holds `batch` pairs, negatives are global. Reports the slowest rank.
int run_multi(const Options& o, DType in, DType comp) {
  const int N = o.gpus;
  const std::string uid = o.emulate ? std::string() : RcclComm::unique_id();
  auto group = o.emulate ? make_thread_comm_group(N) : nullptr;
  ThreadBarrier bar(N);
  std::vector<double> mean_ms(N, 0.0);
  std::vector<std::string> errs(N);
  double flops = 0;
  float loss = 0;
  std::vector<std::thread> th;
  for (int r = 0; r < N; ++r) {
    th.emplace_back([&, r] {
      try {
        NTXENT_HIP_CHECK(hipSetDevice(o.emulate ? 0 : r));
        std::unique_ptr<Comm> comm;
        if (o.emulate) comm = std::make_unique<ThreadComm>(group, r);
        else comm = std::make_unique<RcclComm>(r, N, uid, r);
        Bench bench(o.batch, o.dim, in, comp, o.T, !o.recompute, comm.get(), 1234 + r, true, 0, o.negatives);
        bar.wait();
        const Result fb = stats(bench.time(o.graph ? 3 : 2, o.warmup, o.iters));
        mean_ms[r] = fb.mean;
        if (r == 0) { flops = step_flops(bench.geom()); loss = bench.loss(); }
        bar.wait();
      } catch (const std::exception& e) {
        errs[r] = e.what();
      }
    });
  }
  for (auto& t : th) t.join();
  for (int r = 0; r < N; ++r)
    if (!errs[r].empty()) { std::fprintf(stderr, "rank %d: %s\n", r, errs[r].c_str()); return 1; }
  const double ms = *std::max_element(mean_ms.begin(), mean_ms.end());
  std::printf("%s=%d B/rank=%d D=%d %s %s: fwd+bwd %.4f ms (slowest rank), %.1f samples/s total, "
              "%.1f TFLOP/s/rank, loss %.6f\n", o.emulate ? "emulated ranks" : "gpus", N, o.batch, o.dim, o.dtype.c_str(),
              o.negatives == Negatives::kSymmetric ? "symmetric" : "allgather", ms,
              (double)N * o.batch / (ms * 1e-3), flops / (ms * 1e-3) / 1e12, loss);
  return 0;
}

// One rank of a multi-process data-parallel run (the native counterpart of the torchrun path):
// rank 0 publishes the RCCL unique id through a file (written, then renamed), the others wait
// for it. Each rank prints its loss and mean fwd+bwd time; the launcher compares the ranks' loss
// with the --emulate run of the same seeds.
int run_proc(const Options& o, DType in, DType comp) {
  const int N = o.gpus, r = o.proc_rank;
  NTXENT_CHECK(r >= 0 && r < N && !o.uid_file.empty(), "--proc-rank needs 0 <= r < --gpus and --uid-file");
  std::string uid;
  if (r == 0) {
    uid = RcclComm::unique_id();
    const std::string tmp = o.uid_file + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    NTXENT_CHECK(f && std::fwrite(uid.data(), 1, uid.size(), f) == uid.size(), "cannot write the uid file");
    std::fclose(f);
    NTXENT_CHECK(std::rename(tmp.c_str(), o.uid_file.c_str()) == 0, "cannot publish the uid file");
  } else {
    for (int t = 0; t < 1200 && uid.size() != RcclComm::kIdBytes; ++t) {
      if (FILE* f = std::fopen(o.uid_file.c_str(), "rb")) {
        char b[RcclComm::kIdBytes];
        if (std::fread(b, 1, sizeof(b), f) == sizeof(b)) uid.assign(b, sizeof(b));
        std::fclose(f);
      }
      if (uid.size() != RcclComm::kIdBytes) std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    NTXENT_CHECK(uid.size() == RcclComm::kIdBytes, "timed out waiting for the uid file");
  }
  RcclComm comm(r, N, uid, o.shared_gpu ? 0 : r);
  Bench bench(o.batch, o.dim, in, comp, o.T, !o.recompute, &comm, 1234 + r, true, 0, o.negatives);
  const Result fb = stats(bench.time(o.graph ? 3 : 2, o.warmup, o.iters));
  std::printf("proc rank %d/%d B/rank=%d D=%d %s %s: fwd+bwd %.4f ms, loss %.6f\n", r, N, o.batch, o.dim,
              o.dtype.c_str(), o.negatives == Negatives::kSymmetric ? "symmetric" : "allgather", fb.mean,
              bench.loss());
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  Options o;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() { return std::string(i + 1 < argc ? argv[++i] : ""); };
    if (a == "--batch") o.batch = std::stoi(next());
    else if (a == "--dim") o.dim = std::stoi(next());
    else if (a == "--iters") o.iters = std::stoi(next());
    else if (a == "--warmup") o.warmup = std::stoi(next());
    else if (a == "--dtype") o.dtype = next();
    else if (a == "--compute") o.compute = next();
    else if (a == "--temperature") o.T = std::stof(next());
    else if (a == "--gpus") o.gpus = std::stoi(next());
    else if (a == "--json") o.json = next();
    else if (a == "--check") o.check = true;
    else if (a == "--grad-digest") o.grad_digest = true;
    else if (a == "--graph") o.graph = true;
    else if (a == "--recompute") o.recompute = true;
    else if (a == "--no-small") o.small = false;
    else if (a == "--fp8-bwd") ntxent::set_fp8_backward(true);
    else if (a == "--no-fp8-bwd") ntxent::set_fp8_backward(false);
    else if (a == "--no-raw-fwd") ntxent::set_raw_forward(false);
    else if (a == "--small-splits") o.small_splits = std::stoi(next());
    else if (a == "--negatives") {
      const std::string v = next();
      NTXENT_CHECK(v == "symmetric" || v == "allgather", "--negatives symmetric|allgather");
      o.negatives = v == "symmetric" ? Negatives::kSymmetric : Negatives::kAllGather;
    }
    else if (a == "--emulate") o.emulate = true;
    else if (a == "--proc-rank") o.proc_rank = std::stoi(next());
    else if (a == "--uid-file") o.uid_file = next();
    else if (a == "--shared-gpu") o.shared_gpu = true;
    else if (a == "--small-fuse-rows") ntxent::set_small_fuse_rows(std::stoi(next()));
    else if (a == "-h" || a == "--help") {
      std::printf("usage: ntxent_bench [--batch B --dim D] [--dtype bf16|fp16|fp32] [--compute auto|fp16|bf16|fp32|fp8]\n"
                  "                    [--iters N] [--warmup W] [--temperature T] [--check] [--graph]\n"
                  "                    [--recompute] [--no-small] [--gpus N] [--json out.json]\n"
                  "  --no-small: large-problem pipeline for every shape (no one-launch small path)\n"
                  "  --gpus N [--negatives symmetric|allgather] [--emulate]: data parallel over N GPUs (RCCL),\n"
                  "           or N emulated ranks on GPU 0 (in-process ThreadComm, --emulate)\n"
                  "  --gpus N --proc-rank r --uid-file F [--shared-gpu]: rank r of N processes over RCCL\n"
                  "  --fp8-bwd / --no-fp8-bwd: with --compute fp8, the backward's C and Z^T in e4m3 too (or fp16)\n"
                  "  --no-raw-fwd: unit-row (zq) forward operands instead of the input rows normalised in the epilogue\n"
                  "  --small-fuse-rows R: small forward with the row prologue fused up to R rows (0: prep launch)\n"
                  "  --grad-digest: print a hash of dh after one step (build variants must match bitwise)\n"
                  "  (the measured A/B alternatives of earlier rounds are deleted; build-time variants:\n"
                  "   tools/build_variant.sh)\n");
      return 0;
    }
  }
  int dev = 0;
  NTXENT_HIP_CHECK(hipSetDevice(dev));
  const DeviceInfo& di = device_info(dev);
  std::printf("Device: %s, %d CUs, matrix cores: %s\n", di.arch.c_str(), di.num_cus,
              check_matrix_core_support(dev) ? "yes (gfx950 MFMA)" : "no");
  const DType in = parse_dtype(o.dtype);
  const DType comp = o.compute == "auto" ? (in == DType::F32 ? DType::F32 : DType::F16) : parse_dtype(o.compute);
  if (o.gpus > 1) {
    if (o.batch <= 0) o.batch = 4096;
    if (o.dim <= 0) o.dim = 2048;
    if (o.proc_rank >= 0) return run_proc(o, in, comp);
    return run_multi(o, in, comp);
  }

  std::vector<std::pair<int, int>> shapes;
  if (o.batch > 0) {
    shapes.push_back({o.batch, o.dim > 0 ? o.dim : 2048});
  } else {  // the reference sweep (src/benchmark.cpp:68-71)
    for (int b : {32, 64, 128, 256, 512, 1024})
      for (int d : {64, 128, 256}) shapes.push_back({b, d});
  }
  std::printf("%6s %6s %5s %5s | %-38s | %-38s | %-38s | %-10s | %12s %9s\n", "B", "D", "dtype", "path",
              "fwd ms: mean / std / min / max", "bwd ms: mean / std / min / max",
              "fwd+bwd ms: mean / std / min / max", "graph ms", "samples/s", "TFLOP/s");
  FILE* jf = o.json.empty() ? nullptr : std::fopen(o.json.c_str(), "w");
  if (jf) std::fprintf(jf, "{\"device\": \"%s\", \"results\": {", di.arch.c_str());
  bool first = true;
  for (auto [b, d] : shapes) {
    Bench bench(b, d, in, comp, o.T, !o.recompute, nullptr, 1234, o.small, o.small_splits);
    const char* path = bench.engine().small() ? "small" : "large";
    const Result f = stats(bench.time(0, o.warmup, o.iters));
    const Result bw = stats(bench.time(1, o.warmup, o.iters));
    const Result fb = stats(bench.time(2, o.warmup, o.iters));
    const Result gr = o.graph ? stats(bench.time(3, o.warmup, o.iters)) : Result{};
    const double best = o.graph ? std::min(gr.mean, fb.mean) : fb.mean;
    const double tf = step_flops(bench.geom()) / (best * 1e-3) / 1e12;
    std::printf("%6d %6d %5s %5s | %8.4f %8.4f %8.4f %8.4f   | %8.4f %8.4f %8.4f %8.4f   | %8.4f %8.4f %8.4f %8.4f   | %10.4f | %12.1f %9.1f\n",
                b, d, o.dtype.c_str(), path, f.mean, f.stdev, f.mn, f.mx, bw.mean, bw.stdev, bw.mn, bw.mx, fb.mean,
                fb.stdev, fb.mn, fb.mx, gr.mean, b / (best * 1e-3), tf);
    if (jf) {
      std::fprintf(jf, "%s\n  \"B=%d,d=%d,dtype=%s,world=1\": {\"path\": \"%s\", \"fwd_ms\": [%.5f, %.5f, %.5f, %.5f], "
                   "\"bwd_ms\": [%.5f, %.5f, %.5f, %.5f], \"fwd_bwd_ms\": [%.5f, %.5f, %.5f, %.5f], "
                   "\"graph_ms\": %.5f, \"samples_per_s\": %.1f, \"tflops\": %.2f, \"device_bytes\": %zu}",
                   first ? "" : ",", b, d, o.dtype.c_str(), path, f.mean, f.stdev, f.mn, f.mx, bw.mean, bw.stdev, bw.mn,
                   bw.mx, fb.mean, fb.stdev, fb.mn, fb.mx, gr.mean, b / (best * 1e-3), tf,
                   bench.engine().device_bytes());
      first = false;
    }
    if (o.grad_digest) {
      const auto gd = bench.grad_digest();
      std::printf("       grad digest: %016llx l1 %.9e loss %.6f\n", gd.first, gd.second, bench.loss());
    }
    if (o.check && b <= 1024 && d <= 512) {
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
  if (jf) {
    std::fprintf(jf, "\n}}\n");
    std::fclose(jf);
  }
  return 0;
}

// ntxent_tests — C++ tests of the native runtime (ntxent::Engine) on a gfx950 GPU.
//
// Covers the reference GTest intents (tests/test_forward.cpp:19-52: BasicForward,
// GradientCheck, DifferentBatchSizes; tests/test_backward.cpp:19-49: BasicBackward,
// GradientNorm) but with value checks: every loss and gradient is compared against a host
// fp64 evaluation of the same formulas, not just "not NaN". GTest is not
// installed on this image, so this is a small self-registering runner (ctest runs it).
//
//   ntxent_tests            # all tests
//   ntxent_tests Gradient   # tests whose name contains "Gradient"
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "ntxent/comm.h"
#include "ntxent/engine.h"
#include "ntxent/trace.h"

using namespace ntxent;

namespace {

struct TestCase {
  std::string name;
  std::function<void()> fn;
};
std::vector<TestCase>& registry() {
  static std::vector<TestCase> r;
  return r;
}
struct Reg {
  Reg(const char* n, std::function<void()> f) { registry().push_back({n, std::move(f)}); }
};
#define NT_TEST(name)                          \
  void name();                                 \
  const Reg reg_##name(#name, name);           \
  void name()

struct Failure : std::runtime_error {
  using std::runtime_error::runtime_error;
};
#define EXPECT(cond, ...)                                                              \
  do {                                                                                 \
    if (!(cond)) {                                                                     \
      char _b[512];                                                                    \
      std::snprintf(_b, sizeof(_b), __VA_ARGS__);                                      \
      throw Failure(std::string(__FILE__) + ":" + std::to_string(__LINE__) + ": " + _b); \
    }                                                                                  \
  } while (0)

// ---- host helpers -------------------------------------------------------------------------
uint16_t to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFF + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
float from_bf16(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

// Random embeddings (tests/test_utils.hpp:7-15 generate_random_embeddings analogue, seeded).
std::vector<float> embeddings(int rows, int dim, unsigned seed, float scale = 1.0f) {
  std::mt19937 rng(seed);
  std::normal_distribution<float> nd;
  std::vector<float> h((size_t)rows * dim);
  for (auto& x : h) x = scale * nd(rng);
  return h;
}

// Host fp64 oracle: loss and dL/dh (grad_out = go).
void oracle(const std::vector<float>& h, int R, int d, double T, double go, double& loss, std::vector<double>& dh) {
  const int n = R / 2;
  std::vector<double> z((size_t)R * d), inv(R);
  for (int i = 0; i < R; ++i) {
    double ss = 0;
    for (int e = 0; e < d; ++e) ss += (double)h[(size_t)i * d + e] * h[(size_t)i * d + e];
    inv[i] = 1.0 / std::max(std::sqrt(ss), 1e-12);
    for (int e = 0; e < d; ++e) z[(size_t)i * d + e] = h[(size_t)i * d + e] * inv[i];
  }
  std::vector<double> S((size_t)R * R), lse(R);
  loss = 0;
  for (int i = 0; i < R; ++i) {
    double mx = -1e300;
    for (int j = 0; j < R; ++j) {
      double s = 0;
      for (int e = 0; e < d; ++e) s += z[(size_t)i * d + e] * z[(size_t)j * d + e];
      S[(size_t)i * R + j] = s / T;
      if (j != i) mx = std::max(mx, s / T);
    }
    double se = 0;
    for (int j = 0; j < R; ++j)
      if (j != i) se += std::exp(S[(size_t)i * R + j] - mx);
    lse[i] = mx + std::log(se);
    loss += lse[i] - S[(size_t)i * R + (i + n) % R];
  }
  loss /= R;
  // C = P + P^T - 2 I_pos ; dz = C z * go / (R T) ; dh = inv (dz - z (z.dz))
  dh.assign((size_t)R * d, 0.0);
  std::vector<double> dz(d);
  for (int i = 0; i < R; ++i) {
    std::fill(dz.begin(), dz.end(), 0.0);
    for (int j = 0; j < R; ++j) {
      if (j == i) continue;
      double c = std::exp(S[(size_t)i * R + j] - lse[i]) + std::exp(S[(size_t)j * R + i] - lse[j]);
      if (j == (i + n) % R) c -= 2.0;
      for (int e = 0; e < d; ++e) dz[e] += c * z[(size_t)j * d + e];
    }
    double dot = 0;
    for (int e = 0; e < d; ++e) {
      dz[e] *= go / (R * T);
      dot += z[(size_t)i * d + e] * dz[e];
    }
    for (int e = 0; e < d; ++e) dh[(size_t)i * d + e] = inv[i] * (dz[e] - z[(size_t)i * d + e] * dot);
  }
}

// Data-parallel oracle: W ranks of R rows each (rank r's rows are global rows r*R .. r*R+R-1,
// its positives pair within the rank: i <-> i + R/2), negatives over all W*R rows; the loss is
// the global mean (what every rank's Engine reports) and dh the gradient of the global loss.
void oracle_dp(const std::vector<float>& h, int W, int R, int d, double T, double& loss, std::vector<double>& dh) {
  const int N = W * R, n = R / 2;
  auto pos = [&](int g) { return (g / R) * R + (g % R + n) % R; };
  std::vector<double> z((size_t)N * d), inv(N);
  for (int i = 0; i < N; ++i) {
    double ss = 0;
    for (int e = 0; e < d; ++e) ss += (double)h[(size_t)i * d + e] * h[(size_t)i * d + e];
    inv[i] = 1.0 / std::max(std::sqrt(ss), 1e-12);
    for (int e = 0; e < d; ++e) z[(size_t)i * d + e] = h[(size_t)i * d + e] * inv[i];
  }
  std::vector<double> S((size_t)N * N), lse(N);
  loss = 0;
  for (int i = 0; i < N; ++i) {
    double mx = -1e300;
    for (int j = 0; j < N; ++j) {
      double s = 0;
      for (int e = 0; e < d; ++e) s += z[(size_t)i * d + e] * z[(size_t)j * d + e];
      S[(size_t)i * N + j] = s / T;
      if (j != i) mx = std::max(mx, s / T);
    }
    double se = 0;
    for (int j = 0; j < N; ++j)
      if (j != i) se += std::exp(S[(size_t)i * N + j] - mx);
    lse[i] = mx + std::log(se);
    loss += lse[i] - S[(size_t)i * N + pos(i)];
  }
  loss /= N;
  dh.assign((size_t)N * d, 0.0);
  std::vector<double> dz(d);
  for (int i = 0; i < N; ++i) {
    std::fill(dz.begin(), dz.end(), 0.0);
    for (int j = 0; j < N; ++j) {
      if (j == i) continue;
      double c = std::exp(S[(size_t)i * N + j] - lse[i]) + std::exp(S[(size_t)j * N + i] - lse[j]);
      if (j == pos(i)) c -= 2.0;
      for (int e = 0; e < d; ++e) dz[e] += c * z[(size_t)j * d + e];
    }
    double dot = 0;
    for (int e = 0; e < d; ++e) {
      dz[e] /= N * T;
      dot += z[(size_t)i * d + e] * dz[e];
    }
    for (int e = 0; e < d; ++e) dh[(size_t)i * d + e] = inv[i] * (dz[e] - z[(size_t)i * d + e] * dot);
  }
}

// One engine run on device data; returns loss and dh (as float).
struct Run {
  float loss = 0;
  std::vector<float> dh;
};

class Harness {
 public:
  Harness(std::vector<float> h, int R, int d, DType in, DType comp, float T, bool keep = true, Comm* comm = nullptr,
          bool check_finite = false, Negatives neg = Negatives::kSymmetric)
      : host_(std::move(h)), R_(R), d_(d), in_(in) {
    EngineConfig c;
    c.negatives = neg;
    c.rows = R;
    c.dim = d;
    c.temperature = T;
    c.input = in;
    c.compute = comp;
    c.keep_cos = keep;
    c.check_finite = check_finite;
    const size_t n = host_.size(), es = dtype_size(in);
    NTXENT_HIP_CHECK(hipMalloc(&h_, n * es));
    NTXENT_HIP_CHECK(hipMalloc(&dh_, n * es));
    NTXENT_HIP_CHECK(hipMalloc(&go_, 4));
    if (in == DType::F32) {
      NTXENT_HIP_CHECK(hipMemcpy(h_, host_.data(), n * 4, hipMemcpyHostToDevice));
    } else {  // bf16 inputs; keep host_ equal to what the device sees
      std::vector<uint16_t> b(n);
      for (size_t k = 0; k < n; ++k) {
        b[k] = to_bf16(host_[k]);
        host_[k] = from_bf16(b[k]);
      }
      NTXENT_HIP_CHECK(hipMemcpy(h_, b.data(), n * 2, hipMemcpyHostToDevice));
    }
    NTXENT_HIP_CHECK(hipStreamCreateWithFlags(&s_, hipStreamNonBlocking));
    e_ = std::make_unique<Engine>(c, comm);
  }
  ~Harness() {
    e_.reset();
    hipFree(h_);
    hipFree(dh_);
    hipFree(go_);
    hipStreamDestroy(s_);
  }
  Run run(float grad_out = 1.0f, bool graph = false) {
    NTXENT_HIP_CHECK(hipMemcpyAsync(go_, &grad_out, 4, hipMemcpyHostToDevice, s_));
    if (graph) {
      if (!e_->captured()) e_->capture(h_, dh_, s_);
      e_->replay(s_);
    } else {
      e_->forward(h_, s_);
      e_->backward(grad_out == 1.0f ? nullptr : go_, dh_, s_);
    }
    Run r;
    r.loss = e_->loss(s_);
    const size_t n = host_.size();
    r.dh.resize(n);
    if (in_ == DType::F32) {
      NTXENT_HIP_CHECK(hipMemcpy(r.dh.data(), dh_, n * 4, hipMemcpyDeviceToHost));
    } else {
      std::vector<uint16_t> b(n);
      NTXENT_HIP_CHECK(hipMemcpy(b.data(), dh_, n * 2, hipMemcpyDeviceToHost));
      for (size_t k = 0; k < n; ++k) r.dh[k] = from_bf16(b[k]);
    }
    return r;
  }
  const std::vector<float>& host() const { return host_; }
  Engine& engine() { return *e_; }
  hipStream_t stream() const { return s_; }

 private:
  std::vector<float> host_;
  int R_, d_;
  DType in_;
  void* h_ = nullptr;
  void* dh_ = nullptr;
  float* go_ = nullptr;
  hipStream_t s_ = nullptr;
  std::unique_ptr<Engine> e_;
};

double rel_l2(const std::vector<float>& a, const std::vector<double>& b) {
  double num = 0, den = 0;
  for (size_t k = 0; k < a.size(); ++k) {
    num += (a[k] - b[k]) * (a[k] - b[k]);
    den += b[k] * b[k];
  }
  return std::sqrt(num / std::max(den, 1e-300));
}

double l2(const std::vector<float>& a) {
  double s = 0;
  for (float x : a) s += (double)x * x;
  return std::sqrt(s);
}

// Fixture of the reference tests: T = 0.07, B = 32, D = 128 (tests/test_forward.cpp:13-16).
constexpr float kT = 0.07f;
constexpr int kB = 32, kD = 128;

void check_case(int B, int D, DType in, DType comp, float T, double loss_tol, double grad_tol, unsigned seed) {
  const int R = 2 * B;
  Harness hs(embeddings(R, D, seed), R, D, in, comp, T);
  const Run r = hs.run();
  double lref;
  std::vector<double> gref;
  oracle(hs.host(), R, D, T, 1.0, lref, gref);
  EXPECT(std::isfinite(r.loss), "loss not finite");
  EXPECT(std::fabs(r.loss - lref) <= loss_tol * std::max(1.0, std::fabs(lref)), "B=%d D=%d loss %.7f ref %.7f", B, D,
         r.loss, lref);
  const double gr = rel_l2(r.dh, gref);
  EXPECT(gr <= grad_tol, "B=%d D=%d grad rel err %.3e > %.1e", B, D, gr, grad_tol);
}

// ---- tests -------------------------------------------------------------------------------
NT_TEST(BasicForward) {
  Harness hs(embeddings(2 * kB, kD, 1), 2 * kB, kD, DType::BF16, DType::F16, kT);
  const Run r = hs.run();
  EXPECT(r.loss > 0.f && std::isfinite(r.loss), "loss %f", r.loss);
  double lref;
  std::vector<double> g;
  oracle(hs.host(), 2 * kB, kD, kT, 1.0, lref, g);
  EXPECT(std::fabs(r.loss - lref) < 5e-3 * lref, "loss %.6f vs oracle %.6f", r.loss, lref);
}

NT_TEST(GradientCheck) {
  check_case(kB, kD, DType::F32, DType::F32, kT, 1e-5, 1e-4, 2);   // exact fp32 path
  check_case(kB, kD, DType::BF16, DType::F16, kT, 5e-3, 2e-2, 3);  // fp16 MFMA
  check_case(kB, kD, DType::BF16, DType::BF16, kT, 1e-2, 5e-2, 4); // bf16 MFMA
}

NT_TEST(DifferentBatchSizes) {
  for (int B : {16, 32, 64, 128, 17, 300}) check_case(B, kD, DType::F32, DType::F32, kT, 1e-5, 1e-4, 10 + B);
}

NT_TEST(OddShapes) {
  check_case(17, 100, DType::F32, DType::F32, 0.2f, 1e-5, 1e-4, 21);
  check_case(3, 7, DType::F32, DType::F32, 0.5f, 1e-5, 1e-4, 22);
  check_case(129, 520, DType::BF16, DType::F16, kT, 5e-3, 2e-2, 23);
}

NT_TEST(BasicBackward) {
  Harness hs(embeddings(2 * kB, kD, 5), 2 * kB, kD, DType::BF16, DType::F16, kT);
  const Run r = hs.run();
  for (float x : r.dh) EXPECT(std::isfinite(x), "non-finite gradient");
}

NT_TEST(GradientNorm) {
  Harness hs(embeddings(2 * kB, kD, 6), 2 * kB, kD, DType::F32, DType::F32, kT);
  const Run r = hs.run();
  const double n = l2(r.dh);
  EXPECT(n > 0.0 && n < 100.0, "grad norm %f", n);  // tests/test_backward.cpp:46-48
  double lref;
  std::vector<double> g;
  oracle(hs.host(), 2 * kB, kD, kT, 1.0, lref, g);
  double gn = 0;
  for (double x : g) gn += x * x;
  EXPECT(std::fabs(n - std::sqrt(gn)) < 1e-4 * std::sqrt(gn), "norm %.6e vs %.6e", n, std::sqrt(gn));
}

NT_TEST(GradOutScaling) {
  Harness hs(embeddings(64, 64, 7), 64, 64, DType::F32, DType::F32, kT);
  const Run a = hs.run(1.0f);
  const Run b = hs.run(-2.5f);
  for (size_t k = 0; k < a.dh.size(); ++k)
    EXPECT(std::fabs(b.dh[k] + 2.5f * a.dh[k]) <= 1e-5f * (1.0f + std::fabs(a.dh[k])), "scaling at %zu", k);
}

NT_TEST(StabilityGrid) {  // python/test.py:57-79: scales x temperatures, finite and correct
  for (float scale : {1e-5f, 1.0f, 1e5f})
    for (float T : {0.01f, 0.07f, 1.0f}) {
      Harness hs(embeddings(256, 256, 8, scale), 256, 256, DType::F32, DType::F32, T);
      const Run r = hs.run();
      double lref;
      std::vector<double> g;
      oracle(hs.host(), 256, 256, T, 1.0, lref, g);
      EXPECT(std::isfinite(r.loss) && std::fabs(r.loss - lref) < 1e-4 * std::max(1.0, lref), "scale %g T %g loss %f ref %f",
             scale, T, r.loss, lref);
      EXPECT(rel_l2(r.dh, g) < 1e-3, "scale %g T %g grad err %.3e", scale, T, rel_l2(r.dh, g));
    }
}

NT_TEST(Determinism) {
  Harness hs(embeddings(1024, 256, 9), 1024, 256, DType::BF16, DType::F16, kT);
  const Run a = hs.run(), b = hs.run();
  EXPECT(a.loss == b.loss, "loss differs");
  EXPECT(std::memcmp(a.dh.data(), b.dh.data(), a.dh.size() * 4) == 0, "gradients differ bitwise");
}

NT_TEST(GraphReplayMatchesEager) {
  Harness hs(embeddings(1024, 512, 10), 1024, 512, DType::BF16, DType::F16, kT);
  const Run eager = hs.run();
  const Run g1 = hs.run(1.0f, true);
  const Run g2 = hs.run(1.0f, true);
  EXPECT(eager.loss == g1.loss && g1.loss == g2.loss, "graph loss differs");
  EXPECT(std::memcmp(eager.dh.data(), g2.dh.data(), eager.dh.size() * 4) == 0, "graph gradients differ");
}

NT_TEST(RecomputeMatchesStore) {
  auto h = embeddings(600, 200, 11);
  Harness a(h, 600, 200, DType::F32, DType::F32, kT, true);
  Harness b(h, 600, 200, DType::F32, DType::F32, kT, false);
  const Run ra = a.run(), rb = b.run();
  EXPECT(ra.loss == rb.loss, "loss differs");
  double num = 0, den = 0;
  for (size_t k = 0; k < ra.dh.size(); ++k) {
    num += (ra.dh[k] - rb.dh[k]) * (ra.dh[k] - rb.dh[k]);
    den += (double)ra.dh[k] * ra.dh[k];
  }
  EXPECT(std::sqrt(num / den) < 1e-5, "store vs recompute %.3e", std::sqrt(num / den));
}

NT_TEST(LocalCommWorldOne) {
  auto h = embeddings(512, 128, 12);
  LocalComm lc;
  Harness a(h, 512, 128, DType::BF16, DType::F16, kT);
  Harness b(h, 512, 128, DType::BF16, DType::F16, kT, true, &lc);
  const Run ra = a.run(), rb = b.run();
  EXPECT(ra.loss == rb.loss && std::memcmp(ra.dh.data(), rb.dh.data(), ra.dh.size() * 4) == 0, "LocalComm differs");
}

NT_TEST(RcclCommWorldOne) {
  const std::string id = RcclComm::unique_id();
  EXPECT(id.size() == RcclComm::kIdBytes, "uid size");
  RcclComm comm(0, 1, id, 0);
  auto h = embeddings(512, 128, 13);
  Harness a(h, 512, 128, DType::BF16, DType::F16, kT);
  Harness b(h, 512, 128, DType::BF16, DType::F16, kT, true, &comm);
  const Run ra = a.run(), rb = b.run();
  EXPECT(ra.loss == rb.loss, "RCCL world-1 loss differs");
  comm.check();
}

// Comm extensions at world 1 (the multi-rank behaviour runs on the driver's 8-GPU node): the
// reduce-scatter, the grouped point-to-point batch (self-exchange) and the chunked all-gather
// with per-chunk events, for both the local and the RCCL communicator.
static void comm_primitives(Comm& c, const char* name) {
  hipStream_t s;
  NTXENT_HIP_CHECK(hipStreamCreate(&s));
  const size_t n = 1000, bytes = 3000 * 4 + 44;  // not a multiple of the 256-byte chunk unit
  std::vector<float> hs(n);
  for (size_t i = 0; i < n; ++i) hs[i] = 0.5f * (float)i - 7.f;
  float *a = nullptr, *b = nullptr;
  char *src = nullptr, *dst = nullptr;
  NTXENT_HIP_CHECK(hipMalloc(&a, n * 4));
  NTXENT_HIP_CHECK(hipMalloc(&b, n * 4));
  NTXENT_HIP_CHECK(hipMalloc(&src, bytes));
  NTXENT_HIP_CHECK(hipMalloc(&dst, bytes));
  NTXENT_HIP_CHECK(hipMemcpy(a, hs.data(), n * 4, hipMemcpyHostToDevice));
  c.reduce_scatter_sum(a, b, n, s);
  std::vector<float> out(n);
  NTXENT_HIP_CHECK(hipMemcpyAsync(out.data(), b, n * 4, hipMemcpyDeviceToHost, s));
  NTXENT_HIP_CHECK(hipStreamSynchronize(s));
  EXPECT(out == hs, "%s: reduce_scatter_sum at world 1 is not the identity", name);
  // grouped self send/recv
  NTXENT_HIP_CHECK(hipMemsetAsync(b, 0, n * 4, s));
  c.send_recv({P2POp{true, a, n * 4, 0}, P2POp{false, b, n * 4, 0}}, s);
  NTXENT_HIP_CHECK(hipMemcpyAsync(out.data(), b, n * 4, hipMemcpyDeviceToHost, s));
  NTXENT_HIP_CHECK(hipStreamSynchronize(s));
  EXPECT(out == hs, "%s: send_recv self-exchange", name);
  // chunked all-gather, out of place and in place, with per-chunk events
  std::vector<unsigned char> hb(bytes), ob(bytes);
  for (size_t i = 0; i < bytes; ++i) hb[i] = (unsigned char)(i * 7 + 3);
  NTXENT_HIP_CHECK(hipMemcpy(src, hb.data(), bytes, hipMemcpyHostToDevice));
  hipEvent_t ev[3];
  for (auto& e : ev) NTXENT_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  NTXENT_HIP_CHECK(hipMemsetAsync(dst, 0, bytes, s));
  c.all_gather_chunks(src, dst, bytes, 3, s, ev);
  NTXENT_HIP_CHECK(hipEventSynchronize(ev[2]));
  NTXENT_HIP_CHECK(hipMemcpy(ob.data(), dst, bytes, hipMemcpyDeviceToHost));
  EXPECT(ob == hb, "%s: all_gather_chunks out of place", name);
  c.all_gather_chunks(dst, dst, bytes, 5, s);
  NTXENT_HIP_CHECK(hipStreamSynchronize(s));
  NTXENT_HIP_CHECK(hipMemcpy(ob.data(), dst, bytes, hipMemcpyDeviceToHost));
  EXPECT(ob == hb, "%s: all_gather_chunks in place", name);
  for (auto& e : ev) NTXENT_HIP_CHECK(hipEventDestroy(e));
  NTXENT_HIP_CHECK(hipFree(a));
  NTXENT_HIP_CHECK(hipFree(b));
  NTXENT_HIP_CHECK(hipFree(src));
  NTXENT_HIP_CHECK(hipFree(dst));
  NTXENT_HIP_CHECK(hipStreamDestroy(s));
}

NT_TEST(LocalCommPrimitives) {
  LocalComm lc;
  comm_primitives(lc, "LocalComm");
}

NT_TEST(RcclCommPrimitivesWorldOne) {
  RcclComm comm(0, 1, RcclComm::unique_id(), 0);
  comm_primitives(comm, "RcclComm");
  comm.check();
}

// The multi-rank Engine paths (all-gather and symmetric negatives) on ONE GPU: W emulated ranks,
// one host thread each, over the in-process ThreadComm (RCCL refuses two ranks on a device);
// every rank's loss and gradient against the data-parallel fp64 oracle.
static void multi_rank_case(int W, int R, int d, DType comp, Negatives neg, double loss_tol, double grad_tol) {
  const auto h = embeddings(W * R, d, 100 + W * 7 + (int)neg);
  auto group = make_thread_comm_group(W);
  std::vector<std::unique_ptr<ThreadComm>> comms;
  for (int r = 0; r < W; ++r) comms.push_back(std::make_unique<ThreadComm>(group, r));
  std::vector<std::unique_ptr<Harness>> hs(W);
  for (int r = 0; r < W; ++r)
    hs[r] = std::make_unique<Harness>(std::vector<float>(h.begin() + (size_t)r * R * d, h.begin() + (size_t)(r + 1) * R * d),
                                      R, d, comp == DType::F32 ? DType::F32 : DType::BF16, comp, kT, true,
                                      comms[r].get(), false, neg);
  EXPECT(W == 1 || hs[0]->engine().symmetric() == (neg == Negatives::kSymmetric), "mode not selected");
  std::vector<Run> runs(W);
  std::vector<std::string> errs(W);
  std::vector<std::thread> th;
  for (int r = 0; r < W; ++r)
    th.emplace_back([&, r] {
      try {
        NTXENT_HIP_CHECK(hipSetDevice(0));
        for (int it = 0; it < 2; ++it) runs[r] = hs[r]->run();  // twice: reusable events / buffers
      } catch (const std::exception& e) {
        errs[r] = e.what();
      }
    });
  for (auto& t : th) t.join();
  for (int r = 0; r < W; ++r) EXPECT(errs[r].empty(), "rank %d: %s", r, errs[r].c_str());
  std::vector<float> host;
  for (int r = 0; r < W; ++r) host.insert(host.end(), hs[r]->host().begin(), hs[r]->host().end());
  double lref;
  std::vector<double> gref;
  oracle_dp(host, W, R, d, kT, lref, gref);
  std::vector<float> dh;
  for (int r = 0; r < W; ++r) {
    EXPECT(std::fabs(runs[r].loss - lref) <= loss_tol * std::fabs(lref), "W=%d rank %d loss %.7f ref %.7f", W, r,
           runs[r].loss, lref);
    dh.insert(dh.end(), runs[r].dh.begin(), runs[r].dh.end());
  }
  const double gr = rel_l2(dh, gref);
  EXPECT(gr <= grad_tol, "W=%d %s grad rel err %.3e > %.1e", W, neg == Negatives::kSymmetric ? "symmetric" : "allgather",
         gr, grad_tol);
  std::printf("         W=%d %-9s loss %.6f (oracle %.6f) grad rel err %.2e\n", W,
              neg == Negatives::kSymmetric ? "symmetric" : "allgather", runs[0].loss, lref, gr);
}

NT_TEST(ThreadCommPrimitives) {  // world 1 semantics of the in-process communicator
  auto g = make_thread_comm_group(1);
  ThreadComm c(g, 0);
  comm_primitives(c, "ThreadComm");
}

NT_TEST(MultiRankSymmetric) {
  // W = 8: the driver's scaling-run world size (3 full partner blocks + a split pair per rank)
  for (int W : {2, 3, 4, 8}) multi_rank_case(W, 512, 128, DType::F16, Negatives::kSymmetric, 2e-3, 2e-2);
}

NT_TEST(MultiRankAllGather) {
  for (int W : {2, 3, 8}) multi_rank_case(W, 512, 128, DType::F16, Negatives::kAllGather, 2e-3, 2e-2);
}

NT_TEST(MultiRankSymmetricFp32) {  // fp32 contributions on the wire, one slab stack
  multi_rank_case(3, 512, 96, DType::F32, Negatives::kSymmetric, 1e-5, 1e-4);
}

NT_TEST(FaultInjection) {
  Harness hs(embeddings(128, 64, 14), 128, 64, DType::F32, DType::F32, kT, true, nullptr, /*check_finite=*/true);
  set_fault_sites("dz");
  bool threw = false;
  try {
    hs.run();
  } catch (const InjectedFault&) {
    threw = true;
  }
  set_fault_sites("");
  EXPECT(threw, "injected dz fault did not surface");
  NTXENT_HIP_CHECK(hipStreamSynchronize(hs.stream()));
  set_fault_sites("nonfinite");
  threw = false;
  try {
    hs.run();
  } catch (const std::runtime_error& e) {
    threw = std::string(e.what()).find("non-finite") != std::string::npos;
  }
  set_fault_sites("");
  EXPECT(threw, "non-finite loss not detected");
  const Run ok = hs.run();  // engine still usable after the failures
  EXPECT(std::isfinite(ok.loss), "engine unusable after fault");
}

NT_TEST(BadInputsRejected) {
  bool threw = false;
  try {
    EngineConfig c;
    c.rows = 7;
    c.dim = 16;
    Engine e(c);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  EXPECT(threw, "odd row count accepted");
}

}  // namespace

int main(int argc, char** argv) {
  const std::string filter = argc > 1 ? argv[1] : "";
  int dev_count = 0;
  if (hipGetDeviceCount(&dev_count) != hipSuccess || dev_count == 0) {
    std::printf("no GPU: skipping %zu tests\n", registry().size());
    return 0;
  }
  int pass = 0, fail = 0;
  for (const auto& t : registry()) {
    if (!filter.empty() && t.name.find(filter) == std::string::npos) continue;
    try {
      t.fn();
      std::printf("[ PASS ] %s\n", t.name.c_str());
      ++pass;
    } catch (const std::exception& e) {
      std::printf("[ FAIL ] %s: %s\n", t.name.c_str(), e.what());
      ++fail;
    }
    std::fflush(stdout);
  }
  std::printf("%d passed, %d failed\n", pass, fail);
  return fail ? 1 : 0;
}

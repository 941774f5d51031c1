// gfx950 (CDNA4) kernels of the NT-Xent loss. Written for MI355X directly: wave64, MFMA
// 16x16x32 (f16/bf16) or 16x16x4 (exact f32) tiles, LDS staged by global_load_lds with an
// XOR swizzle, XCD-aware tile order, fused reductions. See include/ntxent/ntxent.h for the
// data layout and SURVEY.md §2.2 for the math.
//
// Parity map to the reference (what each kernel replaces):
//   prep_kernel        -> at::cat({z,z}) + (missing) normalisation   src/ntxent_kernel.cu:161
//   sim_gemm<FWD>      -> cublasSgemm logits + row_max_kernel + softmax_kernel
//                         src/ntxent_kernel.cu:8-103,165-192 (never materialises logits)
//   lse_kernel         -> compute_loss_kernel                         src/ntxent_kernel.cu:105-134
//   coef_kernel        -> grad_logits.diagonal() = ...               src/ntxent_kernel.cu:218-221
//   sim_gemm<DZ>       -> cublasSgemm backward                        src/ntxent_kernel.cu:228-236
//   norm_bwd_kernel    -> (missing) normalisation backward + grad_out scaling

#include "../include/ntxent/ntxent.h"
#include "device_common.h"
#include "sim_gemm.h"

#include <atomic>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>
#include <unordered_map>

namespace ntxent {
namespace dev {

// ------------------------------------------------------------------------------------
// Row prologue: one 256-thread block per positive pair (i, i+n).
// ------------------------------------------------------------------------------------
template <typename T> __device__ __forceinline__ void load8(const T* p, float (&v)[8]);
template <> __device__ __forceinline__ void load8<float>(const float* p, float (&v)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}
template <typename T> __device__ __forceinline__ void load8_h(const T* p, float (&v)[8]) {
  union { uint4 u; T h[8]; } pk;
  pk.u = *reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = to_f32<T>(pk.h[j]);
}
template <> __device__ __forceinline__ void load8<_Float16>(const _Float16* p, float (&v)[8]) { load8_h(p, v); }
template <> __device__ __forceinline__ void load8<__bf16>(const __bf16* p, float (&v)[8]) { load8_h(p, v); }

template <typename T> __device__ __forceinline__ void store8(T* p, const float (&v)[8], float (&q)[8]) {
  if constexpr (sizeof(T) == 2) {
    union { uint4 u; T h[8]; } pk;
#pragma unroll
    for (int j = 0; j < 8; ++j) { pk.h[j] = from_f32<T>(v[j]); q[j] = to_f32<T>(pk.h[j]); }
    *reinterpret_cast<uint4*>(p) = pk.u;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) q[j] = v[j];
    *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
}

// store8 into base[off .. off + 7], 16-bit rows write-through (sc1; base uniform: one buffer
// resource, per-lane offsets): prep -1 us at every BASELINE shape (profiles/r4/variants_r4_v9_wt.md)
template <typename T> __device__ __forceinline__ void store8_at(T* base, long long off, const float (&v)[8], float (&q)[8]) {
  if constexpr (sizeof(T) == 2) {
    union { u32x4 u; T h[8]; } pk;
#pragma unroll
    for (int j = 0; j < 8; ++j) { pk.h[j] = from_f32<T>(v[j]); q[j] = to_f32<T>(pk.h[j]); }
    store16_wt(base, off * 2, pk.u);
  } else {
    store8<T>(base + off, v, q);
  }
}

// fp8 e4m3 of 8 values (x * sc, sc = 2^e the row's scale), packed little-endian into 2 dwords;
// q receives the dequantised values (what the fp8 GEMM multiplies), divided back by sc.
__device__ __forceinline__ u32x2 quant8(const float (&x)[8], float (&q)[8], float sc) {
  u32x2 r;
  const float isc = 1.0f / sc;  // exact: sc is a power of two
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    int v = 0;
    v = __builtin_amdgcn_cvt_pk_fp8_f32(x[4 * h] * sc, x[4 * h + 1] * sc, v, false);
    v = __builtin_amdgcn_cvt_pk_fp8_f32(x[4 * h + 2] * sc, x[4 * h + 3] * sc, v, true);
    r[h] = (unsigned)v;
    q[4 * h + 0] = __builtin_amdgcn_cvt_f32_fp8(v, 0) * isc;
    q[4 * h + 1] = __builtin_amdgcn_cvt_f32_fp8(v, 1) * isc;
    q[4 * h + 2] = __builtin_amdgcn_cvt_f32_fp8(v, 2) * isc;
    q[4 * h + 3] = __builtin_amdgcn_cvt_f32_fp8(v, 3) * isc;
  }
  return r;
}

// Zero one pad row of zq ([ldk] elements) and, for fp8 plans, of zq8 ([ldk8] bytes) with
// 16-byte stores by `nt` cooperating threads.
template <typename Tc, bool Q8>
__device__ __forceinline__ void zero_pad_row(Tc* zq, unsigned char* zq8, int row, int ldk, int ldk8, int t, int nt) {
  const u32x4 z = {0u, 0u, 0u, 0u};
  char* r = reinterpret_cast<char*>(zq + (long long)row * ldk);
  for (int b = t * 16; b < ldk * (int)sizeof(Tc); b += nt * 16) *reinterpret_cast<u32x4*>(r + b) = z;
  if constexpr (Q8) {
    unsigned char* r8 = zq8 + (long long)row * ldk8;
    for (int b = t * 16; b < ldk8; b += nt * 16) *reinterpret_cast<u32x4*>(r8 + b) = z;
  }
}

// Q8: also write the fp8 copy zq8 (row stride ldk8 bytes, zero padded to dk8) used by the fp8
// forward GEMM; the positive logit then comes from the dequantised fp8 rows, consistent with
// the GEMM's logits.
template <typename Tin, typename Tc, bool Q8>
__global__ __launch_bounds__(256) void prep_kernel(const Tin* __restrict__ h, Tc* __restrict__ zq,
                                                   float* __restrict__ inv, float* __restrict__ ypos,
                                                   int R, int d, int dk, int ldk, float y_scale,
                                                   unsigned char* __restrict__ zq8, int dk8, int ldk8) {
  __shared__ float red[16];
  const int n = R >> 1, i = blockIdx.x, pi = i + n;
  if (i >= n) {  // pad row R + (i - n) of zq (and zq8): zeros (replaces a memset launch)
    zero_pad_row<Tc, Q8>(zq, zq8, R + (i - n), ldk, ldk8, threadIdx.x, 256);
    return;
  }
  const Tin* hi = h + (long long)i * d;
  const Tin* hp = h + (long long)pi * d;
  Tc* zi = zq + (long long)i * ldk;
  Tc* zp = zq + (long long)pi * ldk;
  const bool vec = (d % 8) == 0;
  float ssi = 0.f, ssp = 0.f, mxi = 0.f, mxp = 0.f;  // sums of squares, max |h| (fp8 row scales)
  if (vec) {
    for (int e = threadIdx.x * 8; e < d; e += 256 * 8) {
      float a[8], b[8];
      load8<Tin>(hi + e, a);
      load8<Tin>(hp + e, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ssi += a[j] * a[j]; ssp += b[j] * b[j];
        mxi = fmaxf(mxi, fabsf(a[j])); mxp = fmaxf(mxp, fabsf(b[j]));
      }
    }
  } else {
    for (int e = threadIdx.x; e < d; e += 256) {
      const float a = to_f32<Tin>(hi[e]), b = to_f32<Tin>(hp[e]);
      ssi += a * a; ssp += b * b;
      mxi = fmaxf(mxi, fabsf(a)); mxp = fmaxf(mxp, fabsf(b));
    }
  }
  ssi = block_sum(ssi, red);
  ssp = block_sum(ssp, red + 8);
  const float ivi = 1.0f / fmaxf(sqrtf(ssi), 1e-12f);
  const float ivp = 1.0f / fmaxf(sqrtf(ssp), 1e-12f);
  // fp8: per-row power-of-two scale from the row's amax (amax of z = amax of h * inv exactly)
  int ei = 0, ep = 0;
  if constexpr (Q8) {
    ei = fp8_row_exp(block_max(mxi, red) * ivi);
    ep = fp8_row_exp(block_max(mxp, red + 8) * ivp);
  }
  const float sci = __int_as_float((ei + 127) << 23), scp = __int_as_float((ep + 127) << 23);
  float dot = 0.f;
  unsigned char* zi8 = Q8 ? zq8 + (long long)i * ldk8 : nullptr;
  unsigned char* zp8 = Q8 ? zq8 + (long long)pi * ldk8 : nullptr;
  if (vec) {
    for (int e = threadIdx.x * 8; e < d; e += 256 * 8) {
      float a[8], b[8], qa[8], qb[8];
      load8<Tin>(hi + e, a);
      load8<Tin>(hp + e, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[j] *= ivi; b[j] *= ivp; }
      store8<Tc>(zi + e, a, qa);
      store8<Tc>(zp + e, b, qb);
      if constexpr (Q8) {
        *reinterpret_cast<u32x2*>(zi8 + e) = quant8(a, qa, sci);
        *reinterpret_cast<u32x2*>(zp8 + e) = quant8(b, qb, scp);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) dot += qa[j] * qb[j];
    }
  } else {
    for (int e = threadIdx.x; e < d; e += 256) {
      const float af = to_f32<Tin>(hi[e]) * ivi, bf = to_f32<Tin>(hp[e]) * ivp;
      const Tc a = from_f32<Tc>(af);
      const Tc b = from_f32<Tc>(bf);
      zi[e] = a; zp[e] = b;
      if constexpr (Q8) {
        const int va = __builtin_amdgcn_cvt_pk_fp8_f32(af * sci, 0.f, 0, false);
        const int vb = __builtin_amdgcn_cvt_pk_fp8_f32(bf * scp, 0.f, 0, false);
        zi8[e] = (unsigned char)(va & 0xFF);
        zp8[e] = (unsigned char)(vb & 0xFF);
        dot += (__builtin_amdgcn_cvt_f32_fp8(va, 0) / sci) * (__builtin_amdgcn_cvt_f32_fp8(vb, 0) / scp);
      } else {
        dot += to_f32<Tc>(a) * to_f32<Tc>(b);
      }
    }
  }
  for (int e = d + threadIdx.x; e < dk; e += 256) { zi[e] = from_f32<Tc>(0.f); zp[e] = from_f32<Tc>(0.f); }
  if constexpr (Q8) {
    for (int e = d + threadIdx.x; e < dk8; e += 256) { zi8[e] = 0; zp8[e] = 0; }
    if (threadIdx.x == 0) {  // E8M0 scale byte right after the row's K range (see Geometry::ld_k8)
      zi8[dk8] = (unsigned char)(127 - ei);
      zp8[dk8] = (unsigned char)(127 - ep);
    }
  }
  dot = block_sum(dot, red);
  if (threadIdx.x == 0) {
    inv[i] = ivi; inv[pi] = ivp;
    ypos[i] = dot * y_scale; ypos[pi] = dot * y_scale;
  }
}

// Wave-per-pair prologue for d % 8 == 0, d <= 512 * NCH: each lane keeps its NCH chunks of 8
// features of both rows in registers between the norm and the normalise pass (h is read once)
// and every reduction is a wave reduction (no LDS, no block barrier); 4 pairs per block.
// ST (statistics only, the raw-operand forward): inv and ypos from the input rows in fp32, no zq
// (ypos = (h_i . h_p) inv_i inv_p, unrounded; no pad blocks).
template <typename Tin, typename Tc, bool Q8, int NCH, bool ST = false>
__global__ __launch_bounds__(256) void prep_wave_kernel(const Tin* __restrict__ h, Tc* __restrict__ zq,
                                                        float* __restrict__ inv, float* __restrict__ ypos,
                                                        int R, int d, int dk, int ldk, float y_scale,
                                                        unsigned char* __restrict__ zq8, int dk8, int ldk8,
                                                        int pad_end) {
  const int lane = threadIdx.x & 63;
  const int n = R >> 1;
  const int npb = (n + 3) >> 2;  // pair blocks; the blocks after them zero the pad rows
  if ((int)blockIdx.x >= npb) {
    const int row = R + ((int)blockIdx.x - npb) * 4 + (threadIdx.x >> 6);
    if (row < pad_end) zero_pad_row<Tc, Q8>(zq, zq8, row, ldk, ldk8, lane, 64);
    return;
  }
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;  // whole wave
  const int pi = i + n;
  const Tin* hi = h + (long long)i * d;
  const Tin* hp = h + (long long)pi * d;
  Tc* zi = zq + (long long)i * ldk;
  Tc* zp = zq + (long long)pi * ldk;
  float a[NCH][8], b[NCH][8];
  float ssi = 0.f, ssp = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = (c * 64 + lane) * 8;
    if (e < d) {
      load8<Tin>(hi + e, a[c]);
      load8<Tin>(hp + e, b[c]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[c][j] = 0.f; b[c][j] = 0.f; }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) { ssi += a[c][j] * a[c][j]; ssp += b[c][j] * b[c][j]; }
  }
  float hd = 0.f;  // statistics only: the pair's dot joins the two norms' reductions
  if constexpr (ST) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) hd += a[c][j] * b[c][j];
    hd = wave_sum(hd);
  }
  ssi = wave_sum(ssi);
  ssp = wave_sum(ssp);
  const float ivi = 1.0f / fmaxf(sqrtf(ssi), 1e-12f);
  const float ivp = 1.0f / fmaxf(sqrtf(ssp), 1e-12f);
  if constexpr (ST) {
    if (lane == 0) {
      inv[i] = ivi; inv[pi] = ivp;
      ypos[i] = hd * ivi * ivp * y_scale; ypos[pi] = ypos[i];
    }
    return;
  }
  // fp8: per-row power-of-two scale from the row's amax (amax of z = amax of h * inv exactly)
  int ei = 0, ep = 0;
  if constexpr (Q8) {
    float mxi = 0.f, mxp = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) { mxi = fmaxf(mxi, fabsf(a[c][j])); mxp = fmaxf(mxp, fabsf(b[c][j])); }
    ei = fp8_row_exp(xrow_max(row16_max(mxi)) * ivi);
    ep = fp8_row_exp(xrow_max(row16_max(mxp)) * ivp);
  }
  const float sci = __int_as_float((ei + 127) << 23), scp = __int_as_float((ep + 127) << 23);
  float dot = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = (c * 64 + lane) * 8;
    if (e < d) {
      float qa[8], qb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[c][j] *= ivi; b[c][j] *= ivp; }
      store8_at<Tc>(zq, (long long)i * ldk + e, a[c], qa);
      store8_at<Tc>(zq, (long long)pi * ldk + e, b[c], qb);
      if constexpr (Q8) {
        *reinterpret_cast<u32x2*>(zq8 + (long long)i * ldk8 + e) = quant8(a[c], qa, sci);
        *reinterpret_cast<u32x2*>(zq8 + (long long)pi * ldk8 + e) = quant8(b[c], qb, scp);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) dot += qa[j] * qb[j];
    }
  }
  for (int e = d + lane; e < dk; e += 64) { zi[e] = from_f32<Tc>(0.f); zp[e] = from_f32<Tc>(0.f); }
  if constexpr (Q8) {
    for (int e = d + lane; e < dk8; e += 64) { zq8[(long long)i * ldk8 + e] = 0; zq8[(long long)pi * ldk8 + e] = 0; }
    if (lane == 0) {  // E8M0 scale byte right after the row's K range (see Geometry::ld_k8)
      zq8[(long long)i * ldk8 + dk8] = (unsigned char)(127 - ei);
      zq8[(long long)pi * ldk8 + dk8] = (unsigned char)(127 - ep);
    }
  }
  dot = wave_sum(dot);
  if (lane == 0) {
    inv[i] = ivi; inv[pi] = ivp;
    ypos[i] = dot * y_scale; ypos[pi] = dot * y_scale;
  }
}

// Block-per-pair prologue for 2048 < d <= 2048 * NCH (d % 8 == 0): as prep_wave_kernel with 256
// threads per pair, each thread keeping its NCH chunks of 8 features of both rows in registers,
// so h is read once (the generic prep_kernel reads it twice: 1.5x the HBM traffic at d = 8192).
template <typename Tin, typename Tc, bool Q8, int NCH, bool ST = false>
__global__ __launch_bounds__(256) void prep_block_kernel(const Tin* __restrict__ h, Tc* __restrict__ zq,
                                                         float* __restrict__ inv, float* __restrict__ ypos,
                                                         int R, int d, int dk, int ldk, float y_scale,
                                                         unsigned char* __restrict__ zq8, int dk8, int ldk8) {
  __shared__ float red[24];
  const int t = threadIdx.x;
  const int n = R >> 1, i = blockIdx.x, pi = i + n;
  if (i >= n) {  // pad row R + (i - n) of zq (and zq8): zeros
    zero_pad_row<Tc, Q8>(zq, zq8, R + (i - n), ldk, ldk8, t, 256);
    return;
  }
  const Tin* hi = h + (long long)i * d;
  const Tin* hp = h + (long long)pi * d;
  Tc* zi = zq + (long long)i * ldk;
  Tc* zp = zq + (long long)pi * ldk;
  float a[NCH][8], b[NCH][8];
  float ssi = 0.f, ssp = 0.f, mxi = 0.f, mxp = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = (c * 256 + t) * 8;
    if (e < d) {
      load8<Tin>(hi + e, a[c]);
      load8<Tin>(hp + e, b[c]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[c][j] = 0.f; b[c][j] = 0.f; }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ssi += a[c][j] * a[c][j]; ssp += b[c][j] * b[c][j];
      if constexpr (Q8) { mxi = fmaxf(mxi, fabsf(a[c][j])); mxp = fmaxf(mxp, fabsf(b[c][j])); }
    }
  }
  if constexpr (ST) {  // statistics only (see prep_wave_kernel): one reduction of the three sums
    float hd = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) hd += a[c][j] * b[c][j];
    block_sum3(ssi, ssp, hd, red);
    const float ivi = 1.0f / fmaxf(sqrtf(ssi), 1e-12f);
    const float ivp = 1.0f / fmaxf(sqrtf(ssp), 1e-12f);
    if (t == 0) {
      inv[i] = ivi; inv[pi] = ivp;
      ypos[i] = hd * ivi * ivp * y_scale; ypos[pi] = ypos[i];
    }
    return;
  }
  ssi = block_sum(ssi, red);
  ssp = block_sum(ssp, red + 8);
  const float ivi = 1.0f / fmaxf(sqrtf(ssi), 1e-12f);
  const float ivp = 1.0f / fmaxf(sqrtf(ssp), 1e-12f);
  int ei = 0, ep = 0;
  if constexpr (Q8) {
    ei = fp8_row_exp(block_max(mxi, red) * ivi);
    ep = fp8_row_exp(block_max(mxp, red + 8) * ivp);
  }
  const float sci = __int_as_float((ei + 127) << 23), scp = __int_as_float((ep + 127) << 23);
  float dot = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = (c * 256 + t) * 8;
    if (e < d) {
      float qa[8], qb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[c][j] *= ivi; b[c][j] *= ivp; }
      store8_at<Tc>(zq, (long long)i * ldk + e, a[c], qa);
      store8_at<Tc>(zq, (long long)pi * ldk + e, b[c], qb);
      if constexpr (Q8) {
        *reinterpret_cast<u32x2*>(zq8 + (long long)i * ldk8 + e) = quant8(a[c], qa, sci);
        *reinterpret_cast<u32x2*>(zq8 + (long long)pi * ldk8 + e) = quant8(b[c], qb, scp);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) dot += qa[j] * qb[j];
    }
  }
  for (int e = d + t; e < dk; e += 256) { zi[e] = from_f32<Tc>(0.f); zp[e] = from_f32<Tc>(0.f); }
  if constexpr (Q8) {
    for (int e = d + t; e < dk8; e += 256) { zq8[(long long)i * ldk8 + e] = 0; zq8[(long long)pi * ldk8 + e] = 0; }
    if (t == 0) {  // E8M0 scale byte right after the row's K range (see Geometry::ld_k8)
      zq8[(long long)i * ldk8 + dk8] = (unsigned char)(127 - ei);
      zq8[(long long)pi * ldk8 + dk8] = (unsigned char)(127 - ep);
    }
  }
  dot = block_sum(dot, red);
  if (t == 0) {
    inv[i] = ivi; inv[pi] = ivp;
    ypos[i] = dot * y_scale; ypos[pi] = dot * y_scale;
  }
}

// 64x64 tile transpose with 16-byte global accesses on both sides (rows of Zq in, rows of
// ZqT out). LDS: 16-byte chunk c of row r sits at chunk c ^ ((r / V) % CPR), so the column
// gathers (V rows r = V jc + q of one column per lane group) hit distinct banks (the padded
// linear layout alone left them 4-way conflicted: 3.7M SQ_LDS_BANK_CONFLICT per launch at the
// headline, profiles/r2/pmc_final).
// Ts / inv (raw-operand forward): the source rows are the input h (2-byte Ts, same width as T),
// normalised here (z = h * inv[row]) on their way into the tile.
template <typename T, typename Ts = T>
__device__ __forceinline__ void transpose_tile(const Ts* __restrict__ zq, T* __restrict__ zqt, int dk, int ldk, int ldt,
                                               int bx, int by, T (&tile)[64][64 + 16 / sizeof(T)],
                                               const float* __restrict__ inv = nullptr) {
  constexpr int V = 16 / sizeof(T);  // elements per 16 B
  constexpr int CPR = 64 / V;        // 16-B chunks per 64-element row
  static_assert(sizeof(Ts) == sizeof(T), "transpose: source and destination element widths differ");
  const int j0 = bx * 64, e0 = by * 64;
  for (int k = threadIdx.x; k < 64 * CPR; k += 256) {
    const int r = k / CPR, c = k % CPR;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (e0 + c * V < dk) v = *reinterpret_cast<const u32x4*>(zq + (long long)(j0 + r) * ldk + e0 + c * V);
    if constexpr (!std::is_same<Ts, T>::value || sizeof(T) == 2) {
      if (inv) {  // (uniform) raw rows: normalise, convert
        const float s = inv[j0 + r];
        union { Ts h[V]; u32x4 u; } x;
        union { T h[V]; u32x4 u; } y;
        x.u = v;
#pragma unroll
        for (int q = 0; q < V; ++q) y.h[q] = from_f32<T>(to_f32<Ts>(x.h[q]) * s);
        v = y.u;
      }
    }
    *reinterpret_cast<u32x4*>(&tile[r][(c ^ ((r / V) % CPR)) * V]) = v;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 64 * CPR; k += 256) {
    const int er = k / CPR, jc = k % CPR;
    union { T h[V]; u32x4 u; } pk;
#pragma unroll
    for (int q = 0; q < V; ++q) pk.h[q] = tile[jc * V + q][((er / V) ^ (jc % CPR)) * V + er % V];
    store16_wt(zqt, ((long long)(e0 + er) * ldt + j0 + jc * V) * (long long)sizeof(T), pk.u);  // write-through
  }
}

// Z^T = (h inv)^T of the raw-operand forward as the diagonal remainder's side job (diag_up_kernel
// blocks [nup, grid)): 64x64 tiles strided over the side blocks, in 9 KiB of that kernel's LDS.
// (Pairs of tiles per iteration, all four 16-B loads of a thread in flight: the remainder's
// blocks slowed more, headline launch 18.4 -> 20.3 us: profiles/r5/zt_side/.)
template <typename T, typename Ts>
struct DiagSideZt {
  int nup;
  const Ts* h;
  T* zqt;
  const float* inv;
  int dk, ldt, tx, ntiles;
  __device__ void operator()(int b, int nb, char* smem) const {
    typedef T Tile[64][64 + 16 / sizeof(T)];
    static_assert(sizeof(Tile) <= kUpLds, "Z^T side job: tile exceeds the remainder's LDS");
    Tile& tile = *reinterpret_cast<Tile*>(smem);
    for (int t = b; t < ntiles; t += nb) {
      transpose_tile<T, Ts>(h, zqt, dk, dk, ldt, t % tx, t / tx, tile, inv);
      __syncthreads();  // every wave's gathers done before the next tile's rows land
    }
  }
};

// fp8 backward operand: e4m3(256 Z^T) ([dim_n][ldt] bytes) from the fp16 rows, same tiling (the
// gathered 8 elements go out as one 8-byte store). |z| <= 1, so 256 z stays below the e4m3 max.
__device__ __forceinline__ void transpose_tile_q8(const _Float16* __restrict__ zq, unsigned char* __restrict__ zqt,
                                                  int dk, int ldk, int ldt, int bx, int by, _Float16 (&tile)[64][72]) {
  constexpr int V = 8, CPR = 8;
  const int j0 = bx * 64, e0 = by * 64;
  for (int k = threadIdx.x; k < 64 * CPR; k += 256) {
    const int r = k / CPR, c = k % CPR;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (e0 + c * V < dk) v = *reinterpret_cast<const u32x4*>(zq + (long long)(j0 + r) * ldk + e0 + c * V);
    *reinterpret_cast<u32x4*>(&tile[r][(c ^ ((r / V) % CPR)) * V]) = v;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 64 * CPR; k += 256) {
    const int er = k / CPR, jc = k % CPR;
    float x[V];
#pragma unroll
    for (int q = 0; q < V; ++q) x[q] = 256.f * (float)tile[jc * V + q][((er / V) ^ (jc % CPR)) * V + er % V];
    u32x2 o;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int w = __builtin_amdgcn_cvt_pk_fp8_f32(x[4 * h], x[4 * h + 1], 0, false);
      w = __builtin_amdgcn_cvt_pk_fp8_f32(x[4 * h + 2], x[4 * h + 3], w, true);
      o[h] = (unsigned)w;
    }
    *reinterpret_cast<u32x2*>(zqt + (long long)(e0 + er) * ldt + j0 + jc * V) = o;
  }
}

// out[i] = sum_k in[k * count + i], k = 0 .. n-1 in order (deterministic reductions of the
// in-process communicator).
__global__ __launch_bounds__(256) void sum_slabs_kernel(const float* __restrict__ in, int n, size_t count,
                                                        float* __restrict__ out) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < count; i += (size_t)gridDim.x * 256) {
    float s = 0.f;
    for (int k = 0; k < n; ++k) s += in[(size_t)k * count + i];
    out[i] = s;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(const T* __restrict__ zq, T* __restrict__ zqt,
                                                        int dk, int ldk, int ldt) {
  __shared__ __attribute__((aligned(16))) T tile[64][64 + 16 / sizeof(T)];
  transpose_tile<T>(zq, zqt, dk, ldk, ldt, blockIdx.x, blockIdx.y, tile);
}


// Eight lanes per positive pair (i, i+n): lane q merges column tiles q, q+8, ... of both rows,
// an xor-shuffle tree merges the eight states, lane 0 finishes: LSE of both rows, their loss
// terms and the positive coefficient C_ip = P_ip + P_pi - 2 = -(a_i + a_p) (no 1 - P
// cancellation). Pad rows [R, Rpad) get zeros. One thread per pair left the chip ~94% idle
// (16 workgroups for B = 4096) and serialised 32-64 dependent merges per thread.
constexpr int kLseLanes = 8;
struct LseArgs {
  const float2* part;
  const float* ypos;
  float* lse2_all;
  float* cpos;
  float* block_loss;
  float* loss_sum;
  float loss_scale;
  int R, Rpad, Tc, own0;
  // fp8 backward (q8_row_exp): each row's negatives-only max logit and the global min LSE (log2
  // units); null otherwise
  float* mneg2;
  float* lmin;
  // > 0: the loss sum as one fixed-point ticket (lse_block), 2^F units per nat (lse_loss_fx)
  double loss_fx;
};
// Block `bid` of the nb LSE blocks (the last of them to finish sums the loss).
__device__ __forceinline__ void lse_block(const LseArgs& a, int bid, int nb, float* red, int& last) {
  const float2* __restrict__ part = a.part;
  const int R = a.R, Rpad = a.Rpad, Tc = a.Tc, own0 = a.own0;
  float* __restrict__ lse2_all = a.lse2_all;
  float* __restrict__ cpos = a.cpos;
  const int n = R >> 1;
  const int gt = bid * 256 + threadIdx.x;
  const int item = gt / kLseLanes, q = gt % kLseLanes;
  float li = 0.f, lmn = kPosInf;
  if (item < n) {  // uniform across the 8 lanes of an item
    const int i = item, j = item + n;
    float mi = kNegInf, si = 0.f, mj = kNegInf, sj = 0.f;
    // fp8 backward: a bound on each row's largest negative logit, max over the column tiles of
    // m + log2(s) (>= the tile's largest term, <= it + log2(256)). The merged m alone is no bound:
    // the fixed-shift forward epilogue reports m = M (the largest POSSIBLE logit) for every tile,
    // and a scale from it put the negatives' coefficients ~15 bits below their e4m3 range
    // (subnormal or zero: a 5e-2 gradient error, profiles/r5/fp8bwd_diag.log).
    float bi = kNegInf, bj = kNegInf;
    // 4 column tiles per lane per round, all loads issued before the (branchy) merges: one
    // memory round trip per 32 column tiles instead of one per tile
    for (int t0 = q; t0 < Tc; t0 += 4 * kLseLanes) {
      float2 vi[4], vj[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + u * kLseLanes;
        const int tc = t < Tc ? t : t0;  // clamped (no conditional loads); duplicates are skipped below
        vi[u] = part[(long long)tc * Rpad + i];
        vj[u] = part[(long long)tc * Rpad + j];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (t0 + u * kLseLanes < Tc) {
          lse_merge(mi, si, vi[u].x, vi[u].y);
          lse_merge(mj, sj, vj[u].x, vj[u].y);
          if (a.mneg2) {
            bi = fmaxf(bi, vi[u].y > 0.f ? vi[u].x + log2f(vi[u].y) : kNegInf);
            bj = fmaxf(bj, vj[u].y > 0.f ? vj[u].x + log2f(vj[u].y) : kNegInf);
          }
        }
    }
#pragma unroll
    for (int off = 1; off < kLseLanes; off <<= 1) {
      lse_merge(mi, si, __shfl_xor(mi, off), __shfl_xor(si, off));
      lse_merge(mj, sj, __shfl_xor(mj, off), __shfl_xor(sj, off));
      if (a.mneg2) {
        bi = fmaxf(bi, __shfl_xor(bi, off));
        bj = fmaxf(bj, __shfl_xor(bj, off));
      }
    }
    if (q == 0) {
      const float yp = a.ypos[i];
      float l_i, l_j, a_i, a_j;
      const float L2i = finish_row(mi, si, yp, l_i, a_i), L2j = finish_row(mj, sj, yp, l_j, a_j);
      lse2_all[own0 + i] = L2i;
      lse2_all[own0 + j] = L2j;
      cpos[i] = -(a_i + a_j);
      cpos[j] = -(a_i + a_j);
      li = l_i + l_j;
      lmn = fminf(L2i, L2j);
      if (a.mneg2) { a.mneg2[own0 + i] = bi; a.mneg2[own0 + j] = bj; }
    }
  } else if (item < Rpad - n && q == 0) {
    const int i = R + (item - n);
    lse2_all[own0 + i] = 0.f;
    cpos[i] = 0.f;
    if (a.mneg2) a.mneg2[own0 + i] = kNegInf;
  }
  const float tot = block_sum(li, red);
  const bool fx = a.loss_fx > 0.0;
  if (fx) {
    // One 64-bit ticket carries the arrival (bits 0-11), a non-finite partial (bits 12-23) and the
    // partial in fixed point (bits 24-63, loss_fx units: launch_lse sizes it so the whole sum fits
    // 40 bits). Integer adds commute, so the sum is deterministic whoever arrives last, and the
    // partial needs no store + drain + reload around the ticket (two memory round trips fewer on
    // the launch's critical path than the float form below).
    if (threadIdx.x == 0) {
      unsigned long long* tk = reinterpret_cast<unsigned long long*>(a.block_loss + 2);
      const bool fin = tot >= 0.f && tot < 3.0e38f;
      const unsigned long long q = fin ? (unsigned long long)llrint((double)tot * a.loss_fx) : 0ull;
      const unsigned long long add = (q << 24) | (fin ? 1ull : (1ull << 12) | 1ull);
      const unsigned long long old = __hip_atomic_fetch_add(tk, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((int)(old & 0xFFF) == nb - 1) {
        __hip_atomic_store(tk, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long all = old + add;
        a.loss_sum[0] = ((all >> 12) & 0xFFF) ? __builtin_nanf("")
                                               : (float)((double)(all >> 24) / a.loss_fx * (double)a.loss_scale);
      }
    }
    if (!a.lmin) return;  // (fp8 backward: the LSE minimum still takes the partials below)
  }
  const float bmin = a.lmin ? -block_max(-lmn, red) : 0.f;
  // Last-block-done final sum (replaces a separate one-thread launch): publish this block's
  // partial, count arrivals; the last block adds all partials in block order (deterministic)
  // and returns the counter (a fixed slot ahead of the partials) to zero. The partial is a
  // write-through (sc1) 4-byte store and the last block reads the partials with sc1 loads,
  // so no agent release/acquire is needed (MI355X_MICROARCH.md § visibility, Valid forms
  // row 1); a release fence here wrote back every dirty L2 line the forward GEMM left behind.
  int* cnt = reinterpret_cast<int*>(a.block_loss);  // fixed slot 0: the counter
  float* partial = a.block_loss + 64;               // per-block partials after it
  float* pmin = partial + nb;                       // per-block LSE minima (fp8 backward)
  if (threadIdx.x == 0) {
    __hip_atomic_store(partial + bid, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a.lmin) __hip_atomic_store(pmin + bid, bmin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == nb - 1;
    if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (last && threadIdx.x < 64) {
    float s = 0.f;
    for (int b = threadIdx.x; b < nb; b += 64)
      s += __hip_atomic_load(partial + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s = wave_sum(s);  // fixed lane assignment and tree: deterministic
    if (threadIdx.x == 0 && !fx) a.loss_sum[0] = s * a.loss_scale;
    if (a.lmin) {
      float m = kPosInf;
      for (int b = threadIdx.x; b < nb; b += 64)
        m = fminf(m, __hip_atomic_load(pmin + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      m = -xrow_max(row16_max(-m));
      if (threadIdx.x == 0) a.lmin[0] = m;
    }
  }
}

__global__ __launch_bounds__(256) void lse_kernel(const LseArgs a) {
  __shared__ float red[16];
  __shared__ int last;
  lse_block(a, blockIdx.x, gridDim.x, red, last);
}

// The LSE merge and the Z -> Z^T transpose (the dZ GEMM's B operand) in one launch: blocks
// [0, nb) merge, the rest transpose one 64x64 tile each. The merge is latency-bound on few
// blocks and the transpose is bandwidth-bound on many, so they share the chip instead of
// running back to back, and no side stream / event join (a ~5-7 us bubble each) is needed.
// Q8: the transpose writes the fp8 backward's e4m3(256 Z^T) (T = _Float16 rows in).
template <typename T, bool Q8 = false, typename Ts = T>
__global__ __launch_bounds__(256) void lse_transpose_kernel(const LseArgs a, int nb, const Ts* __restrict__ zq,
                                                            void* __restrict__ zqt, int dk, int ldk, int ldt, int tx,
                                                            const float* __restrict__ inv = nullptr) {
  __shared__ __attribute__((aligned(16))) T tile[64][64 + 16 / sizeof(T)];
  __shared__ float red[16];
  __shared__ int last;
  if ((int)blockIdx.x < nb) {
    lse_block(a, blockIdx.x, nb, red, last);
  } else {
    const int t = blockIdx.x - nb;
    if constexpr (Q8)
      transpose_tile_q8(zq, static_cast<unsigned char*>(zqt), dk, ldk, ldt, t % tx, t / tx, tile);
    else
      transpose_tile<T, Ts>(zq, static_cast<T*>(zqt), dk, ldk, ldt, t % tx, t / tx, tile, inv);
  }
}

// Vectorised normalisation backward: one 256-thread block per row; each thread owns NCH
// chunks of 8 contiguous features, kept in registers between the dot pass and the output.
// xs: nx extra fp16 slabs (received partner contributions, symmetric data-parallel mode) added
// to the fp32 sum.
template <typename Tin, int NCH>
__global__ __launch_bounds__(256) void norm_bwd_vec_kernel(const float* __restrict__ slabs, int nslabs,
                                                           long long slab_stride, long long ldo,
                                                           const Tin* __restrict__ h, const float* __restrict__ inv,
                                                           const float* __restrict__ grad_out, float alpha_base,
                                                           Tin* __restrict__ dh, int d, const _Float16* __restrict__ xs,
                                                           int nx) {
  __shared__ float red[16];
  const int i = blockIdx.x;
  const float iv = inv[i];
  const float alpha = grad_out[0] * alpha_base;
  const Tin* hi = h + (long long)i * d;
  const float* gi = slabs + (long long)i * ldo;
  float g[NCH][8], z[NCH][8];
  float dot = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = (c * 256 + threadIdx.x) * 8;
    if (e < d) {
      load8<Tin>(hi + e, z[c]);
      f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = {0.f, 0.f, 0.f, 0.f};
      if (nslabs > 0) {  // nslabs = 0: fp16 slabs only (xs)
        a = *reinterpret_cast<const f32x4*>(gi + e);
        b = *reinterpret_cast<const f32x4*>(gi + e + 4);
      }
      for (int k = 1; k < nslabs; ++k) {
        a += *reinterpret_cast<const f32x4*>(gi + k * slab_stride + e);
        b += *reinterpret_cast<const f32x4*>(gi + k * slab_stride + e + 4);
      }
      for (int k = 0; k < nx; ++k) {
        const half8 x = *reinterpret_cast<const half8*>(xs + k * slab_stride + (long long)i * ldo + e);
        a += f32x4{(float)x[0], (float)x[1], (float)x[2], (float)x[3]};
        b += f32x4{(float)x[4], (float)x[5], (float)x[6], (float)x[7]};
      }
      g[c][0] = a[0]; g[c][1] = a[1]; g[c][2] = a[2]; g[c][3] = a[3];
      g[c][4] = b[0]; g[c][5] = b[1]; g[c][6] = b[2]; g[c][7] = b[3];
#pragma unroll
      for (int j = 0; j < 8; ++j) { z[c][j] *= iv; dot += z[c][j] * g[c][j]; }
    }
  }
  dot = block_sum(dot, red);
  Tin* di = dh + (long long)i * d;
  const float s = alpha * iv;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = (c * 256 + threadIdx.x) * 8;
    if (e < d) {
      float o[8], q[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = s * (g[c][j] - z[c][j] * dot);
      store8<Tin>(di + e, o, q);
    }
  }
}

template <typename Tin>
__global__ __launch_bounds__(256) void norm_bwd_kernel(const float* __restrict__ slabs, int nslabs,
                                                       long long slab_stride, long long ldo,
                                                       const Tin* __restrict__ h, const float* __restrict__ inv,
                                                       const float* __restrict__ grad_out, float alpha_base,
                                                       Tin* __restrict__ dh, int d, const _Float16* __restrict__ xs,
                                                       int nx) {
  const _Float16* xi = xs + (long long)blockIdx.x * ldo;
  __shared__ float red[16];
  const int i = blockIdx.x;
  const float iv = inv[i];
  const float alpha = grad_out[0] * alpha_base;
  const Tin* hi = h + (long long)i * d;
  const float* gi = slabs + (long long)i * ldo;
  float dot = 0.f;
  for (int e = threadIdx.x; e < d; e += 256) {
    float g = 0.f;
    for (int k = 0; k < nslabs; ++k) g += gi[k * slab_stride + e];
    for (int k = 0; k < nx; ++k) g += (float)xi[k * slab_stride + e];
    dot += to_f32<Tin>(hi[e]) * iv * g;
  }
  dot = block_sum(dot, red);
  Tin* di = dh + (long long)i * d;
  for (int e = threadIdx.x; e < d; e += 256) {
    float g = 0.f;
    for (int k = 0; k < nslabs; ++k) g += gi[k * slab_stride + e];
    for (int k = 0; k < nx; ++k) g += (float)xi[k * slab_stride + e];
    const float z = to_f32<Tin>(hi[e]) * iv;
    di[e] = from_f32<Tin>(alpha * iv * (g - z * dot));
  }
}

// dot_i = sum over the coefficient pass's slots dotp[k][i] (slot-major; fixed order: deterministic).
// 32 rows per block (one per CU at the headline: 256 blocks), 8 threads per row: thread (w, lane)
// takes row (lane & 31) and slots sg, sg + 8, ... (sg = 2 w + (lane >> 5)), all its loads in flight
// at once; the 8 partials are then summed in sg order. (64 rows x 4 slot groups per block left half
// the CUs idle and put 32 loads behind each thread: 5.0 us at the headline.)
__global__ __launch_bounds__(256) void dot_reduce_kernel(const float* __restrict__ dotp, int nslot, int rows,
                                                         float* __restrict__ dot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = blockIdx.x * 32 + (lane & 31), sg = 2 * w + (lane >> 5);
  __shared__ float part[8][32];
  // (the same arithmetic as the dZ's folded form, dz_dot_fold: bitwise the same dot)
  part[sg][lane & 31] = i < rows ? dot_slot_sum(dotp, nslot, rows, i, sg) : 0.f;
  __syncthreads();
  if (threadIdx.x < 32 && blockIdx.x * 32 + (int)threadIdx.x < rows) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) t += part[g][threadIdx.x];
    dot[blockIdx.x * 32 + threadIdx.x] = t;
  }
}

}  // namespace dev

// ======================================================================================
// Host side
// ======================================================================================
namespace {
inline int roundup(int x, int m) { return (x + m - 1) / m * m; }

template <typename F>
void dispatch_comp(DType t, F&& f) {
  switch (t) {
    case DType::F32: f(float{}); break;
    case DType::F16: f(_Float16{}); break;
    case DType::BF16: f(__bf16{}); break;
    case DType::FP8: NTXENT_CHECK(false, "fp8 is a GEMM operand type only"); break;
  }
}

// GEMM operand types (fp8 included).
template <typename F>
void dispatch_gemm(DType t, F&& f) {
  if (t == DType::FP8) f(dev::fp8e4m3{});
  else dispatch_comp(t, f);
}

// fp8 forward GEMMs: accumulators are products of e4m3(z * 256) values.
// fp8 forward GEMMs: the block-scaled MFMA applies each row's E8M0 scale (stored right after
// the row's dim_k8 bytes), so accumulators are unscaled dot products like the other dtypes.
void set_operand_scales(dev::SimParams& p, DType comp, const Geometry& g) {
  p.acc_scale = p.y_scale;
  p.scale_off = comp == DType::FP8 ? g.dim_k8 : 0;
}

#if NTXENT_TIMING
// Diagnostic builds: a device buffer of [grid][kTimingItems][kTimingMarks] s_memtime marks per
// launch kind, written after the launch to $NTXENT_TIMING_OUT/<name>_g<grid>.bin (the last launch
// of a kind wins; tools/gemm_timing.py reads them).
struct TimingBuf {
  unsigned long long* buf = nullptr;
  size_t cap = 0, n = 0;
  unsigned long long* prepare(int grid, hipStream_t stream) {
    n = (size_t)grid * dev::kTimingItems * dev::kTimingMarks;
    if (n > cap) {
      if (buf) NTXENT_HIP_CHECK(hipFree(buf));
      NTXENT_HIP_CHECK(hipMalloc(&buf, n * 8));
      cap = n;
    }
    NTXENT_HIP_CHECK(hipMemsetAsync(buf, 0, n * 8, stream));
    return buf;
  }
  void dump(const std::string& name, int grid, hipStream_t stream) const {
    const char* dir = std::getenv("NTXENT_TIMING_OUT");
    if (!dir) return;
    std::vector<unsigned long long> h(n);
    NTXENT_HIP_CHECK(hipStreamSynchronize(stream));
    NTXENT_HIP_CHECK(hipMemcpy(h.data(), buf, n * 8, hipMemcpyDeviceToHost));
    const std::string f = std::string(dir) + "/" + name + "_g" + std::to_string(grid) + ".bin";
    if (FILE* fp = std::fopen(f.c_str(), "wb")) {
      const int hdr[3] = {grid, dev::kTimingItems, dev::kTimingMarks};
      std::fwrite(hdr, sizeof(int), 3, fp);
      std::fwrite(h.data(), 8, n, fp);
      std::fclose(fp);
    }
  }
};
#endif

template <typename Tc, int MODE>
void launch_sim_gemm(int grid, const dev::SimParams& p_in, hipStream_t stream) {
#if NTXENT_TIMING
  static TimingBuf tb;
  dev::SimParams p = p_in;
  p.tstamp = tb.prepare(grid, stream);
#else
  const dev::SimParams& p = p_in;
#endif
  if (MODE == dev::kModeFwd && !p.fixed_shift)
    hipLaunchKernelGGL((dev::sim_gemm_kernel<Tc, MODE, MODE == dev::kModeFwd ? 0 : 1>), dim3(grid), dim3(kGemmThreads), 0,
                       stream, p);
  else
    hipLaunchKernelGGL((dev::sim_gemm_kernel<Tc, MODE>), dim3(grid), dim3(kGemmThreads), 0, stream, p);
#if NTXENT_TIMING
  tb.dump("gemm_m" + std::to_string(MODE) + "_e" + std::to_string(sizeof(Tc)), grid, stream);
#endif
}

dev::SimParams base_params(const Geometry& g) {
  dev::SimParams p{};
  p.R = g.rows;
  p.Rpad = g.rows_pad;
  p.n_half = g.rows / 2;
  p.own0 = g.rank * g.rows_pad;
  p.row_tile0 = g.rank * g.row_tiles;
  p.col_tiles = g.col_tiles;
  p.b_tile0 = 0;
  p.c_ld = g.col_tiles;
  p.c_tile0 = 0;
  p.y_scale = g.inv_temp * dev::kLog2e;
  p.acc_scale = p.y_scale;
  p.fixed_shift = (2.0f * p.y_scale < 120.0f) ? 1 : 0;  // tau > ~0.024
  return p;
}

// Fill the stream-K fields of `p` for `ntiles` tiles of p.kbytes each. The arrival counters at
// the head of the workspace are zero when it is allocated and every launch leaves them zero
// (the last arriver of a tile resets its counter), so no memset node is needed per launch.
// Returns the grid.
// Counter region: 2 per CU for the stream-K tiles, and 14 per diagonal-remainder tile
// (diag_up_kernel: 4 row-group + 10 region tickets) for up to num_cus - 1 remainder tiles.
constexpr int kDiagTickets = 14;
size_t sk_counter_bytes(int num_cus) {
  return ((size_t)std::max(2, kDiagTickets) * std::max(1, num_cus) * 4 + 255) / 256 * 256;
}

int apply_schedule(dev::SimParams& p, int ntiles, const GemmWorkspace& ws, hipStream_t stream) {
  NTXENT_CHECK(p.kbytes % kKStepBytes == 0, "K not aligned to the K step");
  const int nk = (int)(p.kbytes / kKStepBytes);
  const int cus = ws.sched_cus > 0 ? std::min(ws.sched_cus, ws.num_cus) : ws.num_cus;
  const GemmSchedule s = make_schedule(ntiles, nk, cus);
  p.nk = s.nk;
  p.dp_tiles = s.dp_tiles;
  p.sk_tiles = s.sk_tiles;
  p.ipb = s.ipb;
  const size_t cnt_bytes = sk_counter_bytes(ws.num_cus);  // fixed: independent of the launch
  NTXENT_CHECK(s.sk_tiles <= 2 * ws.num_cus, "stream-K tile count exceeds the counter region");
  p.sk_cnt = static_cast<int*>(ws.ptr);
  p.sk_slabs = reinterpret_cast<float*>(static_cast<char*>(ws.ptr) + cnt_bytes);
  if (s.sk_tiles > 0) {  // counters must be zero at launch: zeroed at allocation, self-cleaning
    NTXENT_CHECK(ws.ptr != nullptr && ws.bytes >= gemm_workspace_bytes(ntiles, ws.num_cus),
                 "stream-K workspace too small");
  }
  (void)stream;
  return s.grid;
}

// Leading dimension (elements) for a row of `n` elements: strides of a multiple of 1024
// elements get 64 extra so the rows a tile streams rotate through the L2 channels.
#ifndef NTXENT_NO_LDPAD
#define NTXENT_NO_LDPAD 0  // A/B switch (tools/build_variant.sh -DNTXENT_NO_LDPAD=1: unpadded rows)
#endif
int padded_ld(int n) { return (!NTXENT_NO_LDPAD && n % 1024 == 0) ? n + 64 : n; }

// The coefficient tiles as the dZ GEMM's A operand: tile (I, J) of a row panel of `panel_tiles`
// tiles; 256 K-columns per tile. Row-major tiles: rows of 256 elements, every 256 K-columns jump
// to the next tile of the panel.
dev::OperandDesc coef_tile_operand(const void* base, long long panel_tiles, long long cs) {
  dev::OperandDesc o;
  o.base = static_cast<const char*>(base);
  o.row_tile_stride = panel_tiles * kTileElems * cs;
  o.ld = kTile * cs;
  o.kblk = kTile * cs;
  o.kblk_stride = kTileElems * cs;
  return o;
}

dev::OperandDesc rowmajor_operand(const void* base, long long ld_bytes, long long kbytes) {
  dev::OperandDesc o;
  o.base = static_cast<const char*>(base);
  o.ld = ld_bytes;
  o.row_tile_stride = ld_bytes * kTile;
  o.kblk = kbytes;       // one K block: no blocking
  o.kblk_stride = 0;
  return o;
}
}  // namespace

Geometry make_geometry(int rows, int dim, int world, int rank, float temperature) {
  NTXENT_CHECK(rows > 0 && rows % 2 == 0, "rows must be positive and even (two stacked views)");
  NTXENT_CHECK(dim > 0, "dim must be positive");
  NTXENT_CHECK(world >= 1 && rank >= 0 && rank < world, "bad world/rank");
  NTXENT_CHECK(temperature > 0.f, "temperature must be positive");
  Geometry g;
  g.rows = rows;
  g.rows_pad = roundup(rows, kTile);
  g.dim = dim;
  g.dim_k = roundup(dim, 64);
  g.dim_n = roundup(dim, kTile);
  g.ld_k = padded_ld(g.dim_k);
  g.ld_t = padded_ld(g.rows_pad);
  g.dim_k8 = roundup(dim, 128);
  g.ld_k8 = g.dim_k8 + 64;  // >= 1 spare byte per row for the E8M0 row scale; never a 1 KiB multiple
  g.world = world;
  g.rank = rank;
  g.row_tiles = g.rows_pad / kTile;
  g.col_tiles = world * g.row_tiles;
  g.temperature = temperature;
  g.inv_temp = 1.0f / temperature;
  g.global_rows = (long long)world * rows;
  return g;
}

// Morton (Z-order) key: every aligned run of 2^k consecutive tiles is a compact 2-D block.
static unsigned morton2(unsigned i, unsigned j) {
  unsigned r = 0;
  for (int b = 0; b < 16; ++b) r |= ((i >> b) & 1u) << (2 * b + 1) | ((j >> b) & 1u) << (2 * b);
  return r;
}

static void zorder(std::vector<int4>& t, size_t first, size_t last) {
  std::stable_sort(t.begin() + first, t.begin() + last, [](const int4& a, const int4& b) {
    return morton2((unsigned)a.x, (unsigned)a.y) < morton2((unsigned)b.x, (unsigned)b.y);
  });
}

// Own-block upper triangle: the off-diagonal tiles, then the row_tiles diagonal tiles in order
// (own_diag_tail(g) of them end the list). Off-diagonal order: the GEMM gives each XCD 32
// consecutive tiles per round, and A and B are both row panels of Zq, so a group's L2 traffic is
// its number of distinct panels. Row tiles in superblocks of 8: every pair of superblocks
// (a < b) forms two 4 x 8 groups (12 panels per 32 tiles), then each superblock's own 28 upper
// tiles (8 panels); 13.2 distinct panels per group at 32 row tiles, 12.5 at 64, against 15.4 /
// 15.6 in Z-order (the fallback for row_tiles not a multiple of 8).
static std::vector<int4> own_block_tiles(const Geometry& g) {
  std::vector<int4> tiles;
  const int own = g.rank * g.row_tiles, rt = g.row_tiles;
  if (rt % 8 == 0 && rt >= 16) {
    const int nb = rt / 8;
    for (int a = 0; a < nb; ++a)
      for (int b = a + 1; b < nb; ++b)
        for (int h = 0; h < 2; ++h)
          for (int i = 8 * a + 4 * h; i < 8 * a + 4 * h + 4; ++i)
            for (int j = 8 * b; j < 8 * b + 8; ++j) tiles.push_back(make_int4(i, own + j, kTileSymOff, 0));
    for (int a = 0; a < nb; ++a) {
      const size_t first = tiles.size();
      for (int i = 8 * a; i < 8 * a + 8; ++i)
        for (int j = i + 1; j < 8 * a + 8; ++j) tiles.push_back(make_int4(i, own + j, kTileSymOff, 0));
      zorder(tiles, first, tiles.size());
    }
  } else {
    for (int ti = 0; ti < rt; ++ti)
      for (int local = ti + 1; local < rt; ++local) tiles.push_back(make_int4(ti, own + local, kTileSymOff, 0));
    zorder(tiles, 0, tiles.size());
  }
  for (int ti = 0; ti < rt; ++ti) tiles.push_back(make_int4(ti, own + ti, kTileDiag, 0));
  return tiles;
}

int own_diag_tail(const Geometry& g) { return g.row_tiles; }

std::vector<int4> build_fwd_tiles(const Geometry& g) {
  // Own-rank block first (upper triangle: S is symmetric), then the remote column blocks.
  // Each part in Z-order: the blocks of one XCD (consecutive logical ids after xcd_remap) take
  // consecutive tiles, and a Z-order run of 32 tiles touches ~0.4 distinct row panels per tile
  // (A and B panels of the own block are both rows of Zq) versus ~0.7-1.0 for panel-major
  // order, which is what the forward GEMM's L2 hit rate depends on (measured 48% before).
  // The own block's diagonal tiles come last in it (own_block_tiles): a launch of the own block
  // leaves its whole-round remainder on them, which the strip kernel finishes (launch_fwd_stats).
  std::vector<int4> tiles = own_block_tiles(g);
  const size_t n_own = tiles.size();
  const int own = g.rank * g.row_tiles;
  for (int ti = 0; ti < g.row_tiles; ++ti)
    for (int tj = 0; tj < g.col_tiles; ++tj)
      if (tj < own || tj >= own + g.row_tiles) tiles.push_back(make_int4(ti, tj, kTilePlain, 0));
  zorder(tiles, n_own, tiles.size());
  return tiles;
}

std::vector<int4> build_sym_fwd_tiles(const Geometry& g, const std::vector<SymJob>& jobs, int nchunks) {
  std::vector<int4> tiles = own_block_tiles(g);
  for (const SymJob& j : jobs) {
    NTXENT_CHECK(j.q >= 0 && j.q < g.world && j.q != g.rank, "sym job: bad partner");
    NTXENT_CHECK(0 <= j.m0 && j.m0 <= j.m1 && j.m1 <= g.row_tiles && 0 <= j.k0 && j.k0 <= j.k1 &&
                     j.k1 <= g.row_tiles, "sym job: tile range out of bounds");
  }
  NTXENT_CHECK(nchunks >= 1 && nchunks <= g.row_tiles, "sym tiles: bad chunk count");
  // one contiguous Z-ordered segment per chunk of the partners' row tiles (sym_chunk_bounds):
  // a chunk's tiles can run as soon as that chunk of every partner's rows has arrived
  for (int c = 0; c < nchunks; ++c) {
    const int c0 = (int)((long long)g.row_tiles * c / nchunks), c1 = (int)((long long)g.row_tiles * (c + 1) / nchunks);
    const size_t first = tiles.size();
    for (const SymJob& j : jobs)
      for (int ti = j.m0; ti < j.m1; ++ti)
        for (int tj = std::max(j.k0, c0); tj < std::min(j.k1, c1); ++tj)
          tiles.push_back(make_int4(ti, j.q * g.row_tiles + tj, kTileCross, 0));
    zorder(tiles, first, tiles.size());
  }
  return tiles;
}

int count_own_fwd_tiles(const Geometry& g) { return g.row_tiles * (g.row_tiles + 1) / 2; }

std::vector<SymJob> sym_jobs(int world, int rank, int row_tiles) {
  std::vector<SymJob> jobs;
  const int W = world, r = rank, rt = row_tiles;
  for (int d = 1; d <= (W - 1) / 2; ++d) jobs.push_back(SymJob{(r + d) % W, 0, rt, 0, rt});
  if (W % 2 == 0 && W > 1) {
    const int q = (r + W / 2) % W, h = (rt + 1) / 2;
    const SymJob j = r < q ? SymJob{q, 0, h, 0, rt} : SymJob{q, 0, rt, h, rt};
    if (j.m0 < j.m1 && j.k0 < j.k1) jobs.push_back(j);
  }
  return jobs;
}

std::vector<SymJob> sym_incoming(int world, int rank, int row_tiles) {
  std::vector<SymJob> out;
  for (int p = 0; p < world; ++p) {
    if (p == rank) continue;
    for (const SymJob& j : sym_jobs(world, p, row_tiles))
      if (j.q == rank) out.push_back(SymJob{p, j.m0, j.m1, j.k0, j.k1});
  }
  return out;
}

int sym_num_chunks(int row_tiles) { return std::max(1, std::min(4, row_tiles)); }
int sym_c_ld(const Geometry& g) { return std::min(g.world, g.world / 2 + 1) * g.row_tiles; }

GemmSchedule make_schedule(int ntiles, int nk, int num_cus) {
  // Whole tiles in data-parallel rounds of G = num_cus blocks; only the remainder tiles
  // (ntiles % G) are split, into p K-pieces each, run by the first rem * p blocks after their
  // DP rounds (the classic hybrid that also splits a whole DP round spent 30-74 us per block of
  // the B = 4096 forward in slab traffic). p minimises, in K-step units,
  //   nk / p + (p > 1 ? 10 + 4 (p - 1) : 0):
  // a split costs ~10 K-steps once (slab publish, ticket, the last arriver's extra item) and ~4
  // per partial slab the last arriver sums. Fitted on a same-box sweep of p = 1..8
  // (profiles/r2/sk_split_sweep.log): p = 1 at nk <= 16 (d = 512 / 1024 forward; splitting cost
  // 5-15 %), p = 3-4 at nk = 32 (the headline), p = 6 at nk = 128 (d = 8192, 36 tiles).
  GemmSchedule s;
  s.nk = nk;
  const int G0 = std::max(1, num_cus);
  const int q = ntiles / G0, rem = ntiles % G0;
  s.dp_tiles = q * G0;
  s.sk_tiles = rem;
  if (rem == 0) {
    s.grid = std::min(G0, std::max(1, ntiles));
    s.ipb = 0;
    return s;
  }
  int p = 1;
  double best = 1e30;
  for (int c = 1; c <= std::max(1, std::min(G0 / rem, nk)); ++c) {
    const double cost = (double)nk / c + (c > 1 ? 10.0 + 4.0 * (c - 1) : 0.0);
    if (cost < best - 1e-9) { best = cost; p = c; }
  }
  s.grid = q > 0 ? G0 : rem * p;
  s.ipb = (nk + p - 1) / p;  // K-steps per stream-K block; ceil(rem * nk / ipb) <= rem * p blocks busy
  return s;
}

// Stream-K splits at most 2*G - 1 tiles (one DP round plus the remainder, or all tiles when
// there are fewer than G), so 2*num_cus counters always suffice. The counter region has a
// fixed size so that launches of different tile counts sharing one workspace never place
// their fp32 partial slabs over another launch's (self-cleaning, zero) counters.

// + the split-K forward's column-partial strips (fewer tiles than CUs: < num_cus tiles).
size_t gemm_workspace_bytes(int ntiles, int num_cus) {
  (void)ntiles;
  return sk_counter_bytes(num_cus) + (size_t)2 * std::max(1, num_cus) * kTileElems * sizeof(float) +
         (size_t)std::max(1, num_cus) * dev::kSkColpTile * sizeof(float2);
}

std::vector<int4> build_dz_tiles(const Geometry& g) {
  std::vector<int4> tiles;
  const int nt = g.dim_n / kTile;
  for (int ti = 0; ti < g.row_tiles; ++ti)
    for (int tn = 0; tn < nt; ++tn) tiles.push_back(make_int4(ti, tn, 0, 0));
  return tiles;
}

void launch_prep(DType in, DType comp, const void* h, void* zq, float* inv, float* ypos,
                 const Geometry& g, hipStream_t stream, void* zq8) {
  NTXENT_CHECK(comp != DType::FP8, "prep: pass the fp16 plan dtype and a zq8 buffer for fp8");
  // pad rows [R, Rpad) are zeroed by extra blocks of the prep kernel itself (no memset launch);
  // zq rows are 16-byte multiples (ld_k is a multiple of 64 elements, ld_k8 of 128 bytes)
  const int pad = g.rows_pad - g.rows;
  const float ys = g.inv_temp * dev::kLog2e;
  // wave-per-pair kernel when the rows fit in registers (d <= 2048), else one block per pair
  const int nch = (g.dim % 8 == 0) ? (g.dim + 511) / 512 : 0;
  if (zq == nullptr) {  // statistics only (raw-operand forward): inv, ypos; no zq, no pad rows
    NTXENT_CHECK(zq8 == nullptr && g.dim % 8 == 0 && g.dim <= 16384, "prep (statistics only): d % 8 == 0, d <= 16384");
    dispatch_comp(in, [&](auto tin) {
      using Tin = decltype(tin);
      if (nch >= 1 && nch <= 4) {
        auto go = [&](auto nc) {
          hipLaunchKernelGGL((dev::prep_wave_kernel<Tin, Tin, false, decltype(nc)::value, true>),
                             dim3((g.rows / 2 + 3) / 4), dim3(256), 0, stream, static_cast<const Tin*>(h), nullptr, inv,
                             ypos, g.rows, g.dim, g.dim_k, g.ld_k, ys, nullptr, 0, 0, g.rows);
        };
        if (nch == 1) go(std::integral_constant<int, 1>{});
        else if (nch == 2) go(std::integral_constant<int, 2>{});
        else go(std::integral_constant<int, 4>{});
      } else {
        const int nbl = (g.dim + 2047) / 2048;
        auto go = [&](auto nc) {
          hipLaunchKernelGGL((dev::prep_block_kernel<Tin, Tin, false, decltype(nc)::value, true>), dim3(g.rows / 2),
                             dim3(256), 0, stream, static_cast<const Tin*>(h), nullptr, inv, ypos, g.rows, g.dim,
                             g.dim_k, g.ld_k, ys, nullptr, 0, 0);
        };
        if (nbl <= 2) go(std::integral_constant<int, 2>{});
        else if (nbl <= 4) go(std::integral_constant<int, 4>{});
        else go(std::integral_constant<int, 8>{});
      }
    });
    NTXENT_HIP_CHECK(hipGetLastError());
    return;
  }
  dispatch_comp(in, [&](auto tin) {
    using Tin = decltype(tin);
    dispatch_comp(comp, [&](auto tc) {
      using Tc = decltype(tc);
      if (nch >= 1 && nch <= 4) {
        const dim3 grid((g.rows / 2 + 3) / 4 + (pad + 3) / 4);
        auto go = [&](auto nc, auto q8) {
          constexpr int NC = decltype(nc)::value;
          constexpr bool Q = decltype(q8)::value;
          hipLaunchKernelGGL((dev::prep_wave_kernel<Tin, Tc, Q, NC>), grid, dim3(256), 0, stream,
                             static_cast<const Tin*>(h), static_cast<Tc*>(zq), inv, ypos, g.rows, g.dim, g.dim_k,
                             g.ld_k, ys, static_cast<unsigned char*>(zq8), g.dim_k8, g.ld_k8, g.rows_pad);
        };
        auto by_q = [&](auto nc) {
          if (zq8) go(nc, std::true_type{});
          else go(nc, std::false_type{});
        };
        if (nch == 1) by_q(std::integral_constant<int, 1>{});
        else if (nch == 2) by_q(std::integral_constant<int, 2>{});
        else by_q(std::integral_constant<int, 4>{});
        return;
      }
      const int nbl = (g.dim % 8 == 0) ? (g.dim + 2047) / 2048 : 0;  // chunks per thread, 256 per pair
      if (nbl >= 2 && nbl <= 8) {
        auto go = [&](auto nc, auto q8) {
          constexpr int NC = decltype(nc)::value;
          constexpr bool Q = decltype(q8)::value;
          hipLaunchKernelGGL((dev::prep_block_kernel<Tin, Tc, Q, NC>), dim3(g.rows / 2 + pad), dim3(256), 0, stream,
                             static_cast<const Tin*>(h), static_cast<Tc*>(zq), inv, ypos, g.rows, g.dim, g.dim_k,
                             g.ld_k, ys, static_cast<unsigned char*>(zq8), g.dim_k8, g.ld_k8);
        };
        auto by_q = [&](auto nc) {
          if (zq8) go(nc, std::true_type{});
          else go(nc, std::false_type{});
        };
        if (nbl <= 2) by_q(std::integral_constant<int, 2>{});
        else if (nbl <= 4) by_q(std::integral_constant<int, 4>{});
        else by_q(std::integral_constant<int, 8>{});
        return;
      }
      if (zq8)
        hipLaunchKernelGGL((dev::prep_kernel<Tin, Tc, true>), dim3(g.rows / 2 + pad), dim3(256), 0, stream,
                           static_cast<const Tin*>(h), static_cast<Tc*>(zq), inv, ypos, g.rows, g.dim,
                           g.dim_k, g.ld_k, ys, static_cast<unsigned char*>(zq8), g.dim_k8, g.ld_k8);
      else
        hipLaunchKernelGGL((dev::prep_kernel<Tin, Tc, false>), dim3(g.rows / 2 + pad), dim3(256), 0, stream,
                           static_cast<const Tin*>(h), static_cast<Tc*>(zq), inv, ypos, g.rows, g.dim,
                           g.dim_k, g.ld_k, ys, nullptr, 0, 0);
    });
  });
  NTXENT_HIP_CHECK(hipGetLastError());
}

void launch_sum_slabs(const float* in, int n, size_t count, float* out, hipStream_t stream) {
  if (count == 0) return;
  const int grid = (int)std::min<size_t>((count + 255) / 256, 1024);
  hipLaunchKernelGGL(dev::sum_slabs_kernel, dim3(grid), dim3(256), 0, stream, in, n, count, out);
  NTXENT_HIP_CHECK(hipGetLastError());
}

void launch_transpose(DType comp, const void* zq, void* zqt, const Geometry& g, hipStream_t stream) {
  dispatch_comp(comp, [&](auto tc) {
    using Tc = decltype(tc);
    hipLaunchKernelGGL((dev::transpose_kernel<Tc>), dim3(g.rows_pad / 64, g.dim_n / 64), dim3(256), 0,
                       stream, static_cast<const Tc*>(zq), static_cast<Tc*>(zqt), g.dim_k, g.ld_k, g.ld_t);
  });
  NTXENT_HIP_CHECK(hipGetLastError());
}

// ---- runtime switches: every process-wide toggle of the library lives here (atomics). Only
//      behaviour switches remain: the small-problem path (off = the large-problem pipeline at
//      every shape, so tests can exercise it on small inputs), its two test overrides, and the
//      fp8 backward switch. Measured A/B losers are deleted, not kept behind toggles; the CUs a
//      GEMM leaves free for communication are a per-launch argument (GemmWorkspace::sched_cus).
static std::atomic<bool> g_small_path{true};     // one-launch small-problem forward / backward
static std::atomic<int> g_small_splits{0};       // small backward column splits (0: small_bwd_splits)
static std::atomic<int> g_small_fuse_rows{-1};   // small forward: fused row prologue up to R rows (-1: default)
static std::atomic<bool> g_fp8_bwd{true};        // FP8 plans: e4m3 coefficient / Z^T dZ GEMM (Q8Stats)
static std::atomic<bool> g_raw_fwd{true};        // raw-operand forward (RawRows) where eligible
void set_small_path(bool on) { g_small_path = on; }
bool small_path_enabled() { return g_small_path.load(); }
void set_small_splits(int n) { g_small_splits = std::max(0, n); }
int small_splits_override() { return g_small_splits.load(); }
void set_small_fuse_rows(int rows) { g_small_fuse_rows = rows < 0 ? -1 : rows; }
int small_fuse_rows_override() { return g_small_fuse_rows.load(); }
void set_fp8_backward(bool on) { g_fp8_bwd = on; }
void set_raw_forward(bool on) { g_raw_fwd = on; }

static std::atomic<bool> g_lse_fold{[] {
  const char* e = std::getenv("NTXENT_LSE_FOLD");
  return e == nullptr || std::string(e) != "0";
}()};
void set_lse_fold(bool on) { g_lse_fold = on; }

bool lse_fold_enabled() { return g_lse_fold.load(); }
static double lse_loss_fx(const Geometry& g, int nb);

static std::atomic<bool> g_half_c{[] {
  const char* e = std::getenv("NTXENT_HALF_C");
  return e == nullptr || std::string(e) != "0";
}()};
void set_half_c(bool on) { g_half_c = on; }
bool half_c_enabled() { return g_half_c.load(); }

// The scheduling decisions of launch_dz, replayed: half C needs every dZ item to start at an even
// K-step (whole tiles, or split-K pieces of an even ipb), so that an item's lower-tile K-steps
// (4 per tile) are an even count ahead of its upper ones; stream-K ranges are arbitrary.
bool dz_half_c_eligible(DType comp, const Geometry& g, int n_dz, const GemmWorkspace& ws) {
  if ((comp != DType::F16 && comp != DType::BF16) || g.world != 1 || n_dz <= 0) return false;
  if ((long long)g.row_tiles * g.col_tiles * kTileElems * 2 >= (1ll << 31)) return false;  // 32-bit offsets
  const int cus = ws.sched_cus > 0 ? std::min(ws.sched_cus, ws.num_cus) : ws.num_cus;
  const int nk = (int)((long long)g.rows_pad * 2 / kKStepBytes);
  int pieces = fwd_splitk_pieces(n_dz, nk, cus, 1);
  if (pieces < 3) pieces = 0;
  if (pieces > 0) return ((nk + pieces - 1) / pieces) % 2 == 0;
  return make_schedule(n_dz, nk, cus).sk_tiles == 0;
}
static std::atomic<bool> g_dot_fold{[] {
  const char* e = std::getenv("NTXENT_DOT_FOLD");
  return e == nullptr || std::string(e) != "0";
}()};
void set_dot_fold(bool on) { g_dot_fold = on; }
bool dot_fold_enabled() { return g_dot_fold.load(); }
// polls (s_sleep 8 each, ~0.2 us) before an epilogue sums its rows' dot itself; the count is
// complete a main loop before the first poll, so the bound only guards a grid whose blocks are not
// all resident. Tests set 0: every epilogue takes the fallback (its result must not change).
static std::atomic<int> g_dot_spin{1 << 14};
void set_dot_fold_spin(int polls) { g_dot_spin = polls < 0 ? 0 : polls; }
int dot_fold_spin() { return g_dot_spin.load(); }
// The dot reduce folds into a 16-bit fused dZ (whole / stream-K tiles: published to its own
// epilogues; split-K pieces: to the reduce launch); callers then skip launch_dot_reduce
// (NormFuse::dot_cnt).
bool dz_dot_fold_eligible(DType comp, const Geometry& g, int n_dz, const GemmWorkspace&) {
  return (comp == DType::F16 || comp == DType::BF16) && n_dz > 0 && g.dim % 8 == 0 && dot_fold_enabled();
}
bool raw_forward_enabled() { return g_raw_fwd.load(); }
bool raw_forward_eligible(const Geometry& g, DType in, DType comp) {
  // (fp16 rows on a bf16 plan would keep fp16 cosines for a bf16 backward: not offered)
  return g.world == 1 && (in == DType::F16 || in == DType::BF16) && (comp == DType::F16 || comp == in) &&
         g.rows % kTile == 0 && g.dim % 64 == 0 && g.dim <= 16384;
}
bool fp8_backward_enabled() { return g_fp8_bwd.load(); }
bool fp8_backward_eligible(const Geometry& g, DType comp) { return comp == DType::FP8 && g.world == 1 && g.dim % 8 == 0; }
// padded like the 16-bit Z^T (padded_ld): at a power-of-two stride (16 KiB at config 5) the dZ's
// B half-tiles, 8 rows per DMA instruction, all fell into one L1 set and L2 channel (TD busy 86 %,
// MFMA busy 17 %: profiles/r5/fp8_dz)
int q8_ldt(const Geometry& g) { return (!NTXENT_NO_LDPAD && g.rows_pad % 1024 == 0) ? g.rows_pad + 128 : g.rows_pad; }

#ifndef NTXENT_ZT_SIDE_PER_CU
#define NTXENT_ZT_SIDE_PER_CU 2  // Z^T side blocks of the diagonal remainder per CU (experiment builds: 1)
#endif

// K pieces of the diagonal remainder's off-diagonal regions (diag_up_kernel): 2 from 32 K-steps
// up (the headline: 1 piece +2 us), 1 below (config 2 -1.5 us, config 5 -0.4 us:
// profiles/r4/variants_r4_v29_diagks1.md; 4 pieces measured +6 us at config 5,
// profiles/r4/variants_r4_v2.md)
constexpr int kDiagKS = 2;  // the most pieces any shape uses (workspace sizing)
static int diag_ks(int nk_tile) { return nk_tile >= 32 ? 2 : 1; }

// K pieces per tile of the split-K forward (0: not used): own-block launches with fewer tiles
// than CUs and long K, where the stream-K schedule's last-arriving block would read p - 1
// partial slabs serially (BASELINE config 4: 36 tiles x 128 K-steps, fixup ~40 % of the GEMM).

int fwd_diag_remainder(int ntiles, int nk_tile, int cus, int diag_tail, bool f8) {
  if (diag_tail <= 0 || f8 || nk_tile < 4 || cus <= 0) return 0;
  const int q = ntiles / cus, rem = ntiles % cus;
  return (q >= 1 && rem > 0 && rem <= diag_tail) ? rem : 0;
}

int fwd_splitk_pieces(int ntiles, int nk, int cus, int diag_tail) {
  if (diag_tail <= 0 || ntiles <= 0 || ntiles >= cus || nk < 32) return 0;
  const int pcs = std::min(cus / ntiles, nk / 8);
  return pcs >= 2 ? pcs : 0;
}

bool launch_fwd_stats(DType comp, const void* zq_local, const void* zq_all, const int4* tiles,
                      int ntiles, float2* part, void* sc, const GemmWorkspace& ws, const Geometry& g,
                      hipStream_t stream, const BlockView& bv, float2* part_x, int diag_tail,
                      hipEvent_t main_done, const RawRows* raw) {
  if (ntiles == 0) return false;
  bool zt_done = false;  // raw->zqt written beside the diagonal remainder
  NTXENT_CHECK(diag_tail >= 0 && diag_tail <= ntiles, "fwd_stats: bad diagonal tail");
  const bool f8 = comp == DType::FP8;  // fp8: K = dim_k8 bytes of rows ld_k8 bytes apart
  if (raw) {
    NTXENT_CHECK(raw_forward_eligible(g, raw->in, comp) && raw->inv && part_x == nullptr && bv.b_tile0 == 0,
                 "fwd_stats (raw operands): single-process 2-byte plan, rows % 256 == 0, dim % 64 == 0");
    zq_local = zq_all = raw->h;
  }
  // raw operands: the input rows, dim (= dim_k) elements apart; else the padded zq rows
  const long long kb = f8 ? (long long)g.dim_k8 : (long long)g.dim_k * dtype_size(comp);
  const long long ld = f8 ? (long long)g.ld_k8 : raw ? (long long)g.dim * 2 : (long long)g.ld_k * dtype_size(comp);
  dev::SimParams p = base_params(g);
  if (raw) {
    p.inv_a = raw->inv;
    p.inv_b = raw->inv;
  }
  set_operand_scales(p, comp, g);
  p.A = rowmajor_operand(zq_local, ld, kb);
  p.B = rowmajor_operand(zq_all, ld, kb);
  p.tiles = tiles;
  p.kbytes = kb;
  p.part = part;
  p.sc = static_cast<char*>(sc);
  p.b_tile0 = bv.b_tile0;
  p.part_x = part_x;
  const int cus = ws.sched_cus > 0 ? std::min(ws.sched_cus, ws.num_cus) : ws.num_cus;
  const int nk_tile = (int)(kb / kKStepBytes);
  // Whole rounds on the persistent GEMM. A remainder of diagonal tiles (the own block's tail)
  // runs after them as upper 64x64 regions (diag_up_kernel: 10 of a tile's 16 regions, the
  // coefficient pass mirrors the rest) instead of a third round / stream-K split: 528 forward
  // tiles at B = 4096/view are 2 rounds + 16 diagonal tiles. fp8 launches and short K (< 4
  // K-steps: no K halves) keep the stream-K split of the remainder.
  const int nstrip = fwd_diag_remainder(ntiles, nk_tile, cus, diag_tail, f8);
  // kDiagTickets arrival tickets per tile in the counter region (sized for any remainder below
  // num_cus), 10 KS piece partials per tile in the slab region and [4 row groups][4 slots][64 rows]
  // float2 row-group partials per tile (8 KiB) in the column-partial area (diag_up_kernel's
  // scratch; the area holds num_cus x kSkColpTile float2): every remainder of a whole-round launch fits
  NTXENT_CHECK((size_t)kDiagTickets * nstrip * 4 <= sk_counter_bytes(ws.num_cus) &&
                   (size_t)10 * kDiagKS * nstrip * 4096 <= (size_t)2 * ws.num_cus * kTileElems &&
                   (size_t)nstrip * dev::kDiagScratchTile * sizeof(float2) <=
                       (size_t)ws.num_cus * dev::kSkColpTile * sizeof(float2),
               "diagonal remainder: workspace too small");
  const int nmain = ntiles - nstrip;
  const int pieces = part_x == nullptr ? fwd_splitk_pieces(ntiles, nk_tile, cus, diag_tail) : 0;
  int grid;
  if (pieces > 0) {
    // split-K: tile-aligned pieces, piece-major over the blocks (the XCD-contiguous block runs
    // then stream one K range of every row panel together: L2 reuse across the tiles,
    // profiles/r3/splitk_pm); every piece publishes its slab, sk_reduce_kernel finishes the tiles
    NTXENT_CHECK(kb % kKStepBytes == 0, "K not aligned to the K step");
    p.nk = nk_tile;
    p.dp_tiles = 0;
    p.sk_tiles = ntiles;
    p.ipb = (nk_tile + pieces - 1) / pieces;
    p.sk_cnt = static_cast<int*>(ws.ptr);
    p.sk_slabs = reinterpret_cast<float*>(static_cast<char*>(ws.ptr) + sk_counter_bytes(ws.num_cus));
    p.splitk = 1;
    grid = (int)((nk_tile + p.ipb - 1) / p.ipb) * ntiles;
    // fp16 partial tiles for 2-byte plans: the pieces are normalised-row dot products over a K
    // range (|x| <= 1), summed in fp32 by the reduce; the kept cosines are 2-byte anyway
    p.sk_half = (comp == DType::F16 || comp == DType::BF16) ? 1 : 0;
    NTXENT_CHECK(grid <= ws.num_cus && ws.ptr != nullptr && ws.bytes >= gemm_workspace_bytes(ntiles, ws.num_cus),
                 "split-K forward: workspace too small");
  } else {
    grid = apply_schedule(p, nmain, ws, stream);
  }
  // operand type: the plan's, or for raw bf16 rows on an fp16 plan bf16 operands with fp16 kept
  // cosines (dev::bf16r)
  auto dispatch_fwd = [&](auto&& f) {
    if (raw && raw->in == DType::BF16 && comp == DType::F16) f(dev::bf16r{});
    else dispatch_gemm(comp, f);
  };
  dispatch_fwd([&](auto tc) {
    using Tc = decltype(tc);
    launch_sim_gemm<Tc, dev::kModeFwd>(grid, p, stream);
    if (pieces > 0) {
      using TS = typename dev::StoreT<Tc>::type;
      float2* colp = reinterpret_cast<float2*>(static_cast<char*>(ws.ptr) + sk_counter_bytes(ws.num_cus) +
                                               (size_t)2 * ws.num_cus * kTileElems * sizeof(float));
      // (Z^T of the raw rows beside this reduce as side blocks: config 4 forward +3.5 us, the
      // reduce slowed by more than the LSE launch's transpose costs: profiles/r6/README.md)
      if (p.fixed_shift) hipLaunchKernelGGL((dev::sk_reduce_kernel<TS, 1>), dim3(ntiles * 16), dim3(256), 0, stream, p, colp);
      else hipLaunchKernelGGL((dev::sk_reduce_kernel<TS, 0>), dim3(ntiles * 16), dim3(256), 0, stream, p, colp);
    }
    if (main_done) NTXENT_HIP_CHECK(hipEventRecord(main_done, stream));
    if constexpr (!std::is_same<Tc, dev::fp8e4m3>::value) {
      if (nstrip > 0) {
        NTXENT_CHECK(p.A.kblk_stride == 0 && p.B.kblk_stride == 0, "diagonal remainder: row-major operands only");
        dev::SimParams q = p;
        q.tiles = tiles + nmain;
        if (q.sc) q.sc += (size_t)nmain * kTileElems * sizeof(typename dev::StoreT<Tc>::type);
        q.sk_cnt = static_cast<int*>(ws.ptr);
        q.sk_slabs = reinterpret_cast<float*>(static_cast<char*>(ws.ptr) + sk_counter_bytes(ws.num_cus));
        // row-group partials in the column-partial area of the workspace
        float2* scratch = reinterpret_cast<float2*>(static_cast<char*>(ws.ptr) + sk_counter_bytes(ws.num_cus) +
                                                    (size_t)2 * ws.num_cus * kTileElems * sizeof(float));
        const int nup = nstrip * (diag_ks(nk_tile) == 2 ? dev::diag_up_blocks<2>() : dev::diag_up_blocks<1>());
#if NTXENT_TIMING
        static TimingBuf tb;
        q.tstamp = tb.prepare(nup, stream);
#endif
        // While a transfer is in flight (ws.sched_cus < num_cus) the region blocks are capped to
        // the CUs the schedule leaves to compute and walk the regions (diag_up_kernel: nupg); the
        // plain launch is one block per region
        const int nupg = cus < ws.num_cus ? std::min(nup, cus) : nup;
        // the LSE launch folded into this one (LseFold): the remainder = the diagonal tiles of
        // exactly the second half of the rows, Z^T beside it, raw rows (world 1, R = Rpad)
        dev::LseFold lf{};
        const int nhalf = g.rows / 2;
        // (the launch is build_fwd_tiles' whole own block: its diagonal tiles come last, in panel
        // order, so the remainder is panels [rt - nstrip, rt))
        if (raw && raw->lse2 && raw->zqt && raw->fold_pre && raw->fold_cnt && lse_fold_enabled() && nup <= ws.num_cus &&
            g.world == 1 &&
            g.rows == g.rows_pad && nhalf % kTile == 0 && nstrip * kTile == nhalf && diag_tail == g.row_tiles &&
            ntiles == count_own_fwd_tiles(g)) {
          {
            lf.on = 1;
            lf.n = nhalf;
            lf.ngroups = nstrip * 4;
            lf.ypos = raw->ypos;
            lf.lse2 = raw->lse2;
            lf.cpos = raw->cpos;
            lf.ticket = reinterpret_cast<unsigned long long*>(raw->block_loss + 2);
            lf.loss = raw->loss;
            lf.pre = raw->fold_pre;
            lf.gcnt = raw->fold_cnt;
            lf.loss_scale = (float)(1.0 / (double)g.global_rows);
            lf.loss_fx = lse_loss_fx(g, lf.ngroups);
            NTXENT_CHECK(lf.loss_fx > 0.0, "lse fold: ticket scale");
          }
        }
        auto launch_up = [&](auto side, int nside) {
          using S = decltype(side);
          const dim3 sg(nupg + nside);
          if (diag_ks(nk_tile) == 2) {
            if (p.fixed_shift) hipLaunchKernelGGL((dev::diag_up_kernel<Tc, 1, 2, S>), sg, dim3(256), 0, stream, q, scratch, side, nupg, lf);
            else hipLaunchKernelGGL((dev::diag_up_kernel<Tc, 0, 2, S>), sg, dim3(256), 0, stream, q, scratch, side, nupg, lf);
          } else {
            if (p.fixed_shift) hipLaunchKernelGGL((dev::diag_up_kernel<Tc, 1, 1, S>), sg, dim3(256), 0, stream, q, scratch, side, nupg, lf);
            else hipLaunchKernelGGL((dev::diag_up_kernel<Tc, 0, 1, S>), sg, dim3(256), 0, stream, q, scratch, side, nupg, lf);
          }
        };
        using TS = typename dev::StoreT<Tc>::type;
        bool side_zt = false;
        if constexpr (sizeof(TS) == 2) {
          if (raw && raw->zqt && nup <= ws.num_cus) {
            // Z^T beside the remainder (the LSE launch then only merges): 2 side blocks per CU next
            // to its one block per CU (3 blocks of its ~50 KiB LDS fit a CU). Only when the
            // remainder is at most one block per CU: with more (config 5: 320 blocks) the side
            // blocks hold the slots its second wave needs (+5 us against the LSE launch's transpose)
            using Ts = typename std::conditional<std::is_same<Tc, dev::bf16r>::value, __bf16, Tc>::type;
            NTXENT_CHECK(raw->zt == (std::is_same<TS, __bf16>::value ? DType::BF16 : DType::F16) && g.dim_n % 64 == 0,
                         "fwd_stats: Z^T dtype must be the plan's backward dtype");
            dev::DiagSideZt<TS, Ts> zs;
            zs.nup = nup;
            zs.h = static_cast<const Ts*>(raw->h);
            zs.zqt = static_cast<TS*>(raw->zqt);
            zs.inv = raw->inv;
            zs.dk = g.dim;
            zs.ldt = (int)g.ld_t;
            zs.tx = g.rows_pad / 64;
            zs.ntiles = zs.tx * (g.dim_n / 64);  // (rows [dim, dim_n) of Z^T: zeros)
            const int nside = std::min(zs.ntiles, NTXENT_ZT_SIDE_PER_CU * ws.num_cus);
            if (nside < lf.ngroups) lf.on = 0;  // (every group needs its pre-merging side block)
            launch_up(zs, nside);
            side_zt = true;
          }
        }
        if (!side_zt) {
          lf.on = 0;  // (the LSE launch still runs: it writes Z^T)
          launch_up(dev::NoSide{nup}, 0);
        }
        zt_done = side_zt;
        if (raw) raw->lse_folded = side_zt && lf.on;
#if NTXENT_TIMING
        tb.dump("diag_up", nup, stream);
#endif
      }
    }
  });
  NTXENT_HIP_CHECK(hipGetLastError());
  return zt_done;
}

void launch_coef_gemm(DType comp, const void* zq_local, const void* zq_all, void* cbuf,
                      const float* lse2_all, const float* cpos, const int4* tiles, int ntiles,
                      const GemmWorkspace& ws, const Geometry& g, hipStream_t stream, const BlockView& bv,
                      float* dotp) {
  if (ntiles == 0) return;
  const bool f8 = comp == DType::FP8;  // fp8: K = dim_k8 bytes of rows ld_k8 bytes apart
  const long long kb = f8 ? (long long)g.dim_k8 : (long long)g.dim_k * dtype_size(comp);
  const long long ld = f8 ? (long long)g.ld_k8 : (long long)g.ld_k * dtype_size(comp);
  dev::SimParams p = base_params(g);
  set_operand_scales(p, comp, g);
  p.A = rowmajor_operand(zq_local, ld, kb);
  p.B = rowmajor_operand(zq_all, ld, kb);
  p.tiles = tiles;
  p.kbytes = kb;
  p.cbuf = static_cast<char*>(cbuf);
  p.lse2 = lse2_all;
  p.cpos = cpos;
  p.dotp = dotp;
  p.b_tile0 = bv.b_tile0;
  if (bv.c_ld > 0) p.c_ld = bv.c_ld;
  p.c_tile0 = bv.c_tile0;
  const int grid = apply_schedule(p, ntiles, ws, stream);
  dispatch_gemm(comp, [&](auto tc) {
    using Tc = decltype(tc);
    launch_sim_gemm<Tc, dev::kModeCoef>(grid, p, stream);
  });
  NTXENT_HIP_CHECK(hipGetLastError());
}

static int lse_blocks(const Geometry& g) { return ((g.rows_pad - g.rows / 2) * dev::kLseLanes + 255) / 256; }

int lse_scratch_floats(const Geometry& g) { return 64 + 2 * lse_blocks(g); }  // counter slot + partials (sum, min)

// Fixed-point scale of the LSE launch's loss ticket (lse_block): 2^F units per nat with the whole
// sum below 2^40 units. Every loss term is softplus(lse_neg - y_pos) <= log(2N) + 2 / tau + 1
// (unit rows: logits within +-1/tau), so F = 39 - ceil(log2(R * that)); 0 (the float partials
// and their reload) when nb exceeds the ticket's 12-bit arrival count.
static double lse_loss_fx(const Geometry& g, int nb) {
  if (nb >= 4095) return 0.0;
  const double bound = (double)g.rows * (std::log(2.0 * (double)g.global_rows) + 2.0 / g.temperature + 1.0) + 64.0;
  const int F = 39 - (int)std::ceil(std::log2(bound));
  return std::ldexp(1.0, F);
}

void launch_lse(const float2* part, const float* ypos, float* lse2_all, float* cpos, float* block_loss,
                float* loss_sum, const Geometry& g, hipStream_t stream, DType tr_dtype, const void* zq, void* zqt,
                const Q8Stats* q8, const RawRows* raw) {
  const int nb = lse_blocks(g);  // one workgroup per 32 pairs / pad rows
  dev::LseArgs a{part, ypos, lse2_all, cpos, block_loss, loss_sum, (float)(1.0 / (double)g.global_rows),
                 g.rows, g.rows_pad, g.col_tiles, g.rank * g.rows_pad};
  if (q8) {
    a.mneg2 = q8->mneg2;
    a.lmin = q8->lmin;
  }
  a.loss_fx = lse_loss_fx(g, nb);
  if (raw) {  // Z^T = (h * inv)^T straight from the input rows (raw-operand forward)
    NTXENT_CHECK(zqt != nullptr && q8 == nullptr && raw->inv && (tr_dtype == DType::F16 || tr_dtype == DType::BF16) &&
                     g.rows == g.rows_pad && g.dim == g.dim_k, "lse (raw rows): 2-byte Z^T, rows % 256 == 0, dim % 64 == 0");
    const int tx = g.rows_pad / 64, ty = g.dim_n / 64;
    dispatch_comp(tr_dtype, [&](auto tc) {
      using Tc = decltype(tc);
      auto go = [&](auto ts) {
        using Ts = decltype(ts);
        hipLaunchKernelGGL((dev::lse_transpose_kernel<Tc, false, Ts>), dim3(nb + tx * ty), dim3(256), 0, stream, a, nb,
                           static_cast<const Ts*>(raw->h), zqt, g.dim, g.dim, g.ld_t, tx, raw->inv);
      };
      if constexpr (sizeof(Tc) == 2) {
        if (raw->in == DType::BF16) go(__bf16{});
        else go(_Float16{});
      }
    });
  } else if (zq == nullptr) {
    hipLaunchKernelGGL(dev::lse_kernel, dim3(nb), dim3(256), 0, stream, a);
  } else if (q8 && q8->zq8t) {
    NTXENT_CHECK(tr_dtype == DType::F16 && g.world == 1, "lse: the fp8 backward transposes fp16 rows (world 1)");
    const int tx = g.rows_pad / 64, ty = g.dim_n / 64;
    hipLaunchKernelGGL((dev::lse_transpose_kernel<_Float16, true>), dim3(nb + tx * ty), dim3(256), 0, stream, a, nb,
                       static_cast<const _Float16*>(zq), q8->zq8t, g.dim_k, g.ld_k, q8_ldt(g), tx);
  } else {
    NTXENT_CHECK(zqt != nullptr, "lse: transpose output missing");
    const int tx = g.rows_pad / 64, ty = g.dim_n / 64;
    dispatch_comp(tr_dtype, [&](auto tc) {
      using Tc = decltype(tc);
      hipLaunchKernelGGL((dev::lse_transpose_kernel<Tc>), dim3(nb + tx * ty), dim3(256), 0, stream, a, nb,
                         static_cast<const Tc*>(zq), zqt, g.dim_k, g.ld_k, g.ld_t, tx);
    });
  }
  NTXENT_HIP_CHECK(hipGetLastError());
}

void launch_coef(DType comp, const void* sbuf, void* cbuf, const float* lse2_all, const float* cpos,
                 const int4* tiles, int ntiles, const Geometry& g, hipStream_t stream,
                 void* mbuf, float* dotp, const Q8Stats* q8, bool half_c) {
  if (ntiles == 0) return;
  dev::SimParams p = base_params(g);
  NTXENT_CHECK(!half_c || (mbuf == nullptr && q8 == nullptr && g.world == 1 && (comp == DType::F16 || comp == DType::BF16)),
               "coef: half C needs a 16-bit, single-rank, mirrored-layout pass");
  p.c_half = half_c ? 1 : 0;
  p.dotp = dotp;
  p.tiles = tiles;
  p.sc = const_cast<char*>(static_cast<const char*>(sbuf));
  p.cbuf = static_cast<char*>(cbuf);
  p.mbuf = static_cast<char*>(mbuf);
  if (mbuf != nullptr) {  // symmetric mode: compact cbuf (sym_c_ld)
    p.c_ld = sym_c_ld(g);
    p.c_rot = 1;
  }
  p.lse2 = lse2_all;
  p.cpos = cpos;
  if (q8) {
    NTXENT_CHECK(comp == DType::F16 && mbuf == nullptr && g.world == 1,
                 "coef (fp8 backward): fp16 kept cosines, world 1, mirrored layout");
    p.q8_mneg = q8->mneg2;
    p.q8_lmin = q8->lmin;
    hipLaunchKernelGGL((dev::coef_kernel<_Float16, true>), dim3(16 * ntiles), dim3(64), 0, stream, p);
    NTXENT_HIP_CHECK(hipGetLastError());
    return;
  }
  dispatch_comp(comp, [&](auto tc) {
    using Tc = decltype(tc);
    hipLaunchKernelGGL((dev::coef_kernel<Tc>), dim3(16 * ntiles), dim3(64), 0, stream, p);
  });
  NTXENT_HIP_CHECK(hipGetLastError());
}

int dot_slots(const Geometry& g) { return 4 * g.col_tiles; }

void launch_dot_reduce(const float* dotp, float* dot, const Geometry& g, hipStream_t stream) {
  hipLaunchKernelGGL(dev::dot_reduce_kernel, dim3((g.rows_pad + 31) / 32), dim3(256), 0, stream, dotp, dot_slots(g),
                     g.rows_pad, dot);
  NTXENT_HIP_CHECK(hipGetLastError());
}

// Fused normalisation backward in the dZ epilogue (dz_store), or for split-K pieces in the reduce
// launch (sk_dz_reduce_kernel): rows must be whole 16-byte chunks.
static bool apply_norm_fuse(dev::SimParams& p, const NormFuse* nf, const Geometry& g) {
  if (nf == nullptr || nf->dh == nullptr || g.dim % 8 != 0) return false;
  p.nh = nf->h;
  p.nh_dt = nf->in == DType::F32 ? 0 : (nf->in == DType::F16 ? 1 : 2);
  p.nd = g.dim;
  p.ninv = nf->inv;
  p.ndot = nf->dot;
  p.ngo = nf->grad_out;
  p.nalpha = (float)(1.0 / ((double)g.global_rows * g.temperature));
  p.ndh = nf->dh;
  p.out_f16 = 1;
  p.accum = 0;
  return true;
}

bool launch_dz(DType comp, const void* sc, const void* zqt_all, const int4* tiles, int ntiles,
               void* slabs, const GemmWorkspace& ws, const Geometry& g, hipStream_t stream, bool out_f16,
               const NormFuse* nf, const Q8Stats* q8, const float* cpos, bool half_c) {
  if (ntiles == 0) return false;
  NTXENT_CHECK(!half_c || dz_half_c_eligible(comp, g, ntiles, ws), "dz: half C not eligible for this launch");
  const bool f8 = comp == DType::FP8;
  NTXENT_CHECK(!f8 || (q8 && q8->mneg2 && q8->lmin && q8->zq && cpos && g.world == 1 && out_f16),
               "dz (fp8 backward): Q8Stats, cpos, world 1 and an fp16 slab required");
  const long long cs = (long long)dtype_size(comp);
  dev::SimParams p = base_params(g);
  if (f8) {
    p.q8_mneg = q8->mneg2;
    p.q8_lmin = q8->lmin;
    p.q8_zq = static_cast<const _Float16*>(q8->zq);
    p.q8_ldz = g.ld_k;
    p.cpos = cpos;
  }
  // A = C, tile-blocked (coef_tile_operand)
  p.A = coef_tile_operand(sc, g.col_tiles, cs);
  // B = ZqT_all [W][dim_n][ld_t]: rows = embedding dims, K = global columns, one K block per rank.
  p.B.base = static_cast<const char*>(zqt_all);
  const long long ldt = f8 ? q8_ldt(g) : g.ld_t;
  p.B.ld = ldt * cs;
  p.B.row_tile_stride = (long long)kTile * ldt * cs;
  p.B.kblk = (long long)g.rows_pad * cs;
  p.B.kblk_stride = (long long)g.dim_n * ldt * cs;
  p.tiles = tiles;
  p.kbytes = (long long)g.world * g.rows_pad * cs;
  p.out = static_cast<float*>(slabs);
  p.out_f16 = out_f16 ? 1 : 0;
  p.ldo = g.dim_n;
  p.slab_stride = (long long)g.rows_pad * g.dim_n;
  // tile-starved (d <= 1024 at 8192 rows): split-K pieces + a parallel reduce instead of the
  // stream-K schedule's serial last-arriver fixup (same rule as the forward's)
  const int cus = ws.sched_cus > 0 ? std::min(ws.sched_cus, ws.num_cus) : ws.num_cus;
  const int nk = (int)(p.kbytes / kKStepBytes);
  int pieces = fwd_splitk_pieces(ntiles, nk, cus, 1);
  if (pieces < 3 || f8) pieces = 0;  // 2 pieces: the reduce launch costs more than the fixup it replaces
  // (fp8: the finishing block's dequantisation lives in the GEMM epilogue, not the reduce)
  int grid;
  if (pieces > 0) {
    p.nk = nk;
    p.dp_tiles = 0;
    p.sk_tiles = ntiles;
    p.ipb = (nk + pieces - 1) / pieces;
    p.sk_cnt = static_cast<int*>(ws.ptr);
    p.sk_slabs = reinterpret_cast<float*>(static_cast<char*>(ws.ptr) + sk_counter_bytes(ws.num_cus));
    // piece-major, as the forward's: an XCD streams one K range of every panel. fp32 slabs (fp16
    // ones measured -3 us at config 2 but moved dZ by ~2e-3 of max|g|: profiles/r3/skhalf)
    p.splitk = 1;
    grid = (int)((nk + p.ipb - 1) / p.ipb) * ntiles;
    NTXENT_CHECK(p.kbytes % kKStepBytes == 0 && grid <= ws.num_cus && ws.ptr != nullptr &&
                     ws.bytes >= gemm_workspace_bytes(ntiles, ws.num_cus),
                 "split-K dZ: workspace too small");
  } else {
    grid = apply_schedule(p, ntiles, ws, stream);
  }
  if (half_c)
    NTXENT_CHECK(((pieces == 0 && p.sk_tiles == 0 && p.dp_tiles == ntiles) || (pieces > 0 && p.ipb % 2 == 0)) &&
                     (long long)g.row_tiles * g.col_tiles * kTileElems * cs < (1ll << 31),
                 "dz: half C needs items starting at even K-steps and a C buffer below 2 GiB (32-bit offsets)");
  p.c_half = half_c ? 1 : 0;
  const bool fused = comp != DType::F32 && apply_norm_fuse(p, nf, g);
  if (fused) NTXENT_CHECK(nf->dot != nullptr, "dz: fused normalisation backward without dot");
  if (nf && nf->dot_cnt) {
    // dot reduce folded in (dz_dot_fold): the grid sums nf->dotp into nf->dot itself
    NTXENT_CHECK(fused && !f8 && nf->dotp && dz_dot_fold_eligible(comp, g, ntiles, ws),
                 "dz: dot fold needs the fused 16-bit epilogue");
    p.dotp = const_cast<float*>(nf->dotp);
    p.dot_nslot = dot_slots(g);
    p.dot_cnt = pieces == 0 ? nf->dot_cnt : nullptr;  // split-K: the reduce launch reads dot
    p.dot_spin = dot_fold_spin();
  }
  dispatch_gemm(comp, [&](auto tc) {
    using Tc = decltype(tc);
    launch_sim_gemm<Tc, dev::kModeDz>(grid, p, stream);
  });
  if (pieces > 0) hipLaunchKernelGGL(dev::sk_dz_reduce_kernel, dim3(ntiles * 64), dim3(256), 0, stream, p);
  NTXENT_HIP_CHECK(hipGetLastError());
  return fused;
}

void launch_dz_view(DType comp, const void* a, long long a_panel_tiles, const void* b, long long b_kblk_cols,
                    long long b_kblk_stride, int k_tiles, const int4* tiles, int ntiles, void* out, bool accum,
                    const GemmWorkspace& ws, const Geometry& g, hipStream_t stream, bool out_f16) {
  NTXENT_CHECK(!(accum && out_f16), "dz_view: fp16 output cannot accumulate");
  if (ntiles == 0 || k_tiles == 0) return;
  NTXENT_CHECK(k_tiles > 0 && a_panel_tiles >= k_tiles, "dz_view: bad K extent");
  const long long cs = (long long)dtype_size(comp);
  dev::SimParams p = base_params(g);
  p.A = coef_tile_operand(a, a_panel_tiles, cs);
  // B: K blocks of transposed rows (rows = embedding dims, ld_t apart), one block per rank
  NTXENT_CHECK(b_kblk_cols > 0 && b_kblk_cols % kTile == 0, "dz_view: bad B K block");
  p.B.base = static_cast<const char*>(b);
  p.B.ld = (long long)g.ld_t * cs;
  p.B.row_tile_stride = (long long)kTile * g.ld_t * cs;
  p.B.kblk = b_kblk_cols * cs;
  p.B.kblk_stride = b_kblk_stride * cs;
  p.tiles = tiles;
  p.kbytes = (long long)k_tiles * kTile * cs;
  p.out = static_cast<float*>(out);
  p.ldo = g.dim_n;
  p.slab_stride = (long long)g.rows_pad * g.dim_n;
  p.accum = accum ? 1 : 0;
  p.out_f16 = out_f16 ? 1 : 0;
  const int grid = apply_schedule(p, ntiles, ws, stream);
  dispatch_comp(comp, [&](auto tc) {
    using Tc = decltype(tc);
    launch_sim_gemm<Tc, dev::kModeDz>(grid, p, stream);
  });
  NTXENT_HIP_CHECK(hipGetLastError());
}

void launch_norm_bwd(DType in, const float* slabs, int nslabs, const void* h, const float* inv,
                     const float* grad_out, void* dh, const Geometry& g, hipStream_t stream,
                     const void* xslabs, int nx) {
  const _Float16* xs = static_cast<const _Float16*>(xslabs);
  if (xs == nullptr) nx = 0;
  const float alpha_base = (float)(1.0 / ((double)g.global_rows * g.temperature));
  const long long ss = (long long)g.rows_pad * g.dim_n, ldo = g.dim_n;
  const int nch = (g.dim + 2047) / 2048;  // 8-element chunks per thread
  const bool vec = (g.dim % 8) == 0 && nch <= 4;
  dispatch_comp(in, [&](auto tin) {
    using Tin = decltype(tin);
    const Tin* hp = static_cast<const Tin*>(h);
    Tin* dp = static_cast<Tin*>(dh);
    if (vec && nch == 1)
      hipLaunchKernelGGL((dev::norm_bwd_vec_kernel<Tin, 1>), dim3(g.rows), dim3(256), 0, stream, slabs, nslabs, ss,
                         ldo, hp, inv, grad_out, alpha_base, dp, g.dim, xs, nx);
    else if (vec && nch == 2)
      hipLaunchKernelGGL((dev::norm_bwd_vec_kernel<Tin, 2>), dim3(g.rows), dim3(256), 0, stream, slabs, nslabs, ss,
                         ldo, hp, inv, grad_out, alpha_base, dp, g.dim, xs, nx);
    else if (vec)
      hipLaunchKernelGGL((dev::norm_bwd_vec_kernel<Tin, 4>), dim3(g.rows), dim3(256), 0, stream, slabs, nslabs, ss,
                         ldo, hp, inv, grad_out, alpha_base, dp, g.dim, xs, nx);
    else
      hipLaunchKernelGGL((dev::norm_bwd_kernel<Tin>), dim3(g.rows), dim3(256), 0, stream, slabs, nslabs, ss, ldo,
                         hp, inv, grad_out, alpha_base, dp, g.dim, xs, nx);
  });
  NTXENT_HIP_CHECK(hipGetLastError());
}

// ---- device utilities ------------------------------------------------------------------
const DeviceInfo& device_info(int device) {
  static std::mutex mu;
  static std::unordered_map<int, DeviceInfo> cache;
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(device);
  if (it != cache.end()) return it->second;
  hipDeviceProp_t prop;
  NTXENT_HIP_CHECK(hipGetDeviceProperties(&prop, device));
  DeviceInfo d;
  d.device = device;
  d.num_cus = prop.multiProcessorCount;
  d.lds_per_block = (int)prop.sharedMemPerBlock;
  d.warp_size = prop.warpSize;
  d.arch = prop.gcnArchName;
  d.is_gfx950 = d.arch.rfind("gfx950", 0) == 0;
  return cache.emplace(device, d).first->second;
}

bool check_matrix_core_support(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device >= n) return false;
  return device_info(device).is_gfx950;
}

int get_optimal_block_size(int rows) {
  // Row kernels use one 256-thread (4 x wave64) block per row pair; GEMM tiles use 512.
  return rows >= kTile ? kGemmThreads : 256;
}

}  // namespace ntxent

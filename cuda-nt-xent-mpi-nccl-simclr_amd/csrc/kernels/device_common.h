// Device helpers for the gfx950 NT-Xent kernels: vector types, MFMA wrappers, wave64
// reductions (DPP row ops, no 32-lane masks — cf. the reference's WARP_SIZE=32 and
// 0xffffffff shuffles at src/ntxent_kernel.cu:17-18,31), dtype conversions.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ntxent {
namespace dev {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf168 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int kNumXcdDev = 8;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kNegInf = -__builtin_huge_valf();
constexpr float kPosInf = __builtin_huge_valf();

// ---- dtype conversion --------------------------------------------------------------
template <typename T> __device__ __forceinline__ float to_f32(T x);
template <> __device__ __forceinline__ float to_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ float to_f32<_Float16>(_Float16 x) { return (float)x; }
template <> __device__ __forceinline__ float to_f32<__bf16>(__bf16 x) { return (float)x; }

template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ _Float16 from_f32<_Float16>(float x) { return (_Float16)x; }
template <> __device__ __forceinline__ __bf16 from_f32<__bf16>(float x) { return (__bf16)x; }

// ---- MFMA: one 16-byte K-chunk per lane per operand ----------------------------------
// 16x16x32 f16/bf16: lane l holds A[row l&15][k 8(l>>4)..+7], B[k ...][col l&15];
// C/D: col = l&15, row = 4(l>>4) + reg.
// f32: the same 16-byte chunk (4 consecutive k) drives four 16x16x4 MFMAs; A and B use the
// identical k permutation so the contraction is exact.
template <typename T> struct Mfma;
template <> struct Mfma<_Float16> {
  typedef half8 frag;
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mfma<__bf16> {
  typedef bf168 frag;
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mfma<float> {
  typedef f32x4 frag;
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
    return c;
  }
};

// fp8 e4m3 (OCP, gfx950) operand type: the 128-byte K-step of a row holds 128 elements and runs
// on the CDNA4 block-scaled MFMA v_mfma_scale_f32_16x16x128_f8f6f4 (twice the fp16/bf16 and the
// legacy 16x16x32 fp8 rate). One MFMA per (row block, column block) and K-step: lane l's 32-byte
// operand is the concatenation of its two 16-byte chunks (k-substeps s = 0, 1), i.e. chunks
// {cq, cq + 4} of the K-step for lane group cq = l >> 4 — a fixed permutation of the 128 k
// positions, the same for A and B, so the dot product is exact.
// Scales: every row of Zq8 is quantised with its own power of two 2^e (e4m3(z * 2^e), amax of
// the row mapped into [224, 448]) and carries the E8M0 byte 127 - e; the MFMA applies
// 2^(sa - 127) * 2^(sb - 127), so the accumulator is the unscaled dot product. A lane passes
// the scale of its A row (l & 15 of the row block) and of its B row (= output column).
struct fp8e4m3 {
  unsigned char v;
};
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
template <> struct Mfma<fp8e4m3> {
  typedef u32x4 frag;  // 16 bytes of one k-substep; the MFMA itself: mma_mx_sel in sim_gemm.h
};

// Element type used to store cosines / coefficients produced from a GEMM in operand type T
// (fp8 GEMMs keep their outputs in fp16: the backward runs in fp16).
template <typename T> struct StoreT { typedef T type; };
template <> struct StoreT<fp8e4m3> { typedef _Float16 type; };
// Raw-operand forward on bf16 input rows (the input h itself, normalised in the epilogue): bf16
// MFMA operands, cosines kept in fp16 for the fp16 backward.
struct bf16r {};
template <> struct Mfma<bf16r> : Mfma<__bf16> {};
template <> struct StoreT<bf16r> { typedef _Float16 type; };

// E8M0 byte -> 2^(byte - 127) as fp32 (bytes 1..254: normal powers of two).
__device__ __forceinline__ float e8m0_to_f32(unsigned char b) { return __int_as_float((int)b << 23); }

// Per-row fp8 scale exponent: the largest e with amax * 2^e <= 448 (e4m3 max), clamped to
// [0, 126]; the row's E8M0 scale byte is 127 - e. amax = 0 (a zero / pad row) gives e = 126.
__device__ __forceinline__ int fp8_row_exp(float amax) {
  if (!(amax > 0.f)) return 126;
  const float r = 448.0f / amax;
  const int e = ((__float_as_int(r) >> 23) & 0xff) - 127;  // floor(log2 r) for normal r
  return e < 0 ? 0 : (e > 126 ? 126 : e);
}

// ---- wave64 cross-lane reductions ----------------------------------------------------
// DPP row_ror within a 16-lane row: 0x120 + n. bound_ctrl set (no lane of a rotation is out of
// bounds, so results are unchanged): lets hipcc fold the move into the consuming add / max
// (v_add_f32_dpp: one instruction per reduction step instead of a v_mov_b32_dpp + v_add pair).
template <int CTRL> __device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, true));
}
// Reduce across the 16 lanes of a DPP row (lanes sharing l>>4): every lane gets the result.
__device__ __forceinline__ float row16_max(float x) {
  x = fmaxf(x, dpp_f<0x128>(x));
  x = fmaxf(x, dpp_f<0x124>(x));
  x = fmaxf(x, dpp_f<0x122>(x));
  x = fmaxf(x, dpp_f<0x121>(x));
  return x;
}
__device__ __forceinline__ float row16_sum(float x) {
  x += dpp_f<0x128>(x);
  x += dpp_f<0x124>(x);
  x += dpp_f<0x122>(x);
  x += dpp_f<0x121>(x);
  return x;
}
// Four rows' sums over the 16 lanes of a DPP row at once: x[r] holds this lane's part of row r;
// returns the total of row (lane >> 2) & 3 (a transposing reduction: each exchange halves the
// rows a lane carries, 5 DPP adds + 6 selects instead of 4 x 4 DPP adds). Partners: lane ^ 8
// (row_ror:8), the half-row mirror (lane ^ 7 within 8), then ^ 1 and ^ 2 (quad_perm).
__device__ __forceinline__ float row16_sum4t(const float (&x)[4], int lane) {
  const bool b3 = (lane & 8) != 0, b2 = (lane & 4) != 0;
  float ka = b3 ? x[2] : x[0], kb = b3 ? x[3] : x[1];  // rows kept: {0, 1} or {2, 3}
  const float sa = b3 ? x[0] : x[2], sb = b3 ? x[1] : x[3];  // the partner's rows
  ka += dpp_f<0x128>(sa);
  kb += dpp_f<0x128>(sb);
  float k = b2 ? kb : ka;
  k += dpp_f<0x141>(b2 ? ka : kb);  // row_half_mirror
  k += dpp_f<0xB1>(k);              // quad_perm [1, 0, 3, 2]
  k += dpp_f<0x4E>(k);              // quad_perm [2, 3, 0, 1]
  return k;
}
// Reduce across lanes l, l^16, l^32, l^48 (the 4 DPP rows).
__device__ __forceinline__ float xrow_max(float x) {
  x = fmaxf(x, __shfl_xor(x, 16, 64));
  x = fmaxf(x, __shfl_xor(x, 32, 64));
  return x;
}
__device__ __forceinline__ float xrow_sum(float x) {
  x += __shfl_xor(x, 16, 64);
  x += __shfl_xor(x, 32, 64);
  return x;
}
__device__ __forceinline__ float wave_sum(float x) {
  x = row16_sum(x);
  return xrow_sum(x);
}

// Untracked LDS accesses (inline asm; byte address in LDS). hipcc waits vmcnt(0) for every
// in-flight LDS-DMA before a compiler-visible LDS access, whatever its address; a kernel that
// keeps DMA in flight across an epilogue uses these for regions the DMA never writes, and waits
// lgkmcnt itself (the reads below return only after their own wait).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void lds_put_f2(unsigned addr, f32x2 v) {
  asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(v) : "memory");
}
// untracked 4- and 16-byte LDS reads (usable while LDS-DMA is in flight: a compiler-tracked
// LDS access there makes hipcc wait vmcnt(0))
__device__ __forceinline__ float lds_get_f32(unsigned addr) {
  float v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}
__device__ __forceinline__ f32x4 lds_get_f32x4(unsigned addr) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}
// the raw-operand forward's inverse norms of one item (sim_gemm_kernel epilogue): 4 column
// values at cbase + {0, 64, 512, 576} and 4 row quads at rbase + {0, 64, 128, 192} + rofs, one
// wait for all eight reads (a wait per read exposed ~1 k cycles of LDS latency per tile)
template <int ROFS>
__device__ __forceinline__ void lds_get_inv(unsigned rbase, unsigned cbase, f32x4 (&rs)[4], float (&cs)[4]) {
  asm volatile(
      "ds_read_b128 %0, %8 offset:%c10\n\t"
      "ds_read_b128 %1, %8 offset:%c11\n\t"
      "ds_read_b128 %2, %8 offset:%c12\n\t"
      "ds_read_b128 %3, %8 offset:%c13\n\t"
      "ds_read_b32 %4, %9\n\t"
      "ds_read_b32 %5, %9 offset:64\n\t"
      "ds_read_b32 %6, %9 offset:512\n\t"
      "ds_read_b32 %7, %9 offset:576\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(rs[0]), "=&v"(rs[1]), "=&v"(rs[2]), "=&v"(rs[3]), "=&v"(cs[0]), "=&v"(cs[1]), "=&v"(cs[2]), "=&v"(cs[3])
      : "v"(rbase), "v"(cbase), "i"(ROFS), "i"(ROFS + 64), "i"(ROFS + 128), "i"(ROFS + 192)
      : "memory");
}
// row inverse norms only (the second row half of an item: the column norms are the first half's)
template <int ROFS>
__device__ __forceinline__ void lds_get_rinv(unsigned rbase, f32x4 (&rs)[4]) {
  asm volatile(
      "ds_read_b128 %0, %4 offset:%c5\n\t"
      "ds_read_b128 %1, %4 offset:%c6\n\t"
      "ds_read_b128 %2, %4 offset:%c7\n\t"
      "ds_read_b128 %3, %4 offset:%c8\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(rs[0]), "=&v"(rs[1]), "=&v"(rs[2]), "=&v"(rs[3])
      : "v"(rbase), "i"(ROFS), "i"(ROFS + 64), "i"(ROFS + 128), "i"(ROFS + 192)
      : "memory");
}
// fp8 operand row scales of one item (sim_gemm_kernel): 8 A dwords at abase + {0, 64, 128, 192,
// 512, 576, 640, 704} and 4 B dwords at bbase + {0, 64, 512, 576}, one wait
__device__ __forceinline__ void lds_get_scales(unsigned abase, unsigned bbase, unsigned (&av)[8], unsigned (&bv)[4]) {
  asm volatile(
      "ds_read_b32 %0, %12\n\t"
      "ds_read_b32 %1, %12 offset:64\n\t"
      "ds_read_b32 %2, %12 offset:128\n\t"
      "ds_read_b32 %3, %12 offset:192\n\t"
      "ds_read_b32 %4, %12 offset:512\n\t"
      "ds_read_b32 %5, %12 offset:576\n\t"
      "ds_read_b32 %6, %12 offset:640\n\t"
      "ds_read_b32 %7, %12 offset:704\n\t"
      "ds_read_b32 %8, %13\n\t"
      "ds_read_b32 %9, %13 offset:64\n\t"
      "ds_read_b32 %10, %13 offset:512\n\t"
      "ds_read_b32 %11, %13 offset:576\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3]), "=&v"(av[4]), "=&v"(av[5]), "=&v"(av[6]),
        "=&v"(av[7]), "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(bv[2]), "=&v"(bv[3])
      : "v"(abase), "v"(bbase)
      : "memory");
}
// low bytes of four dwords packed into one (byte i = low byte of x[i])
__device__ __forceinline__ int pack_low_bytes(unsigned x0, unsigned x1, unsigned x2, unsigned x3) {
  return (int)((x0 & 0xffu) | ((x1 & 0xffu) << 8) | ((x2 & 0xffu) << 16) | ((x3 & 0xffu) << 24));
}
// four 8-byte reads at addr + {0, 1, 2, 3} * 2048
__device__ __forceinline__ void lds_get4_f2(unsigned addr, f32x2& a, f32x2& b, f32x2& c, f32x2& d) {
  asm volatile(
      "ds_read_b64 %0, %4\n\t"
      "ds_read_b64 %1, %4 offset:2048\n\t"
      "ds_read_b64 %2, %4 offset:4096\n\t"
      "ds_read_b64 %3, %4 offset:6144\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d)
      : "v"(addr)
      : "memory");
}
// two 8-byte reads at addr + {0, 2048}
__device__ __forceinline__ void lds_get2_f2(unsigned addr, f32x2& a, f32x2& b) {
  asm volatile(
      "ds_read_b64 %0, %2\n\t"
      "ds_read_b64 %1, %2 offset:2048\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(a), "=&v"(b)
      : "v"(addr)
      : "memory");
}

// Wave-uniform 16-byte load of a read-only table (written before the launch) through the scalar
// cache: counted by lgkmcnt, not vmcnt, so it neither waits for nor drains in-flight LDS-DMA
// (hipcc loads such a descriptor with a vector load and waits vmcnt(0) at its first use).
__device__ __forceinline__ int4 sload_int4(const int4* base, int idx) {
  typedef int i4s __attribute__((ext_vector_type(4)));
  i4s r;
  const int4* a = base + __builtin_amdgcn_readfirstlane(idx);
  asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(a) : "memory");
  return make_int4(r[0], r[1], r[2], r[3]);
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float fast_log2(float x) { return __builtin_amdgcn_logf(x); }

// Merge two (max, sum) online-softmax states in the log2 domain.
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == kNegInf) return;  // both empty
  s = s * fast_exp2(m - mn) + s2 * fast_exp2(m2 - mn);
  m = mn;
}

// fp8 backward: power-of-two scale 2^e of row i's coefficients in the e4m3 C matrix. Every
// negative coefficient C_ij = P_ij + P_ji is at most 2^(m_i - lse_i) + 2^(m_i - L) <= 2 * 2^(m_i - L)
// (m_i: row i's largest negative logit, L: the smallest LSE of any row, log2 units; y_ij = y_ji
// <= m_i), so C_ij * 2^e <= 448 (e4m3 max) with e = floor(log2(448 / 2) - (m_i - L)). The positive
// coefficient is not stored in e4m3 (the dZ epilogue adds C_ip z_p exactly). Empty / padded rows
// (m_i = -inf) and extreme rows are clamped.
__device__ __forceinline__ int q8_row_exp(float mneg2, float lmin) {
  const float e = floorf(7.807f - (mneg2 - lmin));
  return (int)fminf(fmaxf(e, -60.f), 60.f);
}
__device__ __forceinline__ float exp2i(int e) { return __int_as_float((e + 127) << 23); }  // |e| <= 126

// Row statistics from a row's merged negatives-only (max, sum) state: returns lse2 and writes
// the natural-log loss term softplus(lse_neg - y_pos) and a = 1 - P_ip = sigmoid(lse_neg - y_pos).
__device__ __forceinline__ float finish_row(float m, float s, float yp, float& loss, float& a) {
  const float neg2 = (m == kNegInf || s <= 0.f) ? kNegInf : m + log2f(s);
  const float mx = fmaxf(neg2, yp);  // lse = logaddexp(lse_neg, y_pos)
  const float l2 = mx + log2f(exp2f(neg2 - mx) + exp2f(yp - mx));
  const float x = (neg2 - yp) * kLn2;
  loss = x > 0.f ? x + log1pf(expf(-x)) : log1pf(expf(x));
  a = 1.0f / (1.0f + exp2f(yp - neg2));
  return l2;
}

// Block-wide sum for up to 1024 threads; `red` must hold >= 16 floats. All threads get it.
__device__ __forceinline__ float block_sum(float x, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  x = wave_sum(x);
  __syncthreads();
  if (lane == 0) red[w] = x;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];  // fixed order: deterministic
  return t;
}

// Three block sums with one pair of barriers (same contract as block_sum; red: 3 * 8 floats).
__device__ __forceinline__ void block_sum3(float& x, float& y, float& z, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  x = wave_sum(x);
  y = wave_sum(y);
  z = wave_sum(z);
  __syncthreads();
  if (lane == 0) { red[w] = x; red[8 + w] = y; red[16 + w] = z; }
  __syncthreads();
  x = y = z = 0.f;
  for (int i = 0; i < nw; ++i) { x += red[i]; y += red[8 + i]; z += red[16 + i]; }  // fixed order
}

// Block-wide max (same contract as block_sum).
__device__ __forceinline__ float block_max(float x, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  x = xrow_max(row16_max(x));
  __syncthreads();
  if (lane == 0) red[w] = x;
  __syncthreads();
  float t = red[0];
  for (int i = 1; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

// XCD-aware, bijective blockIdx remap: blocks that the dispatcher round-robins onto one
// XCD (b % 8) get a contiguous run of the tile list so neighbouring tiles share L2 panels
// (cdna_hip_programming.md §5.5 T1, bijective form).
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  if (nwg < 2 * kNumXcdDev) return b;
  const int q = nwg / kNumXcdDev, r = nwg % kNumXcdDev;
  const int xcd = b % kNumXcdDev, idx = b / kNumXcdDev;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace dev
}  // namespace ntxent

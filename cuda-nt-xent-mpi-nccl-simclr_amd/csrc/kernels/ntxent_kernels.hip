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

#include <algorithm>
#include <mutex>
#include <unordered_map>

namespace ntxent {
namespace dev {

enum SimMode : int { kModeFwd = 0, kModeCoef = 1, kModeDz = 2 };

constexpr int kStageBytes = 2 * kTile * kKStepBytes;  // A + B tile = 64 KiB
constexpr int kGemmLds = 2 * kStageBytes;             // double buffered = 128 KiB

struct OperandDesc {
  const char* base;            // bytes
  long long row_tile_stride;   // bytes between consecutive 256-row tiles
  long long ld;                // bytes between rows inside a tile
  long long kblk;              // K bytes per contiguous K block
  long long kblk_stride;       // bytes between K blocks
};

struct SimParams {
  OperandDesc A, B;
  const int4* tiles;
  long long kbytes;      // K bytes handled by one workgroup
  int R, Rpad, n_half, own0, row_tile0, col_tiles;
  float y_scale;         // inv_temp * log2(e)
  float2* part;          // [col_tiles][Rpad] partial (max, sum) in log2 units
  char* sc;              // tile-blocked cosine / coefficient buffer
  const float* lse2;     // [W*Rpad] lse in log2 units (all ranks)
  const float* ypos;     // [R] positive logit (log2 units, from the quantised rows)
  const float* lseneg2;  // [Rpad] log2-sum-exp2 over the NEGATIVES of each local row
  float* out;            // dZ slabs
  long long ldo;         // elements
  long long slab_stride; // elements
};

// ------------------------------------------------------------------------------------
// Coefficient epilogue shared by the store-mode coef kernel and the recompute GEMM:
// cos tile (MFMA C layout, rows = local rows of tile mt, cols = global cols of tile nt)
//   -> C_ij = 2^(y - lse2_i) + 2^(y - lse2_j) - 2[j == p(i)],  0 on the diagonal / padding
// written row-major into slot (mt, nt) and, for a mirrored tile, transposed into the
// lower-triangular slot (nt_local, row_tile0 + mt). C is symmetric, so the mirror is exact.
// ------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void coef_epilogue(f32x4 (&acc)[8][4], int mt, int nt, int kind,
                                              const SimParams& p, int wm, int wn, int lane) {
  T* base = reinterpret_cast<T*>(p.sc);
  const int col_local0 = (nt * kTile) % p.Rpad;  // rank-local column of this tile's col 0
  float lcol[4];
  bool cvalid[4];
  int gj[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int col_t = 64 * wn + 16 * ni + (lane & 15);
    gj[ni] = nt * kTile + col_t;
    lcol[ni] = p.lse2[gj[ni]];
    cvalid[ni] = (col_local0 + col_t) < p.R;
  }
  T* slot = base + ((long long)mt * p.col_tiles + nt) * kTileElems;
  T* mirror = nullptr;
  if (kind == kTileSymOff)
    mirror = base + ((long long)(nt - p.row_tile0) * p.col_tiles + p.row_tile0 + mt) * kTileElems;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    float c[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row_t = 128 * wm + 16 * mi + 4 * (lane >> 4) + r;
      const int gi = mt * kTile + row_t;
      const bool rvalid = gi < p.R;
      const float lrow = p.lse2[p.own0 + gi];
      const int gself = p.own0 + gi;
      const int lpos = gi < p.n_half ? gi + p.n_half : gi - p.n_half;
      const int gpos = p.own0 + lpos;
      // positive: P_ip - 1 = -sigmoid(lse_neg_i - y_ip) (no 1 - P cancellation when P ~ 1)
      float cpos = 0.f;
      if (rvalid) {
        const float yp = p.ypos[gi];
        cpos = -(1.0f / (1.0f + fast_exp2(yp - p.lseneg2[gi])) + 1.0f / (1.0f + fast_exp2(yp - p.lseneg2[lpos])));
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const float y = acc[mi][ni][r] * p.y_scale;
        float v = fast_exp2(y - lrow) + fast_exp2(y - lcol[ni]);
        v = (gj[ni] == gpos) ? cpos : v;
        v = (rvalid && cvalid[ni] && gj[ni] != gself) ? v : 0.0f;
        c[ni][r] = v;
      }
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int col_t = 64 * wn + 16 * ni + (lane & 15);
      const int row_t0 = 128 * wm + 16 * mi + 4 * (lane >> 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) slot[(row_t0 + r) * kTile + col_t] = from_f32<T>(c[ni][r]);
      if (mirror) {
        T* dst = mirror + col_t * kTile + row_t0;
        if constexpr (sizeof(T) == 2) {
          union { T h[4]; uint2 u; } pk;
#pragma unroll
          for (int r = 0; r < 4; ++r) pk.h[r] = from_f32<T>(c[ni][r]);
          *reinterpret_cast<uint2*>(dst) = pk.u;
        } else {
          *reinterpret_cast<f32x4*>(dst) = f32x4{c[ni][0], c[ni][1], c[ni][2], c[ni][3]};
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// The similarity GEMM: out tile (256x256) = A_tile (256 x K) * B_tile (256 x K)^T, both
// operands K-contiguous. 8 waves (2 M x 4 N), 128x64 outputs per wave as 8x4 MFMA 16x16
// accumulators. K advances 128 bytes per step through a 2-deep LDS ring filled by
// global_load_lds_dwordx4 (lane-linear destination, swizzle applied on the source side:
// physical 16B chunk = logical ^ ((row>>1)&7), conflict-free for the ds_read_b128 lane
// groups of the 16x16x32 operand reads).
// ------------------------------------------------------------------------------------
template <typename T, int MODE>
__global__ __launch_bounds__(kGemmThreads) void sim_gemm_kernel(const SimParams p) {
  typedef typename Mfma<T>::frag frag;
  typedef __attribute__((address_space(3))) const frag lds_frag;
  __shared__ __attribute__((aligned(16))) char smem[kGemmLds];
  lds_char* lds = (lds_char*)smem;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const int4 t = p.tiles[xcd_remap(blockIdx.x, gridDim.x)];
  const int mt = t.x, nt = t.y;

  const char* Ab = p.A.base + (long long)mt * p.A.row_tile_stride;
  const char* Bb = p.B.base + (long long)nt * p.B.row_tile_stride;
  long long k0 = (MODE == kModeDz) ? (long long)t.z * p.kbytes : 0;
  long long a_kin = k0 % p.A.kblk, a_kbo = (k0 / p.A.kblk) * p.A.kblk_stride;
  long long b_kin = k0 % p.B.kblk, b_kbo = (k0 / p.B.kblk) * p.B.kblk_stride;

  // per-lane staging offsets (constant over K)
  unsigned a_off[4], b_off[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = (4 * w + q) * 8 + (lane >> 3);
    const int lchunk = (lane & 7) ^ ((row >> 1) & 7);
    a_off[q] = (unsigned)(row * p.A.ld) + lchunk * 16;
    b_off[q] = (unsigned)(row * p.B.ld) + lchunk * 16;
  }

  auto stage = [&](int buf) {
    lds_char* As = lds + buf * kStageBytes;
    lds_char* Bs = As + kTile * kKStepBytes;
    const char* ak = Ab + a_kbo + a_kin;
    const char* bk = Bb + b_kbo + b_kin;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int g = 4 * w + q;
      __builtin_amdgcn_global_load_lds((const void*)(ak + a_off[q]), (lds_void*)(As + g * 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(bk + b_off[q]), (lds_void*)(Bs + g * 1024),
                                       16, 0, 0);
    }
    a_kin += kKStepBytes;
    if (a_kin == p.A.kblk) { a_kin = 0; a_kbo += p.A.kblk_stride; }
    b_kin += kKStepBytes;
    if (b_kin == p.B.kblk) { b_kin = 0; b_kbo += p.B.kblk_stride; }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int r16 = lane & 15, sw = (r16 >> 1) & 7, cq = lane >> 4;
  auto compute = [&](int buf) {
    const lds_char* As = lds + buf * kStageBytes;
    const lds_char* Bs = As + kTile * kKStepBytes;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int pch = ((4 * s + cq) ^ sw) << 4;
      frag a[8], b[4];
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
        a[mi] = *(lds_frag*)(As + (128 * wm + 16 * mi + r16) * kKStepBytes + pch);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        b[ni] = *(lds_frag*)(Bs + (64 * wn + 16 * ni + r16) * kKStepBytes + pch);
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = (MODE == kModeDz) ? Mfma<T>::mma(b[ni], a[mi], acc[mi][ni])
                                          : Mfma<T>::mma(a[mi], b[ni], acc[mi][ni]);
    }
  };

  const int nk = (int)(p.kbytes / kKStepBytes);
  stage(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int it = 0; it < nk; ++it) {
    if (it + 1 < nk) stage((it + 1) & 1);
    compute(it & 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  if constexpr (MODE == kModeDz) {
    // swapped orientation: lane holds out[m = 16mi + (lane&15)][n = 16ni + 4(lane>>4) + r]
    float* out = p.out + (long long)t.z * p.slab_stride;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const long long row = (long long)mt * kTile + 128 * wm + 16 * mi + (lane & 15);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int col = nt * kTile + 64 * wn + 16 * ni + 4 * (lane >> 4);
        *reinterpret_cast<f32x4*>(out + row * p.ldo + col) = acc[mi][ni];
      }
    }
  } else if constexpr (MODE == kModeCoef) {
    coef_epilogue<T>(acc, mt, nt, t.z, p, wm, wn, lane);
  } else {
    const int kind = t.z;
    if (p.sc) {  // keep cosines for the backward (fragment order; 8/16 B per lane)
      T* st = reinterpret_cast<T*>(p.sc) + ((long long)mt * p.col_tiles + nt) * kTileElems;
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          T* dst = st + ((w * 32 + mi * 4 + ni) * 64 + lane) * 4;
          if constexpr (sizeof(T) == 2) {
            union { T h[4]; uint2 u; } pk;
#pragma unroll
            for (int r = 0; r < 4; ++r) pk.h[r] = from_f32<T>(acc[mi][ni][r]);
            *reinterpret_cast<uint2*>(dst) = pk.u;
          } else {
            *reinterpret_cast<f32x4*>(dst) = acc[mi][ni];
          }
        }
    }
    // masks -> scaled logits in log2 units (-inf where excluded). The partials cover the
    // NEGATIVES only: self and positive are excluded (the positive logit comes from prep), so
    // the loss is softplus(lse_neg - y_pos) with no lse - y cancellation.
    const int col_local0 = (nt * kTile) % p.Rpad;
    const bool own_blk = kind != kTilePlain;
    bool cvalid[4];
    int cloc[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      cloc[ni] = col_local0 + 64 * wn + 16 * ni + (lane & 15);
      cvalid[ni] = cloc[ni] < p.R;
    }
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = mt * kTile + 128 * wm + 16 * mi + 4 * (lane >> 4) + r;
        const bool rvalid = gi < p.R;
        const int lpos = gi < p.n_half ? gi + p.n_half : gi - p.n_half;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const bool ok = rvalid && cvalid[ni] && !(own_blk && (cloc[ni] == gi || cloc[ni] == lpos));
          acc[mi][ni][r] = ok ? acc[mi][ni][r] * p.y_scale : kNegInf;
        }
      }
    float2* rowred = reinterpret_cast<float2*>(smem);             // [4][256]
    float2* colred = reinterpret_cast<float2*>(smem + 4 * 256 * 8);  // [2][256]
    // row partials over this wave's 64 columns
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float m = fmaxf(fmaxf(acc[mi][0][r], acc[mi][1][r]), fmaxf(acc[mi][2][r], acc[mi][3][r]));
        m = row16_max(m);
        const float ms = (m == kNegInf) ? 0.f : m;
        float s = fast_exp2(acc[mi][0][r] - ms) + fast_exp2(acc[mi][1][r] - ms) +
                  fast_exp2(acc[mi][2][r] - ms) + fast_exp2(acc[mi][3][r] - ms);
        s = row16_sum(s);
        if ((lane & 15) == 0) rowred[wn * 256 + 128 * wm + 16 * mi + 4 * (lane >> 4) + r] = make_float2(m, s);
      }
    if (kind == kTileSymOff) {  // column partials = partials of the mirrored rows
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        float m = kNegInf;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
          for (int r = 0; r < 4; ++r) m = fmaxf(m, acc[mi][ni][r]);
        m = xrow_max(m);
        const float ms = (m == kNegInf) ? 0.f : m;
        float s = 0.f;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
          for (int r = 0; r < 4; ++r) s += fast_exp2(acc[mi][ni][r] - ms);
        s = xrow_sum(s);
        if ((lane >> 4) == 0) colred[wm * 256 + 64 * wn + 16 * ni + lane] = make_float2(m, s);
      }
    }
    __syncthreads();
    if (tid < 256) {
      float2 v = rowred[tid];
      float m = v.x, s = v.y;
#pragma unroll
      for (int q = 1; q < 4; ++q) {
        const float2 u = rowred[q * 256 + tid];
        lse_merge(m, s, u.x, u.y);
      }
      p.part[(long long)nt * p.Rpad + mt * kTile + tid] = make_float2(m, s);
    } else if (kind == kTileSymOff) {
      const int c = tid - 256;
      float2 v = colred[c];
      float m = v.x, s = v.y;
      const float2 u = colred[256 + c];
      lse_merge(m, s, u.x, u.y);
      p.part[(long long)(p.row_tile0 + mt) * p.Rpad + (nt - p.row_tile0) * kTile + c] = make_float2(m, s);
    }
  }
}

// Store-mode coefficient pass: read the kept cosine tile (fragment order), emit C in place.
template <typename T>
__global__ __launch_bounds__(kGemmThreads) void coef_kernel(const SimParams p) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const int4 t = p.tiles[xcd_remap(blockIdx.x, gridDim.x)];
  const T* st = reinterpret_cast<const T*>(p.sc) + ((long long)t.x * p.col_tiles + t.y) * kTileElems;
  f32x4 acc[8][4];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const T* src = st + ((w * 32 + mi * 4 + ni) * 64 + lane) * 4;
      if constexpr (sizeof(T) == 2) {
        union { T h[4]; uint2 u; } pk;
        pk.u = *reinterpret_cast<const uint2*>(src);
        acc[mi][ni] = f32x4{to_f32<T>(pk.h[0]), to_f32<T>(pk.h[1]), to_f32<T>(pk.h[2]), to_f32<T>(pk.h[3])};
      } else {
        acc[mi][ni] = *reinterpret_cast<const f32x4*>(src);
      }
    }
  __syncthreads();  // every wave holds its cosines before the tile is overwritten in place
  coef_epilogue<T>(acc, t.x, t.y, t.z, p, wm, wn, lane);
}

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

template <typename Tin, typename Tc>
__global__ __launch_bounds__(256) void prep_kernel(const Tin* __restrict__ h, Tc* __restrict__ zq,
                                                   float* __restrict__ inv, float* __restrict__ ypos,
                                                   int R, int d, int dk, float y_scale) {
  __shared__ float red[16];
  const int n = R >> 1, i = blockIdx.x, pi = i + n;
  const Tin* hi = h + (long long)i * d;
  const Tin* hp = h + (long long)pi * d;
  Tc* zi = zq + (long long)i * dk;
  Tc* zp = zq + (long long)pi * dk;
  const bool vec = (d % 8) == 0;
  float ssi = 0.f, ssp = 0.f;
  if (vec) {
    for (int e = threadIdx.x * 8; e < d; e += 256 * 8) {
      float a[8], b[8];
      load8<Tin>(hi + e, a);
      load8<Tin>(hp + e, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) { ssi += a[j] * a[j]; ssp += b[j] * b[j]; }
    }
  } else {
    for (int e = threadIdx.x; e < d; e += 256) {
      const float a = to_f32<Tin>(hi[e]), b = to_f32<Tin>(hp[e]);
      ssi += a * a; ssp += b * b;
    }
  }
  ssi = block_sum(ssi, red);
  ssp = block_sum(ssp, red + 8);
  const float ivi = 1.0f / fmaxf(sqrtf(ssi), 1e-12f);
  const float ivp = 1.0f / fmaxf(sqrtf(ssp), 1e-12f);
  float dot = 0.f;
  if (vec) {
    for (int e = threadIdx.x * 8; e < d; e += 256 * 8) {
      float a[8], b[8], qa[8], qb[8];
      load8<Tin>(hi + e, a);
      load8<Tin>(hp + e, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[j] *= ivi; b[j] *= ivp; }
      store8<Tc>(zi + e, a, qa);
      store8<Tc>(zp + e, b, qb);
#pragma unroll
      for (int j = 0; j < 8; ++j) dot += qa[j] * qb[j];
    }
  } else {
    for (int e = threadIdx.x; e < d; e += 256) {
      const Tc a = from_f32<Tc>(to_f32<Tin>(hi[e]) * ivi);
      const Tc b = from_f32<Tc>(to_f32<Tin>(hp[e]) * ivp);
      zi[e] = a; zp[e] = b;
      dot += to_f32<Tc>(a) * to_f32<Tc>(b);
    }
  }
  for (int e = d + threadIdx.x; e < dk; e += 256) { zi[e] = from_f32<Tc>(0.f); zp[e] = from_f32<Tc>(0.f); }
  dot = block_sum(dot, red);
  if (threadIdx.x == 0) {
    inv[i] = ivi; inv[pi] = ivp;
    ypos[i] = dot * y_scale; ypos[pi] = dot * y_scale;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(const T* __restrict__ zq, T* __restrict__ zqt,
                                                        int Rpad, int dk) {
  __shared__ T tile[64][65];
  const int j0 = blockIdx.x * 64, e0 = blockIdx.y * 64;
  for (int k = threadIdx.x; k < 4096; k += 256) {
    const int r = k >> 6, c = k & 63;
    tile[r][c] = (e0 + c < dk) ? zq[(long long)(j0 + r) * dk + e0 + c] : from_f32<T>(0.f);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 4096; k += 256) {
    const int r = k >> 6, c = k & 63;
    zqt[(long long)(e0 + r) * Rpad + j0 + c] = tile[c][r];
  }
}

__global__ __launch_bounds__(256) void lse_kernel(const float2* __restrict__ part, const float* __restrict__ ypos,
                                                  float* __restrict__ lse2_all, float* __restrict__ lseneg2,
                                                  float* __restrict__ block_loss, int R, int Rpad, int Tc, int own0) {
  __shared__ float red[16];
  const int i = blockIdx.x * 256 + threadIdx.x;
  float m = kNegInf, s = 0.f;
  for (int t = 0; t < Tc; ++t) {
    const float2 v = part[(long long)t * Rpad + i];
    lse_merge(m, s, v.x, v.y);
  }
  const bool ok = i < R;
  const float yp = ok ? ypos[i] : 0.f;
  const float neg2 = (m == kNegInf || s <= 0.f) ? kNegInf : m + log2f(s);
  // lse = logaddexp(lse_neg, y_pos); loss_i = softplus(lse_neg - y_pos) (natural log)
  const float mx = fmaxf(neg2, yp);
  const float l2 = mx + log2f(exp2f(neg2 - mx) + exp2f(yp - mx));
  lse2_all[own0 + i] = ok ? l2 : 0.f;
  lseneg2[i] = ok ? neg2 : 0.f;
  const float x = (neg2 - yp) * kLn2;
  const float sp = x > 0.f ? x + log1pf(expf(-x)) : log1pf(expf(x));
  const float li = ok ? sp : 0.f;
  const float tot = block_sum(li, red);
  if (threadIdx.x == 0) block_loss[blockIdx.x] = tot;
}

__global__ void loss_final_kernel(const float* __restrict__ block_loss, int nb, float scale, float* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    float s = 0.f;
    for (int b = 0; b < nb; ++b) s += block_loss[b];  // fixed order: deterministic
    out[0] = s * scale;
  }
}

template <typename Tin>
__global__ __launch_bounds__(256) void norm_bwd_kernel(const float* __restrict__ slabs, int ksplit,
                                                       long long slab_stride, long long ldo,
                                                       const Tin* __restrict__ h, const float* __restrict__ inv,
                                                       const float* __restrict__ grad_out, float alpha_base,
                                                       Tin* __restrict__ dh, int d) {
  __shared__ float red[16];
  const int i = blockIdx.x;
  const float iv = inv[i];
  const float alpha = grad_out[0] * alpha_base;
  const Tin* hi = h + (long long)i * d;
  const float* gi = slabs + (long long)i * ldo;
  float dot = 0.f;
  for (int e = threadIdx.x; e < d; e += 256) {
    float g = 0.f;
    for (int k = 0; k < ksplit; ++k) g += gi[k * slab_stride + e];
    dot += to_f32<Tin>(hi[e]) * iv * g;
  }
  dot = block_sum(dot, red);
  Tin* di = dh + (long long)i * d;
  for (int e = threadIdx.x; e < d; e += 256) {
    float g = 0.f;
    for (int k = 0; k < ksplit; ++k) g += gi[k * slab_stride + e];
    const float z = to_f32<Tin>(hi[e]) * iv;
    di[e] = from_f32<Tin>(alpha * iv * (g - z * dot));
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
  }
}

dev::SimParams base_params(const Geometry& g) {
  dev::SimParams p{};
  p.R = g.rows;
  p.Rpad = g.rows_pad;
  p.n_half = g.rows / 2;
  p.own0 = g.rank * g.rows_pad;
  p.row_tile0 = g.rank * g.row_tiles;
  p.col_tiles = g.col_tiles;
  p.y_scale = g.inv_temp * dev::kLog2e;
  return p;
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
  g.world = world;
  g.rank = rank;
  g.row_tiles = g.rows_pad / kTile;
  g.col_tiles = world * g.row_tiles;
  g.temperature = temperature;
  g.inv_temp = 1.0f / temperature;
  g.global_rows = (long long)world * rows;
  return g;
}

std::vector<int4> build_fwd_tiles(const Geometry& g) {
  // Order: panel-major so that a run of consecutive tiles (one XCD's share after the
  // xcd_remap) shares its A row panel and walks neighbouring B panels.
  std::vector<int4> tiles;
  const int own = g.rank * g.row_tiles;
  for (int ti = 0; ti < g.row_tiles; ++ti) {
    for (int tj = 0; tj < g.col_tiles; ++tj) {
      const int local = tj - own;
      if (local >= 0 && local < g.row_tiles) {
        if (local < ti) continue;  // lower triangle: mirrored from (local, ti)
        tiles.push_back(make_int4(ti, tj, local == ti ? kTileDiag : kTileSymOff, 0));
      } else {
        tiles.push_back(make_int4(ti, tj, kTilePlain, 0));
      }
    }
  }
  return tiles;
}

int choose_dz_ksplit(const Geometry& g, int num_cus) {
  const int tiles = g.row_tiles * (g.dim_n / kTile);
  const int ksteps = g.world * g.rows_pad / kTile;  // K in units of 256
  int ks = 1;
  while (tiles * ks < num_cus && ks * 2 <= ksteps && (ksteps % (ks * 2)) == 0) ks *= 2;
  return ks;
}

std::vector<int4> build_dz_tiles(const Geometry& g, int ksplit) {
  std::vector<int4> tiles;
  const int nt = g.dim_n / kTile;
  for (int ti = 0; ti < g.row_tiles; ++ti)
    for (int ks = 0; ks < ksplit; ++ks)
      for (int tn = 0; tn < nt; ++tn) tiles.push_back(make_int4(ti, tn, ks, 0));
  return tiles;
}

void launch_prep(DType in, DType comp, const void* h, void* zq, float* inv, float* ypos,
                 const Geometry& g, hipStream_t stream) {
  const size_t cs = dtype_size(comp);
  if (g.rows_pad > g.rows) {
    NTXENT_HIP_CHECK(hipMemsetAsync(static_cast<char*>(zq) + (size_t)g.rows * g.dim_k * cs, 0,
                                    (size_t)(g.rows_pad - g.rows) * g.dim_k * cs, stream));
  }
  const float ys = g.inv_temp * dev::kLog2e;
  dispatch_comp(in, [&](auto tin) {
    using Tin = decltype(tin);
    dispatch_comp(comp, [&](auto tc) {
      using Tc = decltype(tc);
      hipLaunchKernelGGL((dev::prep_kernel<Tin, Tc>), dim3(g.rows / 2), dim3(256), 0, stream,
                         static_cast<const Tin*>(h), static_cast<Tc*>(zq), inv, ypos, g.rows, g.dim,
                         g.dim_k, ys);
    });
  });
  NTXENT_HIP_CHECK(hipGetLastError());
}

void launch_transpose(DType comp, const void* zq, void* zqt, const Geometry& g, hipStream_t stream) {
  dispatch_comp(comp, [&](auto tc) {
    using Tc = decltype(tc);
    hipLaunchKernelGGL((dev::transpose_kernel<Tc>), dim3(g.rows_pad / 64, g.dim_n / 64), dim3(256), 0,
                       stream, static_cast<const Tc*>(zq), static_cast<Tc*>(zqt), g.rows_pad, g.dim_k);
  });
  NTXENT_HIP_CHECK(hipGetLastError());
}

void launch_fwd_stats(DType comp, const void* zq_local, const void* zq_all, const int4* tiles,
                      int ntiles, float2* part, void* sc, const Geometry& g, hipStream_t stream) {
  if (ntiles == 0) return;
  const long long kb = (long long)g.dim_k * dtype_size(comp);
  dev::SimParams p = base_params(g);
  p.A = rowmajor_operand(zq_local, kb, kb);
  p.B = rowmajor_operand(zq_all, kb, kb);
  p.tiles = tiles;
  p.kbytes = kb;
  p.part = part;
  p.sc = static_cast<char*>(sc);
  dispatch_comp(comp, [&](auto tc) {
    using Tc = decltype(tc);
    hipLaunchKernelGGL((dev::sim_gemm_kernel<Tc, dev::kModeFwd>), dim3(ntiles), dim3(kGemmThreads), 0,
                       stream, p);
  });
  NTXENT_HIP_CHECK(hipGetLastError());
}

void launch_coef_gemm(DType comp, const void* zq_local, const void* zq_all, void* sc,
                      const float* lse2_all, const float* ypos, const float* lseneg2, const int4* tiles,
                      int ntiles, const Geometry& g, hipStream_t stream) {
  if (ntiles == 0) return;
  const long long kb = (long long)g.dim_k * dtype_size(comp);
  dev::SimParams p = base_params(g);
  p.A = rowmajor_operand(zq_local, kb, kb);
  p.B = rowmajor_operand(zq_all, kb, kb);
  p.tiles = tiles;
  p.kbytes = kb;
  p.sc = static_cast<char*>(sc);
  p.lse2 = lse2_all;
  p.ypos = ypos;
  p.lseneg2 = lseneg2;
  dispatch_comp(comp, [&](auto tc) {
    using Tc = decltype(tc);
    hipLaunchKernelGGL((dev::sim_gemm_kernel<Tc, dev::kModeCoef>), dim3(ntiles), dim3(kGemmThreads), 0,
                       stream, p);
  });
  NTXENT_HIP_CHECK(hipGetLastError());
}

void launch_lse(const float2* part, const float* ypos, float* lse2_all, float* lseneg2, float* block_loss,
                float* loss_sum, const Geometry& g, hipStream_t stream) {
  const int nb = g.rows_pad / 256;
  hipLaunchKernelGGL(dev::lse_kernel, dim3(nb), dim3(256), 0, stream, part, ypos, lse2_all, lseneg2, block_loss,
                     g.rows, g.rows_pad, g.col_tiles, g.rank * g.rows_pad);
  NTXENT_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(dev::loss_final_kernel, dim3(1), dim3(64), 0, stream, block_loss, nb,
                     (float)(1.0 / (double)g.global_rows), loss_sum);
  NTXENT_HIP_CHECK(hipGetLastError());
}

void launch_coef(DType comp, void* sc, const float* lse2_all, const float* ypos, const float* lseneg2,
                 const int4* tiles, int ntiles, const Geometry& g, hipStream_t stream) {
  if (ntiles == 0) return;
  dev::SimParams p = base_params(g);
  p.tiles = tiles;
  p.sc = static_cast<char*>(sc);
  p.lse2 = lse2_all;
  p.ypos = ypos;
  p.lseneg2 = lseneg2;
  dispatch_comp(comp, [&](auto tc) {
    using Tc = decltype(tc);
    hipLaunchKernelGGL((dev::coef_kernel<Tc>), dim3(ntiles), dim3(kGemmThreads), 0, stream, p);
  });
  NTXENT_HIP_CHECK(hipGetLastError());
}

void launch_dz(DType comp, const void* sc, const void* zqt_all, const int4* tiles, int ntiles,
               int ksplit, float* slabs, const Geometry& g, hipStream_t stream) {
  if (ntiles == 0) return;
  const long long cs = (long long)dtype_size(comp);
  dev::SimParams p = base_params(g);
  // A = C, tile-blocked: rows of a 256x256 tile are 256 elements; every 256 K-columns jump
  // to the next tile of the row panel.
  p.A.base = static_cast<const char*>(sc);
  p.A.ld = kTile * cs;
  p.A.row_tile_stride = (long long)g.col_tiles * kTileElems * cs;
  p.A.kblk = kTile * cs;
  p.A.kblk_stride = kTileElems * cs;
  // B = ZqT_all [W][dim_n][Rpad]: rows = embedding dims, K = global columns, one K block per rank.
  p.B.base = static_cast<const char*>(zqt_all);
  p.B.ld = (long long)g.rows_pad * cs;
  p.B.row_tile_stride = (long long)kTile * g.rows_pad * cs;
  p.B.kblk = (long long)g.rows_pad * cs;
  p.B.kblk_stride = (long long)g.dim_n * g.rows_pad * cs;
  p.tiles = tiles;
  p.kbytes = (long long)g.world * g.rows_pad * cs / ksplit;
  NTXENT_CHECK(p.kbytes % kKStepBytes == 0, "dz split not aligned to the K step");
  p.out = slabs;
  p.ldo = g.dim_n;
  p.slab_stride = (long long)g.rows_pad * g.dim_n;
  dispatch_comp(comp, [&](auto tc) {
    using Tc = decltype(tc);
    hipLaunchKernelGGL((dev::sim_gemm_kernel<Tc, dev::kModeDz>), dim3(ntiles), dim3(kGemmThreads), 0,
                       stream, p);
  });
  NTXENT_HIP_CHECK(hipGetLastError());
}

void launch_norm_bwd(DType in, const float* slabs, int ksplit, const void* h, const float* inv,
                     const float* grad_out, void* dh, const Geometry& g, hipStream_t stream) {
  const float alpha_base = (float)(1.0 / ((double)g.global_rows * g.temperature));
  dispatch_comp(in, [&](auto tin) {
    using Tin = decltype(tin);
    hipLaunchKernelGGL((dev::norm_bwd_kernel<Tin>), dim3(g.rows), dim3(256), 0, stream, slabs, ksplit,
                       (long long)g.rows_pad * g.dim_n, (long long)g.dim_n, static_cast<const Tin*>(h), inv,
                       grad_out, alpha_base, static_cast<Tin*>(dh), g.dim);
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

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
constexpr int kCtStride = kTile * 2 + 16;                // C^T staging row: 512 B + 16 B pad
constexpr int kCoefLds = kTile * kCtStride;             // 132 KiB
constexpr int kCoefWaveLds = 64 * (128 * 2 + 16);      // 17 KiB: C^T of one 128x64 wave region

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
  float y_scale;         // inv_temp * log2(e) = M, the largest possible logit (log2 units)
  int fixed_shift;       // 1: exponentials use the fixed shift M (2M < 120, see fwd epilogue)
  float2* part;          // [col_tiles][Rpad] partial (max, sum) in log2 units
  char* sc;              // kept cosines: [n_fwd_tiles][256*256] (fragment order)
  char* cbuf;            // coefficients: [row_tiles][col_tiles][256*256] (row-major per tile)
  const float* lse2;     // [W*Rpad] lse in log2 units (all ranks)
  const float* cpos;     // [Rpad] positive coefficient C_i,p(i) = -(a_i + a_p), a = 1 - P_ip
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
// NW = waves of the calling block: 8 (a GEMM block: the whole 256x256 tile) or 1 (a single
// wave owning its 128x64 region; 17 KiB of LDS, so the memory-bound store-mode pass runs
// many independent waves per CU).
template <typename T, int NW>
__device__ __forceinline__ void coef_epilogue(f32x4 (&acc)[8][4], int mt, int nt, int kind, lds_char* lds,
                                              const SimParams& p, int wm, int wn, int lane) {
  constexpr int NROWS = NW == 8 ? kTile : 128;
  constexpr int NCOLS = NW == 8 ? kTile : 64;
  constexpr int S = NROWS * 2 + 16;          // LDS row stride (bytes) of the C^T staging tile
  constexpr int NT = NW * 64;                // threads in the calling block
  const int row_base = NW == 8 ? 0 : 128 * wm;
  const int col_base = NW == 8 ? 0 : 64 * wn;
  T* base = reinterpret_cast<T*>(p.cbuf);
  const int col_local0 = (nt * kTile) % p.Rpad;  // rank-local column of this tile's col 0
  // C_ij = 2^(y - lse2_i) + 2^(y - lse2_j). Fixed-shift form (2M < 120, see the forward
  // epilogue): 2^(y - M) * (2^(M - lse2_i) + 2^(M - lse2_j)), one exp2 per element, the
  // per-row / per-column factors computed once.
  const bool fixed = p.fixed_shift != 0;
  const float M = p.y_scale;
  float lcol[4];
  bool cvalid[4];
  int gj[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int col_t = 64 * wn + 16 * ni + (lane & 15);
    gj[ni] = nt * kTile + col_t;
    const float l = p.lse2[gj[ni]];
    lcol[ni] = fixed ? fast_exp2(M - l) : l;
    cvalid[ni] = (col_local0 + col_t) < p.R;
  }
  T* slot = base + ((long long)mt * p.col_tiles + nt) * kTileElems;
  T* mirror = nullptr;
  if (kind == kTileSymOff)
    mirror = base + ((long long)(nt - p.row_tile0) * p.col_tiles + p.row_tile0 + mt) * kTileElems;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    float c[4][4];
    const int gi0 = mt * kTile + 128 * wm + 16 * mi + 4 * (lane >> 4);  // 4 consecutive rows
    const f32x4 lrow4 = *reinterpret_cast<const f32x4*>(p.lse2 + p.own0 + gi0);
    const f32x4 cpos4 = *reinterpret_cast<const f32x4*>(p.cpos + gi0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gi = gi0 + r;
      const bool rvalid = gi < p.R;
      const float lrow = fixed ? fast_exp2(M - lrow4[r]) : lrow4[r];
      const int gself = p.own0 + gi;
      const int gpos = p.own0 + (gi < p.n_half ? gi + p.n_half : gi - p.n_half);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const float y = acc[mi][ni][r] * p.y_scale;
        float v = fixed ? fast_exp2(y - M) * (lrow + lcol[ni]) : fast_exp2(y - lrow) + fast_exp2(y - lcol[ni]);
        v = (gj[ni] == gpos) ? cpos4[r] : v;  // positive: -(a_i + a_p), no 1 - P cancellation
        v = (rvalid && cvalid[ni] && gj[ni] != gself) ? v : 0.0f;
        c[ni][r] = v;
      }
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int col_t = 64 * wn + 16 * ni + (lane & 15);
      const int row_t0 = 128 * wm + 16 * mi + 4 * (lane >> 4);
      if constexpr (sizeof(T) == 2) {
        // stage C^T in LDS: Ct[col][row0..row0+3] (one ds_write_b64 per fragment)
        union { T h[4]; u32x2 u; } pk;
#pragma unroll
        for (int r = 0; r < 4; ++r) pk.h[r] = from_f32<T>(c[ni][r]);
        *reinterpret_cast<__attribute__((address_space(3))) u32x2*>(lds + (col_t - col_base) * S + (row_t0 - row_base) * 2) = pk.u;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) slot[(row_t0 + r) * kTile + col_t] = c[ni][r];
        if (mirror)
          *reinterpret_cast<f32x4*>(mirror + col_t * kTile + row_t0) = f32x4{c[ni][0], c[ni][1], c[ni][2], c[ni][3]};
      }
    }
  }
  if constexpr (sizeof(T) == 2) {
    __syncthreads();
    const int tid = threadIdx.x, w = tid >> 6;  // w = wave index inside the calling block
    // (a) Ct rows are rows of C^T: coalesced 16-B stores into the mirror slot (SymOff) or,
    //     for a diagonal tile (C symmetric inside it), into the tile's own slot.
    T* rows_dst = mirror;  // only mirrored tiles (a diagonal tile goes through (b) like any other)
    if (rows_dst) {
      constexpr int CPR = NROWS * 2 / 16;  // 16-B chunks per staged row
#pragma unroll 4
      for (int q = 0; q < NCOLS * CPR / NT; ++q) {
        const int k = tid + NT * q;
        const int row = k / CPR, c16 = k % CPR;
        const u32x4 v = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(lds + row * S + c16 * 16);
        *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(rows_dst) + (col_base + row) * (kTile * 2) + row_base * 2 +
                                  c16 * 16) = v;
      }
    }
    // (b) rows of C = columns of Ct via the gfx950 transposed LDS read (ds_read_b64_tr_b16):
    //     a 16-lane group reads a 4 (Ct rows) x 16 (Ct cols) block and lane i receives column
    //     i, i.e. 4 consecutive entries of C row c0+i. Two reads give 16 B per lane.
    {
      typedef short v4s __attribute__((ext_vector_type(4)));
      constexpr int RB = NROWS / 16;                 // 16-row blocks of C in this call
      constexpr int NBLK = RB * (NCOLS / 32) / NW;   // 16x32 blocks per wave (= 16)
      const int g = lane >> 4, i = lane & 15, q4 = i >> 2, p4 = i & 3;
#pragma unroll 2
      for (int b = 0; b < NBLK; ++b) {
        const int blk = w * NBLK + b;
        const int c0 = (blk % RB) * 16;   // C rows row_base+c0 .. +15
        const int rb = (blk / RB) * 32;   // C cols col_base+rb .. +31
        const int r0 = rb + 8 * g;
        const lds_char* a0 = lds + (r0 + q4) * S + (c0 + 4 * p4) * 2;
        const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)a0);
        const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(a0 + 4 * S));
        u32x4 u;
        u[0] = (unsigned short)lo[0] | ((unsigned)(unsigned short)lo[1] << 16);
        u[1] = (unsigned short)lo[2] | ((unsigned)(unsigned short)lo[3] << 16);
        u[2] = (unsigned short)hi[0] | ((unsigned)(unsigned short)hi[1] << 16);
        u[3] = (unsigned short)hi[2] | ((unsigned)(unsigned short)hi[3] << 16);
        *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(slot) + (row_base + c0 + i) * (kTile * 2) +
                                  (col_base + r0) * 2) = u;
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
  __shared__ __attribute__((aligned(16))) char smem[MODE == kModeCoef ? kCoefLds : kGemmLds];
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
    coef_epilogue<T, 8>(acc, mt, nt, t.z, lds, p, wm, wn, lane);
  } else {
    const int kind = t.z;
    if (p.sc) {  // keep cosines for the backward (compact: one slot per computed tile, fragment order)
      T* st = reinterpret_cast<T*>(p.sc) + (long long)xcd_remap(blockIdx.x, gridDim.x) * kTileElems;
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
    // Fixed-shift fast path: rows are unit-norm, so y = cos * M with M = log2(e)/tau and
    // y - M lies in [-2M, 0]. For 2M < 120 every exp2(y - M) is a normal fp32 number, so ONE
    // exp2 per element feeds both the row and the column partial with a common shift M (no
    // max passes). Smaller tau falls back to per-tile max shifting (2 exps per element).
    const bool fixed = p.fixed_shift != 0;
    const float M = p.y_scale;
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
          if (fixed)
            acc[mi][ni][r] = ok ? fast_exp2(acc[mi][ni][r] * p.y_scale - M) : 0.f;
          else
            acc[mi][ni][r] = ok ? acc[mi][ni][r] * p.y_scale : kNegInf;
        }
      }
    float2* rowred = reinterpret_cast<float2*>(smem);             // [4][256]
    float2* colred = reinterpret_cast<float2*>(smem + 4 * 256 * 8);  // [2][256]
    if (fixed) {
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float s = (acc[mi][0][r] + acc[mi][1][r]) + (acc[mi][2][r] + acc[mi][3][r]);
          s = row16_sum(s);
          if ((lane & 15) == 0)
            rowred[wn * 256 + 128 * wm + 16 * mi + 4 * (lane >> 4) + r] = make_float2(s > 0.f ? M : kNegInf, s);
        }
      if (kind == kTileSymOff) {
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          float s = 0.f;
#pragma unroll
          for (int mi = 0; mi < 8; ++mi)
            s += (acc[mi][ni][0] + acc[mi][ni][1]) + (acc[mi][ni][2] + acc[mi][ni][3]);
          s = xrow_sum(s);
          if ((lane >> 4) == 0) colred[wm * 256 + 64 * wn + 16 * ni + lane] = make_float2(s > 0.f ? M : kNegInf, s);
        }
      }
    } else {
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
    }  // !fixed
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
// Store-mode coefficient pass: one wave per 128x64 region of a kept cosine tile (fragment
// order, 16 KiB contiguous per region) -> C into the separate coefficient buffer. 17 KiB of
// LDS per wave keeps many independent waves in flight per CU (the pass is HBM-bound).
template <typename T>
__global__ __launch_bounds__(64) void coef_kernel(const SimParams p) {
  __shared__ __attribute__((aligned(16))) char smem[sizeof(T) == 2 ? kCoefWaveLds : 16];
  const int lane = threadIdx.x;
  const int idx = xcd_remap(blockIdx.x, gridDim.x);
  const int tidx = idx >> 3, w = idx & 7;
  const int wm = w >> 2, wn = w & 3;
  const int4 t = p.tiles[tidx];
  const T* st = reinterpret_cast<const T*>(p.sc) + (long long)tidx * kTileElems;
  f32x4 acc[8][4];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const T* src = st + ((w * 32 + mi * 4 + ni) * 64 + lane) * 4;
      if constexpr (sizeof(T) == 2) {
        union { T h[4]; u32x2 u; } pk;
        pk.u = *reinterpret_cast<const u32x2*>(src);
        acc[mi][ni] = f32x4{to_f32<T>(pk.h[0]), to_f32<T>(pk.h[1]), to_f32<T>(pk.h[2]), to_f32<T>(pk.h[3])};
      } else {
        acc[mi][ni] = *reinterpret_cast<const f32x4*>(src);
      }
    }
  coef_epilogue<T, 1>(acc, t.x, t.y, t.z, (lds_char*)smem, p, wm, wn, lane);
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

// 64x64 tile transpose with 16-byte global accesses on both sides (rows of Zq in, rows of
// ZqT out); the LDS tile is padded by 16 B per row.
template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(const T* __restrict__ zq, T* __restrict__ zqt,
                                                        int Rpad, int dk) {
  constexpr int V = 16 / sizeof(T);  // elements per 16 B
  constexpr int CPR = 64 / V;        // 16-B chunks per 64-element row
  __shared__ __attribute__((aligned(16))) T tile[64][64 + V];
  const int j0 = blockIdx.x * 64, e0 = blockIdx.y * 64;
  for (int k = threadIdx.x; k < 64 * CPR; k += 256) {
    const int r = k / CPR, c = k % CPR;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (e0 + c * V < dk) v = *reinterpret_cast<const u32x4*>(zq + (long long)(j0 + r) * dk + e0 + c * V);
    *reinterpret_cast<u32x4*>(&tile[r][c * V]) = v;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 64 * CPR; k += 256) {
    const int er = k / CPR, jc = k % CPR;
    union { T h[V]; u32x4 u; } pk;
#pragma unroll
    for (int q = 0; q < V; ++q) pk.h[q] = tile[jc * V + q][er];
    *reinterpret_cast<u32x4*>(zqt + (long long)(e0 + er) * Rpad + j0 + jc * V) = pk.u;
  }
}

// Row statistics of one row from its negatives-only partials: returns lse2 and writes the
// natural-log loss term softplus(lse_neg - y_pos) and a = 1 - P_ip = sigmoid(lse_neg - y_pos).
__device__ __forceinline__ float row_stats(const float2* __restrict__ part, int i, int Rpad, int Tc, float yp,
                                           float& loss, float& a) {
  float m = kNegInf, s = 0.f;
  for (int t = 0; t < Tc; ++t) {
    const float2 v = part[(long long)t * Rpad + i];
    lse_merge(m, s, v.x, v.y);
  }
  const float neg2 = (m == kNegInf || s <= 0.f) ? kNegInf : m + log2f(s);
  const float mx = fmaxf(neg2, yp);  // lse = logaddexp(lse_neg, y_pos)
  const float l2 = mx + log2f(exp2f(neg2 - mx) + exp2f(yp - mx));
  const float x = (neg2 - yp) * kLn2;
  loss = x > 0.f ? x + log1pf(expf(-x)) : log1pf(expf(x));
  a = 1.0f / (1.0f + exp2f(yp - neg2));
  return l2;
}

// One thread per positive pair (i, i+n) (plus the pad rows): LSE of both rows, their loss
// terms, and the positive coefficient C_ip = P_ip + P_pi - 2 = -(a_i + a_p), formed without
// the 1 - P cancellation.
__global__ __launch_bounds__(256) void lse_kernel(const float2* __restrict__ part, const float* __restrict__ ypos,
                                                  float* __restrict__ lse2_all, float* __restrict__ cpos,
                                                  float* __restrict__ block_loss, int R, int Rpad, int Tc, int own0) {
  __shared__ float red[16];
  const int n = R >> 1;
  const int t = blockIdx.x * 256 + threadIdx.x;
  float li = 0.f;
  if (t < n) {
    const int i = t, j = t + n;
    const float yp = ypos[i];
    float l_i, l_j, a_i, a_j;
    const float l2i = row_stats(part, i, Rpad, Tc, yp, l_i, a_i);
    const float l2j = row_stats(part, j, Rpad, Tc, yp, l_j, a_j);
    lse2_all[own0 + i] = l2i;
    lse2_all[own0 + j] = l2j;
    cpos[i] = -(a_i + a_j);
    cpos[j] = -(a_i + a_j);
    li = l_i + l_j;
  } else if (t < Rpad - n) {
    const int i = R + (t - n);
    lse2_all[own0 + i] = 0.f;
    cpos[i] = 0.f;
  }
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

// Vectorised normalisation backward: one 256-thread block per row; each thread owns NCH
// chunks of 8 contiguous features, kept in registers between the dot pass and the output.
template <typename Tin, int NCH>
__global__ __launch_bounds__(256) void norm_bwd_vec_kernel(const float* __restrict__ slabs, int ksplit,
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
  float g[NCH][8], z[NCH][8];
  float dot = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = (c * 256 + threadIdx.x) * 8;
    if (e < d) {
      load8<Tin>(hi + e, z[c]);
      f32x4 a = *reinterpret_cast<const f32x4*>(gi + e), b = *reinterpret_cast<const f32x4*>(gi + e + 4);
      for (int k = 1; k < ksplit; ++k) {
        a += *reinterpret_cast<const f32x4*>(gi + k * slab_stride + e);
        b += *reinterpret_cast<const f32x4*>(gi + k * slab_stride + e + 4);
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
  p.fixed_shift = (2.0f * p.y_scale < 120.0f) ? 1 : 0;  // tau > ~0.024
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

void launch_coef_gemm(DType comp, const void* zq_local, const void* zq_all, void* cbuf,
                      const float* lse2_all, const float* cpos, const int4* tiles, int ntiles,
                      const Geometry& g, hipStream_t stream) {
  if (ntiles == 0) return;
  const long long kb = (long long)g.dim_k * dtype_size(comp);
  dev::SimParams p = base_params(g);
  p.A = rowmajor_operand(zq_local, kb, kb);
  p.B = rowmajor_operand(zq_all, kb, kb);
  p.tiles = tiles;
  p.kbytes = kb;
  p.cbuf = static_cast<char*>(cbuf);
  p.lse2 = lse2_all;
  p.cpos = cpos;
  dispatch_comp(comp, [&](auto tc) {
    using Tc = decltype(tc);
    hipLaunchKernelGGL((dev::sim_gemm_kernel<Tc, dev::kModeCoef>), dim3(ntiles), dim3(kGemmThreads), 0,
                       stream, p);
  });
  NTXENT_HIP_CHECK(hipGetLastError());
}

void launch_lse(const float2* part, const float* ypos, float* lse2_all, float* cpos, float* block_loss,
                float* loss_sum, const Geometry& g, hipStream_t stream) {
  const int nb = (g.rows_pad - g.rows / 2 + 255) / 256;  // one thread per pair + pad rows
  hipLaunchKernelGGL(dev::lse_kernel, dim3(nb), dim3(256), 0, stream, part, ypos, lse2_all, cpos, block_loss,
                     g.rows, g.rows_pad, g.col_tiles, g.rank * g.rows_pad);
  NTXENT_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(dev::loss_final_kernel, dim3(1), dim3(64), 0, stream, block_loss, nb,
                     (float)(1.0 / (double)g.global_rows), loss_sum);
  NTXENT_HIP_CHECK(hipGetLastError());
}

void launch_coef(DType comp, const void* sbuf, void* cbuf, const float* lse2_all, const float* cpos,
                 const int4* tiles, int ntiles, const Geometry& g, hipStream_t stream) {
  if (ntiles == 0) return;
  dev::SimParams p = base_params(g);
  p.tiles = tiles;
  p.sc = const_cast<char*>(static_cast<const char*>(sbuf));
  p.cbuf = static_cast<char*>(cbuf);
  p.lse2 = lse2_all;
  p.cpos = cpos;
  dispatch_comp(comp, [&](auto tc) {
    using Tc = decltype(tc);
    hipLaunchKernelGGL((dev::coef_kernel<Tc>), dim3(8 * ntiles), dim3(64), 0, stream, p);
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
  const long long ss = (long long)g.rows_pad * g.dim_n, ldo = g.dim_n;
  const int nch = (g.dim + 2047) / 2048;  // 8-element chunks per thread
  const bool vec = (g.dim % 8) == 0 && nch <= 4;
  dispatch_comp(in, [&](auto tin) {
    using Tin = decltype(tin);
    const Tin* hp = static_cast<const Tin*>(h);
    Tin* dp = static_cast<Tin*>(dh);
    if (vec && nch == 1)
      hipLaunchKernelGGL((dev::norm_bwd_vec_kernel<Tin, 1>), dim3(g.rows), dim3(256), 0, stream, slabs, ksplit, ss,
                         ldo, hp, inv, grad_out, alpha_base, dp, g.dim);
    else if (vec && nch == 2)
      hipLaunchKernelGGL((dev::norm_bwd_vec_kernel<Tin, 2>), dim3(g.rows), dim3(256), 0, stream, slabs, ksplit, ss,
                         ldo, hp, inv, grad_out, alpha_base, dp, g.dim);
    else if (vec)
      hipLaunchKernelGGL((dev::norm_bwd_vec_kernel<Tin, 4>), dim3(g.rows), dim3(256), 0, stream, slabs, ksplit, ss,
                         ldo, hp, inv, grad_out, alpha_base, dp, g.dim);
    else
      hipLaunchKernelGGL((dev::norm_bwd_kernel<Tin>), dim3(g.rows), dim3(256), 0, stream, slabs, ksplit, ss, ldo,
                         hp, inv, grad_out, alpha_base, dp, g.dim);
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

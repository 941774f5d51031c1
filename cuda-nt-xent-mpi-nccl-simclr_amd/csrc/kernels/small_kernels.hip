// Small-problem NT-Xent path for gfx950: one forward and one backward launch after the row
// prologue, for single-rank problems with R <= kSmallMaxRows rows and dim_k <= kSmallMaxDk.
//
// The reference's own benchmark sweeps B in {32..1024} x D in {64,128,256}
// (/root/reference/src/benchmark.cpp:68-71) and its stability harness runs B = 128, D = 256
// (/root/reference/python/test.py:57-79). At these sizes the large-problem pipeline (256 x 256
// persistent tiles, seven launches) is launch- and padding-bound; here:
//
//   small_fwd : grid (col block J, row block I) of 64 x 64 tiles. The row prologue is fused:
//               each tile reads its two row blocks of h, L2-normalises and rounds them into LDS
//               (XOR-swizzled 16-B chunks, K = dim_k whole); the diagonal tile also writes zq and
//               1/|h| for the backward, and the tile holding a row's partner writes the positive
//               logit. 16x16x32 MFMA (4 waves, 32 x 32
//               each), masked per-row (max, sum) partials; the last-arriving tile of a row block
//               merges that block's partials (finish_row: LSE, softplus loss term, positive
//               weight a = 1 - P_ip) and the last row block sums the loss in block order
//               (deterministic). Replaces src/ntxent_kernel.cu:8-134 + the SGEMM at :165-173.
//   small_bwd : grid (row block I, column split s). Each wave owns 16 rows. Per 64-column block
//               J: S^T = Z_J Z_I^T on MFMA (accumulator: a row i per lane, 16 columns j in
//               registers), C_ij = P_ij + P_ji - 2[j = p(i)] in fp32 registers, packed straight
//               into the A operand of dZ_I += C Z_J (no LDS round trip: the accumulator's
//               4-row k groups are exactly the row blocks that ds_read_b64_tr_b16 delivers for
//               the B operand), then the L2-normalisation backward in the epilogue. Column
//               splits publish fp32 partial slabs (write-through) and the last arriver sums
//               them in split order. Replaces src/ntxent_kernel.cu:205-239.
#include "../include/ntxent/ntxent.h"
#include "device_common.h"

#include <algorithm>

namespace ntxent {
namespace dev {

constexpr int kSmallTile = 64;
constexpr int kSmallThreads = 256;

struct SmallParams {
  const void* zq;     // [Rpad][ldk] normalised rows, compute dtype (zero padded)
  const void* h;      // [R][d] input (backward)
  const float* inv;   // [R]
  const void* hin;    // [R][d] input rows (forward: the fused row prologue reads them)
  int hvec;           // hin rows can be read in 16-B vectors (d % 8 == 0, 16-B aligned base)
  void* zq_out;       // [Rp64][ldk] zq written by the forward's diagonal tiles (backward operand)
  float* inv_out;     // [R] 1/|h_i| written by the forward's diagonal tiles
  float* ypos;        // [Rp64] positive logit (log2 units), written by the tile holding the pair
  float2* part;       // [nT][Rp64] per-(column block, row) (max, sum), log2 units
  float* lse2;        // [Rp64] full LSE (log2 units, positive included)
  float* arow;        // [Rp64] a_i = 1 - P_i,p(i)
  int* cnt;           // arrival counters (zero at launch, self-cleaning): [nT] fwd, [1] loss, [nT] bwd
  float* loss_part;   // [nT]
  float* loss;        // scalar
  float* slabs;       // [nT][nS][64 * dk] fp32 partial dZ (bwd, nS > 1)
  const float* grad_out;
  void* dh;
  int R, n_half, ldk, d, dk, nT, Rp64, nS;
  float y_scale;      // log2(e) / tau
  float loss_scale;   // 1 / R
  float alpha_base;   // 1 / (R tau)
};

// Linear LDS image of a [64][dk] row block: 16-B chunk c of row r lives at chunk c ^ (r & 7).
template <int NKS>
__device__ __forceinline__ int sw_off(int row, int chunk) {
  return row * (NKS * 64) + ((chunk ^ (row & 7)) << 4);
}

// Stage rows [row0, row0 + 64) of zq (dk = 32 * NKS elements of 2 bytes) into `dst` by
// global_load_lds: every wave moves NKS pieces of 1 KiB; the swizzle is applied on the source.
template <int NKS>
__device__ __forceinline__ void stage_rows(const char* zq, long long ld_bytes, int row0, lds_char* dst, int w,
                                           int lane) {
  constexpr int RB = NKS * 64;  // bytes per row
#pragma unroll
  for (int q = 0; q < NKS; ++q) {
    const int piece = w * NKS + q;
    const int o = piece * 1024 + lane * 16;
    const int row = o / RB, pc = (o % RB) >> 4;
    const int lc = pc ^ (row & 7);
    __builtin_amdgcn_global_load_lds((const void*)(zq + (long long)(row0 + row) * ld_bytes + lc * 16),
                                     (lds_void*)(dst + piece * 1024), 16, 0, 0);
  }
}

// Fused row prologue: rows [row0, row0 + 64) of h, L2-normalised and rounded to T, into the
// same swizzled LDS image as stage_rows (zero for rows >= R and columns >= d). 4 threads per
// row, thread q of a row owning the 16-B chunks q, q + 4, ...; the row's sum of squares is
// reduced over those 4 lanes. With zq_out set the rounded rows also go to zq (rows up to the
// 64-row pad, zeros included) and 1/|h| to inv_out.
template <typename Tin, typename T, int NKS>
__device__ __forceinline__ void norm_stage(const Tin* h, int R, int d, bool vec, int row0, lds_char* dst, int tid,
                                           T* zq_out, int ldk, float* inv_out) {
  const int r = tid >> 2, q = tid & 3, gr = row0 + r;
  const bool ok = gr < R;
  const Tin* hr = h + (long long)gr * d;
  float v[NKS][8];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < NKS; ++k) {
    const int e0 = 8 * (q + 4 * k);
    if (ok && vec && e0 < d) {  // (d % 8 == 0: the whole chunk is in the row)
      if constexpr (sizeof(Tin) == 4) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(hr + e0), b = *reinterpret_cast<const f32x4*>(hr + e0 + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[k][j] = a[j]; v[k][4 + j] = b[j]; }
      } else {
        union { u32x4 u; Tin x[8]; } pk;
        pk.u = *reinterpret_cast<const u32x4*>(hr + e0);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = to_f32<Tin>(pk.x[j]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = (ok && e0 + j < d) ? to_f32<Tin>(hr[e0 + j]) : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[k][j] * v[k][j];
  }
  ss += __shfl_xor(ss, 1, 64);
  ss += __shfl_xor(ss, 2, 64);
  const float iv = 1.0f / fmaxf(sqrtf(ss), 1e-12f);
#pragma unroll
  for (int k = 0; k < NKS; ++k) {
    const int c = q + 4 * k;
    union { u32x4 u; T x[8]; } pk;
#pragma unroll
    for (int j = 0; j < 8; ++j) pk.x[j] = from_f32<T>(v[k][j] * iv);
    *(__attribute__((address_space(3))) u32x4*)(dst + sw_off<NKS>(r, c)) = pk.u;
    if (zq_out) *reinterpret_cast<u32x4*>(zq_out + (long long)gr * ldk + 8 * c) = pk.u;
  }
  if (zq_out && ok && q == 0) inv_out[gr] = iv;
}

// ---------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------
// FUSE: the row prologue runs inside (norm_stage, above); otherwise launch_prep has written zq
// and the positive logits, and the row blocks are staged from zq by LDS-DMA (large row counts:
// a tile per 64 x 64 block re-normalising its rows costs more than the extra launch).
template <typename Tin, typename T, int NKS, bool FUSE>
__global__ __launch_bounds__(kSmallThreads) void small_fwd_kernel(const SmallParams p) {
  typedef typename Mfma<T>::frag frag;
  constexpr int RB = NKS * 64;
  __shared__ __attribute__((aligned(16))) char smem[2 * kSmallTile * RB];
  __shared__ float2 red[4][kSmallTile];
  __shared__ int flag;
  lds_char* lds = (lds_char*)smem;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int J = blockIdx.x, I = blockIdx.y;
  const Tin* h = static_cast<const Tin*>(p.hin);
  // row block I (A) and J (B); the diagonal tile stages one block, used as both operands, and
  // publishes it (zq, inv) for the backward
  lds_char* bimg = lds + (I == J ? 0 : kSmallTile * RB);
  if constexpr (FUSE) {
    norm_stage<Tin, T, NKS>(h, p.R, p.d, p.hvec != 0, I * kSmallTile, lds, tid,
                            I == J ? static_cast<T*>(p.zq_out) : nullptr, p.ldk, p.inv_out);
    if (I != J) norm_stage<Tin, T, NKS>(h, p.R, p.d, p.hvec != 0, J * kSmallTile, bimg, tid, nullptr, p.ldk, nullptr);
  } else {
    const long long ldb = (long long)p.ldk * 2;
    const char* zq = static_cast<const char*>(p.zq);
    stage_rows<NKS>(zq, ldb, I * kSmallTile, lds, w, lane);
    if (I != J) stage_rows<NKS>(zq, ldb, J * kSmallTile, bimg, w, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  const int wr = w >> 1, wc = w & 1, r16 = lane & 15, g = lane >> 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    frag a[2], b[2];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int row = 32 * wr + 16 * mi + r16;
      a[mi] = *(__attribute__((address_space(3))) const frag*)(lds + sw_off<NKS>(row, 4 * ks + g));
    }
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int row = 32 * wc + 16 * ni + r16;
      b[ni] = *(__attribute__((address_space(3))) const frag*)(bimg + sw_off<NKS>(row, 4 * ks + g));
    }
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = Mfma<T>::mma(a[mi], b[ni], acc[mi][ni]);
  }

  // masked logits (log2 units) -> per-row (max, sum) over this tile's 64 columns
  const float M = p.y_scale;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row_t = 32 * wr + 16 * mi + 4 * g + r;
      const int gi = I * kSmallTile + row_t;
      const int gpos = gi < p.n_half ? gi + p.n_half : gi - p.n_half;
      float y[2];
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int gj = J * kSmallTile + 32 * wc + 16 * ni + r16;
        const bool drop = (gi >= p.R) | (gj >= p.R) | (gj == gi) | (gj == gpos);
        y[ni] = drop ? kNegInf : acc[mi][ni][r] * M;
        // the positive pair lives in exactly one tile of the row: publish its logit (write-through,
        // read by the row block's last arriver after the ticket below)
        if (FUSE && gj == gpos && gi < p.R) __hip_atomic_store(p.ypos + gi, acc[mi][ni][r] * M, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
      }
      float m = row16_max(fmaxf(y[0], y[1]));
      const float ms = m == kNegInf ? 0.f : m;
      float s = row16_sum(fast_exp2(y[0] - ms) + fast_exp2(y[1] - ms));
      if (r16 == 0) red[wc][row_t] = make_float2(m, s);
    }
  __syncthreads();
  if (tid < kSmallTile) {
    float2 v = red[0][tid];
    const float2 u = red[1][tid];
    lse_merge(v.x, v.y, u.x, u.y);
    // write-through (sc1) partial: the last arriver of the row block reads it with sc1 loads
    float2* dst = p.part + (long long)J * p.Rp64 + I * kSmallTile + tid;
    __hip_atomic_store(reinterpret_cast<float*>(dst), v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<float*>(dst) + 1, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (p.nT > 1) {  // (one column block: this tile is the row block's only one)
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(p.cnt + I, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == p.nT - 1;
      if (last) __hip_atomic_store(p.cnt + I, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag = last;
    }
    __syncthreads();
    if (!flag) return;
  }
  // ---- last tile of row block I: merge the block's partials ----
  // 4 threads per row, each over every 4th column block with 8 write-through (sc1) 8-byte loads
  // in flight at a time (a dependent load per partial made this a 32-deep latency chain); the
  // quarters are combined in order, so the result is deterministic.
  {
    const int row = tid & 63, qq = tid >> 6;
    const int gi = I * kSmallTile + row;
    float m = kNegInf, s = 0.f;
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(p.part) + gi;
    for (int t0 = qq; t0 < p.nT; t0 += 32) {
      unsigned long long v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int t = t0 + 4 * k;
        v[k] = t < p.nT ? __hip_atomic_load(src + (long long)t * p.Rp64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : 0ull;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (t0 + 4 * k < p.nT) {
          const float2 u = __builtin_bit_cast(float2, v[k]);
          lse_merge(m, s, u.x, u.y);
        }
    }
    red[qq][row] = make_float2(m, s);
  }
  __syncthreads();
  float li = 0.f;
  if (tid < kSmallTile) {
    const int gi = I * kSmallTile + tid;
    float2 v = red[0][tid];
#pragma unroll
    for (int q2 = 1; q2 < 4; ++q2) lse_merge(v.x, v.y, red[q2][tid].x, red[q2][tid].y);
    if (gi < p.R) {
      const float m = v.x, s = v.y;
      const float yp = FUSE ? __hip_atomic_load(p.ypos + gi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : p.ypos[gi];
      const float neg2 = (m == kNegInf || s <= 0.f) ? kNegInf : m + log2f(s);
      const float mx = fmaxf(neg2, yp);
      p.lse2[gi] = mx + log2f(exp2f(neg2 - mx) + exp2f(yp - mx));
      const float x = (neg2 - yp) * kLn2;
      li = x > 0.f ? x + log1pf(expf(-x)) : log1pf(expf(x));
      p.arow[gi] = 1.0f / (1.0f + exp2f(yp - neg2));
    } else if (gi < p.Rp64) {
      p.lse2[gi] = 0.f;
      p.arow[gi] = 0.f;
    }
  }
  if (w == 0) {
    const float tot = wave_sum(li);
    if (p.nT == 1) {  // single tile: no cross-block sum
      if (lane == 0) p.loss[0] = tot * p.loss_scale;
      return;
    }
    int last = 0;
    if (lane == 0) {
      __hip_atomic_store(p.loss_part + I, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int old = __hip_atomic_fetch_add(p.cnt + p.nT, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = old == p.nT - 1;
      if (last) __hip_atomic_store(p.cnt + p.nT, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    last = __shfl(last, 0, 64);
    if (last) {  // last row block: sum the row-block partials (lane b holds block b; nT <= 64)
      const float v = lane < p.nT ? __hip_atomic_load(p.loss_part + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : 0.f;
      const float tot_all = wave_sum(v);  // fixed lane tree: deterministic
      if (lane == 0) p.loss[0] = tot_all * p.loss_scale;
    }
  }
}

// ---------------------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------------------
typedef short v4s __attribute__((ext_vector_type(4)));

template <typename Tin, typename T, int NKS>
__global__ __launch_bounds__(kSmallThreads) void small_bwd_kernel(const SmallParams p) {
  typedef typename Mfma<T>::frag frag;
  constexpr int RB = NKS * 64;       // LDS bytes per staged row
  constexpr int NEB = NKS * 2;       // 16-column blocks of dZ (dk / 16)
  constexpr int NBUF = 3;            // Z_J ring: two blocks in flight while one is computed
  constexpr int kRing = NBUF * kSmallTile * RB;
  // ONE __shared__ object (a second one beside the LDS-DMA ring can make hipcc drain vmcnt
  // before the ring's ds_reads: cdna_hip_programming.md §5 item 4(a)): ring | lse | a | flag
  __shared__ __attribute__((aligned(16))) char smem[kRing + 2 * kSmallMaxRows * 4 + 16];
  float* s_lse = reinterpret_cast<float*>(smem + kRing);
  float* s_a = s_lse + kSmallMaxRows;
  int& flag = *reinterpret_cast<int*>(s_a + kSmallMaxRows);
  lds_char* lds = (lds_char*)smem;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int I = blockIdx.x, split = blockIdx.y;
  const int r16 = lane & 15, g = lane >> 4;
  const long long ldb = (long long)p.ldk * 2;
  const char* zq = static_cast<const char*>(p.zq);
  const int j0 = (int)((long long)p.nT * split / p.nS), j1 = (int)((long long)p.nT * (split + 1) / p.nS);

  // row statistics of every row (LSE for P_ji, a_j for the positive term) and this wave's
  // Z_I fragments (rows 16w..16w+15 of the block, B operand of S^T = Z_J Z_I^T)
  for (int k = tid; k < p.Rp64; k += kSmallThreads) {
    s_lse[k] = p.lse2[k];
    s_a[k] = p.arow[k];
  }
  frag zi[NKS];
  {
    const char* rowp = zq + (long long)(I * kSmallTile + 16 * w + r16) * ldb;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) zi[ks] = *reinterpret_cast<const frag*>(rowp + (4 * ks + g) * 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int il = 16 * w + r16;            // tile-local row of this lane in S^T / C
  const int gi = I * kSmallTile + il;
  const int gpos = gi < p.n_half ? gi + p.n_half : gi - p.n_half;
  const float lse_i = s_lse[gi], a_i = s_a[gi];
  const bool row_ok = gi < p.R;
  const float M = p.y_scale;

  f32x4 acc[NEB];
#pragma unroll
  for (int e = 0; e < NEB; ++e) acc[e] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: blocks j0 and j0 + 1 in flight
  if (j0 < j1) stage_rows<NKS>(zq, ldb, j0 * kSmallTile, lds, w, lane);
  if (j0 + 1 < j1) stage_rows<NKS>(zq, ldb, (j0 + 1) * kSmallTile, lds + kSmallTile * RB, w, lane);
  for (int J = j0; J < j1; ++J) {
    const int k = J - j0, buf = k % NBUF;
    // block J landed for this wave (block J+1 may stay in flight: NKS pieces per block), then a
    // raw barrier (no vmcnt drain: __syncthreads would retire the prefetch too): J is visible
    // to every wave, and every wave's reads of block J-1 (lgkmcnt) are done -> its slot is free
    if (J + 1 < j1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NKS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (J + 2 < j1) stage_rows<NKS>(zq, ldb, (J + 2) * kSmallTile, lds + ((k + 2) % NBUF) * kSmallTile * RB, w, lane);
    const lds_char* zj = lds + buf * kSmallTile * RB;
    // S^T blocks: D[j = 16b + 4g + r][i = r16]
    f32x4 st[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) st[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const frag a = *(__attribute__((address_space(3))) const frag*)(zj + sw_off<NKS>(16 * b + r16, 4 * ks + g));
        st[b] = Mfma<T>::mma(a, zi[ks], st[b]);
      }
    // C_ij = P_ij + P_ji (positive: -(a_i + a_p), self / padding: 0), packed as the A operand
    // of the dZ MFMA: k-step s element jj of lane group g <-> column 32s + 16(jj>>2) + 4g + (jj&3)
    frag cf[2];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int jl0 = 16 * b + 4 * g;
      const int gj0 = J * kSmallTile + jl0;
      const f32x4 lj = *reinterpret_cast<const f32x4*>(s_lse + gj0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gj = gj0 + r;
        const float y = st[b][r] * M;
        float c = fast_exp2(y - lse_i) + fast_exp2(y - lj[r]);
        if (gj == gpos) c = -(a_i + s_a[gj]);
        c = (row_ok && gj < p.R && gj != gi) ? c : 0.f;
        cf[b >> 1][(b & 1) * 4 + r] = from_f32<T>(c);
      }
    }
    // dZ_I += C Z_J: B operand = columns of Z_J via the transposed LDS read (4 k-rows x 16
    // columns per 16-lane group; lane 4q+p addresses row q, columns 4p..4p+3)
    const int q = r16 >> 2, pp = r16 & 3;
#pragma unroll
    for (int eb = 0; eb < NEB; ++eb) {
      const int chunk = 2 * eb + (pp >> 1);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ra = 32 * s + 4 * g + q, rb_ = ra + 16;
        const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s*)(zj + sw_off<NKS>(ra, chunk) + (pp & 1) * 8));
        const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4s*)(zj + sw_off<NKS>(rb_, chunk) + (pp & 1) * 8));
        union { v4s v[2]; frag f; } bop;
        bop.v[0] = lo;
        bop.v[1] = hi;
        acc[eb] = Mfma<T>::mma(cf[s], bop.f, acc[eb]);
      }
    }
  }

  // the epilogue's inputs, loaded now so that their latency overlaps the split exchange
  const Tin* h = static_cast<const Tin*>(p.h);
  float hz[4][NEB], ivr[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int gr = I * kSmallTile + 16 * w + 4 * g + r;
    const bool ok = gr < p.R;
    ivr[r] = ok ? p.inv[gr] : 0.f;
#pragma unroll
    for (int eb = 0; eb < NEB; ++eb) {
      const int e = 16 * eb + r16;
      hz[r][eb] = (ok && e < p.d) ? to_f32<Tin>(h[(long long)gr * p.d + e]) : 0.f;
    }
  }

  // ---- column splits: sum the fp32 partial slabs in split order (last arriver) ----
  if (p.nS > 1) {
    // write-through (sc1) 16-B stores of this split's partial in fragment order; the last
    // arriver reads every slab with sc1 loads (MI355X_MICROARCH.md, visibility: Valid forms)
    constexpr int kSlab = kSmallTile * 32 * NKS;  // floats per (row block, split)
    const auto srs = __builtin_amdgcn_make_buffer_rsrc(p.slabs + (long long)I * p.nS * kSlab, 0, p.nS * kSlab * 4,
                                                       0x00020000);
    const int base = (w * NEB) * 64 + lane;  // fragment-order unit (16 B) index
#pragma unroll
    for (int eb = 0; eb < NEB; ++eb)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[eb]), srs,
                                             (split * kSlab + (base + eb * 64) * 4) * 4, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      int* c = p.cnt + p.nT + 1 + I;
      const int old = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == p.nS - 1;
      if (last) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag = last;
    }
    __syncthreads();
    if (!flag) return;
#pragma unroll
    for (int eb = 0; eb < NEB; ++eb) acc[eb] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < p.nS; ++sp) {  // split order: bitwise deterministic
      u32x4 v[NEB];
#pragma unroll
      for (int eb = 0; eb < NEB; ++eb)
        v[eb] = __builtin_amdgcn_raw_buffer_load_b128(srs, (sp * kSlab + (base + eb * 64) * 4) * 4, 0, 16);
#pragma unroll
      for (int eb = 0; eb < NEB; ++eb) acc[eb] += __builtin_bit_cast(f32x4, v[eb]);
    }
  }

  // ---- L2-normalisation backward: lane holds rows 16w + 4g + r, columns 16eb + r16 ----
  const float alpha = p.grad_out[0] * p.alpha_base;
  Tin* dh = static_cast<Tin*>(p.dh);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int gr = I * kSmallTile + 16 * w + 4 * g + r;
    const bool ok = gr < p.R;
    const float iv = ivr[r];
    float z[NEB];
    float dot = 0.f;
#pragma unroll
    for (int eb = 0; eb < NEB; ++eb) {
      z[eb] = hz[r][eb] * iv;
      dot += z[eb] * acc[eb][r];
    }
    dot = row16_sum(dot);
    const float sc = alpha * iv;
#pragma unroll
    for (int eb = 0; eb < NEB; ++eb) {
      const int e = 16 * eb + r16;
      if (ok && e < p.d) dh[(long long)gr * p.d + e] = from_f32<Tin>(sc * (acc[eb][r] - z[eb] * dot));
    }
  }
}

}  // namespace dev

// ======================================================================================
// host side
// ======================================================================================
namespace {
inline int rup(int x, int m) { return (x + m - 1) / m * m; }
int small_nt(const Geometry& g) { return rup(g.rows, dev::kSmallTile) / dev::kSmallTile; }
}  // namespace

bool small_path_eligible(const Geometry& g, DType comp) {
  return g.world == 1 && (comp == DType::F16 || comp == DType::BF16) && g.rows <= kSmallMaxRows &&
         g.dim_k <= kSmallMaxDk && g.ld_k == g.dim_k;
}

int small_bwd_splits(const Geometry& g) {
  // measured (profiles/r2/small_splits.log): more splits win up to 8 at every swept shape; the
  // per-split slab exchange costs less than streaming more column blocks per workgroup
  return std::min(small_nt(g), 8);
}

size_t small_scratch_bytes(const Geometry& g, int splits) {
  const int nt = small_nt(g);
  const size_t ints = 64 + 2 * (size_t)nt + 2;  // fwd counters, loss counter, bwd counters
  auto up = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t part = (size_t)nt * nt * dev::kSmallTile * sizeof(float2);
  const size_t slabs = splits > 1 ? (size_t)nt * splits * dev::kSmallTile * g.dim_k * 4 : 0;
  return up(ints * 4) + up(part) + up((size_t)nt * 4) + up((size_t)nt * dev::kSmallTile * 4) + slabs;
}

namespace {
dev::SmallParams small_params(const Geometry& g, const void* zq, void* scratch, int splits) {
  const int nt = small_nt(g);
  auto up = [](size_t b) { return (b + 255) / 256 * 256; };
  char* b = static_cast<char*>(scratch);
  dev::SmallParams p{};
  p.cnt = reinterpret_cast<int*>(b);
  b += up((64 + 2 * (size_t)nt + 2) * 4);
  p.part = reinterpret_cast<float2*>(b);
  b += up((size_t)nt * nt * dev::kSmallTile * sizeof(float2));
  p.loss_part = reinterpret_cast<float*>(b);
  b += up((size_t)nt * 4);
  p.ypos = reinterpret_cast<float*>(b);
  b += up((size_t)nt * dev::kSmallTile * 4);
  p.slabs = reinterpret_cast<float*>(b);
  p.zq = zq;
  p.R = g.rows;
  p.n_half = g.rows / 2;
  p.ldk = g.ld_k;
  p.d = g.dim;
  p.dk = g.dim_k;
  p.nT = nt;
  p.Rp64 = nt * dev::kSmallTile;
  p.nS = splits;
  p.y_scale = g.inv_temp * dev::kLog2e;
  p.loss_scale = (float)(1.0 / (double)g.global_rows);
  p.alpha_base = (float)(1.0 / ((double)g.global_rows * g.temperature));
  return p;
}

template <typename F>
void by_nks(int dk, F&& f) {
  switch (dk / 32) {
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 6: f(std::integral_constant<int, 6>{}); break;
    case 8: f(std::integral_constant<int, 8>{}); break;
    default: NTXENT_CHECK(false, "small path: unsupported dim_k");
  }
}
}  // namespace

int small_rows_pad(const Geometry& g) { return small_nt(g) * dev::kSmallTile; }

bool small_fwd_fused(const Geometry& g) {
  const int o = small_fuse_rows_override();
  return g.rows <= (o >= 0 ? o : kSmallFuseMaxRows);
}

void launch_small_fwd(DType in, DType comp, const void* h, void* zq, float* inv, float* ypos, float* lse2,
                      float* arow, float* loss, void* scratch, const Geometry& g, hipStream_t stream) {
  NTXENT_CHECK(small_path_eligible(g, comp), "small path: problem not eligible");
  dev::SmallParams p = small_params(g, zq, scratch, 1);
  const bool fuse = small_fwd_fused(g);
  NTXENT_CHECK(fuse || ypos != nullptr, "small forward (unfused): launch_prep's positive logits required");
  if (!fuse) p.ypos = ypos;
  p.hin = h;
  p.hvec = (g.dim % 8 == 0) && (reinterpret_cast<uintptr_t>(h) % 16 == 0);
  p.zq_out = zq;
  p.inv_out = inv;
  p.lse2 = lse2;
  p.arow = arow;
  p.loss = loss;
  const dim3 grid(p.nT, p.nT);
  by_nks(g.dim_k, [&](auto nks) {
    constexpr int NKS = decltype(nks)::value;
    auto go = [&](auto tin, auto tc) {
      using Tin = decltype(tin);
      using Tc = decltype(tc);
      if (fuse)
        hipLaunchKernelGGL((dev::small_fwd_kernel<Tin, Tc, NKS, true>), grid, dim3(dev::kSmallThreads), 0, stream, p);
      else  // (zq is already in the compute dtype: the input dtype plays no part)
        hipLaunchKernelGGL((dev::small_fwd_kernel<Tc, Tc, NKS, false>), grid, dim3(dev::kSmallThreads), 0, stream, p);
    };
    auto by_in = [&](auto tc) {
      switch (in) {
        case DType::F32: go(float{}, tc); break;
        case DType::F16: go(_Float16{}, tc); break;
        case DType::BF16: go(__bf16{}, tc); break;
        default: NTXENT_CHECK(false, "small path: bad input dtype");
      }
    };
    if (comp == DType::F16) by_in(_Float16{});
    else by_in(__bf16{});
  });
  NTXENT_HIP_CHECK(hipGetLastError());
}

void launch_small_bwd(DType in, DType comp, const void* zq, const void* h, const float* inv, const float* lse2,
                      const float* arow, const float* grad_out, void* dh, void* scratch, const Geometry& g,
                      hipStream_t stream, int splits) {
  NTXENT_CHECK(small_path_eligible(g, comp), "small path: problem not eligible");
  if (splits <= 0) splits = small_bwd_splits(g);
  NTXENT_CHECK(splits <= small_nt(g), "small path: more column splits than column blocks");
  dev::SmallParams p = small_params(g, zq, scratch, splits);
  p.h = h;
  p.inv = inv;
  p.lse2 = const_cast<float*>(lse2);
  p.arow = const_cast<float*>(arow);
  p.grad_out = grad_out;
  p.dh = dh;
  const dim3 grid(p.nT, splits);
  by_nks(g.dim_k, [&](auto nks) {
    constexpr int NKS = decltype(nks)::value;
    auto go = [&](auto tin, auto tc) {
      using Tin = decltype(tin);
      using Tc = decltype(tc);
      hipLaunchKernelGGL((dev::small_bwd_kernel<Tin, Tc, NKS>), grid, dim3(dev::kSmallThreads), 0, stream, p);
    };
    auto by_in = [&](auto tc) {
      switch (in) {
        case DType::F32: go(float{}, tc); break;
        case DType::F16: go(_Float16{}, tc); break;
        case DType::BF16: go(__bf16{}, tc); break;
        default: NTXENT_CHECK(false, "small path: bad input dtype");
      }
    };
    if (comp == DType::F16) by_in(_Float16{});
    else by_in(__bf16{});
  });
  NTXENT_HIP_CHECK(hipGetLastError());
}

}  // namespace ntxent

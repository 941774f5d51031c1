// The NT-Xent similarity GEMM for gfx950 and its fused epilogues.
//
//   out tile (256 x 256) = A_tile (256 x K) * B_tile (256 x K)^T, both operands K-contiguous.
//
// Workgroup = 8 wave64s. K advances in 128-byte steps (64 fp16/bf16 or 32 fp32 per row).
// LDS holds two K-steps (even/odd buffer) of A and B, laid out [A even | A odd | B even |
// B odd] (32 KiB each, so every operand read is a lane base + a 16-bit immediate), each split
// into two 128-row halves (A0, A1, B0, B1: 16 KiB each), filled by buffer_load_dwordx4 ... lds
// from a scalar V# (lane-linear destination; the bank swizzle phys_chunk = chunk ^ ((row>>1)&7)
// is applied on the source offset and on the ds_read_b128 side, conflict-free for the 16x16x32
// operand lane groups).
//
// Main loop: every K-step is 4 phases, one per 128x128 C-quadrant (A0B0, A0B1, A1B0, A1B1);
// in each phase all 8 waves compute 64x32 of that quadrant (16 MFMA 16x16x32 per wave). A
// half-tile is re-staged as soon as its last LDS read is one barrier behind, so loads run
// ~1.75 K-steps ahead; every wait is a counted `s_waitcnt vmcnt(10)` (5 half-tiles still in
// flight) followed by a raw s_barrier — no vmcnt(0) drains in the loop
// (cdna_hip_programming.md §5 "Pipelining across barriers", T3/T4). The forward streams its
// operands across whole-tile work items: the last two K-steps' prefetches load the next item's
// first two, under the epilogue (see kStreamMode in the kernel).
//
// Accumulator acc[mi][ni] (mi < 8, ni < 4) covers tile rows rbase(mi)..+15 and columns
// cbase(ni)..+15 with rbase(mi) = 128(mi>>2) + 64 wa + 16(mi&3), cbase(ni) = 128(ni>>1) +
// 32 wb + 16(ni&1) for wave w = 4 wa + wb. Kept cosine tiles use a canonical fragment order
// (16x16 block (rb, cb) at ((rb*16 + cb)*64 + lane)*4) so producers and consumers with
// different wave layouts agree.
#pragma once

#include "../include/ntxent/ntxent.h"
#include "device_common.h"

#include <type_traits>

namespace ntxent {
namespace dev {

enum SimMode : int { kModeFwd = 0, kModeCoef = 1, kModeDz = 2 };

constexpr int kStageBytes = 2 * kTile * kKStepBytes;  // one operand, both parities = 64 KiB
// cache-policy bits of the GEMM operand LDS-DMA (0: default policy; experiment builds set
// NTXENT_GEMM_DMA_AUX, e.g. 2 = nt, 1 = sc0: tools/build_variant.sh)
#ifndef NTXENT_GEMM_DMA_AUX
#define NTXENT_GEMM_DMA_AUX 0
#endif
constexpr int kGemmDmaAux = NTXENT_GEMM_DMA_AUX;
// Diagnostic builds (tools/build_variant.sh TAG -DNTXENT_TIMING=1; tools/gemm_timing.py): thread 0
// of every GEMM block records s_memtime at four points of each of its first kTimingItems work
// items -- item start, main loop start (prologue landed), main loop end, epilogue end -- and the
// launcher writes them to $NTXENT_TIMING_OUT. Off in every production build.
#ifndef NTXENT_TIMING
#define NTXENT_TIMING 0
#endif
constexpr int kTimingItems = 8;
constexpr int kTimingMarks = 8;  // per item: start, loop start, loop end, epilogue end, 4-7 epilogue phases
// 16-byte write-through (sc1) store at base + off: the line goes to memory at once, so the kernel
// boundary has no dirty L2 lines of it to write back. The buffer descriptor must be wave-uniform
// (a per-lane one makes hipcc emit a waterfall loop): its base is the first active lane's offset
// less 64 MiB, 1 MiB aligned (SGPR arithmetic), so any lane within 64 MiB below and ~1.9 GiB above
// the first lane's offset stores at a non-negative 32-bit offset from it; callers' waves span a
// few rows of one tensor (at most a few MiB).
__device__ __forceinline__ void store16_wt(void* base, long long off, u32x4 v) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)off);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((unsigned long long)off >> 32));
  const long long f0 = (long long)(((unsigned long long)hi << 32) | lo) - (64ll << 20);
  const long long wb = f0 > 0 ? (f0 & ~0xFFFFFll) : 0;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(static_cast<char*>(base) + wb, 0, 0x7FFFFFFF, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(off - wb), 0, 16);
}

// Byte offset of element (r, c) inside a row-major 256 x 256 coefficient tile of es-byte
// elements. (A K-step-blocked layout, [kstep][row][128 B], measured neutral: profiles/r4/variants.)
__device__ __forceinline__ long long ctile_off(int r, int c, int es) { return ((long long)r * kTile + c) * es; }
constexpr int kGemmLds = 2 * kStageBytes;             // A and B, even/odd K-step = 128 KiB
constexpr int kCtStride = kTile * 2 + 16;             // C^T staging row: 512 B + 16 B pad
constexpr int kCoefLds = kTile * kCtStride;           // 132 KiB
constexpr int kCoefWaveLds = 64 * (64 * 2 + 16);      // C^T of one 64x64 region (8 KiB used when swizzled: ct_swz)
constexpr int kHalfBytes = 128 * kKStepBytes;         // one half-tile of one operand = 16 KiB

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
  int b_tile0;           // B operand: global column tile of the chunk's first row tile (ring mode)
  int c_ld, c_tile0;     // coefficient tile slot = mt * c_ld + (nt - c_tile0)
  int c_rot;             // symmetric mode: column slot (nt - row_tile0) mod col_tiles instead (sym_c_ld)
  // half C (world 1, 16-bit, whole-tile dZ items): the coefficient pass writes only the upper
  // tiles (J >= I; no mirror of an off-diagonal tile) and the dZ reads a lower tile C_IJ (J < I)
  // as the transpose of C_JI (dz_tr_stage / ds_read_b64_tr_b16): 64 MiB fewer C bytes written at
  // the headline
  int c_half;
  // raw-operand forward (RawRows): A / B are the input rows h, not unit rows; the accumulators are
  // normalised by inv_a[A row] * inv_b[B row] before the epilogue (null: unit-row operands)
  const float* inv_a;
  const float* inv_b;
  float y_scale;         // inv_temp * log2(e) = M, the largest possible logit (log2 units)
  float acc_scale;       // logit (log2 units) per accumulator unit (y_scale)
  int scale_off;         // fp8 operands: byte offset of each row's E8M0 scale (= K bytes of a row)
  int fixed_shift;       // 1: exponentials use the fixed shift M (2M < 120, see fwd epilogue)
  float2* part;          // [col_tiles][Rpad] partial (max, sum) in log2 units
  char* sc;              // kept cosines: [n_fwd_tiles][256*256] (canonical fragment order)
  char* cbuf;            // coefficients: [row_tiles][col_tiles][256*256] (row-major per tile)
  const float* lse2;     // [W*Rpad] lse in log2 units (all ranks)
  const float* cpos;     // [Rpad] positive coefficient C_i,p(i) = -(a_i + a_p), a = 1 - P_ip
  float2* part_x;        // symmetric mode: column partials of kTileCross tiles (per partner)
  char* mbuf;            // symmetric mode: mirrored coefficient tiles of kTileCross tiles
  float* out;            // dZ slabs
  long long ldo;         // elements
  long long slab_stride; // elements
  int accum;             // dZ: add the tile into `out` (sub-block GEMMs of one gradient)
  int out_f16;           // dZ: write `out` as fp16 (partner gradient contributions on the wire)
  // Fused normalisation backward (see dot_slots / dz_store):
  float* dotp;           // coefficient pass: partials of dot_i = sum_j C_ij cos_ij, [4 col_tiles][Rpad]
  const void* nh;        // dZ epilogue: input rows h [R][nd] (dtype nh_dt: 0 fp32, 1 fp16, 2 bf16) ...
  int nh_dt, nd;
  const float* ninv;     // ... 1 / |h_i|
  const float* ndot;     // ... dot_i (reduced dotp)
  int dot_nslot;         // ... > 0: the dZ grid reduces dotp (dot_nslot slots) into ndot itself
  int dot_spin;          //     polls before dz_dot's fallback (tests: 0 forces the fallback)
  int* dot_cnt;          //     (dz_dot_fold), published through these [2] zeroed counters (self-
                         //     cleaning) to its own epilogues; null for split-K pieces
  const float* ngo;      // ... grad_out (device scalar)
  float nalpha;          // ... 1 / (2N tau)
  void* ndh;             // ... output dh [R][nd] (non-null: fused epilogue)
  // fp8 backward (Q8Stats): per-row e4m3 scale inputs (q8_row_exp) and the fp16 rows for the
  // dZ epilogue's exact positive term
  const float* q8_mneg;
  const float* q8_lmin;
  const _Float16* q8_zq;
  int q8_ldz;
  // persistent stream-K schedule (see sim_gemm_kernel)
  int nk;                // K-steps per tile
  int dp_tiles;          // whole-tile items processed in rounds of gridDim
  int sk_tiles;          // tiles whose K-steps are split evenly over the grid
  long long ipb;         // stream-K K-steps per block
  float* sk_slabs;       // [2 * gridDim][256*256] fp32 partial tiles
  int* sk_cnt;           // [sk_tiles] arrival counters (zero at launch; self-cleaning)
  int splitk;            // split-K for tile-starved launches: tile-aligned pieces of ipb K-steps,
                         // piece-major (block b = piece b / sk_tiles of tile b % sk_tiles, slab
                         // slot 2 b + 1); every piece only publishes its slab and sk_reduce_kernel /
                         // sk_dz_reduce_kernel sum a tile's slabs and run its epilogue
  int sk_half;           // split-K forward of a 2-byte plan: fp16 partial tiles,
                         // half the slab bytes written and re-read (sk_fixup: fragment pairs of a
                         // lane in 16-B units)
#if NTXENT_TIMING
  unsigned long long* tstamp;  // [grid][kTimingItems][kTimingMarks] s_memtime marks (diagnostic builds only)
#endif
};

// Kept-cosine layout for 2-byte types: one 16-byte unit per lane holds the fragments of the
// 16-column blocks cb and cb + 16 (cb a multiple of 32) of the 16-row block at rb (4 values
// each, MFMA C layout). Element offset of the unit = sc_unit(...) * 8. fp32 tiles keep one
// fragment per 16-byte unit: (((rb >> 4) * 16 + (cb >> 4)) * 64 + lane) * 4.
__device__ __forceinline__ int sc_unit(int rb, int cb, int lane) { return ((rb >> 4) * 8 + (cb >> 5)) * 64 + lane; }

// One monotonically advancing K position of a staged half-tile stream of one operand row tile
// (clamped at the last K-step, so the trailing prefetches of the schedule re-read valid
// memory; forward streaming re-initialises a stream onto the next item instead).
struct KStream {
  const char* ptr;  // the K-step to stage next
  int kin, left;    // byte offset inside its K block; K-steps after it
  int kk;           // K-step index (of the whole K range) of ptr
  __device__ __forceinline__ void init(const char* base, long long k0, const OperandDesc& o, int nk) {
    kin = (int)(k0 % o.kblk);
    ptr = base + (k0 / o.kblk) * o.kblk_stride + kin;
    left = nk - 1;
    kk = (int)(k0 / kKStepBytes);
  }
  __device__ __forceinline__ void advance(const OperandDesc& o) {
    if (left > 0) {
      --left;
      ++kk;
      ptr += kKStepBytes;
      kin += kKStepBytes;
      if (kin == (int)o.kblk) { kin = 0; ptr += o.kblk_stride - o.kblk; }  // (K blocks < 2 GiB: 32-bit test)
    }
  }
  // half C: a K-step staged from the transposed tile advances the position only (ptr was placed
  // at the item's first regular K-step by seek)
  __device__ __forceinline__ void skip() {
    if (left > 0) {
      --left;
      ++kk;
    }
  }
  __device__ __forceinline__ void seek(const char* base, long long k0, const OperandDesc& o) {
    kin = (int)(k0 % o.kblk);
    ptr = base + (k0 / o.kblk) * o.kblk_stride + kin;
  }
};

// C^T staging of one 64x64 region by one wave (coef_kernel): LDS row L (C column L) is 128 B of
// 16 8-byte granules (4 C rows each); granule j sits at slot j ^ ct_swz(L). This is conflict-free
// for all three accesses of the staging (MI355X_MICROARCH.md §LDS banking): the ds_write_b64 of a
// fragment (16 lanes = 16 rows L of one granule, banks mod 32: the low 4 bits of L -> 16 distinct
// slots), the ds_read_b64_tr_b16 row reads (32 lanes = rows {b..b+3, b+8..b+11} x 4 granules,
// banks mod 64: slots' top 2 bits biject (L bit 1, L bit 3)) and the mirror's ds_read_b64 pairs
// (rows L, L+2 of one row parity x 8 granules of one parity: slot bit 0 flips with L bit 1). The
// round-4 form (rows padded to 144 B) was 2-way conflicted on all three (1.58 M conflict cycles
// per headline coefficient pass, profiles/r4/pmc_final).
__device__ __forceinline__ int ct_swz(int L) {
  return ((L >> 1) & 1) | ((L & 1) << 1) | (((L >> 3) & 1) << 2) | ((((L >> 1) ^ (L >> 2)) & 1) << 3);
}

// A dot partial slot (coefficient pass; read by dot_reduce_kernel in the next launch). (Folding
// that reduction into this launch -- each 64-row group's last contributing wave sums its slots,
// found by an agent-scope ticket -- measured 42 -> 64 us for the pass at the headline: every
// wave waits for its ticket's return under contention. profiles/r5/coef_dot/.)
__device__ __forceinline__ void dot_slot_store(float* p, float v) { *p = v; }

// Tile index of coefficient tile (mt, nt) in cbuf (row-major [row_tiles][c_ld] tiles).
__device__ __forceinline__ long long ctile_index(const SimParams& p, int mt, int nt) {
  const int cs = p.c_rot ? (nt - p.row_tile0 + p.col_tiles) % p.col_tiles : nt - p.c_tile0;
  return (long long)mt * p.c_ld + cs;
}

// ------------------------------------------------------------------------------------
// Coefficient epilogue shared by the store-mode coef kernel (NW = 1: one wave, a 128x64
// region at (row_base, col_base)) and the recompute GEMM (NW = 8: the whole tile).
//   C_ij = 2^(y - lse2_i) + 2^(y - lse2_j), C_ip = cpos_i, 0 on the diagonal / padding,
// staged transposed in LDS, then written row-major into slot (mt, nt) with 16-B stores
// (rows via ds_read_b64_tr_b16) and, for a mirrored tile, into the lower-triangular slot.
// ------------------------------------------------------------------------------------
template <typename T, int NW, int NMI = 8>
__device__ __forceinline__ void coef_epilogue(f32x4 (&acc)[NMI][4], const int (&rb)[NMI], const int (&cb)[4],
                                              int row_base, int col_base, int mt, int nt, int kind,
                                              lds_char* lds, const SimParams& p, int lane) {
  constexpr int NROWS = NW == 8 ? kTile : NMI * 16;
  constexpr int NCOLS = NW == 8 ? kTile : 64;
  // C^T staging: one wave (64 x 64 region): 128-B rows, granules swizzled by ct_swz; the whole
  // tile (NW = 8, recompute path): rows padded by 16 B
#ifndef NTXENT_COEF_SWZ
#define NTXENT_COEF_SWZ 1  // A/B switch (tools/build_variant.sh -DNTXENT_COEF_SWZ=0: the round-4 padded rows)
#endif
  constexpr bool SWZ = NW == 1 && NTXENT_COEF_SWZ;
  static_assert(!SWZ || (NROWS == 64 && NCOLS == 64), "swizzled C^T staging is for 64 x 64 regions");
  constexpr int S = SWZ ? 128 : NROWS * 2 + 16;  // LDS row stride (bytes) of the C^T staging tile
  // byte offset of C rows e .. e+3 (e % 4 == 0) of staged column L
  auto ct_at = [&](int L, int e) { return SWZ ? L * S + (((e >> 2) ^ ct_swz(L)) << 3) : L * S + e * 2; };
  constexpr int NT = NW * 64;        // threads in the calling block
  T* base = reinterpret_cast<T*>(p.cbuf);
  const int col_local0 = (nt * kTile) % p.Rpad;  // rank-local column of this tile's col 0
  // Fixed-shift form (2M < 120, see the forward epilogue):
  // C = 2^(y - M) * (2^(M - lse2_i) + 2^(M - lse2_j)), one exp2 per element.
  const bool fixed = p.fixed_shift != 0;
  const float M = p.y_scale;
  float lcol[4];
  bool cvalid[4];
  int gj[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int col_t = cb[ni] + (lane & 15);
    gj[ni] = nt * kTile + col_t;
    const float l = p.lse2[gj[ni]];
    lcol[ni] = fixed ? fast_exp2(M - l) : l;
    cvalid[ni] = (col_local0 + col_t) < p.R;
  }
  T* slot = base + ctile_index(p, mt, nt) * kTileElems;
  T* mirror = nullptr;
  // (kTileDiagUp: the same tile's slot; half C: no lower off-diagonal tiles, the dZ reads C_JI^T)
  if ((kind == kTileSymOff && !p.c_half) || kind == kTileDiagUp)
    mirror = base + ctile_index(p, nt - p.row_tile0, p.row_tile0 + mt) * kTileElems;
  else if (kind == kTileCross) {  // partner block C_{q,rank}: mbuf tile (slot, nt % rt, mt)
    const int rt = p.Rpad / kTile, W = p.col_tiles / rt, q = nt / rt;
    const int slot = (q - p.row_tile0 / rt - 1 + W) % W;  // partners r+1, r+2, ... -> slots 0, 1, ...
    mirror = reinterpret_cast<T*>(p.mbuf) + ((long long)(slot * rt + nt % rt) * rt + mt) * kTileElems;
  }
  // dot partial slots of row i: 4 per column tile J (the quarter of J's columns a wave covered, or
  // for the column partials of a mirrored tile the quarter of its rows); each written once,
  // slot-major ([slot][Rpad]: a store instruction's lanes hold neighbouring rows)
  const int wq = NW == 8 ? ((threadIdx.x >> 6) & 3) : (col_base >> 6);  // column quarter of this wave
  float cdot[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  // plain region (uniform): no self or positive element and no padding among this call's rows x
  // columns, so C is the exponential alone, without the per-element compares and selects
  // (coefficient pass -10 % at the headline and config 2: profiles/r4/variants_r4_v25_coefplain.md)
  const int r_lo = mt * kTile + row_base, r_hi = r_lo + NROWS;
  const int c_lo = nt * kTile + col_base, c_hi = c_lo + NCOLS;
  auto hits = [&](int a0) { return a0 < c_hi && c_lo < a0 + NROWS; };
  const bool plain = fixed && r_hi <= p.R && col_local0 + col_base + NCOLS <= p.R && !hits(p.own0 + r_lo) &&
                     !hits(p.own0 + r_lo + p.n_half) && !hits(p.own0 + r_lo - p.n_half);
  // (row LSEs of all blocks loaded up front and the dot partials stored after the block loop,
  // one transposing reduction per 4 rows: the pass measured 42 -> 44 us at the headline and
  // 149 -> 154 us at config 5, not kept; the e4m3 epilogue below gains from the same change)
#pragma unroll
  for (int mi = 0; mi < NMI; ++mi) {
    float c[4][4];
    const int row_t0 = rb[mi] + 4 * (lane >> 4);
    const int gi0 = mt * kTile + row_t0;  // 4 consecutive rows
    const f32x4 lrow4 = *reinterpret_cast<const f32x4*>(p.lse2 + p.own0 + gi0);
    const f32x4 cpos4 = *reinterpret_cast<const f32x4*>(p.cpos + gi0);
    if (plain) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float lrow = fast_exp2(M - lrow4[r]);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) c[ni][r] = fast_exp2(acc[mi][ni][r] * p.acc_scale - M) * (lrow + lcol[ni]);
      }
    } else
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gi = gi0 + r;
      const bool rvalid = gi < p.R;
      const float lrow = fixed ? fast_exp2(M - lrow4[r]) : lrow4[r];
      const int gself = p.own0 + gi;
      const int gpos = p.own0 + (gi < p.n_half ? gi + p.n_half : gi - p.n_half);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const float y = acc[mi][ni][r] * p.acc_scale;
        float v = fixed ? fast_exp2(y - M) * (lrow + lcol[ni]) : fast_exp2(y - lrow) + fast_exp2(y - lcol[ni]);
        v = (gj[ni] == gpos) ? cpos4[r] : v;  // positive: -(a_i + a_p), no 1 - P cancellation
        v = (rvalid && cvalid[ni] && gj[ni] != gself) ? v : 0.0f;
        c[ni][r] = v;
      }
    }
    if (p.dotp) {
      // dot_i = sum_j C_ij cos_ij (= z_i . g_i of the normalisation backward), with C as the dZ
      // GEMM reads it (rounded to T): row partials over this wave's columns; for a mirrored tile
      // also column partials (the lower tile's rows) over this wave's rows.
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float d = 0.f;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) d += to_f32<T>(from_f32<T>(c[ni][r])) * acc[mi][ni][r];
        d = row16_sum(d);
        const int row = mt * kTile + rb[mi] + 4 * (lane >> 4) + r;
        if ((lane & 15) == 0) dot_slot_store(p.dotp + (long long)(nt * 4 + wq) * p.Rpad + row, d);
      }
      const int h2 = NMI == 8 ? (mi >> 2) : 0;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) cdot[h2][ni] += to_f32<T>(from_f32<T>(c[ni][r])) * acc[mi][ni][r];
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int col_t = cb[ni] + (lane & 15);
      if constexpr (sizeof(T) == 2) {
        // stage C^T in LDS: Ct[col][row0..row0+3] (one ds_write_b64 per fragment)
        union { T h[4]; u32x2 u; } pk;
#pragma unroll
        for (int r = 0; r < 4; ++r) pk.h[r] = from_f32<T>(c[ni][r]);
        *reinterpret_cast<__attribute__((address_space(3))) u32x2*>(lds + ct_at(col_t - col_base, row_t0 - row_base)) =
            pk.u;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          *reinterpret_cast<float*>(reinterpret_cast<char*>(slot) + ctile_off(row_t0 + r, col_t, 4)) = c[ni][r];
        if (mirror)
          *reinterpret_cast<f32x4*>(reinterpret_cast<char*>(mirror) + ctile_off(col_t, row_t0, 4)) =
              f32x4{c[ni][0], c[ni][1], c[ni][2], c[ni][3]};
      }
    }
  }
  if (p.dotp) {
    if (kind == kTileSymOff || kind == kTileDiagUp) {
      const int wa8 = (threadIdx.x >> 6) >> 2;
#pragma unroll
      for (int h2 = 0; h2 < (NMI == 8 ? 2 : 1); ++h2)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const float d = xrow_sum(cdot[h2][ni]);
          const int rq = NMI == 8 ? 2 * h2 + wa8 : (row_base >> 6);  // row quarter of this wave's rows
          const int row = (nt - p.row_tile0) * kTile + cb[ni] + (lane & 15);
          if (lane < 16) dot_slot_store(p.dotp + (long long)((p.row_tile0 + mt) * 4 + rq) * p.Rpad + row, d);
        }
    }
  }
  if constexpr (sizeof(T) == 2) {
    __syncthreads();
    const int tid = threadIdx.x, w = tid >> 6;  // w = wave index inside the calling block
    // (a) mirrored tile: Ct rows are rows of C^T -> coalesced 16-B stores into the mirror slot.
    if (mirror) {
      constexpr int CPR = NROWS * 2 / 16;  // 16-B chunks per staged row
#pragma unroll 4
      for (int q = 0; q < NCOLS * CPR / NT; ++q) {
        const int k = tid + NT * q;
        const int row = k / CPR, c16 = k % CPR;
        u32x4 v;
        if constexpr (SWZ) {  // two 8-byte granules (not adjacent once swizzled)
          typedef __attribute__((address_space(3))) const u32x2 lds_u2;
          const u32x2 lo = *(lds_u2*)(lds + ct_at(row, 8 * c16)), hi = *(lds_u2*)(lds + ct_at(row, 8 * c16 + 4));
          v = u32x4{lo[0], lo[1], hi[0], hi[1]};
        } else {
          v = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(lds + row * S + c16 * 16);
        }
        *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(mirror) + ctile_off(col_base + row, row_base + 8 * c16, 2)) = v;
      }
    }
    // (b) rows of C = columns of Ct via the gfx950 transposed LDS read (ds_read_b64_tr_b16):
    //     a 16-lane group reads a 4 (Ct rows) x 16 (Ct cols) block and lane i receives column
    //     i, i.e. 4 consecutive entries of C row c0+i. Two reads give 16 B per lane.
    typedef short v4s __attribute__((ext_vector_type(4)));
    constexpr int RB = NROWS / 16;                // 16-row blocks of C in this call
    constexpr int NBLK = RB * (NCOLS / 32) / NW;  // 16x32 blocks per wave (= 16)
    const int g = lane >> 4, i = lane & 15, q4 = i >> 2, p4 = i & 3;
#pragma unroll 2
    for (int b = 0; b < NBLK; ++b) {
      const int blk = w * NBLK + b;
      const int c0 = (blk % RB) * 16;  // C rows row_base+c0 .. +15
      const int r0 = (blk / RB) * 32 + 8 * g;  // C cols col_base+r0 .. +7
      const lds_char* a0 = lds + ct_at(r0 + q4, c0 + 4 * p4);
      const lds_char* a1 = lds + ct_at(r0 + q4 + 4, c0 + 4 * p4);
      const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)a0);
      const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)a1);
      u32x4 u;
      u[0] = (unsigned short)lo[0] | ((unsigned)(unsigned short)lo[1] << 16);
      u[1] = (unsigned short)lo[2] | ((unsigned)(unsigned short)lo[3] << 16);
      u[2] = (unsigned short)hi[0] | ((unsigned)(unsigned short)hi[1] << 16);
      u[3] = (unsigned short)hi[2] | ((unsigned)(unsigned short)hi[3] << 16);
      // lanes i + 16 g hold 16-byte chunk g of row c0 + i: permute so that lane 4 i + g holds it,
      // and each 4-lane quad stores one contiguous 64-byte row segment (one row per quad
      // instead of four: a quad spanning four rows cost the store path ~4x its cycles)
      const int src = ((lane >> 2) + 16 * (lane & 3)) << 2;
      u32x4 v;
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)u[k]);
      char* cdst = reinterpret_cast<char*>(slot) +
                   ctile_off(row_base + c0 + (lane >> 2), col_base + (blk / RB) * 32 + 8 * (lane & 3), 2);
#ifndef NTXENT_COEF_STORE
#define NTXENT_COEF_STORE 0  // A/B switch: 0 default policy, 1 non-temporal, 2 write-through
#endif
      if constexpr (NTXENT_COEF_STORE == 1)
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(cdst));
      else if constexpr (NTXENT_COEF_STORE == 2)
        store16_wt(slot, cdst - reinterpret_cast<char*>(slot), v);
      else
        *reinterpret_cast<u32x4*>(cdst) = v;
    }
  }
}

// fp8 backward coefficient epilogue (store mode, one wave per 64 x 64 region of a kept cosine
// tile): C as coef_epilogue, quantised to e4m3 with the row scale 2^e_i (q8_row_exp) for the
// stored tile and 2^e_j for its mirror (row j of the lower tile); the positive entry is stored as
// 0 (the dZ epilogue adds C_ip z_p exactly). Both byte tiles are staged in LDS (stride 80 B: the
// column-major writes hit distinct banks) and leave as 16-byte row segments. A lane's 4 rows of
// one column pack into a dword (the mirror's layout); for the stored tile a quad of lanes
// transposes its 4 x 4 bytes in two DPP + v_perm stages, so that each lane holds 4 consecutive
// columns of one row. The dot partials use the dequantised C (as the dZ GEMM reads it) with the
// power-of-two scale factored out of the sums. The pass is VALU-bound (at 2.6 TB/s in round 4),
// so the plain regions (no self, positive or padding element: uniform per wave) skip the masks.
__device__ __forceinline__ unsigned q8_pack4(float x0, float x1, float x2, float x3) {  // x >= 0
  const int w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(x0, 448.f), fminf(x1, 448.f), 0, false);
  return (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(fminf(x2, 448.f), fminf(x3, 448.f), w, true);
}
// sum_r e4m3(w byte r) * a[r]
__device__ __forceinline__ float q8_dot4(unsigned w, const f32x4& a) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, false), hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, true);
  return fmaf(lo[0], a[0], fmaf(lo[1], a[1], fmaf(hi[0], a[2], hi[1] * a[3])));
}

template <typename TS>
__device__ __forceinline__ void coef_epilogue_q8(f32x4 (&acc)[4][4], const int (&rb)[4], const int (&cb)[4],
                                                 int row_base, int col_base, int mt, int nt, int kind, lds_char* lds,
                                                 const SimParams& p, int lane) {
  constexpr int S8 = 80;  // LDS row stride of both staged byte tiles (64 B + 16 B)
  lds_char* ld_d = lds;             // stored tile: [64 rows][64 cols]
  lds_char* ld_m = lds + 64 * S8;   // mirror: [64 cols][64 rows]
  unsigned char* base = reinterpret_cast<unsigned char*>(p.cbuf);
  unsigned char* slot = base + ctile_index(p, mt, nt) * kTileElems;
  const bool mirrored = kind == kTileSymOff || kind == kTileDiagUp;
  unsigned char* mirror = mirrored ? base + ctile_index(p, nt - p.row_tile0, p.row_tile0 + mt) * kTileElems : nullptr;
  const int col_local0 = (nt * kTile) % p.Rpad;
  const bool fixed = p.fixed_shift != 0;
  const float M = p.y_scale;
  const float lmin = p.q8_lmin[0];
  float lcol[4], scol[4], icol[4];
  bool cvalid[4];
  int gj[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int col_t = cb[ni] + (lane & 15);
    gj[ni] = nt * kTile + col_t;
    const float l = p.lse2[gj[ni]];
    lcol[ni] = fixed ? fast_exp2(M - l) : l;
    cvalid[ni] = (col_local0 + col_t) < p.R;
    const int e = q8_row_exp(p.q8_mneg[gj[ni]], lmin);
    scol[ni] = exp2i(e);
    icol[ni] = exp2i(-e);
  }
  float dsv[4];  // row partial of row (lane >> 2) & 3 of each 4-row block (stored after the loop)
  // plain region: as coef_epilogue
  const int r_lo = mt * kTile + row_base, r_hi = r_lo + 64;
  const int c_lo = nt * kTile + col_base, c_hi = c_lo + 64;
  auto hits = [&](int a0) { return a0 < c_hi && c_lo < a0 + 64; };
  const bool plain = fixed && r_hi <= p.R && col_local0 + col_base + 64 <= p.R && !hits(p.own0 + r_lo) &&
                     !hits(p.own0 + r_lo + p.n_half) && !hits(p.own0 + r_lo - p.n_half);
  const int wq = col_base >> 6;
  float cdot[4] = {0.f, 0.f, 0.f, 0.f}, cposd[4] = {0.f, 0.f, 0.f, 0.f};
  // quad byte transpose (lane q of a quad holds bytes M[q][0..3]; afterwards T[q][r] = M[r][q]):
  // exchange 16-bit halves with lane q ^ 2, then bytes with lane q ^ 1
  const int qd = lane & 3;
  const unsigned sel1 = qd < 2 ? 0x05040100u : 0x03020706u;
  const unsigned sel2 = (qd & 1) ? 0x03070105u : 0x06020400u;
  f32x4 lrow_h[4], mneg_h[4];  // loaded up front (as coef_epilogue)
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int gi0 = mt * kTile + rb[mi] + 4 * (lane >> 4);
    lrow_h[mi] = *reinterpret_cast<const f32x4*>(p.lse2 + p.own0 + gi0);
    mneg_h[mi] = *reinterpret_cast<const f32x4*>(p.q8_mneg + p.own0 + gi0);
  }
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int row_t0 = rb[mi] + 4 * (lane >> 4);
    const int gi0 = mt * kTile + row_t0;
    const f32x4 lrow4 = lrow_h[mi];
    const f32x4 mneg4 = mneg_h[mi];
    float srow[4], lrow[4], rdot[4] = {0.f, 0.f, 0.f, 0.f}, rposd[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      srow[r] = exp2i(q8_row_exp(mneg4[r], lmin));
      lrow[r] = fixed ? fast_exp2(M - lrow4[r]) : lrow4[r];
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      float c[4];
      if (plain) {
#pragma unroll
        for (int r = 0; r < 4; ++r) c[r] = fast_exp2(acc[mi][ni][r] * p.acc_scale - M) * (lrow[r] + lcol[ni]);
      } else {
        const f32x4 cpos4 = *reinterpret_cast<const f32x4*>(p.cpos + gi0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gi = gi0 + r;
          const int gself = p.own0 + gi;
          const int gpos = p.own0 + (gi < p.n_half ? gi + p.n_half : gi - p.n_half);
          const float y = acc[mi][ni][r] * p.acc_scale;
          const float v = fixed ? fast_exp2(y - M) * (lrow[r] + lcol[ni]) : fast_exp2(y - lrow[r]) + fast_exp2(y - lcol[ni]);
          const bool ok = gi < p.R && cvalid[ni] && gj[ni] != gself;
          const bool pos = ok && gj[ni] == gpos;
          c[r] = (ok && !pos) ? v : 0.0f;
          // the positive entry is exact in the dZ epilogue; its dot term likewise
          const float pd = pos ? cpos4[r] * acc[mi][ni][r] : 0.f;
          rposd[r] += pd;
          cposd[ni] += pd;
        }
      }
      const unsigned w_d = q8_pack4(c[0] * srow[0], c[1] * srow[1], c[2] * srow[2], c[3] * srow[3]);
      const unsigned w_m = q8_pack4(c[0] * scol[ni], c[1] * scol[ni], c[2] * scol[ni], c[3] * scol[ni]);
      if (p.dotp) {
        typedef float f2 __attribute__((ext_vector_type(2)));
        const f2 lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)w_d, false), hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)w_d, true);
        rdot[0] = fmaf(lo[0], acc[mi][ni][0], rdot[0]);
        rdot[1] = fmaf(lo[1], acc[mi][ni][1], rdot[1]);
        rdot[2] = fmaf(hi[0], acc[mi][ni][2], rdot[2]);
        rdot[3] = fmaf(hi[1], acc[mi][ni][3], rdot[3]);
        if (mirrored) cdot[ni] += q8_dot4(w_m, acc[mi][ni]);
      }
      const unsigned t1 = __builtin_amdgcn_perm((unsigned)__builtin_amdgcn_mov_dpp((int)w_d, 0x4e, 0xf, 0xf, false), w_d, sel1);
      const unsigned o = __builtin_amdgcn_perm((unsigned)__builtin_amdgcn_mov_dpp((int)t1, 0xb1, 0xf, 0xf, false), t1, sel2);
      const int cl = cb[ni] - col_base + (lane & 12);  // first of the 4 columns (region-local)
      *(__attribute__((address_space(3))) unsigned*)(ld_d + (row_t0 - row_base + qd) * S8 + cl) = o;
      *(__attribute__((address_space(3))) unsigned*)(ld_m + (cb[ni] - col_base + (lane & 15)) * S8 +
                                                    (row_t0 - row_base)) = w_m;
    }
    if (p.dotp) {
      float dd[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) dd[r] = fmaf(rdot[r], exp2i(-q8_row_exp(mneg4[r], lmin)), rposd[r]);
      dsv[mi] = row16_sum4t(dd, lane);
    }
  }
  if (p.dotp) {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
      if ((lane & 3) == 0)
        dot_slot_store(p.dotp + (long long)(nt * 4 + wq) * p.Rpad + mt * kTile + rb[mi] + 4 * (lane >> 4) + ((lane >> 2) & 3),
                       dsv[mi]);
  }
  if (p.dotp && mirrored) {
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const float d = xrow_sum(fmaf(cdot[ni], icol[ni], cposd[ni]));
      const int row = (nt - p.row_tile0) * kTile + cb[ni] + (lane & 15);
      if (lane < 16) dot_slot_store(p.dotp + (long long)((p.row_tile0 + mt) * 4 + (row_base >> 6)) * p.Rpad + row, d);
    }
  }
  __syncthreads();
  // 64 rows x 64 B of each tile: lane l moves 16-B chunk (l & 3) of rows l >> 2 + 16 q
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = (lane >> 2) + 16 * q, c16 = lane & 3;
    const u32x4 v = *(__attribute__((address_space(3))) const u32x4*)(ld_d + row * S8 + c16 * 16);
    *reinterpret_cast<u32x4*>(slot + ctile_off(row_base + row, col_base + c16 * 16, 1)) = v;
    if (mirror) {
      const u32x4 m = *(__attribute__((address_space(3))) const u32x4*)(ld_m + row * S8 + c16 * 16);
      *reinterpret_cast<u32x4*>(mirror + ctile_off(col_base + row, row_base + c16 * 16, 1)) = m;
    }
  }
}

// Block-scaled fp8 MFMA with the scale bytes selected by op_sel: byte IA of sa, byte IB of sb
// (the builtin's op_sel operands must be literals).
template <int IA, int IB>
__device__ __forceinline__ f32x4 mma_mx_c(const i32x8& a, const i32x8& b, f32x4 c, int sa, int sb) {
  // cbsz = blgp = 0: both operands fp8 e4m3
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, IA, sa, IB, sb);
}

// ------------------------------------------------------------------------------------
// Stream-K fixup of a partial K-range of tile `stile` (shared by the similarity GEMM and the
// symmetric dZ GEMM; acc in the GEMM's fragment order, wave w = 4 wa + wb of 8). Returns true
// when this block now holds the complete tile in acc and runs the epilogue.
// ------------------------------------------------------------------------------------
template <bool kF8>
__device__ __forceinline__ bool sk_fixup(f32x4 (&acc)[8][4], const SimParams& p, int stile, int bid, int G, int tid,
                                         char* smem) {
  const int lane = tid & 63, w = tid >> 6;
  const int nk = p.nk;
  // ---- stream-K fixup: partial K-range of tile `stile` -------------------------------
  // Publish the fp32 partial (fragment order, 256 KiB) with write-through (sc1) 16-B
  // stores, drain every wave, then one lane counts the arrival. The last arriver sums the
  // segments in block order with sc1 loads (MI355X_MICROARCH.md § visibility, Valid forms
  // row 1: sc1 payload both sides + ticket, so neither an agent release — whose L2
  // write-back of every dirty line of the XCD cost ~30 us per episode here — nor an
  // acquire). Its own segment stays in registers: fp32 addition is commutative, so
  // ((s_b0 + s_b1) + s_b2) ... comes out bitwise identical whoever arrives last.
  const int b0 = (int)((long long)stile * nk / p.ipb);
  const int b1 = (int)(((long long)(stile + 1) * nk - 1) / p.ipb);
  auto slot_off = [&](int bb) {  // byte offset of block bb's slab for this tile
    const long long s = (long long)bb * p.ipb;
    const bool first_partial = !p.splitk && (s / nk == stile) && (s % nk != 0);
    return (unsigned)((2 * bb + (first_partial ? 0 : 1)) * (kTileElems * 4));
  };
  const auto srs = __builtin_amdgcn_make_buffer_rsrc(p.sk_slabs, 0, 2 * G * kTileElems * 4, 0x00020000);
  const unsigned lane_off = (unsigned)((w * 32 * 64 + lane) * 16);
  if (p.sk_half) {
    // fp16 partials (the reduce launch sums them in fp32; forward and dZ split-K): fragments
    // 2q, 2q + 1 of a lane (same mi, ni pair) share one 16-B unit, ((w * 16 + q) * 64 + lane)
    const unsigned mine = slot_off(bid) + (unsigned)((w * 16 * 64 + lane) * 16);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const f32x4 a = acc[q >> 1][2 * (q & 1)], b = acc[q >> 1][2 * (q & 1) + 1];
      union { _Float16 h[8]; u32x4 u; } pk;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pk.h[r] = (_Float16)a[r];
        pk.h[4 + r] = (_Float16)b[r];
      }
      __builtin_amdgcn_raw_buffer_store_b128(pk.u, srs, (int)(mine + q * 64 * 16), 0, 16);
    }
  } else {
    const unsigned mine = slot_off(bid) + lane_off;
#pragma unroll
    for (int f = 0; f < 32; ++f) {
      const f32x4 a = acc[f >> 2][f & 3];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, a), srs, (int)(mine + f * 64 * 16), 0, 16);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (p.splitk) return false;  // split-K: the reduce launch finishes the tile
  int* flag = reinterpret_cast<int*>(smem);
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(p.sk_cnt + stile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == b1 - b0;
    // every contributor has arrived: return the counter to zero for the next launch
    if (last) __hip_atomic_store(p.sk_cnt + stile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = last;
  }
  __syncthreads();
  const bool last = flag[0] != 0;
  __syncthreads();
  if (!last) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
  // The own segment stays in registers when it is the first or second term of the sum
  // ((s_b0 + s_me) = (s_me + s_b0) bitwise); a later position re-reads it from its slab.
  const bool reload_all = bid - b0 >= 2;
  if constexpr (kF8) {
    // (the pipelined form below made hipcc spill ~0.5 KiB per lane in the fp8 kernels)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      for (int bb = b0; bb <= b1; ++bb) {
        if (bb == bid && !reload_all) continue;
        const unsigned off = slot_off(bb) + lane_off;
        u32x4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[j] = __builtin_amdgcn_raw_buffer_load_b128(srs, (int)(off + (g * 8 + j) * 64 * 16), 0, 16);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const f32x4 x = __builtin_bit_cast(f32x4, v[j]);
          f32x4& a = acc[(g * 8 + j) >> 2][(g * 8 + j) & 3];
          a = (reload_all && bb == b0) ? x : (bb < bid && !reload_all) ? x + a : a + x;
        }
      }
    }
  } else {
    // Slab reads are software-pipelined: the next contributor's 8 loads are in flight while the
    // current ones are added (one serial round trip per (g, slab) made the fixup of a tile split
    // 7 ways ~14 us at d = 8192). The next index is clamped, not branched on, so no load is
    // conditional (hipcc would wait vmcnt(0) around it).
    auto next_bb = [&](int bb) {
      int nb = bb + 1;
      if (nb == bid && !reload_all) ++nb;
      return nb;
    };
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      int bb = (b0 == bid && !reload_all) ? b0 + 1 : b0;  // <= b1: the last arriver is never alone
      u32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[j] = __builtin_amdgcn_raw_buffer_load_b128(srs, (int)(slot_off(bb) + lane_off + (g * 8 + j) * 64 * 16), 0, 16);
      for (;;) {
        const int nb = next_bb(bb);
        const bool more = nb <= b1;
        const unsigned noff = slot_off(more ? nb : bb) + lane_off;
        u32x4 nv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          nv[j] = __builtin_amdgcn_raw_buffer_load_b128(srs, (int)(noff + (g * 8 + j) * 64 * 16), 0, 16);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const f32x4 x = __builtin_bit_cast(f32x4, v[j]);
          f32x4& a = acc[(g * 8 + j) >> 2][(g * 8 + j) & 3];
          a = (reload_all && bb == b0) ? x : (bb < bid && !reload_all) ? x + a : a + x;
        }
        if (!more) break;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = nv[j];
        bb = nb;
      }
    }
  }
  return true;
}

// fp8 backward dZ (e4m3 C rows scaled by 2^e_m, e4m3 Z^T by 256): dequantise per row and add the
// positive term C_mp z_p exactly from the fp16 rows (it is stored as 0 in the e4m3 C), after the
// stream-K fixup (the finishing block only), before dz_store.
__device__ __forceinline__ void dz8_finish(f32x4 (&acc)[8][4], const SimParams& p, int mt, int nt,
                                           const int (&rb)[8], const int (&cb)[4], int lane) {
  const float lmin = p.q8_lmin[0];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    const int m = mt * kTile + rb[mi] + (lane & 15);
    const bool mv = m < p.R;
    const float f = exp2i(-q8_row_exp(p.q8_mneg[m], lmin) - 8);
    const float cp = mv ? p.cpos[m] : 0.f;
    const int pm = mv ? (m < p.n_half ? m + p.n_half : m - p.n_half) : 0;
    const _Float16* zp = p.q8_zq + (long long)pm * p.q8_ldz;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int n = nt * kTile + cb[ni] + 4 * (lane >> 4);
      union { _Float16 h[4]; u32x2 u; } z4;
      z4.u = (mv && n < p.q8_ldz) ? *reinterpret_cast<const u32x2*>(zp + n) : u32x2{0u, 0u};
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[mi][ni][r] = acc[mi][ni][r] * f + cp * (float)z4.h[r];
    }
  }
}

// Slot group sg (of 8) of dot_i = sum_k dotp[k][i]: slots sg, sg + 8, ... in increasing order, 16
// loads in flight. dot_reduce_kernel sums the 8 groups in sg order; dz_dot_fold and dz_dot's
// fallback use the same order, so every path gives dot_i bitwise.
__device__ __forceinline__ float dot_slot_sum(const float* dotp, int nslot, int rows, int i, int sg) {
  float s = 0.f;
  int k = sg;
  for (; k + 120 < nslot; k += 128) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = dotp[(long long)(k + 8 * u) * rows + i];
#pragma unroll
    for (int u = 0; u < 16; ++u) s += v[u];
  }
  for (; k < nslot; k += 8) s += dotp[(long long)k * rows + i];
  return s;
}

// dZ with the dot reduce folded in (SimParams::dot_nslot; replaces the dot_reduce launch): every
// block of the persistent grid, before its first item, sums dot_i for its share of rows (32-row
// chunks, dot_reduce_kernel's arithmetic) and stores them sc1; one lane adds 1 to dot_cnt[0]
// after a block barrier that follows every wave's retirement of those stores. The epilogue's
// reads (dz_dot) come one whole main loop later. Split-K pieces (no epilogue here:
// sk_dz_reduce_kernel reads dot after the kernel boundary) fold without the count.
__device__ __forceinline__ void dz_dot_fold(const SimParams& p, lds_char* lds, int tid) {
  typedef __attribute__((address_space(3))) float lds_fl;
  lds_fl* part = (lds_fl*)lds;  // [2 halves][8 slot groups][32 rows]
  const int G = gridDim.x, rows = p.Rpad;
  const int rpb = ((rows + G - 1) / G + 31) & ~31;
  const int r0 = blockIdx.x * rpb, r1 = r0 + rpb < rows ? r0 + rpb : rows;
  const int hf = tid >> 8, lt = tid & 255, ln = lt & 63, sg = 2 * (lt >> 6) + (ln >> 5);
  const auto drs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.ndot), 0, 0x7FFFFFFF, 0x00020000);
  for (int c0 = r0; c0 < r1; c0 += 64) {
    const int i = c0 + 32 * hf + (ln & 31);
    part[(hf * 8 + sg) * 32 + (ln & 31)] = i < r1 ? dot_slot_sum(p.dotp, p.dot_nslot, rows, i, sg) : 0.f;
    __syncthreads();
    if (lt < 32 && c0 + 32 * hf + lt < r1) {
      float t = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) t += part[(hf * 8 + g) * 32 + lt];
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(t), drs, (c0 + 32 * hf + lt) * 4, 0, 16);  // sc1
    }
    __syncthreads();
  }
  // (counted by the caller once the stores have retired: after the first item's prologue wait,
  // or at the exit of a block without items, dz_dot_exit; split-K pieces are not counted: the
  // reduce launch reads dot after the kernel boundary)
}
// dot_i for the dZ epilogue. With the fold, the calling wave first polls (once: `state` 0 -> 1)
// until every block has counted; a poll that runs out (blocks not co-resident: never seen) makes
// the wave sum the slots itself from then on (state 2), in the same order. sc1 loads (the
// producer stored sc1: MI355X_MICROARCH.md, visibility, first table row).
template <bool FOLD>
__device__ __forceinline__ float dz_dot(const SimParams& p, int row, int& state) {
  if (!FOLD || p.dot_cnt == nullptr) return p.ndot[row];
  if (state == 0) {
    int n = 0;
    bool done = false;
    while (!(done = __hip_atomic_load(p.dot_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (int)gridDim.x) &&
           n < p.dot_spin) {
      __builtin_amdgcn_s_sleep(8);
      ++n;
    }
    state = done && p.dot_spin > 0 ? 1 : 2;
  }
  if (state == 2) {  // (serial: dot_slot_sum's additions in the same order, few registers)
    float t = 0.f;
    for (int g = 0; g < 8; ++g) {
      float s = 0.f;
      for (int k = g; k < p.dot_nslot; k += 8) s += p.dotp[(long long)k * p.Rpad + row];
      t += s;
    }
    return t;
  }
  const auto drs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.ndot), 0, 0x7FFFFFFF, 0x00020000);
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(drs, row * 4, 0, 16));
}
// Kernel exit of a folding dZ: a block that had no item counts its fold now; the last block out
// returns both counters to zero (every poll has ended: a block polls before it leaves).
__device__ __forceinline__ void dz_dot_exit(const SimParams& p, int tid, bool counted) {
  if (!counted) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the fold's sc1 stores
  __syncthreads();
  if (tid == 0) {
    if (!counted) __hip_atomic_fetch_add(p.dot_cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int old = __hip_atomic_fetch_add(p.dot_cnt + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (int)gridDim.x - 1) {
      __hip_atomic_store(p.dot_cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p.dot_cnt + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// h tile of the fused dZ epilogue prefetched into the ring (dz_store_h): 8 pieces of 128 rows x
// 128 B (piece i = rows 128 (i & 1).., bytes 128 (i >> 1).. of the tile's 512-byte row segment,
// the ring's chunk swizzle), DMA'd by the last two K-steps in place of their trailing (clamped)
// stages: pieces 0-6 into the ring slots those stages would fill, piece 7 into 16 KiB past the
// per-row coefficients. LDS byte offset of piece i:
__device__ __forceinline__ constexpr int hpiece_lds(int i) {
  return i == 0 ? 0 : i == 1 ? kStageBytes : i == 2 ? kStageBytes + kHalfBytes : i == 3 ? kHalfBytes
       : i == 4 ? kTile * kKStepBytes : i == 5 ? kStageBytes + kTile * kKStepBytes
       : i == 6 ? kStageBytes + kTile * kKStepBytes + kHalfBytes : kGemmLds + 2048;
}
constexpr int kHPieceExtra = 16384;  // piece 7's LDS (dZ kernels of 16-bit plans)

// Fused normalisation backward from the prefetched h tile (hpiece_lds): each lane reads the h
// values of its own accumulator fragments (8 B = 4 columns of one row, conflict-free: 16 lanes =
// 16 rows of distinct swizzled granules), writes dh over them in place, and the tile leaves as
// 128-byte row segments. No fp16 staging of g and no h loads after the main loop, where they
// waited on memory with the whole chip at once (dz_store below).
__device__ __forceinline__ void dz_store_h(f32x4 (&acc)[8][4], const SimParams& p, int mt, int nt, int tid,
                                           const int (&rb)[8], const int (&cb)[4], lds_char* lds, float iv0, float dt0) {
  typedef __attribute__((address_space(3))) u32x2 lds_u2;
  typedef __attribute__((address_space(3))) u32x4 lds_u4;
  typedef __attribute__((address_space(3))) f32x2 lds_f2;
  const int lane = tid & 63, wb = (tid >> 6) & 3;
  const float sgo = p.ngo[0] * p.nalpha;
  lds_f2* cf = (lds_f2*)(lds + kTile * 512);  // [256] per-row (c1, c2)
  if (tid < kTile) cf[tid] = f32x2{sgo * iv0, sgo * iv0 * iv0 * dt0};
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's h pieces landed
  __syncthreads();                                   // everyone's, and the coefficients
  const bool bf = p.nh_dt == 2;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    const int r = (rb[mi] & 127) + (lane & 15);  // row inside piece half mi >> 2
    const f32x2 c = cf[rb[mi] + (lane & 15)];
    const int rofs = r * kKStepBytes;
    const int sw = (r >> 1) & 7;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int nn = (cb[ni] + 4 * (lane >> 4)) & 63;  // column inside the piece's 64
      // piece 2 cq + rh: cq = 2 (ni >> 1) + (wb >> 1) (wave-uniform), rh = mi >> 2
      const int a = (wb >> 1) ? hpiece_lds(4 * (ni >> 1) + 2 + (mi >> 2)) : hpiece_lds(4 * (ni >> 1) + (mi >> 2));
      lds_u2* hp = (lds_u2*)(lds + a + rofs + (((nn >> 3) ^ sw) << 4) + ((nn & 7) << 1));
      union { _Float16 f[4]; __bf16 b[4]; u32x2 u; } x, y;
      x.u = *hp;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float g = (float)(_Float16)acc[mi][ni][e];
        const float hv = bf ? (float)x.b[e] : (float)x.f[e];
        const float o = c.x * g - c.y * hv;
        if (bf) y.b[e] = (__bf16)o;
        else y.f[e] = (_Float16)o;
      }
      *hp = y.u;
    }
  }
  __syncthreads();
  const long long nd = p.nd;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int i = k >> 1, r = (tid >> 3) + 64 * (k & 1), c = tid & 7;
    const u32x4 v = *(lds_u4*)(lds + hpiece_lds(i) + r * kKStepBytes + ((c ^ ((r >> 1) & 7)) << 4));
    const long long m = (long long)mt * kTile + 128 * (i & 1) + r;
    store16_wt(p.ndh, (m * nd + nt * kTile + 64 * (i >> 1) + 8 * c) * 2, v);
  }
}

// dZ epilogue (swapped orientation: lane holds out[m = rb + (lane&15)][n = cb + 4(lane>>4) + r])
// of output tile (mt, nt); `lds` (>= 128 KiB, free) stages the fp16 tile for coalesced rows.
template <typename T>
__device__ __forceinline__ void dz_store(f32x4 (&acc)[8][4], const SimParams& p, int mt, int nt, int tid,
                                         const int (&rb)[8], const int (&cb)[4], lds_char* lds, int& dstate) {
  constexpr bool kFold = !std::is_same<T, fp8e4m3>::value && sizeof(T) == 2;  // dz_dot_fold: 16-bit dZ
  typedef __attribute__((address_space(3))) u32x4 lds_u4;
  const int lane = tid & 63;
  // swapped orientation: lane holds out[m = rb + (lane&15)][n = cb + 4(lane>>4) + r]
  float* out = p.out;
  if (p.out_f16 && !p.accum) {
    // fp16 tile through LDS (free after the main loop): fragments -> row-major [256][256] with
    // the 16-byte chunk index XORed by (row & 15) (conflict-free both ways), then 512-byte
    // coalesced rows out. A fragment's direct 8-byte stores put 16 rows in every instruction.
    typedef __attribute__((address_space(3))) u32x2 lds_u2;
    // fused normalisation backward: this thread's row statistics are loaded before the staging
    // and its 16 chunks of h (16-bit inputs) right after it, so their latency hides under the
    // staging and the barriers instead of following the tile's last MFMA one load at a time
    float iv0 = 0.f, dt0 = 0.f;
    if (p.ndh && tid < kTile && mt * kTile + tid < p.R) {
      iv0 = p.ninv[mt * kTile + tid];
      dt0 = dz_dot<kFold>(p, mt * kTile + tid, dstate);
    }
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int rt = rb[mi] + (lane & 15);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int ct = cb[ni] + 4 * (lane >> 4);
        union { _Float16 h[4]; u32x2 u; } pk;
#pragma unroll
        for (int r = 0; r < 4; ++r) pk.h[r] = (_Float16)acc[mi][ni][r];
        *(lds_u2*)(lds + rt * 512 + ((((ct >> 3) ^ (rt & 15))) << 4) + ((ct >> 2) & 1) * 8) = pk.u;
      }
    }
    const bool h16 = p.ndh && p.nh_dt != 0;
    u32x4 hq[16];
    if (h16) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int idx = tid + kGemmThreads * k, rt = idx >> 5, c = idx & 31;
        const int m = mt * kTile + rt, d0 = nt * kTile + 8 * c;
        hq[k] = (m < p.R && d0 < p.nd)
                    ? *reinterpret_cast<const u32x4*>(static_cast<const char*>(p.nh) + ((long long)m * p.nd + d0) * 2)
                    : u32x4{0u, 0u, 0u, 0u};
      }
    }
    __syncthreads();
    if (p.ndh) {
      // Fused normalisation backward (replaces the norm_bwd launch and the dZ slab round trip):
      //   dh = c1 * g - c2 * h,  c1 = s inv_m, c2 = s inv_m^2 dot_m,  s = grad_out / (2N tau),
      // with dot_m = z_m . g_m = sum_j C_mj cos_mj from the coefficient pass. g is the fp16 tile
      // staged above (the precision of the unfused fp16 dZ slab).
      const float sgo = p.ngo[0] * p.nalpha;
      typedef __attribute__((address_space(3))) float lds_fl;
      lds_fl* cf = (lds_fl*)(lds + kTile * 512);  // [256][2] per-row c1, c2
      if (tid < kTile) {
        cf[2 * tid] = sgo * iv0;
        cf[2 * tid + 1] = sgo * iv0 * iv0 * dt0;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int idx = tid + kGemmThreads * k, rt = idx >> 5, c = idx & 31;
        const int m = mt * kTile + rt, d0 = nt * kTile + 8 * c;
        if (m >= p.R || d0 >= p.nd) continue;
        union { _Float16 h[8]; u32x4 u; } g;
        g.u = *(lds_u4*)(lds + rt * 512 + ((c ^ (rt & 15)) << 4));
        const float c1 = cf[2 * rt], c2 = cf[2 * rt + 1];
        const long long off = (long long)m * p.nd + d0;
        float hv[8], o[8];
        if (p.nh_dt == 2) {
          union { __bf16 h[8]; u32x4 u; } x;
          x.u = hq[k];
#pragma unroll
          for (int e = 0; e < 8; ++e) hv[e] = (float)x.h[e];
        } else if (p.nh_dt == 1) {
          union { _Float16 h[8]; u32x4 u; } x;
          x.u = hq[k];
#pragma unroll
          for (int e = 0; e < 8; ++e) hv[e] = (float)x.h[e];
        } else {
          const f32x4* hp = reinterpret_cast<const f32x4*>(static_cast<const float*>(p.nh) + off);
          const f32x4 a = hp[0], b = hp[1];
#pragma unroll
          for (int e = 0; e < 4; ++e) { hv[e] = a[e]; hv[4 + e] = b[e]; }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = c1 * (float)g.h[e] - c2 * hv[e];
        if (p.nh_dt == 2) {
          union { __bf16 h[8]; u32x4 u; } y;
#pragma unroll
          for (int e = 0; e < 8; ++e) y.h[e] = (__bf16)o[e];
          store16_wt(p.ndh, off * 2, y.u);  // write-through (profiles/r4/variants_r4_v8_wt.md)
        } else if (p.nh_dt == 1) {
          union { _Float16 h[8]; u32x4 u; } y;
#pragma unroll
          for (int e = 0; e < 8; ++e) y.h[e] = (_Float16)o[e];
          store16_wt(p.ndh, off * 2, y.u);
        } else {
          f32x4* op = reinterpret_cast<f32x4*>(static_cast<float*>(p.ndh) + off);
          op[0] = f32x4{o[0], o[1], o[2], o[3]};
          op[1] = f32x4{o[4], o[5], o[6], o[7]};
        }
      }
      return;
    }
    _Float16* o16 = reinterpret_cast<_Float16*>(out) + ((long long)mt * kTile) * p.ldo + nt * kTile;
#pragma unroll 4
    for (int k = 0; k < 16; ++k) {
      const int idx = tid + kGemmThreads * k, rt = idx >> 5, c = idx & 31;
      const u32x4 v = *(lds_u4*)(lds + rt * 512 + ((c ^ (rt & 15)) << 4));
      *reinterpret_cast<u32x4*>(o16 + (long long)rt * p.ldo + c * 8) = v;
    }
  } else {
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    const long long row = (long long)mt * kTile + rb[mi] + (lane & 15);
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int col = nt * kTile + cb[ni] + 4 * (lane >> 4);
      if (p.out_f16) {
        union { _Float16 h[4]; u32x2 u; } pk;
#pragma unroll
        for (int r = 0; r < 4; ++r) pk.h[r] = (_Float16)acc[mi][ni][r];
        *reinterpret_cast<u32x2*>(reinterpret_cast<_Float16*>(out) + row * p.ldo + col) = pk.u;
      } else {
        f32x4* o = reinterpret_cast<f32x4*>(out + row * p.ldo + col);
        *o = p.accum ? *o + acc[mi][ni] : acc[mi][ni];
      }
    }
  }
  }
}

// ------------------------------------------------------------------------------------
// The similarity GEMM with its three epilogues (see the file header for the schedule).
// ------------------------------------------------------------------------------------
// FX: the forward epilogue's exponential form, fixed shift (1, tau > ~0.024) or per-tile max
// (0). A compile-time choice: with both forms in one kernel the allocator spilled the main loop.
template <typename T, int MODE, int FX = 1>
__global__ __launch_bounds__(kGemmThreads) void sim_gemm_kernel(const SimParams p) {
  typedef typename Mfma<T>::frag frag;
  typedef __attribute__((address_space(3))) const frag lds_frag;
  // fp8: 2 KiB more hold the dwords carrying the tile's 256 A-row and 256 B-row E8M0 scales (one
  // array: a second __shared__ object makes hipcc drain the LDS-DMA before every ds_read)
  constexpr int kScaleLds = MODE == kModeCoef ? kCoefLds : kGemmLds;
  // (+2 KiB: fp8 row scales, or the fused dZ epilogue's per-row coefficients; forward: + 12 KiB
  // of row / column reductions above the stage buffers, see the prologue prefetch)
  constexpr int kFwdRed = kScaleLds + ((std::is_same<T, fp8e4m3>::value || MODE == kModeDz) ? 2048 : 0);
  // forward: + 12 KiB of row / column reductions, + 4 KiB: the raw-operand ring of row inverse
  // norms (2 slots x [256 A rows | 256 B rows], filled by 4-byte LDS-DMA one item ahead)
  constexpr int kInvLds = kFwdRed + (MODE == kModeFwd ? 6 * 256 * 8 : 0);
  __shared__ __attribute__((aligned(16))) char smem[kInvLds + (MODE == kModeFwd && !std::is_same<T, fp8e4m3>::value ? 4096 : 0) +
                                                     (MODE == kModeDz && !std::is_same<T, fp8e4m3>::value ? kHPieceExtra : 0)];
  lds_char* lds = (lds_char*)smem;
  typedef __attribute__((address_space(3))) u32x4 lds_u4;

  // the wave index as a scalar: the stage's LDS destinations (M0) stay scalar arithmetic instead
  // of a VALU add + v_readfirstlane per DMA piece (main loop 39 -> 22 VALU per K-step and wave;
  // headline dZ -2 %, forward -1.8 %, config 2 -4 %: profiles/r4/variants_r4_v18_wsgpr.md)
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wa = w >> 2, wb = w & 3;
  const int G = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, G);  // persistent block id (XCD-contiguous runs)
  const int nk = p.nk;                       // K-steps of a whole tile
  KStream sa0, sa1, sb0, sb1;

  // source offsets of this wave's two 8-row pieces j of each half-tile h: row 128 h + 16 w + 8 j +
  // (lane >> 3); the per-lane part (row in the piece, swizzled 16-B chunk: bits 1-3 of the row
  // come from 8 j + (lane >> 3) alone) in 2 VGPRs per operand, the wave-uniform part as the DMA's
  // scalar offset (8 VGPRs of per-(h, j) offsets made the fp8 dZ spill them inside the main loop:
  // 18 VGPRs: the fp8 dZ 641 -> 196 us at config 5 with the read bases below, profiles/r5/fp8_dz)
  unsigned a_vo[2], b_vo[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int rl = 8 * j + (lane >> 3);
    const int lchunk = (lane & 7) ^ ((rl >> 1) & 7);
    a_vo[j] = (unsigned)((lane >> 3) * p.A.ld) + lchunk * 16;
    b_vo[j] = (unsigned)((lane >> 3) * p.B.ld) + lchunk * 16;
  }
  // Half C (p.c_half, 16-bit dZ): the item's K-steps below tr_end (its row panel I's lower tiles
  // J < I) are staged from C_JI, which the coefficient pass wrote instead of C_IJ. Half-tile h of
  // K-step kk = rows kc .. kc + 63 (kc = 64 (kk & 3)) of tile (J = kk >> 2, I), bytes 256 h ..
  // 256 h + 255 of each 512-byte row: 16 pieces of 4 rows, wave w issuing pieces 2 w, 2 w + 1.
  // 16-B slot L of piece P holds row q = (L >> 1) & 3, chunk ch = 8 (((L >> 3) & 1) ^ x) +
  // 2 (L >> 4) + (L & 1), x = (P >> 1) & 1 (= w & 1): the transposed reads of read_a_tr are then
  // bank-conflict-free (a 32-lane half's two 4-row blocks sit in opposite 32-bank halves) and every
  // one of them is ONE lane base + an immediate (the 16-column block index lands in slot bits 4-5).
  constexpr bool kTrCap = MODE == kModeDz && sizeof(T) == 2 && !std::is_same<T, fp8e4m3>::value;
  int tr_end = 0;               // (set per item by the prologue)
  const char* tr_base = nullptr;  // tile (0, I) of the item's row panel I
  unsigned a_tr_vo = 0, rd_tr = 0;
  if constexpr (kTrCap) {
    const int x = w & 1;
    const int ch = 8 * (((lane >> 3) & 1) ^ x) + 2 * (lane >> 4) + (lane & 1);
    a_tr_vo = (unsigned)(((lane >> 1) & 3) * p.A.ld + 16 * ch);
    // read side: lane 4 q + pp of 16-lane group g supplies row q, columns 4 pp .. 4 pp + 3 of the
    // block (ds_read_b64_tr_b16): piece 8 s + 2 g + hi, slot 16 mi + 8 (wa ^ (g & 1)) + 2 q + (pp >> 1)
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    rd_tr = (unsigned)(2048 * g + 128 * (wa ^ (g & 1)) + 32 * q + 16 * (pp >> 1) + 8 * (pp & 1));
    asm volatile("" : "+v"(a_tr_vo), "+v"(rd_tr));
  }
  // stage half-tile h of operand A (isB = 0) or B (isB = 1) for the stream's K-step into buf
  // trm (half C, operand A): 0 the staged K-step is a regular one (a regular K-step only stages
  // K-steps past the item's lower tiles), 2 a lower tile's (a half-C K-step two or more steps
  // before the last one), 1 either: tested (the prologue and the last two half-C K-steps)
  auto stage = [&](int isB, int h, KStream& s, int buf, int trm = 1) {
    // LDS layout [A even | A odd | B even | B odd] (32 KiB each): every operand read of either
    // parity is its lane base + a 16-bit immediate (headline dZ -2.1 %: variants_r4_v23_ldsab.md)
    lds_char* dst = lds + isB * kStageBytes + buf * (kTile * kKStepBytes) + (128 * h + 16 * w) * kKStepBytes;
    if constexpr (kTrCap) {
      if (!isB && (trm == 2 || (trm == 1 && s.kk < tr_end))) {  // a lower tile: rows of C_JI (see above)
        // 32-bit scalar offset from the panel's tile (0, I) (the host checks the C buffer < 2 GiB)
        const unsigned so = (unsigned)(s.kk >> 2) * (unsigned)p.A.row_tile_stride +
                            (unsigned)(((s.kk & 3) * 64 + 8 * w) * (int)p.A.ld + 256 * h);
        const auto trs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(tr_base), 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(trs, (lds_void*)(dst + 8 * j * kKStepBytes), 16, a_tr_vo,
                                                   so + (unsigned)(4 * j * (int)p.A.ld), 0, kGemmDmaAux);
        s.skip();
        return;
      }
    }
    // buffer_load ... lds from a scalar V# at the stream's K-step + the lane's 32-bit offset: no
    // 64-bit VALU address add per piece as global_load_lds needs (main loop 22 -> 14 VALU per
    // K-step and wave; headline dZ -2.9 %, forward -2.6 %: profiles/r4/variants_r4_v20_bufdma.md)
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(s.ptr), 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + 8 * j * kKStepBytes), 16, isB ? b_vo[j] : a_vo[j],
                                               (unsigned)((128 * h + 16 * w + 8 * j) * (isB ? p.B.ld : p.A.ld)), 0,
                                               kGemmDmaAux);
    s.advance(isB ? p.B : p.A);
  };
  // dZ (hpre below): piece i of the epilogue's h tile (hpiece_lds) for output tile (mt_, nt_):
  // tile rows 128 (i & 1) + 16 w + 8 j + (lane >> 3), bytes 128 (i >> 1) + the ring's swizzled
  // 16-B chunk of their 512-byte segment, into this wave's 16 rows of the piece's LDS
  auto stage_h = [&](int i, int mt_, int nt_) {
    const long long hld = (long long)p.nd * 2;
    const char* hb = static_cast<const char*>(p.nh) + ((long long)mt_ * kTile + 128 * (i & 1)) * hld +
                     (long long)nt_ * kTile * 2 + 128 * (i >> 1);
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(hb), 0, 0x7FFFFFFF, 0x00020000);
    lds_char* dst = lds + hpiece_lds(i) + 16 * w * kKStepBytes;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int rl = 8 * j + (lane >> 3);
      const unsigned vo = (unsigned)((lane >> 3) * hld) + (unsigned)((((lane & 7) ^ ((rl >> 1) & 7))) << 4);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + 8 * j * kKStepBytes), 16, vo,
                                               (unsigned)((16 * w + 8 * j) * hld), 0, kGemmDmaAux);
    }
  };

  f32x4 acc[8][4];
  constexpr bool kF8 = std::is_same<T, fp8e4m3>::value;
  // raw-operand forward: thread t stages inv of A row t (t < 256) or B row t - 256 of tile (mt, nt)
  // into ring slot `slot` (one 4-byte LDS-DMA per lane, wave-linear destination)
  auto stage_inv = [&](int mt_, int nt_, int slot) {
    if constexpr (MODE == kModeFwd && !kF8) {
      const int t = threadIdx.x;
      const float* src = t < kTile ? p.inv_a + (long long)mt_ * kTile + t : p.inv_b + (long long)(nt_ - p.b_tile0) * kTile + (t - kTile);
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds + kInvLds + slot * 2048 + 256 * w), 4, 0, 0);
    }
  };
  // fp8: the block-scaled MFMA applies the rows' power-of-two E8M0 scales itself (exact): per
  // item, each lane packs the scale bytes of its 8 A row blocks (byte mi of sa_v[h]) and 4 B
  // column blocks (byte i of sb_v) from the prologue's LDS copy, read by untracked LDS reads after
  // the first counted wait (a plain global load there made hipcc drain the prologue DMA). Round 4
  // ran unit scales and multiplied the accumulators in the epilogue (-1.5 k cycles per item).
  // The dZ's C and Z^T carry no E8M0 scales (unit; per-row dequantisation in dz8_finish).
  const int kUnitScale = 0x7f7f7f7f;
  int sa_v[2] = {kUnitScale, kUnitScale}, sb_v = kUnitScale;

  const int r16 = lane & 15, sw = (r16 >> 1) & 7, cq = lane >> 4;
  // Operand registers [k-substep][block]. fp8: ONE 32-byte register set per block holding both
  // k-substeps (low half = s 0, high half = s 1) for the block-scaled MFMA.
  typedef typename std::conditional<kF8, i32x8, frag>::type OP;
  constexpr int NS = kF8 ? 1 : 2;
  typedef __attribute__((address_space(3))) const i32x4 lds_i4;
  OP af[NS][4], bf0[NS][2], bf1[NS][2];
  // operand-read lane bases, one per k-substep s and operand (row 64 wa + r16 of A / 32 wb + r16 of
  // B, swizzled chunk 4 s + cq): every read is one of them + a compile-time immediate (buffer,
  // half-tile, row block). Opaque: formed inside the reads, the fp8 kernels' substep-1 addresses
  // were (row base + block offset) + chunk, three more loop-invariant VGPRs that the dZ spilled
  // and reloaded behind a vmcnt(0) in every K-step (profiles/r5/fp8_dz).
  unsigned rd_a[2], rd_b[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const unsigned pch = (unsigned)(((4 * s + cq) ^ sw) << 4);
    rd_a[s] = (unsigned)((64 * wa + r16) * kKStepBytes) + pch;
    rd_b[s] = (unsigned)(kStageBytes + (32 * wb + r16) * kKStepBytes) + pch;
    asm volatile("" : "+v"(rd_a[s]), "+v"(rd_b[s]));
  }
  auto read_a = [&](int buf, int h, OP (&af)[NS][4]) {
    i32x4 lo[4];  // fp8: k-substep 0, joined with substep 1 into a fully (re)defined operand (a
                  // .lo/.hi partial write would keep the other half live across the whole kernel)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const lds_char* src = lds + rd_a[s] + (buf * kTile + 128 * h + 16 * mi) * kKStepBytes;
        if constexpr (kF8) {
          if (s == 0) lo[mi] = *(lds_i4*)src;
          else af[0][mi] = __builtin_shufflevector(lo[mi], *(lds_i4*)src, 0, 1, 2, 3, 4, 5, 6, 7);
        } else {
          af[s][mi] = *(lds_frag*)src;
        }
      }
    }
  };
  // A fragments of a transposed K-step (half C): two 4-row transposed reads per fragment. Untracked
  // (asm) reads: the compiler's own wait for a tracked LDS read behind the in-flight LDS-DMA is a
  // vmcnt(0) (it drained the operand prefetch every K-step); the K-step's counted lgkmcnt waits
  // (a0_retire, lds_drain) retire them before their MFMAs.
  auto read_a_tr = [&](auto buf_c, auto h_c, OP (&af)[NS][4]) {
    if constexpr (kTrCap) {
      constexpr int OFF0 = decltype(buf_c)::value * (kTile * kKStepBytes) + decltype(h_c)::value * kHalfBytes;
      const unsigned base = (unsigned)(uintptr_t)lds + rd_tr;
      auto one = [&](auto s_c, auto mi_c) {
        constexpr int sv = decltype(s_c)::value, mv = decltype(mi_c)::value;
        constexpr int off = OFF0 + 8 * sv * 1024 + 256 * mv;
        u32x2 lo, hi;
        asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%c3\n\tds_read_b64_tr_b16 %1, %2 offset:%c4"
                     : "=&v"(lo), "=&v"(hi)
                     : "v"(base), "i"(off), "i"(off + 1024)
                     : "memory");
        af[sv][mv] = __builtin_bit_cast(OP, u32x4{lo[0], lo[1], hi[0], hi[1]});
      };
      typedef std::integral_constant<int, 0> J0;
      typedef std::integral_constant<int, 1> J1;
      typedef std::integral_constant<int, 2> J2;
      typedef std::integral_constant<int, 3> J3;
      one(J0{}, J0{}); one(J0{}, J1{}); one(J0{}, J2{}); one(J0{}, J3{});
      one(J1{}, J0{}); one(J1{}, J1{}); one(J1{}, J2{}); one(J1{}, J3{});
    }
  };
  auto read_b = [&](int buf, int h, OP (&bf)[NS][2]) {
    i32x4 lo[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const lds_char* src = lds + rd_b[s] + (buf * kTile + 128 * h + 16 * ni) * kKStepBytes;
        if constexpr (kF8) {
          if (s == 0) lo[ni] = *(lds_i4*)src;
          else bf[0][ni] = __builtin_shufflevector(lo[ni], *(lds_i4*)src, 0, 1, 2, 3, 4, 5, 6, 7);
        } else {
          bf[s][ni] = *(lds_frag*)src;
        }
      }
    }
  };
  // s_setprio(1)/(0) around each MFMA cluster keeps hipcc from sinking the cluster across the
  // next s_barrier (cdna_hip_programming.md §5.5 T5).
  auto mma_quadrant = [&](auto qa_c, auto qb_c, OP (&af)[NS][4], OP (&bf)[NS][2]) {
    constexpr int qa = decltype(qa_c)::value, qb = decltype(qb_c)::value;
    __builtin_amdgcn_s_setprio(1);
    if constexpr (kF8) {
      // one block-scaled MFMA per (row block, column block) over the whole 128-element K-step
      // (dZ: operands swapped, as the 16-bit path, for the epilogue's row-per-lane orientation)
      auto mx = [&](auto mi_c, auto ni_c) {  // op_sel (scale byte) must be a literal
        constexpr int mi = decltype(mi_c)::value, ni = decltype(ni_c)::value;
        f32x4& c = acc[qa * 4 + mi][qb * 2 + ni];
        if constexpr (MODE == kModeDz)
          c = mma_mx_c<qb * 2 + ni, mi>(bf[0][ni], af[0][mi], c, kUnitScale, kUnitScale);
        else
          c = mma_mx_c<mi, qb * 2 + ni>(af[0][mi], bf[0][ni], c, sa_v[qa], sb_v);
        // The block-scaled MFMA intrinsic is not convergent, so LLVM's IR sinking moved every
        // cluster of a K-step into the loop latch (one 32-MFMA cluster, operands of all phases
        // live at once -> spills and a vmcnt(0) in the loop). An empty asm use pins it here.
        asm volatile("" ::"v"(c));
      };
      typedef std::integral_constant<int, 0> I0;
      typedef std::integral_constant<int, 1> I1;
      typedef std::integral_constant<int, 2> I2;
      typedef std::integral_constant<int, 3> I3;
      mx(I0{}, I0{}); mx(I0{}, I1{}); mx(I1{}, I0{}); mx(I1{}, I1{});
      mx(I2{}, I0{}); mx(I2{}, I1{}); mx(I3{}, I0{}); mx(I3{}, I1{});
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni) {
            f32x4& c = acc[qa * 4 + mi][qb * 2 + ni];
            c = MODE == kModeDz ? Mfma<T>::mma(bf[s][ni], af[s][mi], c) : Mfma<T>::mma(af[s][mi], bf[s][ni], c);
          }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  const std::integral_constant<int, 0> kI0{};
  const std::integral_constant<int, 1> kI1{};
  auto barrier = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto lds_drain = [&]() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
  // phase 1 issues the 8 A0 reads before the 4 B0 reads; LDS reads retire in order
  auto a0_retire = [&]() { asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory"); };
  // Forward streaming (MODE == kModeFwd, 16-bit operands, whole-tile items): the operand
  // streams run from one item into the next, so the schedule's trailing stages (K-steps n and
  // n + 1 of an n-step item: A0 B0 B1 A1, A0 B0 B1 — exactly a prologue) stage the NEXT item's
  // first two K-steps, and its epilogue runs with them in flight: no drain after the main loop,
  // no prologue latency, only raw barriers and untracked (asm) LDS accesses in the epilogue (a
  // __syncthreads or a compiler-tracked LDS access would wait vmcnt(0) for the in-flight DMA).
  // The epilogue's kept-cosine stores are younger than those DMAs: they only make the next
  // item's first counted waits stricter (vmcnt: all but the N youngest), so they drain under
  // the exponentials and the first phases. (Waits relaxed by the store count for those phases
  // measured slower: the per-phase selection cost more than the stores' drain.)
  // (fp8 forward streamed as well, its scale bytes in two LDS slots staged one item ahead:
  // config 5 fp8 forward 182-184 -> 188-189 us, not kept: profiles/r5/README.md)
  constexpr bool kStreamMode = MODE == kModeFwd && !kF8;
  // DMA wait, issued one phase AHEAD of the read it protects: the half-tile read in the NEXT
  // phase has retired for this wave (4 younger half-tiles may stay in flight).
  auto dma_wait = [&]() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); };
  // Wave group (0: waves 0-3, 1: waves 4-7); each SIMD hosts one wave of each group.
  const int grp = __builtin_amdgcn_readfirstlane(w) >> 2;

  // Each K-step: 4 phases (C-quadrants), each split into a load interval L (re-stage one
  // half-tile, read this phase's operands into registers, drain the reads) and a compute
  // interval C (16 MFMA from registers), separated by barriers. Group 1 runs one barrier
  // behind group 0 (staggered ping-pong), so on every SIMD one wave's L overlaps its partner's
  // C and the MFMA pipe alternates between them (cdna_hip_programming.md §5, 8-phase).
  //   phase 1: read A0(t) B0(t) | stage A1(t+1) | MFMA A0B0
  //   phase 2: read B1(t)       | stage A0(t+2) | MFMA A0B1
  //   phase 3: read A1(t)       | stage B0(t+2) | MFMA A1B0
  //   phase 4:                  | stage B1(t+2) | MFMA A1B1
  // (reads are issued before the DMA pieces: a phase costs ~2 x max(L, C), and L is then
  // the DMA issue time rather than DMA issue + read latency.)
  // Correctness under the stagger. WAR: B0, B1 and A1 are re-staged two phases after their
  // last read, and a read retires at the latest at the lgkmcnt(0) right after the next
  // barrier, i.e. before the barrier that starts the re-staging phase of either group; A0 is
  // re-staged ONE phase after its read, so its 8 reads (issued first) retire before the
  // barrier ending their L interval (counted lgkmcnt(4)). RAW: DMA waits run one phase ahead,
  // so both groups' copies of a half-tile retired before a barrier that precedes either
  // group's read.
  //
  // Persistent stream-K schedule: the first dp_tiles tiles are whole-tile work items
  // (rounds of G); the remaining sk_tiles * nk K-steps are split evenly (ipb steps per block).
  // A tile split across blocks is finished by its last-arriving block (fixup below).
  const long long sk_total = (long long)p.sk_tiles * nk;
  const long long it0 = (long long)bid * p.ipb;
  const long long it1 = it0 + p.ipb < sk_total ? it0 + p.ipb : sk_total;
  const int n_dp = p.dp_tiles > bid ? (p.dp_tiles - bid + G - 1) / G : 0;
  long long it = it0;
  // work item `item` of this block -> (tile, K range, stream-K tile); false: no more work
  auto fetch = [&](int item, int& tile, int& kb, int& ke, int& stile) -> bool {
    stile = -1;
    if (item < n_dp) {
      tile = bid + item * G;
      kb = 0;
      ke = nk;
      return true;
    }
    if (p.splitk) {  // piece-major aligned split: one piece per block
      if (item > 0) return false;
      stile = bid % p.sk_tiles;
      kb = (int)((bid / p.sk_tiles) * p.ipb);
      ke = kb + (int)p.ipb < nk ? kb + (int)p.ipb : nk;
      tile = p.dp_tiles + stile;
      return true;
    }
    if (it >= it1) return false;
    stile = (int)(it / nk);
    kb = (int)(it % nk);
    ke = (int)((long long)kb + (it1 - it) < nk ? kb + (it1 - it) : nk);
    it += ke - kb;
    tile = p.dp_tiles + stile;
    return true;
  };
  // operand streams of an item + its prologue DMA: A0 B0 B1 A1 of step 0, A0 B0 B1 of step 1
  // (the stream clamps keep the trailing prefetches in bounds, so every wait count is uniform)
  auto prologue = [&](int tile, int kb, int ke, int slot) {
    const int4 tt = sload_int4(p.tiles, tile);
    if (p.inv_a) stage_inv(tt.x, tt.y, slot);
    if constexpr (kTrCap) {
      tr_base = p.A.base + (long long)tt.x * p.A.kblk_stride;
      tr_end = p.c_half ? 4 * tt.x : 0;  // K-steps of the lower tiles J < I (4 per tile)
    }
    const int ns = ke - kb;
    const char* Ab = p.A.base + (long long)tt.x * p.A.row_tile_stride;
    const char* Bb = p.B.base + (long long)(tt.y - p.b_tile0) * p.B.row_tile_stride;
    const long long k0 = (long long)kb * kKStepBytes;
    sa0.init(Ab, k0, p.A, ns); sa1.init(Ab, k0, p.A, ns);
    if constexpr (kTrCap) {
      if (tr_end > kb) {  // half C: the regular K-steps start at tr_end (the lower ones use tr_base)
        sa0.seek(Ab, (long long)tr_end * kKStepBytes, p.A);
        sa1.seek(Ab, (long long)tr_end * kKStepBytes, p.A);
      }
    }
    sb0.init(Bb, k0, p.B, ns); sb1.init(Bb, k0, p.B, ns);
    if constexpr (kF8 && MODE != kModeDz) {
      // fp8: thread t fetches the dword whose low byte is the E8M0 scale of A row t (t < 256) or
      // B row t - 256 (stored right after the row's K range) into smem[kScaleLds + 4 t] by a
      // 4-byte LDS-DMA issued before the half-tiles: the vmcnt(10) below retires it with A0(0), B0(0)
      const int t = threadIdx.x;
      const char* src = (t < 256 ? Ab + (long long)t * p.A.ld : Bb + (long long)(t - 256) * p.B.ld) + p.scale_off;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds + kScaleLds + 256 * w), 4, 0, 0);
    }
    stage(0, 0, sa0, 0); stage(1, 0, sb0, 0); stage(1, 1, sb1, 0); stage(0, 1, sa1, 0);
    stage(0, 0, sa0, 1); stage(1, 0, sb0, 1); stage(1, 1, sb1, 1);
  };
  // Forward streaming needs whole-tile items with an even number of >= 2 K-steps (the streams
  // run two K-steps into the next item; even: its K-step 0 lands in buffer 0, as after a
  // prologue).
  const bool streaming = kStreamMode && p.sk_tiles == 0 && nk >= 2 && (nk & 1) == 0;
  bool streamed = false;  // this item's first two K-steps were staged by the previous item
  int dstate = 0;         // dZ, dot fold: dz_dot's poll state
  bool dot_counted = false;  // ... this block's fold counted (at its first item)
  if constexpr (MODE == kModeDz && !kF8 && sizeof(T) == 2) {
    // every block (one with no work too) folds its share of the dot reduce before its first item
    // and counts it once its first prologue wait has retired the stores (below); inside
    // the item loop the fold put ~30 more SGPR spills around it, and a peeled first prologue
    // (the fold under its DMA) put 4x the lane reads into the K-loop. The fold's LDS (2 KiB) is
    // the epilogue's per-row coefficients.
    if (p.dot_nslot > 0) dz_dot_fold(p, lds + kGemmLds, threadIdx.x);
  }
  auto tmark = [&](int item, int k) {
#if NTXENT_TIMING
    if (threadIdx.x == 0 && item < kTimingItems)
      p.tstamp[((long long)blockIdx.x * kTimingItems + item) * kTimingMarks + k] = __builtin_amdgcn_s_memtime();
#endif
  };
  for (int item = 0;; ++item) {
  tmark(item, 0);
  int tile, kb, ke, stile;
  if (streamed) {
    tile = bid + item * G; kb = 0; ke = nk; stile = -1;
  } else {
    if (!fetch(item, tile, kb, ke, stile)) break;
    prologue(tile, kb, ke, item & 1);
  }
  const bool cont = streaming && item + 1 < n_dp;  // the trailing stages stage the next item
  const char* na = nullptr;
  const char* nb = nullptr;
  int nmt = 0, nnt = 0;
  if (cont) {
    const int4 tn = sload_int4(p.tiles, bid + (item + 1) * G);
    na = p.A.base + (long long)tn.x * p.A.row_tile_stride;
    nb = p.B.base + (long long)(tn.y - p.b_tile0) * p.B.row_tile_stride;
    nmt = tn.x;
    nnt = tn.y;
  }
  const int4 t = sload_int4(p.tiles, tile);
  const int mt = t.x, nt = t.y;
  const int nsteps = ke - kb;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

  asm volatile("s_waitcnt vmcnt(10)" ::: "memory");  // A0(0), B0(0) retired
  barrier();
  if constexpr (MODE == kModeDz && !kF8 && sizeof(T) == 2) {
    // the fold's sc1 stores preceded this item's 14 DMA pieces: every wave's wait above retired
    // them (in order), and the barrier follows every wave's wait
    if (item == 0 && p.dot_cnt != nullptr && threadIdx.x == 0)
      __hip_atomic_fetch_add(p.dot_cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    dot_counted = true;
  }
  if constexpr (kF8 && MODE != kModeDz) {  // this item's scale bytes (landed with A0(0), B0(0))
    const int r16_ = lane & 15;
    unsigned av[8], bv[4];
    lds_get_scales((unsigned)(uintptr_t)(lds + kScaleLds) + 4 * (64 * wa + r16_),
                   (unsigned)(uintptr_t)(lds + kScaleLds) + 4 * (256 + 32 * wb + r16_), av, bv);
    sa_v[0] = pack_low_bytes(av[0], av[1], av[2], av[3]);
    sa_v[1] = pack_low_bytes(av[4], av[5], av[6], av[7]);
    sb_v = pack_low_bytes(bv[0], bv[1], bv[2], bv[3]);
  }
  tmark(item, 1);
  if (grp == 1) barrier();  // stagger group 1 by one barrier
  // K-steps in pairs: the buffer parity is a compile-time constant in each copy, so the LDS
  // read addresses are loop-invariant registers + immediates (headline dZ -1.9 %, forward -1.5 %,
  // config 5 dZ -3.4 %: profiles/r4/variants_r4_v21_unroll2.md)
  // dZ with the fused normalisation backward of 16-bit rows on a whole tile: the last two K-steps
  // (TAIL 1, 2) stage the epilogue's h tile (dz_store_h) instead of their trailing clamped stages
  bool hpre = false;
  if constexpr (MODE == kModeDz && !kF8)
    hpre = p.ndh != nullptr && (p.nh_dt == 1 || p.nh_dt == 2) && stile < 0 && nsteps == nk && nsteps >= 4 &&
           (nsteps & 1) == 0 && p.R % kTile == 0 && p.nd % kTile == 0;
  auto kstep = [&](const int ks, auto cur_c, auto tail_c, auto tr_c) {
    constexpr int cur = decltype(cur_c)::value, nxt = cur ^ 1;
    constexpr int TAIL = decltype(tail_c)::value;
    // A of this K-step staged transposed (half C); 2: one of the last two such K-steps (its A
    // stages may be regular ones)
    constexpr bool TR = decltype(tr_c)::value != 0;
    constexpr int TRM = decltype(tr_c)::value == 0 ? 0 : (decltype(tr_c)::value == 2 ? 1 : 2);
    if constexpr (kStreamMode) {
      // hand-over: A0, B0, B1 of K-step ks + 2 and A1 of ks + 1 are the next item's K-step 0
      if (cont && ks == nsteps - 2) {
        sa0.init(na, 0, p.A, nk); sb0.init(nb, 0, p.B, nk); sb1.init(nb, 0, p.B, nk);
        // the next item's row inverse norms, into the other ring slot (older than every stage
        // still to come: the counted waits before its epilogue retire it)
        if (p.inv_a) stage_inv(nmt, nnt, (item + 1) & 1);
      }
      if (cont && ks == nsteps - 1) sa1.init(na, 0, p.A, nk);
    }
    dma_wait(); barrier();          // phase 1 L (wait covers B1(t) for phase 2)
    if constexpr (TR) read_a_tr(cur_c, kI0, af);
    else read_a(cur, 0, af);        //   operand reads first: their latency hides under the
    __builtin_amdgcn_sched_barrier(0);  // pin: the 8 A0 reads precede the B0 reads (a0_retire)
    read_b(cur, 0, bf0);            //   DMA issue that follows (~100-200 cycles per piece)
    if constexpr (TAIL == 2) stage_h(3, mt, nt);
    else stage(0, 1, sa1, nxt, TRM);  // A1 of step ks+1
    a0_retire(); barrier();         // phase 1 C: A0 is restaged next phase -> its 8 reads retire
    lds_drain();                    //   before the barrier; the 4 B0 reads may retire after it
    if constexpr (TR) __builtin_amdgcn_sched_barrier(0);  // (asm A reads: no MFMA above the wait)
    mma_quadrant(kI0, kI0, af, bf0);
    dma_wait(); barrier();          // phase 2 L (covers A1(t) for phase 3)
    read_b(cur, 1, bf1);
    if constexpr (TAIL != 0) stage_h(TAIL == 1 ? 0 : 4, mt, nt);
    else stage(0, 0, sa0, cur, TRM);  // A0 of step ks+2
    barrier(); lds_drain();         // phase 2 C (B1 is restaged two phases later)
    mma_quadrant(kI0, kI1, af, bf1);
    barrier();                      // phase 3 L
    if constexpr (TR) read_a_tr(cur_c, kI1, af);
    else read_a(cur, 1, af);
    if constexpr (TAIL != 0) stage_h(TAIL == 1 ? 1 : 5, mt, nt);
    else stage(1, 0, sb0, cur);     //   B0 of step ks+2
    barrier(); lds_drain();         // phase 3 C (A1 is restaged two phases later)
    if constexpr (TR) __builtin_amdgcn_sched_barrier(0);
    mma_quadrant(kI1, kI0, af, bf0);
    // phase 4 L (covers A0(t+1), B0(t+1) for the next phase 1; the last K-step of an h-prefetch
    // tail has none, and its wait would be the first to hold for the h pieces' memory latency)
    if constexpr (TAIL != 2) dma_wait();
    barrier();
    if constexpr (TAIL != 0) {
      stage_h(TAIL == 1 ? 2 : 6, mt, nt);
      if constexpr (TAIL == 2) stage_h(7, mt, nt);  // (its own LDS: no wait counted after it)
    } else {
      stage(1, 1, sb1, cur);        //   B1 of step ks+2
    }
    barrier();                      // phase 4 C
    mma_quadrant(kI1, kI1, af, bf1);
  };
  const std::integral_constant<int, 2> kI2{};
  int ks2 = 0;
  const int nmain = nsteps - (hpre ? 2 : 0);
  if constexpr (kTrCap) {
    // half C: the lower tiles' K-steps first (an even count: the host enables half C only when
    // every item starts at an even K-step, dz_half_c_eligible; 4 K-steps per tile)
    const int ntr = tr_end > kb ? (tr_end < ke ? tr_end : ke) - kb : 0;
    for (; ks2 + 3 < ntr; ks2 += 2) {  // their stages are all lower-tile K-steps
      kstep(ks2, kI0, kI0, kI1);
      kstep(ks2 + 1, kI1, kI0, kI1);
    }
    if (ks2 + 1 < ntr) {  // the last two: their stages cross into the regular K-steps
      kstep(ks2, kI0, kI0, kI2);
      kstep(ks2 + 1, kI1, kI0, kI2);
      ks2 += 2;
    }
  }
  for (; ks2 + 1 < nmain; ks2 += 2) {
    kstep(ks2, kI0, kI0, kI0);
    kstep(ks2 + 1, kI1, kI0, kI0);
  }
  if constexpr (MODE == kModeDz && !kF8) {
    if (hpre) {
      kstep(ks2, kI0, kI1, kI0);
      kstep(ks2 + 1, kI1, kI2, kI0);
      ks2 += 2;
    }
  }
  if (ks2 < nsteps) kstep(ks2, kI0, kI0, kI0);
  if (grp == 0) barrier();  // re-align the groups
  tmark(item, 2);
  // dZ, h prefetched: this thread's row statistics for the epilogue, loaded before the drain
  float hiv = 0.f, hdt = 0.f;
  if constexpr (MODE == kModeDz && !kF8) {
    if (hpre && threadIdx.x < kTile) {
      hiv = p.ninv[mt * kTile + threadIdx.x];
      hdt = dz_dot<sizeof(T) == 2>(p, mt * kTile + threadIdx.x, dstate);
    }
  }
  if (kStreamMode && cont) {
    // the trailing stages are the next item's K-steps 0 and 1 (buffers of parity nk): leave
    // them in flight; this epilogue's stores will be younger than them
    streamed = true;
  } else {
    streamed = false;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the trailing (clamped) prefetches
  }
  if constexpr (kStreamMode) {
    lds_drain();  // raw barrier: a __syncthreads would drain the next item's DMA
    barrier();
  } else {
    __syncthreads();
  }
  {
  // Thread indices re-derived through an opaque copy: keeps the compiler from hoisting the
  // epilogue's address arithmetic out of the persistent loop, where it would stay live across
  // the MFMA main loop and spill.
  int tid_e = threadIdx.x;
  asm volatile("" : "+v"(tid_e));
  const int tid = tid_e, lane = tid_e & 63, w = tid_e >> 6;
  const int wa = w >> 2, wb = w & 3;
  int rb[8], cb[4];
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) rb[mi] = 128 * (mi >> 2) + 64 * wa + 16 * (mi & 3);
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) cb[ni] = 128 * (ni >> 1) + 32 * wb + 16 * (ni & 1);

  if constexpr (MODE == kModeFwd && !kF8) {
    if (p.inv_a) {
      // raw operands: cos = acc * inv_a[row] * inv_b[col], before any split-K publication (linear)
      // and the epilogue; the ring slot was filled one item ahead (or by this item's prologue)
      // and retired by the main loop's counted waits and barriers (untracked reads: the next
      // item's DMA may be in flight)
      const unsigned ib = (unsigned)(uintptr_t)(lds + kInvLds) + (unsigned)((item & 1) * 2048);
      // (cb[ni] = cb[0] + {0, 16, 128, 144}, rb[mi] = rb[0] + 16 (mi & 3) + 128 (mi >> 2))
      const unsigned rbase = ib + 4 * (rb[0] + 4 * (lane >> 4)), cbase = ib + 4 * (kTile + cb[0] + (lane & 15));
      float cs[4];
      f32x4 rs[4];
      auto scale4 = [&](int m0) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) acc[m0 + q][ni] *= rs[q] * cs[ni];
      };
      lds_get_inv<0>(rbase, cbase, rs, cs);
      scale4(0);
      lds_get_rinv<512>(rbase, rs);
      scale4(4);
    }
  }
  tmark(item, 4);
  if (nsteps != nk && !sk_fixup<kF8>(acc, p, stile, bid, G, tid, smem)) continue;

  if constexpr (MODE == kModeDz) {
    if constexpr (kF8) dz8_finish(acc, p, mt, nt, rb, cb, lane);
    if (!kF8 && hpre) dz_store_h(acc, p, mt, nt, tid, rb, cb, lds, hiv, hdt);
    else dz_store<T>(acc, p, mt, nt, tid, rb, cb, lds, dstate);
  } else if constexpr (MODE == kModeCoef) {
    coef_epilogue<typename StoreT<T>::type, 8>(acc, rb, cb, 0, 0, mt, nt, t.z, lds, p, lane);
  } else {
    const int kind = t.z;
    // keep cosines (compact slot per tile, canonical order): the stores of 16-row block mi
    typedef typename StoreT<T>::type TS;
    TS* const st = p.sc ? reinterpret_cast<TS*>(p.sc) + (long long)tile * kTileElems : nullptr;
    // the tile's 128 KiB slot as one buffer resource (wave-uniform base: store16_wt's per-store
    // scalar base arithmetic is not needed inside one tile)
    const auto st_rs = __builtin_amdgcn_make_buffer_rsrc(st, 0, 0x7FFFFFFF, 0x00020000);
    auto store_cos = [&](int mi) {
#pragma unroll
      for (int np = 0; np < 2; ++np) {
        if constexpr (sizeof(TS) == 2) {
          // 16-B stores (half the store-issue time of 8-B ones): the fragments of the column
          // blocks cb and cb + 16 share one unit, see sc_unit()
          union { TS h[8]; u32x4 u; } pk;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            pk.h[r] = from_f32<TS>(acc[mi][2 * np][r]);
            pk.h[4 + r] = from_f32<TS>(acc[mi][2 * np + 1][r]);
          }
          // write-through: -1.1 % headline, -2.3 % config 2 fwd+bwd vs default-policy stores, config
          // 5 as the non-temporal form (profiles/r4/variants_r4_v7_wt.md)
          __builtin_amdgcn_raw_buffer_store_b128(pk.u, st_rs, sc_unit(rb[mi], cb[2 * np], lane) * 16, 0, 16);
        } else {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int ni = 2 * np + q;
            *reinterpret_cast<f32x4*>(st + (((rb[mi] >> 4) * 16 + (cb[ni] >> 4)) * 64 + lane) * 4) = acc[mi][ni];
          }
        }
      }
    };
    // masks -> scaled logits in log2 units. The partials cover the NEGATIVES only: self and
    // positive are excluded (the positive logit comes from prep), so the loss is
    // softplus(lse_neg - y_pos) with no lse - y cancellation.
    // Fixed-shift fast path: rows are unit-norm, so y = cos * M with M = log2(e)/tau and
    // y - M lies in [-2M, 0]. For 2M < 120 every exp2(y - M) is a normal fp32 number, so ONE
    // exp2 per element feeds both the row and the column partial with a common shift M (no
    // max passes). Smaller tau falls back to per-tile max shifting (2 exps per element).
    const int col_local0 = (nt * kTile) % p.Rpad;
    const bool own_blk = kind == kTileDiag || kind == kTileSymOff;
    const bool col_out = kind == kTileSymOff || kind == kTileCross;  // column partials too
    constexpr bool fixed = FX != 0;  // launch_sim_gemm picks FX = p.fixed_shift
    const float M = p.y_scale;
    // Masks set the masked raw values of a 16-row block to -inf (exp2 -> 0). Element (tile row
    // tr, tile col tc) is the self pair when tc - tr == r0 - c0 and a positive when tc - tr ==
    // r0 - c0 +- n_half; a 16x16 fragment can hold such an element only if its block offset
    // cb - rb is within 15 of that difference, and padding only at the tile edge. These tests
    // are wave-uniform, so only the few fragments that need it run per-lane selects; the
    // per-element masked form compiled to per-element control flow (~15 us per tile) and the
    // fully unrolled select form spilled the main loop.
    const int r0 = mt * kTile, c0 = col_local0;
    const int D0 = r0 - c0, D1 = D0 + p.n_half, D2 = D0 - p.n_half;
    const bool pad = (r0 + kTile > p.R) || (c0 + kTile > p.R);
    // fragment offsets cb - rb span [-240, 240]: only tiles with some |D| <= 255 hold a self
    // or positive element (the diagonal band and the two positive bands of the own block)
    const bool tile_near = own_blk && ((D0 <= 255 && D0 >= -255) || (D1 <= 255 && D1 >= -255) ||
                                       (D2 <= 255 && D2 >= -255));
    const bool mask_any = tile_near || pad;
    // block offsets from the wave index in an SGPR: the tests compile to scalar branches
    const int ws = __builtin_amdgcn_readfirstlane(w);
    const int was = ws >> 2, wbs = ws & 3;
    auto mask_rows = [&](int mi) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int rbs = 128 * (mi >> 2) + 64 * was + 16 * (mi & 3);
        const int cbs = 128 * (ni >> 1) + 32 * wbs + 16 * (ni & 1);
        const int off = cbs - rbs;
        const bool near = tile_near && ((off - D0 <= 15 && D0 - off <= 15) || (off - D1 <= 15 && D1 - off <= 15) ||
                                        (off - D2 <= 15 && D2 - off <= 15));
        const bool edge = (r0 + rbs + 16 > p.R) || (c0 + cbs + 16 > p.R);
        if (near || edge) {
          const int tc = cb[ni] + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int tr = rb[mi] + 4 * (lane >> 4) + r;
            const int gi = r0 + tr, d = tc - tr;
            const bool drop = (gi >= p.R) | (c0 + tc >= p.R) |
                              (tile_near & ((d == D0) | ((d == D1) & (gi < p.n_half)) | ((d == D2) & (gi >= p.n_half))));
            acc[mi][ni][r] = drop ? kNegInf : acc[mi][ni][r];
          }
        }
      }
    };
    if constexpr (!fixed) {
      if (st) {
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) store_cos(mi);
      }
      if (mask_any) {
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) mask_rows(mi);
      }
    }
    const float sc_ = p.acc_scale;
    // row / column partial scratch above the stage buffers, [4 wb][256] and [2 wa][256] float2,
    // written and read by untracked LDS accesses (the next item's DMA may be in flight)
    const unsigned rowred = (unsigned)(uintptr_t)(lds + kFwdRed);
    const unsigned colred = rowred + 4 * 256 * 8;
    if constexpr (fixed) {
      // Streamed per 16-row block: exponentiate (exp2(-inf) = 0 for the masked elements),
      // reduce the 4 rows, fold into the column sums; acc[mi] is dead afterwards, which keeps
      // the epilogue's register footprint at the accumulators'.
      f32x2 csum2[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
      f32x2 sc2 = {sc_, sc_}, mM2 = {-M, -M};
      asm volatile("" : "+v"(sc2), "+v"(mM2));  // VGPR pairs: the packed FMA's operands
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        // this block's cosine stores go out between the exponentials of the blocks: the CU's
        // store stream (HBM-write-bound while every CU ends a tile) drains under the VALU work
        // instead of stalling every wave at its 16th store before any exponential
        if (st) store_cos(mi);
        if (mask_any) mask_rows(mi);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {  // packed FMAs: two arguments per instruction
            const f32x2 y = __builtin_elementwise_fma(f32x2{acc[mi][ni][2 * h2], acc[mi][ni][2 * h2 + 1]}, sc2, mM2);
            acc[mi][ni][2 * h2] = fast_exp2(y[0]);
            acc[mi][ni][2 * h2 + 1] = fast_exp2(y[1]);
          }
        }
        {
          // row sums of the block's 4 rows (packed adds over the column blocks, one transposing
          // 16-lane reduction, one LDS write per lane: lane holds row (lane >> 2) & 3), then the
          // column partials as packed pairs
          const f32x4 rsum = (acc[mi][0] + acc[mi][1]) + (acc[mi][2] + acc[mi][3]);
          const float s4[4] = {rsum[0], rsum[1], rsum[2], rsum[3]};
          const float s = row16_sum4t(s4, lane);
          lds_put_f2(rowred + 8 * (wb * 256 + rb[mi] + 4 * (lane >> 4) + ((lane >> 2) & 3)), f32x2{s > 0.f ? M : kNegInf, s});
        }
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          csum2[ni] += f32x2{acc[mi][ni][0], acc[mi][ni][1]} + f32x2{acc[mi][ni][2], acc[mi][ni][3]};
        __builtin_amdgcn_sched_barrier(0);  // keep the blocks streamed (no hoisted exps to spill)
      }
      if (col_out) {
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const float s = xrow_sum(csum2[ni][0] + csum2[ni][1]);
          lds_put_f2(colred + 8 * (wa * 256 + cb[ni] + (lane & 15)), f32x2{s > 0.f ? M : kNegInf, s});
        }
      }
    } else {
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[mi][ni][r] *= sc_;
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
          lds_put_f2(rowred + 8 * (wb * 256 + rb[mi] + 4 * (lane >> 4) + r), f32x2{m, s});
        }
      if (col_out) {  // column partials = partials of the mirrored rows
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
          lds_put_f2(colred + 8 * (wa * 256 + cb[ni] + (lane & 15)), f32x2{m, s});
        }
      }
    }
    tmark(item, 5);
    lds_drain();  // the untracked partial writes
    if constexpr (kStreamMode) {
      barrier();
    } else {
      __syncthreads();
    }
    tmark(item, 6);
    if (tid < 256) {
      f32x2 v[4];
      lds_get4_f2(rowred + 8 * tid, v[0], v[1], v[2], v[3]);
      float m = v[0].x, s = v[0].y;
#pragma unroll
      for (int q = 1; q < 4; ++q) lse_merge(m, s, v[q].x, v[q].y);
      p.part[(long long)nt * p.Rpad + mt * kTile + tid] = make_float2(m, s);
    } else if (col_out) {
      const int c = tid - 256;
      f32x2 v, u;
      lds_get2_f2(colred + 8 * c, v, u);
      float m = v.x, s = v.y;
      lse_merge(m, s, u.x, u.y);
      if (kind == kTileSymOff) {
        p.part[(long long)(p.row_tile0 + mt) * p.Rpad + (nt - p.row_tile0) * kTile + c] = make_float2(m, s);
      } else {  // kTileCross: partner q = nt / rt receives slot (rank, mt) for its rows
        const int rt = p.Rpad / kTile;
        p.part_x[(long long)((nt / rt) * rt + mt) * p.Rpad + (nt % rt) * kTile + c] = make_float2(m, s);
      }
    }
  }
  }  // epilogue scope
  tmark(item, 3);
  // LDS of this item's epilogue is reused by the next item's staging (streaming: the partial
  // scratch lies above the stage buffers and the next epilogue writes it after the next main
  // loop's barriers, so no barrier here)
  if constexpr (!kStreamMode) __syncthreads();
  }  // work items
  if constexpr (MODE == kModeDz && !kF8 && sizeof(T) == 2) {
    if (p.dot_cnt) dz_dot_exit(p, threadIdx.x, dot_counted);
  }
}

// Store-mode coefficient pass: one wave per 64x64 region (wm, wn, half) of a kept cosine tile
// (canonical fragment order: 16 fragments of 512 B) -> C into the coefficient buffer. 9 KiB of
// LDS per wave keeps many independent waves in flight per CU (the pass is HBM-bound), and 16
// waves per tile keep a small problem's few tiles (36 at B = 1024/view) spread over the chip.
template <typename T, bool Q8 = false>
__global__ __launch_bounds__(64) void coef_kernel(const SimParams p) {
  __shared__ __attribute__((aligned(16))) char smem[Q8 ? 2 * 64 * 80 : (sizeof(T) == 2 ? kCoefWaveLds : 16)];
  const int lane = threadIdx.x;
  const int idx = xcd_remap(blockIdx.x, gridDim.x);
  const int tidx = idx >> 4, w = (idx >> 1) & 7, half = idx & 1;
  const int wm = w >> 2, wn = w & 3;
  const int4 t = p.tiles[tidx];
  // A diagonal tile is symmetric: only its regions a <= b (64-row group a = 2 wm + half, column
  // group b = wn) are read, a region a < b writes C with its mirror (b, a) in the same tile, and
  // the kept cosines of its lower regions may be absent (diag_up_kernel computes only the upper).
  int kind = t.z;
  if (kind == kTileDiag) {
    const int ga = 2 * wm + half;
    if (ga > wn) return;
    if (ga < wn) kind = kTileDiagUp;
  }
  const T* st = reinterpret_cast<const T*>(p.sc) + (long long)tidx * kTileElems;
  int rb[4], cb[4];
  f32x4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) rb[mi] = 128 * wm + 64 * half + 16 * mi;
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) cb[ni] = 64 * wn + 16 * ni;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int np = 0; np < 2; ++np) {
      if constexpr (sizeof(T) == 2) {
        union { T h[8]; u32x4 u; } pk;
        // read once: non-temporal (config 5 coefficient pass -8 us, headline -1 us:
        // profiles/r4/variants_r4_v12_ntld.md)
        pk.u = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(st + sc_unit(rb[mi], cb[2 * np], lane) * 8));
        acc[mi][2 * np] = f32x4{to_f32<T>(pk.h[0]), to_f32<T>(pk.h[1]), to_f32<T>(pk.h[2]), to_f32<T>(pk.h[3])};
        acc[mi][2 * np + 1] = f32x4{to_f32<T>(pk.h[4]), to_f32<T>(pk.h[5]), to_f32<T>(pk.h[6]), to_f32<T>(pk.h[7])};
      } else {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int ni = 2 * np + q;
          acc[mi][ni] = *reinterpret_cast<const f32x4*>(st + (((rb[mi] >> 4) * 16 + (cb[ni] >> 4)) * 64 + lane) * 4);
        }
      }
    }
  if constexpr (Q8)
    coef_epilogue_q8<T>(acc, rb, cb, 128 * wm + 64 * half, 64 * wn, t.x, t.y, kind, (lds_char*)smem, p, lane);
  else
    coef_epilogue<T, 1, 4>(acc, rb, cb, 128 * wm + 64 * half, 64 * wn, t.x, t.y, kind, (lds_char*)smem, p, lane);
}

// Ring of the diagonal-remainder kernel below: a stage holds 64 A + 64 B rows of one K-step.
constexpr int kSubStage = 128 * kKStepBytes;   // 16 KiB
// ring stages of the diagonal remainder's off-diagonal-region blocks (diagonal-region blocks: twice
// as many half-size stages; 6 measured the same at the headline, +8 us at config 5:
// profiles/r4/variants_r4_v11_up6.md)
constexpr int kSubStages = 3;

// ------------------------------------------------------------------------------------
// Diagonal tiles by their upper 64x64 regions only (the coefficient pass mirrors a diagonal
// tile's regions a < b into (b, a), coef_kernel), 16 blocks per tile that each stream the same
// operand bytes (the remainder is bound by the per-CU load path, so balance is the lever):
//   blocks 0-3: the diagonal regions (a, a) over the whole K, 64 rows staged (A = B);
//   blocks 4-15: the six regions a < b, each as two K halves, 128 rows staged.
// The second half of a region to arrive (ticket) adds the first one's fp32 partial (write-through
// slab, as sk_fixup) and runs the epilogue: kept cosines of (a, b), masks, row partials of group
// a over b's 64 columns and column partials of group b over a's 64 rows (the mirrored region's
// row partials). The 4th contribution to a row group (ticket) merges the 4 in b order, so the
// result does not depend on arrival order. Half the L2 -> CU bytes of a full 16-region split
// (and 2.5x fewer than 16-row strips, the round-2 form: profiles/r3/diag_up); the
// loop is bound by load latency over the few K-steps in flight, so the diagonal-region blocks
// (half the rows per K-step) run a 6-stage ring of 8 KiB stages in the same LDS (5 in flight).
// ------------------------------------------------------------------------------------
// KS: K pieces of an off-diagonal region (a diagonal region gets KS / 2, at least 1); the pieces'
// fp32 partials go to write-through slabs and the last piece to arrive (ticket) sums them in piece
// order. 4 + 10 tickets and 10 KS 16 KiB slabs per tile (launch_fwd_stats checks the workspace).
// row-group partial scratch of one diagonal tile: [4 row groups][4 contribution slots][64 rows] float2
constexpr int kDiagScratchTile = 4 * 4 * 64;
constexpr int kUpLds = kSubStages * kSubStage + 4 * 64 * 8 + 64;  // ring + column-partial exchange + flags
// (diagonal regions in KS pieces as well: remainder 15.2 -> 16.4 us at the headline, the extra
// piece merges cost more than the shorter K loop saves: profiles/r5/gemm_timing/diag_up.md)
template <int KS> constexpr int diag_ksd() { return KS / 2 > 1 ? KS / 2 : 1; }
template <int KS> constexpr int diag_up_blocks() { return 4 * diag_ksd<KS>() + 6 * KS; }
// The LSE launch folded into the diagonal remainder (LseFold::on; launch_fwd_stats decides). When
// the remainder is the diagonal tiles of exactly the second half of the rows (panels [n/256, rt):
// the headline's 16 of 32), every partial of the first-half rows i and all but the diagonal
// tile's partial of the second-half rows j = i + n are complete before the launch. So, per 64-row
// group G of the remainder (rows j = n + 64 G ..): a side wave pre-merges those (lse_fold_pre),
// the region block that completes the group's diagonal partial merges it (the 4th contributor),
// and whichever of the two arrives second at the group's ticket finishes the 64 pairs with one
// wave (lse_fold_finish: lse2 and the positive coefficient as lse_block, the loss into the LSE
// launch's 64-bit fixed-point ticket, one arrival per group). Neither waits for the other, and
// the LSE launch and its boundary go away.
struct LseFold {
  int on;
  int n;                      // pairs (rows / 2)
  int ngroups;                // 64-row groups of the remainder (loss-ticket arrivals)
  const float* ypos;          // [n] positive logits (log2 units)
  float* lse2;                // [Rpad] (world 1)
  float* cpos;                // [Rpad]
  unsigned long long* ticket; // the LSE scratch's loss ticket (zero; self-cleaning)
  float* loss;                // mean loss
  float2* pre;                // [Rpad] pre-merged (max, sum) states (rows i complete, rows j w/o the diagonal)
  int* gcnt;                  // [ngroups] pre / diagonal arrival tickets (zero; self-cleaning)
  float loss_scale;
  double loss_fx;
};

// Side job of the launch: blocks [nup, gridDim.x) run side(block, count, smem) instead (the LDS is
// this kernel's one array). The remainder waits on load latency with one 4-wave block per CU, so a
// bandwidth-bound job (the raw forward's Z^T, DiagSideZt) runs beside it instead of in a later launch.
struct NoSide {
  int nup;
  __device__ void operator()(int, int, char*) const {}
};
// The 64 pairs of group G finished by one wave (lane = pair): the pre-merged states of rows i and
// j, the diagonal tile's partial (m, s) of row j, then as lse_block.
__device__ __forceinline__ void lse_fold_finish(const LseFold& lf, int G, float2 pi_, float2 pj, float m, float s) {
  const int lane = threadIdx.x & 63;
  const int i = 64 * G + lane, j = i + lf.n;
  float mj = pj.x, sj = pj.y;
  lse_merge(mj, sj, m, s);
  const float yp = lf.ypos[i];
  float l_i, l_j, a_i, a_j;
  const float L2i = finish_row(pi_.x, pi_.y, yp, l_i, a_i), L2j = finish_row(mj, sj, yp, l_j, a_j);
  lf.lse2[i] = L2i;
  lf.lse2[j] = L2j;
  lf.cpos[i] = -(a_i + a_j);
  lf.cpos[j] = -(a_i + a_j);
  const float tot = wave_sum(l_i + l_j);  // fixed tree: deterministic
  if (lane == 0) {  // the LSE launch's ticket (lse_block): arrival, non-finite count, fixed-point sum
    const bool fin = tot >= 0.f && tot < 3.0e38f;
    const unsigned long long qv = fin ? (unsigned long long)llrint((double)tot * lf.loss_fx) : 0ull;
    const unsigned long long add = (qv << 24) | (fin ? 1ull : (1ull << 12) | 1ull);
    const unsigned long long old = __hip_atomic_fetch_add(lf.ticket, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((int)(old & 0xFFF) == lf.ngroups - 1) {
      __hip_atomic_store(lf.ticket, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long all = old + add;
      lf.loss[0] = ((all >> 12) & 0xFFF) ? __builtin_nanf("") : (float)((double)(all >> 24) / lf.loss_fx * (double)lf.loss_scale);
    }
  }
}

// Group G's arrival ticket (lane 0 of the calling wave; agent scope, after the caller's
// write-through stores drained): true for the second of the two arrivals, which resets it.
__device__ __forceinline__ bool lse_fold_ticket(const LseFold& lf, int G) {
  int last = 0;
  if ((threadIdx.x & 63) == 0) {
    const int old = __hip_atomic_fetch_add(lf.gcnt + G, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == 1;
    if (last) __hip_atomic_store(lf.gcnt + G, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return __builtin_amdgcn_readfirstlane(last) != 0;
}

// Side block of group G (4 waves, lane = pair): wave w pre-merges column tiles [Tc w / 4, Tc (w + 1)
// / 4) of rows i (all) and j (all but the diagonal tile nt), one round of loads each; wave 0 merges
// the four states in wave order, publishes them write-through and takes the ticket; the second
// arrival finishes the group.
__device__ __forceinline__ void lse_fold_pre(const SimParams& p, const LseFold& lf, int G, char* smem) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = 64 * G + lane, j = i + lf.n;
  const int nt = j / kTile;  // the remainder's diagonal tile of row j's panel (world 1)
  const int Tc = p.col_tiles, Rpad = p.Rpad;
  const int t0 = Tc * w / 4, t1 = Tc * (w + 1) / 4;
  float mi = kNegInf, si = 0.f, mj = kNegInf, sj = 0.f;
  for (int tb = t0; tb < t1; tb += 8) {  // (8 tiles: Tc <= 32 is one round)
    float2 vi[8], vj[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = tb + u < t1 ? tb + u : tb;
      vi[u] = p.part[(long long)t * Rpad + i];
      vj[u] = p.part[(long long)t * Rpad + j];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (tb + u < t1) {
        lse_merge(mi, si, vi[u].x, vi[u].y);
        if (tb + u != nt) lse_merge(mj, sj, vj[u].x, vj[u].y);
      }
  }
  float4* xs = reinterpret_cast<float4*>(smem);  // [4 waves][64 pairs] (mi, si, mj, sj)
  xs[w * 64 + lane] = make_float4(mi, si, mj, sj);
  __syncthreads();
  if (w != 0) return;
#pragma unroll
  for (int ww = 1; ww < 4; ++ww) {
    const float4 v = xs[ww * 64 + lane];
    lse_merge(mi, si, v.x, v.y);
    lse_merge(mj, sj, v.z, v.w);
  }
  const auto prs = __builtin_amdgcn_make_buffer_rsrc(lf.pre, 0, 0x7FFFFFFF, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(mi), __float_as_uint(si)}, prs, i * 8, 0, 16);
  __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(mj), __float_as_uint(sj)}, prs, j * 8, 0, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (!lse_fold_ticket(lf, G)) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
  const auto drs = __builtin_amdgcn_make_buffer_rsrc(p.part + (long long)nt * Rpad, 0, 0x7FFFFFFF, 0x00020000);
  const u32x2 d = __builtin_amdgcn_raw_buffer_load_b64(drs, j * 8, 0, 16);
  lse_fold_finish(lf, G, make_float2(mi, si), make_float2(mj, sj), __uint_as_float(d[0]), __uint_as_float(d[1]));
}

template <typename T, int FX, int KS>
__device__ __forceinline__ void diag_up_region(const SimParams& p, float2* __restrict__ scratch, const int nup,
                                               const int vb, char* smem, const LseFold& lf) {
#if NTXENT_TIMING
  auto dmark = [&](int k) {
    if (threadIdx.x == 0) p.tstamp[(long long)vb * kTimingItems * kTimingMarks + k] = __builtin_amdgcn_s_memtime();
  };
#else
  auto dmark = [](int) {};
#endif
  dmark(0);
  using MM = Mfma<T>;
  typedef typename MM::frag frag;
  typedef typename StoreT<T>::type TS;
  typedef __attribute__((address_space(3))) const frag lds_frag;
  lds_char* lds = (lds_char*)smem;
  // scalar wave index (scalar M0 arithmetic for the DMA pieces, as sim_gemm_kernel: -0.3 us)
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int KSD = diag_ksd<KS>();                  // K pieces of a diagonal region
  constexpr int NB = diag_up_blocks<KS>();            // blocks per tile
  const int nt_d = nup / NB;                    // diagonal tiles in this launch
  const int idx = xcd_remap(vb, nup);          // a tile's blocks share one XCD
  const int tile = idx / NB, s = idx % NB;
  const bool dg = s < 4 * KSD;
  const int q = dg ? 0 : (s - 4 * KSD) / KS;                     // off-diagonal pair 0..5
  const int hk = dg ? s % KSD : (s - 4 * KSD) % KS;               // K piece
  const int nkp = dg ? KSD : KS;                                  // pieces of this region
  const int rq = dg ? s / KSD : 4 + q;                            // region slot 0..9
  const int a = dg ? s / KSD : (q < 3 ? 0 : (q < 5 ? 1 : 2));
  const int b = dg ? s / KSD : (q < 3 ? q + 1 : (q < 5 ? q - 1 : 3));
  const int4 t = p.tiles[tile];
  const int mt = t.x, nt = t.y;
  const int nk = (int)(p.kbytes / kKStepBytes);
  const int k0 = nk * hk / nkp, k1 = nk * (hk + 1) / nkp;
  // DMA pieces: diagonal region 2 per wave (ring rows 16 w + 8 j + (lane >> 3) = A rows 64 a..),
  // off-diagonal 4 per wave (ring rows 32 w + 8 j + ..: 0-63 A = rows 64 a.., 64-127 B = 64 b..)
  const int np = dg ? 2 : 4;
  const char* src[4];
  int ldst[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = dg ? 16 * w + 8 * j + (lane >> 3) : 32 * w + 8 * j + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    ldst[j] = (dg ? 16 * w + 8 * j : 32 * w + 8 * j) * kKStepBytes;
    src[j] = row < 64 ? p.A.base + (long long)mt * p.A.row_tile_stride + (long long)(64 * a + row) * p.A.ld + 16 * chunk
                      : p.B.base + (long long)(nt - p.b_tile0) * p.B.row_tile_stride +
                            (long long)(64 * b + row - 64) * p.B.ld + 16 * chunk;
  }
  const int SS = dg ? kSubStage / 2 : kSubStage;  // ring stage bytes
  const int NSt = dg ? 2 * kSubStages : kSubStages;
  auto stage = [&](int st, int buf) {
    const long long o = (long long)st * kKStepBytes;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < np)
        __builtin_amdgcn_global_load_lds((const void*)(src[j] + o), (lds_void*)(lds + buf * SS + ldst[j]), 16, 0, 0);
  };
  const int r16 = lane & 15, sw = (r16 >> 1) & 7, cq = lane >> 4;
  const int brow = dg ? 0 : 64;  // ring row of B row 0
  f32x4 acc[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int P = NSt - 1;  // K-steps in flight: 5 (diagonal region) or 2
  for (int i = 0; i < P; ++i) stage(k0 + i < k1 ? k0 + i : k1 - 1, i);
  dmark(1);
  int buf = 0;
  for (int st = k0; st < k1; ++st) {
    // own pieces of step st landed (the P - 1 younger steps' np each in flight: 2 x 4 or 4 x 1);
    // after the barrier every wave's have, and every wave has finished reading the buffer
    // refilled next (the one read in the previous step)
    static_assert(kSubStages == 3, "wait counts assume 6- and 3-stage rings");
    if (dg) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int nb2 = buf == 0 ? NSt - 1 : buf - 1;  // (st + P) % NSt
    stage(st + P < k1 ? st + P : k1 - 1, nb2);
    const lds_char* sb = lds + buf * SS;
    frag af[2], bf[2][4];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int pch = ((4 * c + cq) ^ sw) << 4;
      af[c] = *(lds_frag*)(sb + (16 * w + r16) * kKStepBytes + pch);
#pragma unroll
      for (int f = 0; f < 4; ++f) bf[c][f] = *(lds_frag*)(sb + (brow + 16 * f + r16) * kKStepBytes + pch);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int f = 0; f < 4; ++f) acc[f] = MM::mma(af[c], bf[c][f], acc[f]);
    buf = buf == NSt - 1 ? 0 : buf + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the trailing prefetches
  dmark(2);
  if (p.inv_a) {  // raw operands: normalise (lane: rows 64a + 16w + 4 (lane >> 4) + r, cols 64b + 16f + (lane & 15))
    const f32x4 rs = *reinterpret_cast<const f32x4*>(p.inv_a + (long long)mt * kTile + 64 * a + 16 * w + 4 * (lane >> 4));
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const float cs = p.inv_b[(long long)(nt - p.b_tile0) * kTile + 64 * b + 16 * f + (lane & 15)];
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[f][r] *= rs[r] * cs;
    }
  }
  int* flag = reinterpret_cast<int*>(smem + kSubStages * kSubStage + 4 * 64 * 8);
  int* cnt_pair = p.sk_cnt + 4 * nt_d;  // [nt_d][10] after the [nt_d][4] row-group tickets
  if (nkp > 1) {
    // K pieces: publish this piece's fp32 partial (write-through); the last to arrive sums the
    // region's pieces in piece order (its own from registers), so the result does not depend on
    // the arrival order
    const auto prs = __builtin_amdgcn_make_buffer_rsrc(p.sk_slabs + (size_t)((tile * 10 + rq) * KS) * 4096, 0,
                                                      KS * 4096 * 4, 0x00020000);
#pragma unroll
    for (int f = 0; f < 4; ++f)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[f]), prs,
                                             (int)((hk * 4096 + ((w * 4 + f) * 64 + lane) * 4) * 4), 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(cnt_pair + tile * 10 + rq, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == nkp - 1;
      if (last) __hip_atomic_store(cnt_pair + tile * 10 + rq, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
    f32x4 sum[4];
    for (int h = 0; h < nkp; ++h) {
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        f32x4 v = acc[f];
        if (h != hk)
          v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            prs, (int)((h * 4096 + ((w * 4 + f) * 64 + lane) * 4) * 4), 0, 16));
        sum[f] = h == 0 ? v : sum[f] + v;
      }
    }
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[f] = sum[f];
  }
  dmark(3);
  // lane holds S[row 64a + 16w + 4 (lane >> 4) + r][col 64b + 16 f + (lane & 15)] (tile-local)
  const int rb0 = 64 * a + 16 * w;
  if (p.sc) {  // kept cosines of region (a, b), canonical fragment order, before the masks
    TS* sto = reinterpret_cast<TS*>(p.sc) + (long long)tile * kTileElems;
    if constexpr (sizeof(TS) == 2) {
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        union { TS h[8]; u32x4 u; } pk;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pk.h[r] = from_f32<TS>(acc[2 * h2][r]);
          pk.h[4 + r] = from_f32<TS>(acc[2 * h2 + 1][r]);
        }
        *reinterpret_cast<u32x4*>(sto + sc_unit(rb0, 64 * b + 32 * h2, lane) * 8) = pk.u;
      }
    } else {
#pragma unroll
      for (int f = 0; f < 4; ++f)
        *reinterpret_cast<f32x4*>(sto + (((rb0 >> 4) * 16 + ((64 * b + 16 * f) >> 4)) * 64 + lane) * 4) = acc[f];
    }
  }
  const int r0 = mt * kTile, c0 = (nt * kTile) % p.Rpad;
  const int D0 = r0 - c0, D1 = D0 + p.n_half, D2 = D0 - p.n_half;
  const float sc_ = p.acc_scale, M = p.y_scale;
  // masked logits (log2 units)
  float y[4][4];  // [r][f]
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int tr = rb0 + 4 * (lane >> 4) + r, gi = r0 + tr;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int tc = 64 * b + 16 * f + (lane & 15), d = tc - tr;
      const bool drop = (gi >= p.R) | (c0 + tc >= p.R) | (d == D0) | ((d == D1) & (gi < p.n_half)) |
                        ((d == D2) & (gi >= p.n_half));
      y[r][f] = drop ? kNegInf : acc[f][r] * sc_;
    }
  }
  // row partials of group a over b's 64 columns -> contribution (a, slot b)
  const auto rrs = __builtin_amdgcn_make_buffer_rsrc(scratch + (size_t)(tile * 4 + a) * 4 * 64, 0, 4 * 64 * 8, 0x00020000);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float m = M;
    if constexpr (!FX) m = row16_max(fmaxf(fmaxf(y[r][0], y[r][1]), fmaxf(y[r][2], y[r][3])));
    const float ms = (m == kNegInf) ? 0.f : m;
    float sr = (fast_exp2(y[r][0] - ms) + fast_exp2(y[r][1] - ms)) + (fast_exp2(y[r][2] - ms) + fast_exp2(y[r][3] - ms));
    sr = row16_sum(sr);
    const float mo = FX ? (sr > 0.f ? M : kNegInf) : m;
    if ((lane & 15) == 0)  // write-through: merged by the row group's last contributor on any XCD
      __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(mo), __float_as_uint(sr)}, rrs,
                                            (b * 64 + 16 * w + 4 * (lane >> 4) + r) * 8, 0, 16);
  }
  // column partials of group b over a's 64 rows (off-diagonal regions) -> contribution (b, slot a):
  // per wave over its 16 rows, then the 4 waves merged in wave order through LDS
  if (!dg) {
    typedef __attribute__((address_space(3))) f32x2 lds_f2;
    lds_f2* xw = (lds_f2*)(lds + kSubStages * kSubStage);  // [4 waves][64 cols]
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      float m = M;
      if constexpr (!FX) m = xrow_max(fmaxf(fmaxf(y[0][f], y[1][f]), fmaxf(y[2][f], y[3][f])));
      const float ms = (m == kNegInf) ? 0.f : m;
      float sc = (fast_exp2(y[0][f] - ms) + fast_exp2(y[1][f] - ms)) + (fast_exp2(y[2][f] - ms) + fast_exp2(y[3][f] - ms));
      sc = xrow_sum(sc);
      const float mo = FX ? (sc > 0.f ? M : kNegInf) : m;
      if (lane < 16) xw[w * 64 + 16 * f + lane] = f32x2{mo, sc};
    }
    __syncthreads();
    if (tid < 64) {
      f32x2 v = xw[tid];
      float m = v.x, sm = v.y;
#pragma unroll
      for (int ww = 1; ww < 4; ++ww) {
        const f32x2 u = xw[ww * 64 + tid];
        lse_merge(m, sm, u.x, u.y);
      }
      const auto crs = __builtin_amdgcn_make_buffer_rsrc(scratch + (size_t)(tile * 4 + b) * 4 * 64, 0, 4 * 64 * 8, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(m), __float_as_uint(sm)}, crs, (a * 64 + tid) * 8, 0, 16);
    }
  }
  dmark(4);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  dmark(5);
  if (tid == 0) {  // one ticket per contributed row group; the 4th contributor merges the group
    int lastm = 0;
    const int ga[2] = {a, b};
    for (int k = 0; k < (dg ? 1 : 2); ++k) {
      const int old = __hip_atomic_fetch_add(p.sk_cnt + tile * 4 + ga[k], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == 3) {
        __hip_atomic_store(p.sk_cnt + tile * 4 + ga[k], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lastm |= 1 << k;
      }
    }
    flag[1] = lastm;
  }
  __syncthreads();
  const int lastm = flag[1];
  dmark(6);
  const int k = tid >> 6;  // wave 0 merges group a, wave 1 group b
  if (k > 1 || !((lastm >> k) & 1)) return;
  {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
    const int g = k == 0 ? a : b;
    const auto srs = __builtin_amdgcn_make_buffer_rsrc(scratch + (size_t)(tile * 4 + g) * 4 * 64, 0, 4 * 64 * 8, 0x00020000);
    u32x2 qv[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) qv[kk] = __builtin_amdgcn_raw_buffer_load_b64(srs, (kk * 64 + lane) * 8, 0, 16);
    float m = __uint_as_float(qv[0][0]), sm = __uint_as_float(qv[0][1]);
#pragma unroll
    for (int kk = 1; kk < 4; ++kk) lse_merge(m, sm, __uint_as_float(qv[kk][0]), __uint_as_float(qv[kk][1]));
    if (!lf.on) {
      p.part[(long long)nt * p.Rpad + r0 + 64 * g + lane] = make_float2(m, sm);
      return;
    }
    // LseFold: publish the diagonal partial write-through, then group G's ticket (lse_fold_pre)
    const auto prs = __builtin_amdgcn_make_buffer_rsrc(p.part + (long long)nt * p.Rpad, 0, 0x7FFFFFFF, 0x00020000);
    const int j = r0 + 64 * g + lane, G = (r0 + 64 * g - lf.n) >> 6;
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(m), __float_as_uint(sm)}, prs, j * 8, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!lse_fold_ticket(lf, G)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const auto qrs = __builtin_amdgcn_make_buffer_rsrc(lf.pre, 0, 0x7FFFFFFF, 0x00020000);
    const u32x2 ui = __builtin_amdgcn_raw_buffer_load_b64(qrs, (j - lf.n) * 8, 0, 16);
    const u32x2 uj = __builtin_amdgcn_raw_buffer_load_b64(qrs, j * 8, 0, 16);
    lse_fold_finish(lf, G, make_float2(__uint_as_float(ui[0]), __uint_as_float(ui[1])),
                    make_float2(__uint_as_float(uj[0]), __uint_as_float(uj[1])), m, sm);
  }
}

// nupg: blocks of the grid that run regions (the first nupg; the rest run the side job). Normally
// nupg = side.nup, one block per region; while a transfer is in flight the launcher caps it to the
// CUs the schedule leaves to compute (ws.sched_cus) and each block walks regions nupg apart: a
// region's block never waits on another one (arrival tickets only), so any nupg >= 1 completes.
template <typename T, int FX, int KS, typename SIDE = NoSide>
__global__ __launch_bounds__(256) void diag_up_kernel(const SimParams p, float2* __restrict__ scratch, const SIDE side,
                                                      const int nupg, const LseFold lf) {
  __shared__ __attribute__((aligned(16))) char smem[kUpLds];  // one array: a second __shared__ object drains the LDS-DMA
  if ((int)blockIdx.x >= nupg) {
    const int sb = (int)blockIdx.x - nupg;
    // LseFold: the first ngroups side blocks pre-merge one remainder row group each, first
    if (lf.on && sb < lf.ngroups) {
      lse_fold_pre(p, lf, sb, smem);
      __syncthreads();
    }
    side(sb, (int)gridDim.x - nupg, smem);
    return;
  }
  for (int vb = (int)blockIdx.x; vb < side.nup; vb += nupg) {
    diag_up_region<T, FX, KS>(p, scratch, side.nup, vb, smem, lf);
    __syncthreads();  // the next region restages the ring and the exchange area
  }
}

// ------------------------------------------------------------------------------------
// Split-K forward for tile-starved launches (fewer tiles than CUs, long K: BASELINE config 4,
// 36 tiles x 128 K-steps): every K piece of the persistent GEMM publishes its fp32 partial tile
// (SimParams::splitk), and this launch sums each tile's pieces (fixed block order: deterministic) and runs
// the forward epilogue in 16 row strips per tile instead of one last-arriving block per tile
// reading all p - 1 slabs serially. A strip block writes its rows' partials (complete over the
// tile) and the kept cosines; for a kTileSymOff tile it also publishes its 16-row column
// partials (sc1 stores into colp), and the tile's last strip block to arrive (ticket) merges
// the 16 strips per column in strip order. A slab holds the tile in the GEMM's fragment order:
// float ((w * 32 + f) * 64 + lane) * 4 + r for wave w, fragment f = 4 mi + ni.
// ------------------------------------------------------------------------------------
constexpr int kSkColpTile = 16 * kTile;  // float2 column partials per tile: [16 strips][256 cols]

__device__ __forceinline__ int sk_frag_off(int row, int col) {  // float offset of element (row, col)
  const int mi = 4 * (row >> 7) + ((row >> 4) & 3), wa = (row >> 6) & 1;
  const int ni = 2 * (col >> 7) + ((col >> 4) & 1), wb = (col >> 5) & 3;
  const int lane = 16 * ((row >> 2) & 3) + (col & 15);
  return (((4 * wa + wb) * 32 + 4 * mi + ni) * 64 + lane) * 4 + (row & 3);
}

template <typename TS, int FX>
__global__ __launch_bounds__(256) void sk_reduce_kernel(const SimParams p, float2* __restrict__ colp) {
  __shared__ float red[4][16][2];
  __shared__ int last_flag;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int tile = blockIdx.x >> 4, strip = blockIdx.x & 15;
  const int4 t = p.tiles[tile];
  const int mt = t.x, nt = t.y, kind = t.z;
  const int s16 = 16 * strip;
  const int nk = p.nk;
  const long long ipb = p.ipb;
  // the tile's pieces: blocks pc * sk_tiles + tile, pc = 0 .. npc - 1, summed in piece order
  const int b0 = 0, b1 = (int)((nk + ipb - 1) / ipb) - 1;
  // this thread's 4 fragments (s16, cb[j] = 64 w + 16 j), MFMA C layout: rows s16 + r4 + r,
  // column cb[j] + c1; a wave reads 1 KiB contiguous per fragment and slab
  const int r4 = 4 * (lane >> 4), c1 = lane & 15;
  int off[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) off[j] = sk_frag_off(s16 + r4, 64 * w + 16 * j + c1);
  f32x4 v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* slabs = reinterpret_cast<const float*>(p.sk_slabs);
  auto slab = [&](int bb) { return slabs + (size_t)(2 * (bb * p.sk_tiles + tile) + 1) * kTileElems; };  // piece bb
  if (p.sk_half) {
    // fp16 slabs (sk_fixup): fragments j = 2 jp, 2 jp + 1 of this thread are one 16-B unit, at
    // ((W * 16 + f / 2) * 64 + lane) of the slab for the float offset ((W * 32 + f) * 64 + lane) * 4
    unsigned hoff[2];
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      const int u = off[2 * jp] >> 2;
      hoff[jp] = (unsigned)((((u >> 7) << 6) + (u & 63)) * 16);
    }
    const char* hs = reinterpret_cast<const char*>(p.sk_slabs);
    // 8 loads in flight (clamped, weighted as below; 16 measured +0.9 us at config 4)
    for (int bb = b0; bb <= b1; bb += 4) {
      u32x4 x[4][2];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const char* sl = hs + (size_t)(2 * ((bb + u <= b1 ? bb + u : b1) * p.sk_tiles + tile) + 1) * kTileElems * 4;
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) x[u][jp] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sl + hoff[jp]));
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float k = bb + u <= b1 ? 1.f : 0.f;
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          union { u32x4 u; _Float16 h[8]; } pk;
          pk.u = x[u][jp];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[2 * jp][r] += (float)pk.h[r] * k;
            v[2 * jp + 1][r] += (float)pk.h[4 + r] * k;
          }
        }
      }
    }
  } else
  // 4 slabs per round, all 16 loads issued before the adds (clamped indices: no conditional
  // load; a clamped duplicate is multiplied by 0)
  for (int bb = b0; bb <= b1; bb += 4) {
    f32x4 x[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float* sl = slab(bb + u <= b1 ? bb + u : b1);
#pragma unroll
      for (int j = 0; j < 4; ++j) x[u][j] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(sl + off[j]));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float k = bb + u <= b1 ? 1.f : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] += x[u][j] * k;
    }
  }
  if (p.sc) {  // kept cosines (canonical fragment order), before the masks
    TS* st = reinterpret_cast<TS*>(p.sc) + (long long)tile * kTileElems;
    if constexpr (sizeof(TS) == 2) {
#pragma unroll
      for (int np = 0; np < 2; ++np) {
        union { TS h[8]; u32x4 u; } pk;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pk.h[r] = from_f32<TS>(v[2 * np][r]);
          pk.h[4 + r] = from_f32<TS>(v[2 * np + 1][r]);
        }
        *reinterpret_cast<u32x4*>(st + sc_unit(s16, 64 * w + 32 * np, lane) * 8) = pk.u;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<f32x4*>(st + (((s16 >> 4) * 16 + ((64 * w + 16 * j) >> 4)) * 64 + lane) * 4) = v[j];
    }
  }
  const int r0 = mt * kTile, c0 = (nt * kTile) % p.Rpad;
  const int D0 = r0 - c0, D1 = D0 + p.n_half, D2 = D0 - p.n_half;
  const float sc_ = p.acc_scale, M = p.y_scale;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int tr = s16 + r4 + r, tc = 64 * w + 16 * j + c1, gi = r0 + tr, d = tc - tr;
      const bool drop = (gi >= p.R) | (c0 + tc >= p.R) | (d == D0) | ((d == D1) & (gi < p.n_half)) |
                        ((d == D2) & (gi >= p.n_half));
      v[j][r] = drop ? kNegInf : v[j][r] * sc_;
    }
  // row partials over this wave's 64 columns (the 16 lanes of a DPP row), merged over the waves
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float m = M;
    if constexpr (!FX) m = row16_max(fmaxf(fmaxf(v[0][r], v[1][r]), fmaxf(v[2][r], v[3][r])));
    const float ms = (m == kNegInf) ? 0.f : m;
    float sr = (fast_exp2(v[0][r] - ms) + fast_exp2(v[1][r] - ms)) + (fast_exp2(v[2][r] - ms) + fast_exp2(v[3][r] - ms));
    sr = row16_sum(sr);
    if (c1 == 0) {
      red[w][r4 + r][0] = FX ? (sr > 0.f ? M : kNegInf) : m;
      red[w][r4 + r][1] = sr;
    }
  }
  const bool sym = kind == kTileSymOff;
  if (sym) {  // this strip's column partials (16 rows): the 4 rows of a lane, lanes l ^ 16, 32, 48
    const auto crs = __builtin_amdgcn_make_buffer_rsrc(colp + (size_t)tile * kSkColpTile, 0, kSkColpTile * 8, 0x00020000);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float m = M;
      if constexpr (!FX) m = xrow_max(fmaxf(fmaxf(v[j][0], v[j][1]), fmaxf(v[j][2], v[j][3])));
      const float ms = (m == kNegInf) ? 0.f : m;
      float sc2 = (fast_exp2(v[j][0] - ms) + fast_exp2(v[j][1] - ms)) + (fast_exp2(v[j][2] - ms) + fast_exp2(v[j][3] - ms));
      sc2 = xrow_sum(sc2);
      const float mo = FX ? (sc2 > 0.f ? M : kNegInf) : m;
      if (lane < 16)  // write-through (sc1): read by the tile's last strip block on any XCD
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(mo), __float_as_uint(sc2)}, crs,
                                              (strip * kTile + 64 * w + 16 * j + c1) * 8, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (threadIdx.x < 16) {
    const int i = threadIdx.x;
    float m = red[0][i][0], s = red[0][i][1];
#pragma unroll
    for (int q = 1; q < 4; ++q) lse_merge(m, s, red[q][i][0], red[q][i][1]);
    p.part[(long long)nt * p.Rpad + r0 + s16 + i] = make_float2(m, s);
  }
  if (!sym) return;
  if (threadIdx.x == 0) {  // ticket: the 16th strip block of the tile merges the column partials
    const int old = __hip_atomic_fetch_add(p.sk_cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == 15;
    if (last) __hip_atomic_store(p.sk_cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_flag = last;
  }
  __syncthreads();
  if (!last_flag) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
  const auto crs = __builtin_amdgcn_make_buffer_rsrc(colp + (size_t)tile * kSkColpTile, 0, kSkColpTile * 8, 0x00020000);
  const int c = threadIdx.x;  // one column per thread, strips in order (deterministic)
  u32x2 q[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) q[k] = __builtin_amdgcn_raw_buffer_load_b64(crs, (k * kTile + c) * 8, 0, 16);
  float m = __uint_as_float(q[0][0]), s = __uint_as_float(q[0][1]);
#pragma unroll
  for (int k = 1; k < 16; ++k) lse_merge(m, s, __uint_as_float(q[k][0]), __uint_as_float(q[k][1]));
  p.part[(long long)(p.row_tile0 + mt) * p.Rpad + (nt - p.row_tile0) * kTile + c] = make_float2(m, s);
}

// ------------------------------------------------------------------------------------
// Split-K dZ for tile-starved dZ GEMMs (d <= 1024 at 8192 rows: 64 tiles x 128 K-steps on 256
// CUs): the K pieces publish fp32 partial tiles (SimParams::splitk) and this launch sums each tile's
// pieces in block order (deterministic) and writes the dZ tile exactly as the GEMM's epilogue
// would (fp16 or fp32, optionally accumulated), 64 blocks per tile: block (w, k) = fragments
// 4k..4k+3 of GEMM wave w, one (fragment, lane) per thread (one batch of slab loads in flight).
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sk_dz_reduce_kernel(const SimParams p) {
  const int tile = blockIdx.x >> 6, w = (blockIdx.x >> 3) & 7, kq = blockIdx.x & 7;
  const int4 t = p.tiles[tile];
  const int mt = t.x, nt = t.y;
  const int nk = p.nk;
  const long long ipb = p.ipb;
  // the tile's pieces (piece-major, as sk_reduce_kernel): piece pc is block pc * sk_tiles + tile
  const int b0 = 0, b1 = (int)((nk + ipb - 1) / ipb) - 1;
  const float* slabs = reinterpret_cast<const float*>(p.sk_slabs);
  auto slab = [&](int bb) { return slabs + (size_t)(2 * (bb * p.sk_tiles + tile) + 1) * kTileElems; };
  const int wa = w >> 2, wb = w & 3;
  // one output fragment f of GEMM wave w for this lane, summed over the pieces (v)
  auto emit = [&](int f, int lane, f32x4 v) {
    const int mi = f >> 2, ni = f & 3;
    const int rb = 128 * (mi >> 2) + 64 * wa + 16 * (mi & 3), cb = 128 * (ni >> 1) + 32 * wb + 16 * (ni & 1);
    // swapped orientation (as the dZ epilogue): out[m = rb + (lane & 15)][n = cb + 4 (lane >> 4) + r]
    const long long row = (long long)mt * kTile + rb + (lane & 15);
    const int col = nt * kTile + cb + 4 * (lane >> 4);
    if (p.ndh) {
      // fused normalisation backward (as dz_store): g rounded to fp16 like the unfused slab
      if (row >= p.R || col >= p.nd) return;  // (nd % 8 == 0: the 4 columns are all in or all out)
      const float sgo = p.ngo[0] * p.nalpha, iv = p.ninv[row];
      const float c1 = sgo * iv, c2 = sgo * iv * iv * p.ndot[row];
      const long long off = row * p.nd + col;
      float hv[4], o[4];
      if (p.nh_dt == 0) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(static_cast<const float*>(p.nh) + off);
#pragma unroll
        for (int r = 0; r < 4; ++r) hv[r] = a[r];
      } else {
        union { _Float16 f[4]; __bf16 b[4]; u32x2 u; } x;
        x.u = *reinterpret_cast<const u32x2*>(static_cast<const char*>(p.nh) + off * 2);
#pragma unroll
        for (int r = 0; r < 4; ++r) hv[r] = p.nh_dt == 1 ? (float)x.f[r] : (float)x.b[r];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = c1 * (float)(_Float16)v[r] - c2 * hv[r];
      if (p.nh_dt == 0) {
        *reinterpret_cast<f32x4*>(static_cast<float*>(p.ndh) + off) = f32x4{o[0], o[1], o[2], o[3]};
      } else {
        union { _Float16 f[4]; __bf16 b[4]; u32x2 u; } y;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (p.nh_dt == 1) y.f[r] = (_Float16)o[r];
          else y.b[r] = (__bf16)o[r];
        }
        *reinterpret_cast<u32x2*>(static_cast<char*>(p.ndh) + off * 2) = y.u;
      }
    } else if (p.out_f16) {
      union { _Float16 h[4]; u32x2 u; } pk;
#pragma unroll
      for (int r = 0; r < 4; ++r) pk.h[r] = (_Float16)v[r];
      *reinterpret_cast<u32x2*>(reinterpret_cast<_Float16*>(p.out) + row * p.ldo + col) = pk.u;
    } else {
      f32x4* o = reinterpret_cast<f32x4*>(p.out + row * p.ldo + col);
      *o = p.accum ? *o + v : v;
    }
  };
  {
    const int u = threadIdx.x + 256 * kq, f = u >> 6, lane = u & 63;
    const int off = ((w * 32 + f) * 64 + lane) * 4;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int bb = b0; bb <= b1; bb += 4) {  // 4 slab loads in flight (clamped, weighted)
      f32x4 x[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) x[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(slab(bb + q <= b1 ? bb + q : b1) + off));
#pragma unroll
      for (int q = 0; q < 4; ++q) v += x[q] * (bb + q <= b1 ? 1.f : 0.f);
    }
    emit(f, lane, v);
  }
}

}  // namespace dev
}  // namespace ntxent

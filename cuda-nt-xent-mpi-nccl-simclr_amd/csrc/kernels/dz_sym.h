// The dZ GEMM of the single-process / all-gather flows on the symmetric coefficient matrix:
//
//   dZ[m][d] = sum_j C[m][j] Z[j][d],   C = P + P^T - 2 I_pos  (symmetric)
//
// reading C only from the tiles the coefficient pass writes — the own block's upper triangle
// (C_IJ, I <= J, row-major [m][j] per 256x256 tile) and every remote tile — and Z straight from
// the normalised rows Zq[j][d] (no transposed copy of Z, no mirrored C tiles: the round-2 flow
// wrote a full C and a ZqT, 64 MiB + 32 MiB more HBM writes per step at the headline). A K-step
// whose column tile J lies in the own block below the diagonal (J < own0 + mt) is the transpose
// of the stored tile C_{J, mt}: its A half-tile is staged from that tile's rows (j-major) and its
// fragments are read transposed (ds_read_b64_tr_b16), exactly like every Z fragment.
//
// Same 256x256 tile, 8 waves, 4-phase staggered ping-pong and counted waits as sim_gemm_kernel
// (see sim_gemm.h). LDS images per K-step (64 j-columns) and half-tile (16 KiB each):
//   direct A   [128 m][64 j]   128-B rows, chunk ^ ((row >> 1) & 7)       read by ds_read_b128
//   mirrored A [64 j][128 m]   256-B rows, chunk ^ tr_swz(j)               read by ds_read_b64_tr_b16
//   Z          [64 j][128 d]   256-B rows, chunk ^ tr_swz(j)               read by ds_read_b64_tr_b16
// tr_swz(j) = 2 * ((j & 3) + 4 * ((j >> 3) & 1)) makes a 32-lane half's 8 rows (two 4-row blocks
// 8 rows apart) land in 8 distinct 32-byte bank segments: the transposed reads are conflict-free.
// The swizzles are applied on the per-lane SOURCE address of the lane-linear LDS-DMA
// (cdna_hip_programming.md §5.4 rule 21) and on the read address.
//
// Replaces the reference's backward SGEMM (/root/reference/src/ntxent_kernel.cu:229-236).
#pragma once

#include "sim_gemm.h"

namespace ntxent {
namespace dev {

__device__ __forceinline__ int tr_swz(int j) { return 2 * ((j & 3) + 4 * ((j >> 3) & 1)); }

// SimParams fields used: A.base = coefficient tiles [row_tiles][c_ld] (tile (I, J) at
// (I * c_ld + J - c_tile0) tiles), B.base = Zq_all rows (B.ld bytes apart), tiles / nk / stream-K
// schedule, out / ldo / out_f16 / accum (dz_store), own0 -> row_tile0 (own block's first global
// column tile), Rpad (row_tiles = Rpad / 256).
template <typename T>
__global__ __launch_bounds__(kGemmThreads) void dz_sym_kernel(const SimParams p) {
  static_assert(sizeof(T) == 2, "transposed LDS reads: 16-bit operands only");
  typedef typename Mfma<T>::frag frag;
  typedef __attribute__((address_space(3))) const frag lds_frag;
  __shared__ __attribute__((aligned(16))) char smem[kGemmLds + 2048];  // + the fused epilogue's row coefficients
  lds_char* lds = (lds_char*)smem;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wa = w >> 2, wb = w & 3;
  const int G = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, G);
  const int nk = p.nk;
  const int rt = p.Rpad / kTile, t0 = p.row_tile0;
  const long long tile_bytes = (long long)kTileElems * 2;

  // ---- per-lane staging offsets (bytes from the wave-uniform source base) ----
  // direct A: piece j of half h = rows 128 h + 16 w + 8 j + (lane >> 3) of the C tile, 16-B
  // chunk (lane & 7) ^ ((row >> 1) & 7) of the K-step's 128 bytes
  // mirrored A / Z: piece j = rows 8 w + 4 j + (lane >> 4) of the K-step's 64 j-rows, 16-B chunk
  // (lane & 15) ^ tr_swz(row) of the half's 256 bytes
  // (named scalars, not arrays: a select between array elements went through scratch)
  auto dir_off = [&](int h, int j) {
    const int row = 128 * h + 16 * w + 8 * j + (lane >> 3);
    return (unsigned)(row * kTile * 2 + (((lane & 7) ^ ((row >> 1) & 7)) << 4));
  };
  auto tr_row_off = [&](int j, unsigned ld) {
    const int jr = 8 * w + 4 * j + (lane >> 4);
    return (unsigned)(jr * ld + ((((lane & 15) ^ tr_swz(jr))) << 4));
  };
  const unsigned a_d00 = dir_off(0, 0), a_d01 = dir_off(0, 1), a_d10 = dir_off(1, 0), a_d11 = dir_off(1, 1);
  const unsigned a_m0 = tr_row_off(0, kTile * 2), a_m1 = tr_row_off(1, kTile * 2);  // + 256 h
  const unsigned z_o0 = tr_row_off(0, (unsigned)p.B.ld), z_o1 = tr_row_off(1, (unsigned)p.B.ld);  // + 256 h
  int mt = 0, nt = 0;
  // K-step k of the current tile: mirrored when its column tile lies below the own diagonal
  auto is_mir = [&](int k) {
    const int J = k >> 2;
    return J >= t0 && J < t0 + mt;
  };
  // stage half-tile h of A (isB = 0: coefficients) or B (isB = 1: Zq) for K-step k into buf.
  // Branch-free (a branch in the staging path costs the DMA-issue-bound load interval): the
  // direct and the mirrored A pieces land at the same LDS offsets (1 KiB pieces 2 w + j), the
  // source base is a scalar select and the per-lane offset a mask blend.
  auto stage = [&](int isB, int h, int k, int buf) {
    lds_char* dst = lds + buf * kStageBytes + isB * (kTile * kKStepBytes) + h * kHalfBytes + w * 2048;
    const int J = k >> 2, kk = k & 3;
    const char* src;
    unsigned o0, o1;
    if (isB) {
      src = p.B.base + (long long)k * 64 * p.B.ld + (long long)nt * kTile * 2 + h * 256;
      o0 = z_o0;
      o1 = z_o1;
    } else {
      const bool mir = J >= t0 && J < t0 + mt;
      const long long ti = mir ? (long long)(J - t0) * p.c_ld + (t0 + mt - p.c_tile0)
                               : (long long)mt * p.c_ld + (J - p.c_tile0);
      src = p.A.base + ti * tile_bytes + (mir ? kk * (64 * kTile * 2) + h * 256 : kk * 128);
      const unsigned msk = mir ? 0xffffffffu : 0u;  // wave-uniform
      const unsigned d0 = h ? a_d10 : a_d00, d1 = h ? a_d11 : a_d01;
      o0 = d0 ^ ((d0 ^ a_m0) & msk);
      o1 = d1 ^ ((d1 ^ a_m1) & msk);
    }
    __builtin_amdgcn_global_load_lds((const void*)(src + o0), (lds_void*)dst, 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(src + o1), (lds_void*)(dst + 1024), 16, 0, 0);
  };

  f32x4 acc[8][4];
  const int r16 = lane & 15, sw = (r16 >> 1) & 7, cq = lane >> 4;
  // Transposed reads of a [64 j][128 col] 256-B-row image for the fragment whose 16 columns start
  // at c0: lane 4q + p of group g supplies row 32 s + 8 g + q (+4 for the second read), columns
  // c0 + 4p .. +3. tr_swz(row) = 2 tq + 8 (cq & 1) does not depend on s or on the +4, so the four
  // reads of a fragment share one lane address and differ by immediates (+8192 s, +1024).
  const int tq = (lane >> 2) & 3, tp = lane & 3;
  const int trx = 2 * tq + 8 * (cq & 1);
  auto tr_lane = [&](int c0) {  // byte offset of the (s = 0, first) read for columns c0
    return (8 * cq + tq) * 256 + ((((c0 >> 3) ^ trx) | (tp >> 1)) << 4) + 8 * (tp & 1);
  };
  // The transposed reads are inline asm: as a builtin, hipcc cannot tell them apart from the
  // in-flight LDS-DMA and drains vmcnt(0) before every group (it did: 45 drains in this kernel,
  // the dZ GEMM 25 % slower). Untracked by the compiler, each read's two 8-byte halves are
  // joined into the MFMA operand only after the explicit lgkmcnt drain of the compute interval
  // (an empty asm marks the halves as written there).
  typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
  typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
#define NTXENT_TR8(dst, addr, imm) asm volatile("ds_read_b64_tr_b16 %0, %1 offset:" #imm : "=v"(dst) : "v"(addr))
  // both k-substeps of one fragment: h[s] = {first, second} halves
  auto tr_issue2 = [&](unsigned a, u32x2v (&h)[2][2]) {
    NTXENT_TR8(h[0][0], a, 0);
    NTXENT_TR8(h[0][1], a, 1024);
    NTXENT_TR8(h[1][0], a, 8192);
    NTXENT_TR8(h[1][1], a, 9216);
  };
#undef NTXENT_TR8
  u32x4v bh0[2][2], bh1[2][2];  // [s][ni] raw B operands (joined after the drain)
  u32x4v araw[2][4];            // [s][mi] raw A operands (direct or transposed)
  frag af[2][4], bf0[2][2], bf1[2][2];
  // A reads: one runtime branch on the K-step's kind; both paths leave raw dwords in araw (asm
  // loads, untracked), so the two paths share registers
  auto read_a = [&](int buf, int h, bool mir) {
    const unsigned As = (unsigned)(uintptr_t)(lds + buf * kStageBytes + h * kHalfBytes);
    if (mir) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        u32x2v t[2][2];
        tr_issue2(As + tr_lane(64 * wa + 16 * mi), t);
#pragma unroll
        for (int s = 0; s < 2; ++s) araw[s][mi] = __builtin_shufflevector(t[s][0], t[s][1], 0, 1, 2, 3);
      }
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        // rows 16 mi apart: immediates 2048 mi
        const unsigned a = As + (64 * wa + r16) * kKStepBytes + (((4 * s + cq) ^ sw) << 4);
        asm volatile("ds_read_b128 %0, %1" : "=v"(araw[s][0]) : "v"(a));
        asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(araw[s][1]) : "v"(a));
        asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(araw[s][2]) : "v"(a));
        asm volatile("ds_read_b128 %0, %1 offset:6144" : "=v"(araw[s][3]) : "v"(a));
      }
    }
  };
  auto join_a = [&]() {  // after the lgkmcnt drain
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        asm volatile("" : "+v"(araw[s][mi]));
        af[s][mi] = __builtin_bit_cast(frag, araw[s][mi]);
      }
  };
  auto read_b = [&](int buf, int h, u32x4v (&bh)[2][2]) {
    const unsigned Bs = (unsigned)(uintptr_t)(lds + buf * kStageBytes + kTile * kKStepBytes + h * kHalfBytes);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      u32x2v t[2][2];
      tr_issue2(Bs + tr_lane(32 * wb + 16 * ni), t);
#pragma unroll
      for (int s = 0; s < 2; ++s) bh[s][ni] = __builtin_shufflevector(t[s][0], t[s][1], 0, 1, 2, 3);
    }
  };
  auto join_b = [&](u32x4v (&bh)[2][2], frag (&bf)[2][2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        asm volatile("" : "+v"(bh[s][ni]));
        bf[s][ni] = __builtin_bit_cast(frag, bh[s][ni]);
      }
  };
  auto mma_quadrant = [&](auto qa_c, auto qb_c, frag (&bf)[2][2]) {
    constexpr int qa = decltype(qa_c)::value, qb = decltype(qb_c)::value;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          f32x4& c = acc[qa * 4 + mi][qb * 2 + ni];
          c = Mfma<T>::mma(bf[s][ni], af[s][mi], c);
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
  auto dma_wait = [&]() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); };
  const int grp = __builtin_amdgcn_readfirstlane(w) >> 2;

  const long long sk_total = (long long)p.sk_tiles * nk;
  const long long it0 = (long long)bid * p.ipb;
  const long long it1 = it0 + p.ipb < sk_total ? it0 + p.ipb : sk_total;
  const int n_dp = p.dp_tiles > bid ? (p.dp_tiles - bid + G - 1) / G : 0;
  long long it = it0;
  for (int item = 0;; ++item) {
    int tile, kb, ke, stile = -1;
    if (item < n_dp) {
      tile = bid + item * G;
      kb = 0;
      ke = nk;
    } else {
      if (it >= it1) break;
      stile = (int)(it / nk);
      kb = (int)(it % nk);
      ke = (int)((long long)kb + (it1 - it) < nk ? kb + (it1 - it) : nk);
      it += ke - kb;
      tile = p.dp_tiles + stile;
    }
    const int4 t = p.tiles[tile];
    mt = t.x;
    nt = t.y;
    const int nsteps = ke - kb;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
    // K positions of the four half-tile streams (clamped: the trailing prefetches re-read the
    // last step, so every wait count is uniform)
    int ka0 = kb, ka1 = kb, kb0 = kb, kb1 = kb;
    const int klast = ke - 1;
    auto adv = [&](int& k) { k = k < klast ? k + 1 : k; };
    // prologue: A0 B0 B1 A1 of step 0, A0 B0 B1 of step 1 (the issue order the waits assume)
    stage(0, 0, ka0, 0); adv(ka0);
    stage(1, 0, kb0, 0); adv(kb0);
    stage(1, 1, kb1, 0); adv(kb1);
    stage(0, 1, ka1, 0); adv(ka1);
    stage(0, 0, ka0, 1); adv(ka0);
    stage(1, 0, kb0, 1); adv(kb0);
    stage(1, 1, kb1, 1); adv(kb1);
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");  // A0(0), B0(0) retired
    barrier();
    if (grp == 1) barrier();  // stagger group 1 by one barrier
    for (int ks = 0; ks < nsteps; ++ks) {
      const int cur = ks & 1, nxt = cur ^ 1;
      const bool mir = is_mir(kb + ks);
      // phases as sim_gemm_kernel (see its comment for the WAR / RAW argument)
      dma_wait(); barrier();          // phase 1 L
      read_a(cur, 0, mir);
      __builtin_amdgcn_sched_barrier(0);
      read_b(cur, 0, bh0);
      stage(0, 1, ka1, nxt); adv(ka1);   // A1 of step ks+1
      // A0's reads (issued first; 8 b128 or 16 tr reads) retire before the barrier: A0 is
      // re-staged next phase. The B0 reads (8) may retire after it.
      asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      barrier();                      // phase 1 C
      lds_drain();
      join_a();
      join_b(bh0, bf0);
      mma_quadrant(kI0, kI0, bf0);
      dma_wait(); barrier();          // phase 2 L
      read_b(cur, 1, bh1);
      stage(0, 0, ka0, cur); adv(ka0);   // A0 of step ks+2
      barrier(); lds_drain();         // phase 2 C
      join_b(bh1, bf1);
      mma_quadrant(kI0, kI1, bf1);
      barrier();                      // phase 3 L
      read_a(cur, 1, mir);
      stage(1, 0, kb0, cur); adv(kb0);   // B0 of step ks+2
      barrier(); lds_drain();         // phase 3 C
      join_a();
      mma_quadrant(kI1, kI0, bf0);
      dma_wait(); barrier();          // phase 4 L
      stage(1, 1, kb1, cur); adv(kb1);   // B1 of step ks+2
      barrier();                      // phase 4 C
      mma_quadrant(kI1, kI1, bf1);
    }
    if (grp == 0) barrier();  // re-align the groups
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    {
      int tid_e = threadIdx.x;
      asm volatile("" : "+v"(tid_e));
      const int tid = tid_e, w = tid_e >> 6;
      const int wa = w >> 2, wb = w & 3;
      int rb[8], cb[4];
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) rb[mi] = 128 * (mi >> 2) + 64 * wa + 16 * (mi & 3);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) cb[ni] = 128 * (ni >> 1) + 32 * wb + 16 * (ni & 1);
      if (nsteps != nk && !sk_fixup<false>(acc, p, stile, bid, G, tid, smem)) continue;
      dz_store(acc, p, mt, nt, tid, rb, cb, lds);
    }
    __syncthreads();  // the next item's staging reuses the LDS
  }
}

}  // namespace dev
}  // namespace ntxent

// ntxent-mi355x — public C++ API (raw device pointers, no libtorch dependency).
//
// MI355X-native (gfx950 / CDNA4) NT-Xent (SimCLR) loss. This header replaces the
// reference's `include/ntxent_kernel.cuh` (decls at :31-52, constants :10-13,
// CUDA_CHECK :16-22, utils :79-110, cuBLAS singleton :112-135) with an API that is
// correct for the *intended* math and shaped for MI355X:
//
//   * one 256x256 MFMA tile per workgroup (8 wave64s), K staged 128 B/row per step
//     through LDS by global_load_lds (no BLAS in the hot path);
//   * the 2N x 2N logits are never materialised in fp32: the forward GEMM reduces each
//     tile to per-row (max, sum-exp2) partials in its epilogue and (optionally) keeps
//     the cosine tile in the compute dtype for the backward;
//   * S is symmetric, so within a rank's own column block only the upper-triangular
//     tiles are computed; each produces row AND column partials;
//   * the backward is rank-local: C = P + P^T - 2*I_pos is formed from the stored
//     cosines + all-gathered LSE (no atomics, deterministic), then dZ = C * Z runs on
//     MFMA; the dZ GEMM's epilogue applies grad_out/(2N*tau) and the L2-normalisation
//     backward (dh = c1 g - c2 h, with dot_i = z_i . g_i from the coefficient pass).
//
// Layout conventions (see Geometry):
//   * R local rows = [view1 (n rows); view2 (n rows)], positive p(i) = (i + n) mod R.
//   * Global column index = rank * Rpad + local row (padded rank blocks).
//   * Zq   [Rpad][ld_k]      normalised rows in the compute dtype (zero padded to dim_k).
//   * ZqT  [dim_n][ld_t]     its transpose (B operand of the dZ GEMM), columns [0, Rpad).
//     ld_k / ld_t add 128 B to strides that are multiples of 2 KiB, so the 256 rows a GEMM
//     tile streams do not all land in the same L2 channel.
//   * SC   [row_tiles][col_tiles][256*256]  tile-blocked cosines / coefficients.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace ntxent {

// ---- gfx950 constants (reference `WARP_SIZE=32` etc. at include/ntxent_kernel.cuh:10-13
//      are CUDA-isms; CDNA4 is wave64 with 160 KiB LDS per CU) -------------------------
constexpr int kWaveSize = 64;
constexpr int kTile = 256;          // square output tile of every similarity GEMM
constexpr int kTileElems = kTile * kTile;
constexpr int kKStepBytes = 128;    // bytes of K staged per row per pipeline step
constexpr int kGemmThreads = 512;   // 8 waves: 2 (M) x 4 (N), 128x64 per wave
constexpr int kLdsPerCU = 160 * 1024;
constexpr int kNumXcd = 8;

// FP8 (e4m3, OCP) is a forward-GEMM operand type only: an fp8 plan runs the similarity GEMM
// on fp8 MFMA and keeps cosines / runs the backward in fp16.
enum class DType : int { F32 = 0, F16 = 1, BF16 = 2, FP8 = 3 };

inline size_t dtype_size(DType t) { return t == DType::F32 ? 4 : (t == DType::FP8 ? 1 : 2); }
inline const char* dtype_name(DType t) {
  return t == DType::F32 ? "fp32" : (t == DType::F16 ? "fp16" : (t == DType::BF16 ? "bf16" : "fp8"));
}
// dtype of zq / ZqT / kept cosines / coefficients (the backward operands) for a plan dtype
inline DType backward_dtype(DType t) { return t == DType::FP8 ? DType::F16 : t; }

// Status-typed error check (the reference mis-types a cuBLAS status into AT_CUDA_CHECK at
// src/ntxent_kernel.cu:166; here every HIP call goes through a hipError_t check).
#define NTXENT_HIP_CHECK(expr)                                                        \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) {                                                           \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +   \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__) +   \
                               " in " #expr);                                         \
    }                                                                                 \
  } while (0)

#define NTXENT_CHECK(cond, msg)                                                       \
  do {                                                                                \
    if (!(cond)) throw std::invalid_argument(std::string("ntxent: ") + (msg));        \
  } while (0)

// Problem geometry shared by every kernel of one NT-Xent evaluation.
struct Geometry {
  int rows = 0;        // R: local rows (2 * per-view batch on this rank)
  int rows_pad = 0;    // Rpad = roundup(R, 256)
  int dim = 0;         // d
  int dim_k = 0;       // roundup(d, 64): row stride of Zq (K of the forward GEMM)
  int dim_n = 0;       // roundup(d, 256): rows of ZqT (N of the dZ GEMM)
  int ld_k = 0;        // row stride (elements) of Zq: dim_k, de-aliased from powers of two
  int ld_t = 0;        // row stride (elements) of ZqT: rows_pad, de-aliased likewise
  int dim_k8 = 0;      // roundup(d, 128): K bytes of an fp8 row (one 128-byte K-step = 128 elements)
  int ld_k8 = 0;       // row stride (bytes) of the fp8 copy Zq8
  int world = 1;       // W ranks sharing negatives
  int rank = 0;
  int row_tiles = 0;   // Rpad / 256
  int col_tiles = 0;   // W * Rpad / 256
  float temperature = 0.07f;
  float inv_temp = 1.0f / 0.07f;
  long long global_rows = 0;  // W * R  (the 2N of the loss normalisation)
};

Geometry make_geometry(int rows, int dim, int world, int rank, float temperature);

// Tile kinds of the forward / coefficient pass. kTileCross: a tile of another rank's column
// block that this rank computes for BOTH ranks (symmetric data-parallel mode): its column
// partials and mirrored coefficients go to per-partner buffers instead of this rank's own.
enum TileKind : int { kTilePlain = 0, kTileDiag = 1, kTileSymOff = 2, kTileCross = 3,
                      // coefficient pass only: an upper off-diagonal 64x64 region of a diagonal tile,
                      // written with its mirror (the transposed region of the same tile)
                      kTileDiagUp = 4 };

// Symmetric data-parallel mode: rank `rank` computes rows [m0, m1) (its row tiles) x columns
// [k0, k1) (rank q's row tiles) of the similarity block (rank, q); each unordered rank pair's
// block is computed once across the group (see parallel/symmetric.py for the assignment).
struct SymJob {
  int q, m0, m1, k0, k1;
};
// Own-block upper triangle (as build_fwd_tiles) followed by the kTileCross tiles of `jobs`
// grouped by chunk of the partners' row tiles (chunk c = tiles [rt*c/n, rt*(c+1)/n)), each
// segment in Z-order.
std::vector<int4> build_sym_fwd_tiles(const Geometry& g, const std::vector<SymJob>& jobs, int nchunks = 1);
// The assignment itself (parallel/symmetric.py sym_jobs / sym_incoming / sym_num_chunks): the
// blocks rank `rank` computes, and the other ranks' jobs that involve its rows (q = the
// computing rank there). Rows travel in sym_num_chunks(row_tiles) chunks of row tiles.
std::vector<SymJob> sym_jobs(int world, int rank, int row_tiles);
std::vector<SymJob> sym_incoming(int world, int rank, int row_tiles);
int sym_num_chunks(int row_tiles);
// Symmetric mode's compact coefficient buffer: a rank writes only the column blocks at distance
// 0 .. W/2 from itself (its own block, the full partner blocks, the split block), so cbuf holds
// [row_tiles][sym_c_ld(g)] tiles with global column tile nt at column slot (nt - rank * row_tiles)
// mod col_tiles: min(W, W/2 + 1) blocks instead of W (5 of 8 at W = 8).
int sym_c_ld(const Geometry& g);

// Forward tiles (ti, tj_global, kind, 0). Own-rank block: upper triangle only, listed
// first (count_own_fwd_tiles of them) so they can run while the remote rows are gathered; its
// last own_diag_tail(g) entries are the diagonal tiles (kTileDiag).
std::vector<int4> build_fwd_tiles(const Geometry& g);
int count_own_fwd_tiles(const Geometry& g);
int own_diag_tail(const Geometry& g);
// dZ tiles (ti, tn, 0, 0): the persistent stream-K schedule balances K itself (no split-K).
std::vector<int4> build_dz_tiles(const Geometry& g);

// Persistent stream-K schedule of the similarity GEMMs: `grid` blocks first process
// `dp_tiles` whole tiles in rounds, then split the K-steps of the remaining `sk_tiles` tiles
// evenly (`ipb` steps per block); a split tile is reduced and finished deterministically by
// its last-arriving block. This removes the tile-count quantisation of a plain one-block-per-
// tile launch (e.g. 528 forward tiles on 256 CUs would need 3 rounds instead of 2.06).
struct GemmSchedule {
  int grid = 0, nk = 0, dp_tiles = 0, sk_tiles = 0;
  long long ipb = 0;
};
GemmSchedule make_schedule(int ntiles, int nk, int num_cus);

// Scratch of one similarity-GEMM launch: arrival counters + 2 fp32 partial tiles per block.
// Must be ZERO when first used; every launch leaves the counters zero again, so one
// workspace serves any number of stream-ordered launches (no per-launch memset).
struct GemmWorkspace {
  void* ptr = nullptr;
  size_t bytes = 0;
  int num_cus = 256;    // sizes the counter region and the slabs (the device's CU count)
  // Grid cap of the persistent schedule (0: num_cus), set per launch. A GEMM launched while an
  // RCCL transfer is in flight leaves num_cus - sched_cus CUs free for the communication kernels:
  // the persistent blocks (128 KiB LDS, the whole register file) would otherwise hold every CU
  // until the GEMM ends and the "overlapped" transfer would start only then.
  int sched_cus = 0;
};
size_t gemm_workspace_bytes(int ntiles, int num_cus);

// ---- device-side launchers (all asynchronous on `stream`, no host syncs, no mallocs:
//      safe under hipGraph capture) -----------------------------------------------------

// Row L2-normalisation prologue: inv[i] = 1/max(||h_i||, 1e-12); zq = h*inv (compute
// dtype, zero padded to dim_k); ypos[i] = <zq_i, zq_p(i)> * inv_temp * log2(e).
// Pad rows [R, Rpad) of zq are zeroed.
// zq8 (optional): also write the fp8 copy Zq8[Rpad][ld_k8] = e4m3(z * 256) for an fp8 forward;
// ypos is then computed from the dequantised fp8 rows.
void launch_prep(DType in, DType comp, const void* h, void* zq, float* inv, float* ypos,
                 const Geometry& g, hipStream_t stream, void* zq8 = nullptr);

// out[i] = sum over k = 0 .. n-1 (in order) of in[k * count + i].
void launch_sum_slabs(const float* in, int n, size_t count, float* out, hipStream_t stream);

// zqt[e][j] = zq[j][e] (zero for e >= dim_k). zqt is [dim_n][Rpad].
void launch_transpose(DType comp, const void* zq, void* zqt, const Geometry& g,
                      hipStream_t stream);

// Column-block view for the ring-negatives mode (O(local) memory): the B operand rows of the
// global column tiles [b_tile0, b_tile0 + row_tiles) live in a one-rank chunk, and the
// coefficient tiles are written to a compact buffer with c_ld tiles per row starting at
// global column tile c_tile0. Defaults (c_ld = 0 -> col_tiles) are the all-gather layout.
struct BlockView {
  int b_tile0 = 0;
  int c_ld = 0;
  int c_tile0 = 0;
};

// Forward similarity GEMM: tiles of S = zq_local * zq_all^T with the per-row (max, sum)
// partials epilogue written to part[col_tile][Rpad] (log2 domain). If `sc` is non-null the
// cosine tile is kept (compute dtype, fragment order) for the backward.
// part_x (symmetric mode, kTileCross tiles): column partials for the partner's rows,
// part_x[(q * row_tiles + mt) * Rpad + (nt % row_tiles) * 256 + c] with q = nt / row_tiles,
// i.e. rank q's part slots [rank*row_tiles + mt] for its rows.
// diag_tail: the last `diag_tail` entries of `tiles` are kTileDiag tiles (own_diag_tail(g) for
// a launch that ends with the own block, else 0). When the persistent GEMM's tile count leaves a
// remainder of at most that many tiles after its whole rounds, the remainder runs as upper 64x64
// regions in a second, short launch (diag_up_kernel) instead of a third round or a stream-K
// split (528 forward tiles at B = 4096/view: 2 rounds + 16 diagonal tiles instead of ~2.9 rounds).
// Raw-operand forward (single process, 2-byte input rows, kept cosines): the forward GEMM reads
// the input rows h themselves (their own dtype: bf16 input -> bf16 MFMA operands, exact; fp16 ->
// fp16) and normalises in its epilogue (cos = acc inv_i inv_j), the LSE launch transposes h * inv
// into Z^T, and the row prologue only computes inv and the positive logits (launch_prep with
// zq = null): no zq rows are written or read (prep 32 MiB lighter at the headline).
// zqt (optional): launch_fwd_stats writes Z^T = (h inv)^T there itself when the launch has a
// diagonal remainder (side blocks of diag_up_kernel, which is load-latency-bound on one block per
// CU) and returns true; the LSE launch then only merges. Otherwise launch_lse transposes.
struct RawRows {
  const void* h = nullptr;      // [rows][dim] input rows
  DType in = DType::BF16;       // their dtype (F16 or BF16)
  const float* inv = nullptr;   // [rows] 1 / |h_i|
  void* zqt = nullptr;          // [dim_n][ld_t] Z^T in `zt` (the plan's backward dtype), or null
  DType zt = DType::F16;
  // Optional: the LSE launch's outputs (launch_lse's arguments). When set and the diagonal
  // remainder is exactly the second half's diagonal tiles (with Z^T beside it), the remainder
  // launch computes them itself (LseFold) and sets lse_folded: the caller then skips launch_lse.
  const float* ypos = nullptr;
  float* lse2 = nullptr;
  float* cpos = nullptr;
  float* block_loss = nullptr;
  float* loss = nullptr;
  float2* fold_pre = nullptr;   // [Rpad] scratch of the folded LSE (pre-merged row states)
  int* fold_cnt = nullptr;      // [Rpad / 64] zeroed counters (self-cleaning)
  mutable bool lse_folded = false;
};
void set_lse_fold(bool on);  // default: NTXENT_LSE_FOLD (unset: on)
bool lse_fold_enabled();
bool raw_forward_eligible(const Geometry& g, DType in, DType comp);  // world 1, 2-byte in & comp, rows % 256, dim % 64
void set_raw_forward(bool on);  // default on (off: the zq path, for A/B and tests)
bool raw_forward_enabled();
// Returns true when it wrote raw->zqt.
bool launch_fwd_stats(DType comp, const void* zq_local, const void* zq_all,
                      const int4* tiles, int ntiles, float2* part, void* sc,
                      const GemmWorkspace& ws, const Geometry& g, hipStream_t stream,
                      const BlockView& bv = BlockView{}, float2* part_x = nullptr,
                      int diag_tail = 0, hipEvent_t main_done = nullptr, const RawRows* raw = nullptr);
// main_done (optional): recorded on `stream` right after the persistent GEMM, before the remainder.
// Split-K for own-block launches with fewer tiles than CUs and long K (BASELINE config 4): K
// pieces of every tile publish partial slabs and a second launch sums them and runs the
// epilogue in strips; fwd_splitk_pieces = pieces per tile (0: the stream-K schedule).
int fwd_splitk_pieces(int ntiles, int nk, int cus, int diag_tail);
// Diagonal-remainder tiles of a launch (0: none, the stream-K schedule splits the remainder):
// the tiles left after whole rounds on `cus` CUs when they are all diagonal tiles (ntiles % cus
// <= diag_tail), for 2-byte / fp32 plans with >= 4 K-steps per tile.
int fwd_diag_remainder(int ntiles, int nk_tile, int cus, int diag_tail, bool f8);
// Small-problem path (on by default; off = the large-problem pipeline for every shape) and its
// backward column splits (0 = small_bwd_splits). Test hooks: process-wide.
void set_small_path(bool on);
bool small_path_enabled();
void set_small_splits(int n);
int small_splits_override();

// Merge the negatives-only partials per positive pair -> lse2 = logaddexp2(lse_neg, ypos)
// into lse2_all[rank*Rpad + i] and the positive coefficient cpos[i] = C_i,p(i) =
// -(sigmoid(lse_neg_i - y) + sigmoid(lse_neg_p - y)) (well conditioned when P_ip -> 1).
// loss_sum[0] receives sum_i softplus(lse_neg_i - y_i) / (W*R) over this rank's rows
// (all-reduce SUM across ranks gives the loss). `block_loss` is scratch of
// lse_scratch_floats(g) floats that must be ZERO when first used (the kernel leaves it
// reusable: its arrival counter returns to zero).
int lse_scratch_floats(const Geometry& g);
// zq / zqt (optional, rank-local [Rpad, ld_k] rows in tr_dtype): the same launch also writes the
// transpose zqt = zq^T (launch_transpose) from extra blocks that run beside the merge.
//
// fp8 backward (FP8 plans, set_fp8_backward; world 1, kept cosines): the coefficient matrix and
// Z^T go to the dZ GEMM as e4m3. C row i is scaled by 2^q8_row_exp(mneg2_i, lmin) (a bound on
// its negatives from the LSE pass; the positive C_ip is excluded and added exactly in the dZ
// epilogue), Z^T by 256. Q8Stats carries the LSE pass's extra outputs: mneg2 [Rpad] (a bound on
// each row's largest negative logit, log2 units: max over the column tiles of m + log2 s, within
// log2(256) of it), lmin [1] (the smallest LSE), and zq8t [dim_n][q8_ldt]
// bytes = e4m3(256 zq^T) written instead of zqt (zq: fp16 rows).
void set_fp8_backward(bool on);  // default on (gradient within bf16 rounding of the fp16 backward's)
bool fp8_backward_enabled();
bool fp8_backward_eligible(const Geometry& g, DType comp);  // FP8 plan, world 1, dim % 8 == 0
int q8_ldt(const Geometry& g);                               // row stride of zq8t (bytes): Rpad, padded
struct Q8Stats {
  float* mneg2 = nullptr;
  float* lmin = nullptr;
  void* zq8t = nullptr;
  const void* zq = nullptr;  // fp16 rows (the dZ epilogue's positive term C_ip z_p)
};
// raw (raw-operand forward): the transpose reads raw->h and writes Z^T = (h * inv)^T in tr_dtype.
void launch_lse(const float2* part, const float* ypos, float* lse2_all, float* cpos,
                float* block_loss, float* loss_sum, const Geometry& g, hipStream_t stream,
                DType tr_dtype = DType::F16, const void* zq = nullptr, void* zqt = nullptr,
                const Q8Stats* q8 = nullptr, const RawRows* raw = nullptr);

// Kept cosine tiles `sbuf` ([n_fwd_tiles][256*256], fragment order) -> coefficient tiles
// `cbuf` ([row_tiles][col_tiles][256*256], row-major per tile) with C = P + P^T - 2 I_pos;
// upper-triangular tiles of the own-rank block are mirrored; the positive entry is cpos[i].
// mbuf (symmetric mode): cbuf is the compact [row_tiles][sym_c_ld(g)] layout (see sym_c_ld), and
// the mirrored coefficient tiles of kTileCross tiles go to mbuf, [slots][row_tiles][row_tiles]
// tiles with slot = (q - rank - 1) mod W (partners rank+1, rank+2, ... in order): tile (mt, nt)
// lands transposed at mbuf tile (slot, nt % row_tiles, mt), i.e. the block C_{q,rank} that
// multiplies this rank's rows in rank q's gradient; consecutive slots stack into one tall A.
// dotp (optional, [dot_slots(g)][Rpad] floats, slot-major): partials of dot_i = sum_j C_ij cos_ij, the
// z_i . g_i of the normalisation backward, for the fused dZ epilogue (NormFuse); every slot is
// written (all-gather layout, own-block tiles + remote tiles of the plan).
int dot_slots(const Geometry& g);
// q8 (fp8 backward): cbuf receives e4m3 tiles (1 byte per element, same tile layout, mirrored
// own-block tiles written: launch_dz reads them), scaled per row as Q8Stats says; dotp then holds
// the partials of the dequantised coefficients (plus the exact positive term).
void launch_coef(DType comp, const void* sbuf, void* cbuf, const float* lse2_all, const float* cpos,
                 const int4* tiles, int ntiles, const Geometry& g, hipStream_t stream,
                 void* mbuf = nullptr, float* dotp = nullptr, const Q8Stats* q8 = nullptr, bool half_c = false);
// half_c: write only the upper coefficient tiles (an off-diagonal tile's mirror is skipped; the
// dZ launched with half_c reads C_IJ, J < I, as C_JI^T). Only with dz_half_c_eligible.
// dot[Rpad] = row sums of dotp.
void launch_dot_reduce(const float* dotp, float* dot, const Geometry& g, hipStream_t stream);

// Recompute variant (no stored cosines): GEMM S tiles again and emit C tiles into `cbuf`.
void launch_coef_gemm(DType comp, const void* zq_local, const void* zq_all, void* cbuf,
                      const float* lse2_all, const float* cpos, const int4* tiles, int ntiles,
                      const GemmWorkspace& ws, const Geometry& g, hipStream_t stream,
                      const BlockView& bv = BlockView{}, float* dotp = nullptr);

// dZ[Rpad][dim_n] = C * Z (fp32), C = the coefficient buffer, zqt_all = [W][dim_n][Rpad]
// (all-gathered ZqT blocks); tiles from build_dz_tiles(g).
// out_f16: write dZ as fp16 (the reduced-precision plans: half the bytes of the dZ store and of
// the normalisation backward's read; |dZ| <= ~4, fp16 keeps 11 bits against the bf16/fp16 dh).
// Fused normalisation backward of the dZ GEMM's epilogue: dh = grad_out/(2N tau) inv (g - z dot)
// computed per tile from the fp16-staged g, h, inv and dot; the dZ slab is not written. The
// launchers return whether they fused (not for fp32 plans or d % 8 != 0: then the slab is
// written and launch_norm_bwd runs).
// dot: the reduced z_i . g_i (launch_dot_reduce). (Summing the coefficient pass's slots in every
// dZ tile's epilogue measured slower: dZ +4.6 / +6.3 / +10 us at the headline / config 4 /
// config 5 against the 5-6 us launch it removes, profiles/r5/variants_dotfold.)
// dot_cnt (with dotp = the coefficient pass's slots; only where dz_dot_fold_eligible): the dZ grid
// reduces dotp into dot itself instead, each block its 1/G share of the rows before its first
// item, published through dot_cnt[0] (sc1 stores, one count per block); the epilogues read dot a
// main loop later (split-K pieces: the reduce launch does). dot_cnt: 2 ints, zero before the
// first use (self-cleaning).
struct NormFuse {
  const void* h = nullptr;
  DType in = DType::BF16;
  const float* inv = nullptr;
  const float* dot = nullptr;
  const float* grad_out = nullptr;  // device scalar
  void* dh = nullptr;
  const float* dotp = nullptr;      // dot fold: the slots
  int* dot_cnt = nullptr;           // dot fold: counters (non-null: fold)
};
// comp = FP8 with q8: the fp8 backward's dZ (cbuf = e4m3 C tiles, zqt_all = Q8Stats::zq8t;
// block-scaled MFMA, per-row dequantisation and the exact positive term in the epilogue).
bool launch_dz(DType comp, const void* cbuf, const void* zqt_all, const int4* tiles, int ntiles,
               void* dz, const GemmWorkspace& ws, const Geometry& g, hipStream_t stream, bool out_f16 = false,
               const NormFuse* nf = nullptr, const Q8Stats* q8 = nullptr, const float* cpos = nullptr,
               bool half_c = false);
// Half C (SimParams::c_half): the coefficient pass writes the upper tiles only and the dZ stages a
// lower K tile C_IJ (J < I) from C_JI through a transposing LDS image (ds_read_b64_tr_b16, one
// lane base per wave). Needs a 16-bit backward, one rank and whole-tile dZ items (the schedule of
// launch_dz: no split-K, no stream-K remainder). (Round 3's dz_sym also read Z through transposed
// LDS reads, 33 us slower at the headline, ~10 us of it the mirrored A K-steps: profiles/r3/dzexp.)
bool dz_half_c_eligible(DType comp, const Geometry& g, int n_dz, const GemmWorkspace& ws);
void set_half_c(bool on);  // default: NTXENT_HALF_C (unset: on)
bool half_c_enabled();
// NormFuse::dot_cnt allowed: a 16-bit fused dZ, fold enabled.
bool dz_dot_fold_eligible(DType comp, const Geometry& g, int n_dz, const GemmWorkspace& ws);
void set_dot_fold(bool on);  // default: NTXENT_DOT_FOLD (unset: on)
bool dot_fold_enabled();
void set_dot_fold_spin(int polls);  // test hook: 0 forces the epilogues' fallback sum
int dot_fold_spin();

// Sub-block dZ GEMM (symmetric mode): out[rows of `tiles`] (+)= A * B over K = k_tiles * 256
// columns, A = tile-blocked coefficients starting at `a` (the tile of row panel 0 and the first
// K column; `a_panel_tiles` tiles per row panel), B = transposed rows starting at `b` (column
// offset already applied; rows ld_t apart) in K blocks of `b_kblk_cols` columns, consecutive
// blocks `b_kblk_stride` elements apart (the rank blocks of ZqT_all). accum: add into `out`.
// out_f16: write `out` as fp16 (rows ldo = dim_n elements apart), no accumulation.
void launch_dz_view(DType comp, const void* a, long long a_panel_tiles, const void* b, long long b_kblk_cols,
                    long long b_kblk_stride, int k_tiles, const int4* tiles, int ntiles, void* out, bool accum,
                    const GemmWorkspace& ws, const Geometry& g, hipStream_t stream, bool out_f16 = false);

// dh = grad_out/(2N tau) * inv * (g - z (z.g)), g = sum_ks slabs, z = h*inv (fp32).
// xslabs (optional): nx more fp16 slabs [nx][Rpad][dim_n] added to the sum (received partner
// contributions of the symmetric data-parallel mode, or the fp16 dZ of a reduced-precision plan
// and nslabs = 0 fp32 slabs).
void launch_norm_bwd(DType in, const float* slabs, int nslabs, const void* h,
                     const float* inv, const float* grad_out, void* dh, const Geometry& g,
                     hipStream_t stream, const void* xslabs = nullptr, int nx = 0);

// ---- small-problem path (kernels/small_kernels.hip) -------------------------------------
// Single-rank problems with R <= kSmallMaxRows and dim_k <= kSmallMaxDk in fp16/bf16: ONE
// forward launch (row prologue fused for R <= kSmallFuseMaxRows, else after launch_prep; 64 x 64
// MFMA tiles, in-kernel LSE merge and deterministic loss sum) and ONE backward launch (S recomputed, C formed in registers and fed straight to
// the dZ MFMA, normalisation backward fused). `scratch` (small_scratch_bytes) must be ZERO when
// first used (its arrival counters return to zero after every launch); launches sharing it must
// be stream-ordered. lse2 / arow ([small_rows_pad(g)] floats) carry the row statistics from the
// forward to the backward: LSE in log2 units and a_i = 1 - P_i,p(i).
constexpr int kSmallMaxRows = 2048;
constexpr int kSmallMaxDk = 256;
bool small_path_eligible(const Geometry& g, DType comp);
int small_bwd_splits(const Geometry& g);  // default column splits of the backward grid
int small_rows_pad(const Geometry& g);    // roundup(R, 64)
size_t small_scratch_bytes(const Geometry& g, int splits);
constexpr int kSmallFuseMaxRows = 1024;  // measured: see profiles/r3/small/
bool small_fwd_fused(const Geometry& g);  // the forward runs the row prologue itself
void set_small_fuse_rows(int rows);       // override kSmallFuseMaxRows (-1: default)
int small_fuse_rows_override();
// h: [R][dim] input (dtype `in`). Writes zq ([small_rows_pad][ld_k], compute dtype, pad rows zero)
// and inv ([R]) when small_fwd_fused(g); otherwise zq / inv / ypos are launch_prep's outputs
// (ypos ignored when fused).
void launch_small_fwd(DType in, DType comp, const void* h, void* zq, float* inv, float* ypos, float* lse2,
                      float* arow, float* loss, void* scratch, const Geometry& g, hipStream_t stream);
// splits <= 0: small_bwd_splits(g). grad_out: device fp32 scalar.
void launch_small_bwd(DType in, DType comp, const void* zq, const void* h, const float* inv, const float* lse2,
                      const float* arow, const float* grad_out, void* dh, void* scratch, const Geometry& g,
                      hipStream_t stream, int splits = 0);

// ---- device utilities (reference utils::get_optimal_block_size / check_tensor_core_support
//      at include/ntxent_kernel.cuh:80-110) ------------------------------------------------
struct DeviceInfo {
  int device = 0;
  int num_cus = 0;
  int lds_per_block = 0;
  int warp_size = 0;
  std::string arch;  // gcnArchName, e.g. "gfx950:sramecc+:xnack-"
  bool is_gfx950 = false;
};
const DeviceInfo& device_info(int device);  // cached per device
// True when the device has matrix cores usable by these kernels (gfx950 MFMA).
bool check_matrix_core_support(int device);
// Launch config a kernel family would use for `rows` rows (parity with the reference's
// get_optimal_block_size, which is undefined there: include/ntxent_kernel.cuh:92).
int get_optimal_block_size(int rows);

}  // namespace ntxent

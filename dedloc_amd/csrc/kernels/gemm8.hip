// bf16 GEMM on MFMA with LDS-DMA staging and an 8-phase K loop (the
// structure of cdna_hip_programming.md §5 "The 256² 8-phase template", written for this repo).
//
//   C[M,N] = sum_k A(m,k) B(n,k)      fp32 accumulation, v_mfma_f32_16x16x32_bf16
//
// Operand storage (template flags), as in gemm.hip:
//   K-inner : element (r, k) at p[r * ld + k]   (activations, forward weights [out][in])
//   K-outer : element (r, k) at p[k * ld + r]   (dgrad weights, wgrad operands)
//
// Tile 256 x 256 x 64, 512 threads = 8 waves as 2 (M) x 4 (N), 128 x 64 outputs per wave held as
// four 64 x 32 quadrants.  Each operand tile is staged as two half-tiles of 128 rows x 64 k (16 KiB)
// by global_load_lds (16 B per lane, two instructions per thread per half-tile, no VGPR staging):
// A half h holds the tile rows with bit 6 == h, B half h the columns with bit 5 == h, so quadrant
// (qm, qn) of every wave reads exactly half-tiles A_qm and B_qn.  The K loop runs 4 phases per K-tile,
// one quadrant each, in the order (0,0) (0,1) (1,1) (1,0):
//
//   phase: ds_read this quadrant's new fragments | issue one half-tile of prefetch (2 glds) |
//          s_barrier | 16 MFMA (setprio 1) | s_barrier
//
// Waves 4-7 run one barrier behind waves 0-3 (stagger), so on each SIMD one wave computes while its
// partner reads and prefetches.  Prefetch runs 6 half-tiles (1.5 K-tiles) ahead: each half-tile
// of the double buffer is restaged two phases after its last read — safe for the lagging group
// too — and the only vmcnt wait is a counted vmcnt(4) in the last phase of each K-tile (two
// half-tiles stay in flight across the barriers; never vmcnt(0) in steady state).  All LDS is one __shared__ array and
// every barrier is a raw s_barrier, so no compiler-inserted vmcnt(0) drains the pipeline.
//
// LDS images (bank-conflict free, checked by simulation of the gfx950 lane groups):
//   K-inner half-tile: [128 rows][8 x 16 B], chunk c of row r at c ^ ((r >> 1) & 7)  -> ds_read_b128
//   K-outer half-tile: [64 k][16 x 16 B],   chunk c of k-row k at c ^ (((k&3)<<2)|((k>>2)&3))
//                      -> ds_read_b64_tr_b16 (hardware transpose to the MFMA operand layout)
// LDS-DMA writes each 1 KiB piece lane-linearly; the swizzle is applied on the per-lane global
// source address and on the read (both sides, cdna_hip_programming.md rule 21).
//
// Epilogues (staged through LDS as fp32, 64 rows per round, written as 16-B row chunks):
//   EPI_STORE  C = acc (+ bias[n]) (+ R[m,n])                                 bf16
//   EPI_GELU   H = bf16(acc + bias); C = gelu_new(H)                          bf16 x2
//   EPI_GELUD  h = bf16(acc + bias); C = gelu_new(h), H = gelu_new'(h)        bf16 x2
//   EPI_DGELU  C = bf16(acc) * gelu_new'(R[m,n]); dbias[n] += sum_m C         bf16 (+ fp32 atomics)
//   EPI_DMUL   C = bf16(acc) * R[m,n] (R = gelu_new' stored by EPI_GELUD);   bf16 (+ fp32 atomics)
//              dbias[n] += sum_m C — the FFN backward with no transcendental in its epilogue
//   EPI_F32    Cf[z][m,n] = acc  or  += acc (reduction split z)                fp32
//   EPI_STATS  EPI_STORE, plus per-column sum and sum of squares of the stored bf16 values into
//              stats[g][0..N) / stats[g][N..2N) (fp32 atomics), g = m / stat_rows: the batch
//              statistics of a BatchNorm over this output (SwAV's 1x1 convs), so the BN forward
//              does not re-read the tensor
//   EPI_BNBWD  the data gradient dY of a BatchNorm+ReLU's output (+ R: the identity-branch
//              gradient), prepared for that BN's backward: g = bf16(acc + R) masked by the ReLU
//              (y = Y[m,n] > 0, or x*gamma*rstd + beta - mean*gamma*rstd > 0 from the BN input X),
//              stored; stats[grp][n] += g, stats[grp][N + n] += g * (X[m,n] - mean) * rstd — the
//              BN backward's two column sums, so it skips its statistics pass over dY and X
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "dl_common.h"
#include "dl_kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4_t lds_s4;
typedef __attribute__((address_space(3))) void lds_void;

enum { EPI_STORE = 0, EPI_GELU = 1, EPI_DGELU = 2, EPI_F32 = 3, EPI_STATS = 4, EPI_BNBWD = 5, EPI_GELUD = 6,
       EPI_DMUL = 7 };

constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
constexpr int HALF = 16384;     // one half-tile image
constexpr int BUF = 4 * HALF;   // slots in stage order: 0 = A0, 1 = B1, 2 = A1, 3 = B0
constexpr int SMEM = 2 * BUF;   // double buffer: 128 KiB

__device__ __forceinline__ int kin_swz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int kout_swz(int k) { return ((k & 3) << 2) | ((k >> 2) & 3); }

// Tile row / column of local index l (0..127) of half-tile h: A halves interleave 64-row blocks
// (bit 6 of the tile row), B halves 32-column blocks (bit 5), matching the waves' quadrants.
template <bool ISB>
__device__ __forceinline__ int half_to_tile(int l, int h) {
  return ISB ? ((l >> 5) << 6) + (h << 5) + (l & 31) : ((l >> 6) << 7) + (h << 6) + (l & 63);
}

// Column permutation of a K-outer B tile (swap bits 5 and 6 of the tile column).  A B half-tile
// holds the 32-column blocks with bit 5 == half (the waves' N quadrants); K-outer, a 32-column
// block of a k-row is only 64 bytes, so each half-tile DMA would fetch half cache lines (and every
// line twice, one half per phase).  Tile column c is therefore mapped to global column
// colperm(c): the blocks of one half land on two 64-column (128-byte, whole-line) runs of global
// columns.  The epilogue writes column colperm(c) for the accumulator of tile column c, so the
// permutation is invisible outside the kernel.  K-inner B tiles are not permuted (P = false).
template <bool P>
__device__ __forceinline__ int colperm(int c) {
  return P ? (c & ~0x60) | ((c >> 1) & 0x20) | ((c << 1) & 0x40) : c;
}

// One 16-byte-per-lane LDS-DMA (global_load_lds_dwordx4; M0 = the wave's LDS destination), issued
// from inline asm.  With __builtin_amdgcn_global_load_lds the compiler's wait-count pass cannot
// tell the half-tile slots apart and, in front of every ds_read_b64_tr_b16 that follows an
// in-flight DMA, inserts s_waitcnt vmcnt(0) — three full drains of the prefetch per K-tile in
// every kernel with a K-outer operand (the weight gradients ran ~30% below the K-inner forms).
// Hidden in asm, the DMAs are ordered only by the pipeline's own counted vmcnt waits; the
// compiler's waits for its own loads can only get stricter.
__device__ __forceinline__ void dma16(const bf16_t* src, uint8_t* lds_dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds_void*)lds_dst);
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m0), "v"(src) : "memory", "m0");
}

// Issue the two LDS-DMA pieces of this thread for one half-tile.
template <bool KO, bool ISB>
__device__ __forceinline__ void stage_half(const bf16_t* __restrict__ g, long ld, int r0, int rows_valid, int k0,
                                           int half, uint8_t* slot, int w, int lane) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int region = j * 8 + w;  // 1 KiB piece of the 16 KiB image
    const bf16_t* src;
    if constexpr (!KO) {
      const int lrow = region * 8 + (lane >> 3);
      const int c = (lane & 7) ^ kin_swz(lrow);
      const int trow = half_to_tile<ISB>(lrow, half);
      const int grow = min(r0 + trow, rows_valid - 1);  // M tail: clamp (rows are masked on store)
      src = g + (long)grow * ld + k0 + c * 8;
    } else {
      const int k = region * 4 + (lane >> 4);
      const int c = (lane & 15) ^ kout_swz(k);
      const int tcol = colperm<ISB>(half_to_tile<ISB>(c * 8, half));  // 8-column chunks never straddle a block
      src = g + (long)(k0 + k) * ld + r0 + tcol;
    }
    dma16(src, slot + region * 1024);
  }
}

// The per-lane global source of both LDS-DMA pieces of a half-tile at k0 = 0 (stage_half's address
// math, done once per workgroup): a K-tile's stage is then base + k offset — two 64-bit adds
// instead of ~12 VALU address instructions per piece in the K loop
template <bool KO, bool ISB>
__device__ __forceinline__ void src_base(const bf16_t* __restrict__ g, long ld, int r0, int rows_valid, int half,
                                         int w, int lane, const bf16_t* (&base)[2]) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int region = j * 8 + w;
    if constexpr (!KO) {
      const int lrow = region * 8 + (lane >> 3);
      const int c = (lane & 7) ^ kin_swz(lrow);
      const int grow = min(r0 + half_to_tile<ISB>(lrow, half), rows_valid - 1);
      base[j] = g + (long)grow * ld + c * 8;
    } else {
      const int k = region * 4 + (lane >> 4);
      const int c = (lane & 15) ^ kout_swz(k);
      base[j] = g + (long)k * ld + r0 + colperm<ISB>(half_to_tile<ISB>(c * 8, half));
    }
  }
}

__device__ __forceinline__ void stage_pre(const bf16_t* const (&base)[2], long koff, uint8_t* slot, int w) {
#pragma unroll
  for (int j = 0; j < 2; ++j) dma16(base[j] + koff, slot + (j * 8 + w) * 1024);
}

// MFMA operand fragment: 16 rows (r0..) x 32 k (k-step ks) of a half-tile image; lane l holds
// (row r0 + (l & 15), k = 32 ks + 8 (l >> 4) + j), j = 0..7.
template <bool KO>
__device__ __forceinline__ bf16x8 frag(const uint8_t* img, int r0, int ks, int lane) {
  if constexpr (!KO) {
    const int row = r0 + (lane & 15), c = 4 * ks + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + row * 128 + ((c ^ kin_swz(row)) << 4));
  } else {
    const int g = lane >> 4, i = lane & 15;
    const int kr = 32 * ks + 8 * g + (i >> 2);
    const int col = r0 + 4 * (i & 3);
    const int o1 = kr * 256 + (((col >> 3) ^ kout_swz(kr)) << 4) + ((col & 7) << 1);
    const int o2 = (kr + 4) * 256 + (((col >> 3) ^ kout_swz(kr + 4)) << 4) + ((col & 7) << 1);
    const s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + o1));
    const s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + o2));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Output tiles are written once and not re-read by this kernel: with `nt` the 16-byte stores are
// non-temporal (streamed past the L2 instead of allocating in it), which keeps the operand tiles
// of the other workgroups resident while 256 CUs flush their epilogues at once.
__device__ __forceinline__ void store8_bf16(bf16_t* dst, const float* v, bool nt = false) {
  const uint4 u = pack8_bf16(v);
  if (nt) {
    const u32x4 w = {u.x, u.y, u.z, u.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(dst));
  } else {
    *reinterpret_cast<uint4*>(dst) = u;
  }
}

struct Args {
  const bf16_t* A; long lda;
  const bf16_t* B; long ldb;
  int M, N, K;                   // K per split
  bf16_t* C; long ldc;
  float* Cf; long ldcf; long slab; int accumulate;
  const float* bias;
  const bf16_t* R; long ldr;     // residual (STORE) or pre-activation (DGELU)
  bf16_t* H; long ldh;           // pre-activation out (GELU)
  float* dbias;                  // column sums out (DGELU)
  float* stats; long stat_rows;  // EPI_STATS: [M / stat_rows][2N] column sums / sums of squares
  DlBnBwdEpi bn;                 // EPI_BNBWD operands (BN input, ReLU mask source, mean / rstd)
  int group_m;                   // tile order: column-major inside bands of group_m row blocks
};

// Tile (m0, n0) of linear tile index bid.  group_m = 1: row-major (all column tiles of one row
// block, then the next).  group_m = G: bands of G row blocks walked column by column, so the 32
// consecutive tiles one XCD runs at a time cover ~G row blocks x 32/G column blocks instead of
// ~2.7 x 12 (QKV): fewer distinct operand panels per L2 (e.g. 6 MiB instead of 7.3 for QKV's
// 3072-column weight, which does not fit one XCD's 4 MiB L2).
__device__ __forceinline__ void tile_of(int bid, int tiles_m, int tiles_n, int G, int& m0, int& n0) {
  const int band = G * tiles_n;
  const int first = (bid / band) * G;
  const int gsz = min(tiles_m - first, G);
  const int r = bid % band;
  m0 = (first + r % gsz) * BM;
  n0 = (r / gsz) * BN;
}

#define DL_MFMA_QUAD_B(QM, QN, BF)                                                    \
  do {                                                                                \
    __builtin_amdgcn_s_setprio(1);                                                    \
    _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                  \
      _Pragma("unroll") for (int mi = 0; mi < 4; ++mi)                                \
        _Pragma("unroll") for (int ni = 0; ni < 2; ++ni)                              \
          acc[QM][QN][mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(              \
              af[mi][ks], BF[ni][ks], acc[QM][QN][mi][ni], 0, 0, 0);                  \
    __builtin_amdgcn_s_setprio(0);                                                    \
  } while (0)
#define DL_MFMA_QUAD(QM, QN) DL_MFMA_QUAD_B(QM, QN, bfr)

// The B0 fragments read in phase 0 stay in registers for phase 3 (16 more VGPRs) instead of being
// read again — 24 instead of 28 KiB of LDS reads per wave and K-tile, and phase 3 issues no LDS
// reads at all.
// PRESRC: DMA source addresses from per-lane bases computed once (src_base / stage_pre)
template <bool AKO, bool BKO, int EPI, bool PRESRC>
__global__ __launch_bounds__(NT, 2) void gemm8_kernel(Args p) {
  // EPI_BNBWD: + [4][256] fp32 BatchNorm coefficients of the tile's columns (read per pass from LDS
  // instead of holding 32 registers, which pay for reading the BN input one pass ahead)
  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM + (EPI == EPI_BNBWD ? 4096 : 0)];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 2, wn = w & 3;
  const int tiles_n = p.N / BN;
  const int tiles_m = (p.M + BM - 1) / BM;
  // one linear grid over (split, tile), remapped so that each XCD runs whole splits: the
  // workgroups sharing an XCD's L2 then read the same token range (weight gradients: every tile of
  // a split reads the same rows of both operands), so each operand byte comes from HBM about once
  // instead of once per XCD
  const int tiles = tiles_m * tiles_n;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);  // grid = tiles * splits
  const int split = lid / tiles, bid = lid % tiles;
  int m0, n0;
  tile_of(bid, tiles_m, tiles_n, p.group_m, m0, n0);
  const int kbase = split * p.K;
  const int nk = p.K / BK;

  floatx4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int d = 0; d < 2; ++d) acc[a][b][c][d] = floatx4{0.f, 0.f, 0.f, 0.f};

  const bf16_t* bA0[2];
  const bf16_t* bA1[2];
  const bf16_t* bB0[2];
  const bf16_t* bB1[2];
  if constexpr (PRESRC) {
    src_base<AKO, false>(p.A, p.lda, m0, p.M, 0, w, lane, bA0);
    src_base<AKO, false>(p.A, p.lda, m0, p.M, 1, w, lane, bA1);
    src_base<BKO, true>(p.B, p.ldb, n0, p.N, 0, w, lane, bB0);
    src_base<BKO, true>(p.B, p.ldb, n0, p.N, 1, w, lane, bB1);
  }
  // half-tile h = 4 t + k of the stream: k = 0 A0, 1 B1, 2 A1, 3 B0 -> slot k of buffer t & 1
#define DL_STAGE(T, KSLOT)                                                                          \
  do {                                                                                              \
    uint8_t* slot_ = smem + ((T) & 1) * BUF + (KSLOT) * HALF;                                       \
    const int k0_ = kbase + (T) * BK;                                                               \
    if constexpr (PRESRC) {                                                                         \
      const long ka_ = AKO ? (long)k0_ * p.lda : (long)k0_, kb_ = BKO ? (long)k0_ * p.ldb : (long)k0_; \
      if ((KSLOT) == 0) stage_pre(bA0, ka_, slot_, w);                                              \
      else if ((KSLOT) == 1) stage_pre(bB1, kb_, slot_, w);                                         \
      else if ((KSLOT) == 2) stage_pre(bA1, ka_, slot_, w);                                         \
      else stage_pre(bB0, kb_, slot_, w);                                                           \
    } else {                                                                                        \
      if ((KSLOT) == 0) stage_half<AKO, false>(p.A, p.lda, m0, p.M, k0_, 0, slot_, w, lane);        \
      else if ((KSLOT) == 1) stage_half<BKO, true>(p.B, p.ldb, n0, p.N, k0_, 1, slot_, w, lane);    \
      else if ((KSLOT) == 2) stage_half<AKO, false>(p.A, p.lda, m0, p.M, k0_, 1, slot_, w, lane);   \
      else stage_half<BKO, true>(p.B, p.ldb, n0, p.N, k0_, 0, slot_, w, lane);                      \
    }                                                                                               \
  } while (0)

  // prologue: tile 0 and the first two half-tiles (A0, B1) of tile 1
  DL_STAGE(0, 0); DL_STAGE(0, 1); DL_STAGE(0, 2); DL_STAGE(0, 3);
  if (nk > 1) {
    DL_STAGE(1, 0); DL_STAGE(1, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  // Stagger (cdna_hip_programming.md §5 template, MI355X_MICROARCH.md "Two waves per SIMD"): waves
  // 4-7 (the M half wm = 1; wave w and w + 4 share a SIMD) run one barrier behind waves 0-3, so on
  // every SIMD one wave issues its 16 MFMAs while its partner reads fragments and issues the
  // prefetch.  Every half-tile is restaged two phases after its last read, so even the lagging
  // group's reads (retired by the lgkmcnt wait in front of its MFMAs) are done before the leading
  // group's LDS-DMA into that region is issued.
  if (wm == 1) __builtin_amdgcn_s_barrier();
  const int ra = wm * 64;  // this wave's rows inside an A half-tile image
  const int cb = wn * 32;  // this wave's columns inside a B half-tile image
  bf16x8 af[4][2], bfr[2][2], bf0[2][2];
  // One K-tile; M1 / M2: K-tiles t+1 / t+2 exist (prefetch them).  PRESRC peels the last two K-tiles
  // so the steady-state loop carries no prefetch conditions (no scalar compare/branch pairs around
  // the DMAs); otherwise the flags are run-time.
  auto ktile = [&](int t, auto m1, auto m2) {
    constexpr bool M1 = decltype(m1)::value, M2 = decltype(m2)::value;
    const uint8_t* buf = smem + (t & 1) * BUF;
    const uint8_t* iA0 = buf;
    const uint8_t* iB1 = buf + HALF;
    const uint8_t* iA1 = buf + 2 * HALF;
    const uint8_t* iB0 = buf + 3 * HALF;

    // ---- phase 0: quadrant (0,0); prefetch A1 of tile t+1
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) bf0[ni][ks] = frag<BKO>(iB0, cb + ni * 16, ks, lane);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi][ks] = frag<AKO>(iA0, ra + mi * 16, ks, lane);
    if constexpr (M1) DL_STAGE(t + 1, 2);
    __builtin_amdgcn_s_barrier();
    DL_MFMA_QUAD_B(0, 0, bf0);
    __builtin_amdgcn_s_barrier();

    // ---- phase 1: quadrant (0,1); prefetch B0 of tile t+1
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) bfr[ni][ks] = frag<BKO>(iB1, cb + ni * 16, ks, lane);
    if constexpr (M1) DL_STAGE(t + 1, 3);
    __builtin_amdgcn_s_barrier();
    DL_MFMA_QUAD(0, 1);
    __builtin_amdgcn_s_barrier();

    // ---- phase 2: quadrant (1,1); prefetch A0 of tile t+2
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi][ks] = frag<AKO>(iA1, ra + mi * 16, ks, lane);
    if constexpr (M2) DL_STAGE(t + 2, 0);
    __builtin_amdgcn_s_barrier();
    DL_MFMA_QUAD(1, 1);
    __builtin_amdgcn_s_barrier();

    // ---- phase 3: quadrant (1,0); prefetch B1 of tile t+2; retire tile t+1
    if constexpr (M2) {
      DL_STAGE(t + 2, 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    DL_MFMA_QUAD_B(1, 0, bf0);
    __builtin_amdgcn_s_barrier();
    };
  if constexpr (PRESRC) {
    for (int t = 0; t < nk - 2; ++t) ktile(t, std::true_type{}, std::true_type{});
    if (nk >= 2) ktile(nk - 2, std::true_type{}, std::false_type{});
    ktile(nk - 1, std::false_type{}, std::false_type{});
  } else {
    for (int t = 0; t < nk; ++t) {
      const uint8_t* buf = smem + (t & 1) * BUF;
      const uint8_t* iA0 = buf;
      const uint8_t* iB1 = buf + HALF;
      const uint8_t* iA1 = buf + 2 * HALF;
      const uint8_t* iB0 = buf + 3 * HALF;
      const bool more1 = t + 1 < nk, more2 = t + 2 < nk;

    // ---- phase 0: quadrant (0,0); prefetch A1 of tile t+1
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) bf0[ni][ks] = frag<BKO>(iB0, cb + ni * 16, ks, lane);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi][ks] = frag<AKO>(iA0, ra + mi * 16, ks, lane);
    if (more1) DL_STAGE(t + 1, 2);
    __builtin_amdgcn_s_barrier();
    DL_MFMA_QUAD_B(0, 0, bf0);
    __builtin_amdgcn_s_barrier();

    // ---- phase 1: quadrant (0,1); prefetch B0 of tile t+1
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) bfr[ni][ks] = frag<BKO>(iB1, cb + ni * 16, ks, lane);
    if (more1) DL_STAGE(t + 1, 3);
    __builtin_amdgcn_s_barrier();
    DL_MFMA_QUAD(0, 1);
    __builtin_amdgcn_s_barrier();

    // ---- phase 2: quadrant (1,1); prefetch A0 of tile t+2
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi][ks] = frag<AKO>(iA1, ra + mi * 16, ks, lane);
    if (more2) DL_STAGE(t + 2, 0);
    __builtin_amdgcn_s_barrier();
    DL_MFMA_QUAD(1, 1);
    __builtin_amdgcn_s_barrier();

    // ---- phase 3: quadrant (1,0); prefetch B1 of tile t+2; retire tile t+1
    if (more2) {
      DL_STAGE(t + 2, 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    DL_MFMA_QUAD_B(1, 0, bf0);
    __builtin_amdgcn_s_barrier();
      }
  }
#undef DL_STAGE
  if (wm == 0) __builtin_amdgcn_s_barrier();  // balance the stagger: every wave passes the same barriers
  float* const bnt = reinterpret_cast<float*>(smem + SMEM);  // EPI_BNBWD: [brs | bxh | bsc | bsh][256]
  if constexpr (EPI == EPI_BNBWD) {
    if (threadIdx.x < BN) {  // tile column t -> global column n0 + colperm(t)
      const int t = threadIdx.x, c = n0 + colperm<BKO>(t);
      const long go = (long)(m0 / p.stat_rows) * p.N;
      const float mu = p.bn.mean[go + c], rs = p.bn.rstd[go + c];
      const float sc = p.bn.Y ? 0.f : p.bn.gamma[c] * rs;
      bnt[t] = rs;
      bnt[BN + t] = -mu * rs;  // xhat = x * rstd + bxh
      bnt[2 * BN + t] = sc;
      bnt[3 * BN + t] = p.bn.Y ? 0.f : p.bn.beta[c] - mu * sc;
    }
  }
  __builtin_amdgcn_s_barrier();               // all fragment reads done before the epilogue reuses LDS

  // ---------------------------------------------------------------- epilogue
  // Each wave stages 64 x 64 fp32 per round (quadrant row qm) in its own 16 KiB LDS region:
  // row r at r * 256 B, 16-B chunk q of it at q ^ (r & 1) (conflict-free row reads).
  uint8_t* ep = smem + w * 16384;
  const int crow = 4 * (lane >> 4), ccol = lane & 15;
  float bias_v[2][2];
#pragma unroll
  for (int qn = 0; qn < 2; ++qn)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      bias_v[qn][ni] = 0.f;
      if constexpr (EPI == EPI_STORE || EPI == EPI_GELU || EPI == EPI_GELUD || EPI == EPI_STATS)
        if (p.bias) bias_v[qn][ni] = p.bias[n0 + colperm<BKO>(wn * 64 + qn * 32 + ni * 16 + ccol)];
    }
  float colsum[8], colsq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) colsum[j] = colsq[j] = 0.f;
  const int rch = lane & 7;   // 8-column chunk handled in the row phase
  const int rr = lane >> 3;   // row within a pass of 8 rows
  const int gn = n0 + colperm<BKO>(wn * 64 + rch * 8);
  // Rows m0 + wm * 128 + qm * 64 + pass * 8 + rr: every global address is a per-lane base (row
  // rbase, column gn, computed once) plus a wave-uniform row offset (scalar multiply), and the row
  // bound is tested only in a tail tile (the per-pass 64-bit multiplies and exec-masked row checks
  // were ~15% of the epilogue's VALU).
  const int rbase = m0 + wm * 128 + rr;
  const bool full = m0 + BM <= p.M;

  const int tc8 = wn * 64 + rch * 8;  // EPI_BNBWD: this lane's 8 tile columns in bnt

  // HR: a residual / pre-activation operand R is read.  Its rows are read ahead: all 8 of a row half
  // before its passes, and the next half's row j right after pass j consumed this half's — ahead of
  // that pass's store.  Loaded inside each pass instead, every pass waited (vmcnt(0)) for its load's
  // full HBM latency and, the counter being in issue order, for every store before it.  Whether R is
  // present is a template flag of the pass loop (a run-time flag turned every add into a select).
  // per-lane row-rbase pointers of every operand the epilogue touches
  bf16_t* const cb0 = EPI == EPI_F32 ? nullptr : p.C + (long)rbase * p.ldc + gn;
  bf16_t* const hb0 = (EPI == EPI_GELU || EPI == EPI_GELUD) ? p.H + (long)rbase * p.ldh + gn : nullptr;
  float* const fb0 = EPI == EPI_F32 ? p.Cf + (long)split * p.slab + (long)rbase * p.ldcf + gn : nullptr;
  // HY (EPI_BNBWD): the ReLU mask comes from the BN output Y (a residual branch) instead of from X
  auto run = [&](auto hr_tag, auto hy_tag) {
    constexpr bool HR = decltype(hr_tag)::value, HY = decltype(hy_tag)::value;
    const bf16_t* rb0 = HR ? p.R + (long)rbase * p.ldr + gn : nullptr;
    auto rrow = [&](int qm, int pass) -> uint4 {
      const int off = qm * 64 + pass * 8;
      const bf16_t* src = rb0 + (long)off * p.ldr;
      if (!full) src = p.R + (long)min(rbase + off, p.M - 1) * p.ldr + gn;  // tail rows: clamped, unused
      return *reinterpret_cast<const uint4*>(src);
    };
    uint4 rbuf[8];
    if constexpr (HR) {
#pragma unroll
      for (int pass = 0; pass < 8; ++pass) rbuf[pass] = rrow(0, pass);
    }
    // EPI_BNBWD: the BN input (and output) rows are read one pass ahead
    auto xoff = [&](int k) {  // pass k of the 16 (qm = k / 8)
      int row = rbase + (k >> 3) * 64 + (k & 7) * 8;
      if (!full) row = min(row, p.M - 1);
      return (long)row * p.bn.ldx + gn;
    };
    uint4 xq, yq;
    if constexpr (EPI == EPI_BNBWD) {
      xq = *reinterpret_cast<const uint4*>(p.bn.X + xoff(0));
      if constexpr (HY) yq = *reinterpret_cast<const uint4*>(p.bn.Y + xoff(0));
    }
#pragma unroll
    for (int qm = 0; qm < 2; ++qm) {
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int r = mi * 16 + crow + i;
              const int c = qn * 32 + ni * 16 + ccol;
              const int q = (c >> 2) ^ (r & 1);
              *reinterpret_cast<float*>(ep + r * 256 + q * 16 + (c & 3) * 4) =
                  acc[qm][qn][mi][ni][i] + bias_v[qn][ni];
            }
#pragma unroll
      for (int pass = 0; pass < 8; ++pass) {
        const int r = pass * 8 + rr;
        const float4 lo = *reinterpret_cast<const float4*>(ep + r * 256 + (((2 * rch) ^ (r & 1)) << 4));
        const float4 hi = *reinterpret_cast<const float4*>(ep + r * 256 + (((2 * rch + 1) ^ (r & 1)) << 4));
        float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        const int off = qm * 64 + pass * 8;  // wave-uniform
        float rv[8];
        if constexpr (HR) {
          unpack8_bf16(rbuf[pass], rv);
          if (qm == 0) rbuf[pass] = rrow(1, pass);
        }
        if (full || rbase + off < p.M) {
          if constexpr (EPI == EPI_STORE) {
            if constexpr (HR) {
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] += rv[j];
            }
            store8_bf16(cb0 + (long)off * p.ldc, v, true);
          } else if constexpr (EPI == EPI_STATS) {
            if constexpr (HR) {
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] += rv[j];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              v[j] = round_bf16(v[j]);
              colsum[j] += v[j];
              colsq[j] = fmaf(v[j], v[j], colsq[j]);
            }
            store8_bf16(cb0 + (long)off * p.ldc, v, true);
          } else if constexpr (EPI == EPI_BNBWD) {
            float xv[8], yv[8], brs[8], bmu[8], bsc[8], bsh[8];
            unpack8_bf16(xq, xv);
            if constexpr (HY) unpack8_bf16(yq, yv);
            const int kn = qm * 8 + pass + 1;
            if (kn < 16) {
              xq = *reinterpret_cast<const uint4*>(p.bn.X + xoff(kn));
              if constexpr (HY) yq = *reinterpret_cast<const uint4*>(p.bn.Y + xoff(kn));
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const float4 a = *reinterpret_cast<const float4*>(bnt + tc8 + 4 * h);
              const float4 b = *reinterpret_cast<const float4*>(bnt + BN + tc8 + 4 * h);
              brs[4 * h] = a.x; brs[4 * h + 1] = a.y; brs[4 * h + 2] = a.z; brs[4 * h + 3] = a.w;
              bmu[4 * h] = b.x; bmu[4 * h + 1] = b.y; bmu[4 * h + 2] = b.z; bmu[4 * h + 3] = b.w;
              if constexpr (!HY) {
                const float4 c4 = *reinterpret_cast<const float4*>(bnt + 2 * BN + tc8 + 4 * h);
                const float4 d4 = *reinterpret_cast<const float4*>(bnt + 3 * BN + tc8 + 4 * h);
                bsc[4 * h] = c4.x; bsc[4 * h + 1] = c4.y; bsc[4 * h + 2] = c4.z; bsc[4 * h + 3] = c4.w;
                bsh[4 * h] = d4.x; bsh[4 * h + 1] = d4.y; bsh[4 * h + 2] = d4.z; bsh[4 * h + 3] = d4.w;
              }
            }
            if constexpr (HR) {
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] += rv[j];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              // xhat = (x - mean) rstd = x * brs + bxh (bxh = -mean * rstd: one FMA)
              const float xh = fmaf(xv[j], brs[j], bmu[j]);
              const bool live = HY ? yv[j] > 0.f : fmaf(xv[j], bsc[j], bsh[j]) > 0.f;
              const float g = live ? round_bf16(v[j]) : 0.f;
              v[j] = g;
              colsum[j] += g;
              colsq[j] = fmaf(g, xh, colsq[j]);
            }
            store8_bf16(cb0 + (long)off * p.ldc, v, true);
          } else if constexpr (EPI == EPI_GELU) {
            float h[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) h[j] = round_bf16(v[j]);
            store8_bf16(hb0 + (long)off * p.ldh, h, true);
#pragma unroll
            for (int j = 0; j < 8; ++j) h[j] = gelu_tanh_sig(h[j]);
            store8_bf16(cb0 + (long)off * p.ldc, h, true);
          } else if constexpr (EPI == EPI_GELUD) {
            float g[8], d[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) gelu_and_grad_sig(round_bf16(v[j]), g[j], d[j]);
            store8_bf16(hb0 + (long)off * p.ldh, d, true);
            store8_bf16(cb0 + (long)off * p.ldc, g, true);
          } else if constexpr (EPI == EPI_DGELU) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              v[j] = round_bf16(round_bf16(v[j]) * gelu_tanh_grad_sig(rv[j]));
              colsum[j] += v[j];
            }
            store8_bf16(cb0 + (long)off * p.ldc, v, true);
          } else if constexpr (EPI == EPI_DMUL) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              v[j] = round_bf16(round_bf16(v[j]) * rv[j]);
              colsum[j] += v[j];
            }
            store8_bf16(cb0 + (long)off * p.ldc, v, true);
          } else {
            float* dst = fb0 + (long)off * p.ldcf;
            if (p.accumulate) {
              const float4 o0 = *reinterpret_cast<const float4*>(dst);
              const float4 o1 = *reinterpret_cast<const float4*>(dst + 4);
              v[0] += o0.x; v[1] += o0.y; v[2] += o0.z; v[3] += o0.w;
              v[4] += o1.x; v[5] += o1.y; v[6] += o1.z; v[7] += o1.w;
            }
            *reinterpret_cast<float4*>(dst) = float4{v[0], v[1], v[2], v[3]};
            *reinterpret_cast<float4*>(dst + 4) = float4{v[4], v[5], v[6], v[7]};
          }
        }
      }
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  if constexpr (EPI == EPI_DGELU || EPI == EPI_DMUL) {
    run(T_{}, F_{});
  } else if constexpr (EPI == EPI_BNBWD) {
    if (p.R != nullptr) {
      if (p.bn.Y) run(T_{}, T_{});
      else run(T_{}, F_{});
    } else {
      if (p.bn.Y) run(F_{}, T_{});
      else run(F_{}, F_{});
    }
  } else if constexpr (EPI == EPI_STORE || EPI == EPI_STATS) {
    if (p.R != nullptr) run(T_{}, F_{});
    else run(F_{}, F_{});
  } else {
    run(F_{}, F_{});
  }
  if constexpr (EPI == EPI_DGELU || EPI == EPI_DMUL) {
    if (p.dbias) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float s = colsum[j];
        s += __shfl_xor(s, 8, 64);
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        colsum[j] = s;
      }
      if (lane < 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) atomicAdd(&p.dbias[n0 + colperm<BKO>(wn * 64 + lane * 8) + j], colsum[j]);
      }
    }
  }
  if constexpr (EPI == EPI_STATS || EPI == EPI_BNBWD) {
    // lanes with the same 8-column chunk (lane & 7) hold disjoint rows: fold them, then one atomic
    // per column and moment from lanes 0..7
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = colsum[j], q = colsq[j];
      s += __shfl_xor(s, 8, 64);
      q += __shfl_xor(q, 8, 64);
      s += __shfl_xor(s, 16, 64);
      q += __shfl_xor(q, 16, 64);
      s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 32, 64);
      colsum[j] = s;
      colsq[j] = q;
    }
    // every lane now holds its chunk's eight totals; lane l adds column (l & 7) * 8 + (l >> 3):
    // 64 distinct columns, one wave-instruction per moment (atomics are issue-bound)
    const int jl = lane >> 3;
    float s = colsum[0], q = colsq[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      s = jl == j ? colsum[j] : s;
      q = jl == j ? colsq[j] : q;
    }
    float* st = p.stats + (m0 / p.stat_rows) * 2L * p.N + n0 + colperm<BKO>(wn * 64 + rch * 8) + jl;
    atomicAdd(st, s);
    atomicAdd(st + p.N, q);
  }
}

#undef DL_MFMA_QUAD
#undef DL_MFMA_QUAD_B

// B0 fragments kept in registers for phase 3 (+1-4% per GEMM, +1.8% on the power-capped step) and
// DMA source bases computed once with the K-loop tail peeled (weight gradients +5-7%, forward / data
// gradients +1-3%; the bias+GELU form measured 2% slower with it and keeps the per-K-tile address
// math) — round 3, profiles/r3_gemm8_keep_b0_*, r3_gemm8_presrc_*.  The losing forms (B0 re-read,
// persistent deferred-store tiles, 256 x 128 co-resident tiles: profiles/README.md) are gone.
template <bool AKO, bool BKO, int EPI>
int launch8(const Args& a, int splits, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * (a.N / BN);
  const dim3 grid(tiles * splits);
  if constexpr (EPI == EPI_GELU || EPI == EPI_GELUD) gemm8_kernel<AKO, BKO, EPI, false><<<grid, NT, 0, st>>>(a);
  else gemm8_kernel<AKO, BKO, EPI, true><<<grid, NT, 0, st>>>(a);
  return 0;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

// Returns -1 when the shape is outside the kernel's contract: N % 256 == 0, K % (64 * splits) == 0,
// a K-outer A needs M % 256 == 0, every leading dimension a multiple of 8 elements and every base
// pointer 16-byte aligned.
int dl_gemm8(int a_kouter, int b_kouter, int epi, const bf16_t* A, long lda, const bf16_t* B, long ldb, int M, int N,
             int K, bf16_t* C, long ldc, float* Cf, long ldcf, long slab, int accumulate, const float* bias,
             const bf16_t* R, long ldr, bf16_t* H, long ldh, float* dbias, int splits, hipStream_t st, float* stats,
             long stat_rows, const DlBnBwdEpi* bn) {
  if (M <= 0 || N <= 0 || K <= 0 || splits < 1) return -1;
  if (N % BN || K % (BK * splits)) return -1;
  if (a_kouter && M % BM) return -1;
  if (lda % 8 || ldb % 8 || !aligned16(A) || !aligned16(B)) return -1;
  if (epi == EPI_F32) {
    if (!Cf || ldcf % 4 || !aligned16(Cf) || slab % 4) return -1;
  } else {
    if (!C || ldc % 8 || !aligned16(C)) return -1;
    if (R && (ldr % 8 || !aligned16(R))) return -1;
    if ((epi == EPI_GELU || epi == EPI_GELUD) && (!H || ldh % 8 || !aligned16(H))) return -1;
    if ((epi == EPI_DGELU || epi == EPI_DMUL) && !R) return -1;
    if (splits != 1) return -1;
    // EPI_STATS: every 256-row tile inside one statistics group
    if ((epi == EPI_STATS || epi == EPI_BNBWD) && (!stats || stat_rows < BM || stat_rows % BM || M % stat_rows))
      return -1;
    if (epi == EPI_BNBWD && (!bn || !bn->X || bn->ldx % 8 || !aligned16(bn->X) || (bn->Y && !aligned16(bn->Y)) ||
                             (!bn->Y && (!bn->gamma || !bn->beta))))
      return -1;
  }
  // tile order (tile_of): bands of 4 row blocks.  Against row-major at T = 262144 the QKV forward
  // 1507 -> 1468 us, FFN-up + GELU 2409 -> 2324 us, FFN-down data gradient 2027 -> 1970 us, the rest
  // within +-1.5% (profiles/r3_gemm8_tile_order_T262144.jsonl)
  constexpr int group_m = 4;
  Args a{A, lda, B, ldb, M, N, K / splits, C, ldc, Cf, ldcf, slab, accumulate, bias, R, ldr, H, ldh, dbias,
         stats, stat_rows, DlBnBwdEpi{}, group_m};
  if (epi == EPI_BNBWD) a.bn = *bn;  // by value: the kernel reads it from its argument buffer
#define DL_GEMM8_CASE(AK, BK_, E) \
  if (a_kouter == AK && b_kouter == BK_ && epi == E) return launch8<AK, BK_, E>(a, splits, st);
  DL_GEMM8_CASE(0, 0, EPI_STORE)
  DL_GEMM8_CASE(0, 0, EPI_GELU)
  DL_GEMM8_CASE(0, 1, EPI_STORE)
  DL_GEMM8_CASE(0, 1, EPI_GELU)
  DL_GEMM8_CASE(0, 1, EPI_DGELU)
  DL_GEMM8_CASE(0, 0, EPI_DGELU)
  DL_GEMM8_CASE(0, 0, EPI_GELUD)
  DL_GEMM8_CASE(0, 1, EPI_GELUD)
  DL_GEMM8_CASE(0, 1, EPI_DMUL)
  DL_GEMM8_CASE(0, 0, EPI_DMUL)
  DL_GEMM8_CASE(1, 1, EPI_F32)
  DL_GEMM8_CASE(0, 0, EPI_F32)
  DL_GEMM8_CASE(0, 0, EPI_STATS)
  DL_GEMM8_CASE(0, 1, EPI_BNBWD)
  DL_GEMM8_CASE(0, 0, EPI_BNBWD)
#undef DL_GEMM8_CASE
  return -1;
}

// General-shape bf16 MFMA GEMM for the shapes outside the 256x256-tiled kernels' contracts
// (SURVEY.md §2.7 K20/K23): any M, N, K and any element strides.  In ALBERT these are the
// factorized-embedding GEMMs (hidden 1024 <-> embedding 128: N = 128) and the tied MLM decoder's
// gradients (vocabulary 30000 on one side, 128 on the other); in SwAV the prototypes (N = K = 3000)
// and the small heads.  Several of them have a very long reduction and few output tiles (the
// embedding-mapping weight gradient: 1024 x 128 outputs over 262144 tokens), so the reduction is
// split over gridDim.z into fp32 slabs that a second pass sums (fixed order: deterministic) and
// finishes (bias, residual, bf16 rounding, or fp32 (+)= into the gradient).
//
//   C[m, n] = sum_k A(m, k) B(n, k)    A(m, k) = A[m*sam + k*sak], B(n, k) = B[n*sbn + k*sbk]
//
// Tile 128 x 128 x 32 (128 x 64 when N <= 64), 256 threads = 4 waves (2 x 2), 64 x 64 (64 x 32)
// outputs per wave = 4 x 4 (4 x 2) v_mfma_f32_16x16x32_bf16.  Operands go global -> registers (next K-step prefetched while the
// current one computes) -> LDS rows of 32 k (+8 pad: 80-byte rows keep the 16-byte fragment reads
// aligned and spread over the banks).  The global walk follows the unit-stride side of each
// operand, 16 bytes per lane when it is aligned:
//   KIN  k is unit stride: 8 consecutive k of one row per lane, one 16-B LDS write
//   RIN  rows are unit stride (transposed operands: weight-gradient inputs): 8 consecutive rows
//        of one k per lane, scattered into the k-rows of LDS as eight 2-byte writes
// A partial 8-chunk at a tile edge (or an operand that is not 16-byte aligned) is read
// element-wise with bounds checks (zero fill).
//
// Epilogues: EPI_STORE C = acc (+ bias[n]) (+ R[m, n])  bf16 (row stride ldc)
//            EPI_F32   Cf[m, n] = acc  or  += acc        fp32 (row stride ldcf)
// EPI_STORE with `stats`: also the per-column sum / sum of squares of the stored bf16 values into
// stats[m / stat_rows][0..N) / [N..2N) (BatchNorm statistics of a 64 / 128-channel 1x1 conv or the
// stem, fp32 atomics; a tile's rows never straddle two groups: stat_rows % 128 == 0)
#include <algorithm>

#include "dl_common.h"
#include "dl_kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int TM = 128, TK = 32, ROW = TK + 8, NTH = 256;
enum { L_KIN = 0, L_RIN = 1 };

struct SmallArgs {
  const bf16_t* A; long sam, sak;
  const bf16_t* B; long sbn, sbk;
  int M, N, K, kchunk;
  bf16_t* C; long ldc;
  float* Cf; long ldcf; long slab; int accumulate;
  const float* bias;
  const bf16_t* R; long ldr;
  float* stats; long stat_rows;
  DlBnBwdEpi bn; int bnbwd;  // BN backward preparation (dl_kernels.h DlBnBwdEpi): stats are then the
                             // BN backward's sums and the stored values the ReLU-masked gradient
  long sab, sbb, scb; int batched;  // batched mode: gridDim.z = batch, operand / output strides per
                                    // batch entry (fp32 outputs use `slab` as theirs), no K split
};

// U 8-element chunks of a (64 U) x 32 operand tile per thread, into registers.
template <int L, bool VEC, int U>
__device__ __forceinline__ void gload(const bf16_t* __restrict__ p, long srow, long sk, int r0, int rows, int k0,
                                      int kend, uint4 (&v)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int idx = threadIdx.x + NTH * u;
    int gr, gk;
    if constexpr (L == L_KIN) {
      gr = r0 + (idx >> 2);
      gk = k0 + (idx & 3) * 8;
    } else {  // 8 U row chunks of 8 per k
      gr = r0 + (idx & (8 * U - 1)) * 8;
      gk = k0 + idx / (8 * U);
    }
    const bool whole = L == L_KIN ? (gr < rows && gk + 8 <= kend) : (gk < kend && gr + 8 <= rows);
    if (VEC && whole) {
      v[u] = *reinterpret_cast<const uint4*>(p + (long)gr * srow + (long)gk * sk);
    } else {
      uint16_t e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = L == L_KIN ? gr : gr + j, k = L == L_KIN ? gk + j : gk;
        e[j] = (r < rows && k < kend) ? p[(long)r * srow + (long)k * sk] : (uint16_t)0;
      }
      v[u] = uint4{e[0] | ((uint32_t)e[1] << 16), e[2] | ((uint32_t)e[3] << 16), e[4] | ((uint32_t)e[5] << 16),
                   e[6] | ((uint32_t)e[7] << 16)};
    }
  }
}

// K-outer image of a 128-row operand (U = 2 chunks per thread): [32 k][128 rows], 256-byte k-rows,
// 16-byte chunk c of k-row k at c ^ kswz(k) (conflict-free for the ds_read_b64_tr_b16 lane groups,
// the layout of gemm8.hip's K-outer half-tiles).  A row-walked (L_RIN) operand lands here with one
// 16-byte write per chunk instead of eight 2-byte writes into a K-inner image.
__device__ __forceinline__ int kswz(int k) { return ((k & 3) << 2) | ((k >> 2) & 3); }
__device__ __forceinline__ void lds_put_kout(bf16_t* img, const uint4 (&v)[2]) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int idx = threadIdx.x + NTH * u;
    const int c = idx & 15, k = idx >> 4;
    *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(img) + k * 256 + ((c ^ kswz(k)) << 4)) = v[u];
  }
}
typedef short s4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4_t lds_s4;
// MFMA operand fragment (rows r0 + (lane & 15), k = 8 (lane >> 4) + j) from the K-outer image
__device__ __forceinline__ bf16x8 frag_kout(const bf16_t* img, int r0, int lane) {
  const uint8_t* b = reinterpret_cast<const uint8_t*>(img);
  const int g = lane >> 4, i = lane & 15;
  const int kr = 8 * g + (i >> 2);
  const int col = r0 + 4 * (i & 3);
  const int o1 = kr * 256 + (((col >> 3) ^ kswz(kr)) << 4) + ((col & 7) << 1);
  const int o2 = (kr + 4) * 256 + (((col >> 3) ^ kswz(kr + 4)) << 4) + ((col & 7) << 1);
  const s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(b + o1));
  const s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(b + o2));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int L, int U>
__device__ __forceinline__ void lds_put(bf16_t* img, const uint4 (&v)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int idx = threadIdx.x + NTH * u;
    if constexpr (L == L_KIN) {
      *reinterpret_cast<uint4*>(img + (idx >> 2) * ROW + (idx & 3) * 8) = v[u];
    } else {
      const int r = (idx & (8 * U - 1)) * 8, k = idx / (8 * U);
      const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        img[(r + 2 * j) * ROW + k] = (bf16_t)(w[j] & 0xffff);
        img[(r + 2 * j + 1) * ROW + k] = (bf16_t)(w[j] >> 16);
      }
    }
  }
}

// TN = 128: 4 waves as 2 x 2 of 64 x 64; TN = 64 (outputs of at most 64 columns, e.g. the
// ResNet stem and 64-channel 1x1 convs): 2 x 2 of 64 x 32, half the B tile and no wasted MFMAs
template <int EPI, int TN, int LA, bool VA, int LB, bool VB>
__global__ __launch_bounds__(NTH) void gemm_small_kernel(SmallArgs p) {
  constexpr int UB = TN / 64, NJ = TN / 32;
  __shared__ __attribute__((aligned(16))) bf16_t sa[TM * ROW];
  __shared__ __attribute__((aligned(16))) bf16_t sb[TN * ROW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
  const int kbeg = p.batched ? 0 : blockIdx.z * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const bf16_t* __restrict__ Ap = p.A + (p.batched ? (long)blockIdx.z * p.sab : 0L);
  const bf16_t* __restrict__ Bp = p.B + (p.batched ? (long)blockIdx.z * p.sbb : 0L);
  bf16_t* Cp = p.C + (p.batched ? (long)blockIdx.z * p.scb : 0L);
  floatx4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // row-walked operands of 128-row tiles go through the K-outer image (lds_put_kout / frag_kout)
  constexpr bool AKO = LA == L_RIN, BKO = LB == L_RIN && TN == 128;
  uint4 ra[2], rb[UB];
  gload<LA, VA, 2>(Ap, p.sam, p.sak, m0, p.M, kbeg, kend, ra);
  gload<LB, VB, UB>(Bp, p.sbn, p.sbk, n0, p.N, kbeg, kend, rb);
  for (int k0 = kbeg; k0 < kend; k0 += TK) {
    if constexpr (AKO) lds_put_kout(sa, ra);
    else lds_put<LA, 2>(sa, ra);
    if constexpr (BKO) lds_put_kout(sb, reinterpret_cast<const uint4(&)[2]>(rb));
    else lds_put<LB, UB>(sb, rb);
    __syncthreads();
    if (k0 + TK < kend) {  // next K-step's loads are in flight during this one's MFMAs
      gload<LA, VA, 2>(Ap, p.sam, p.sak, m0, p.M, k0 + TK, kend, ra);
      gload<LB, VB, UB>(Bp, p.sbn, p.sbk, n0, p.N, k0 + TK, kend, rb);
    }
    bf16x8 af[4], bfr[NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (AKO) af[i] = frag_kout(sa, wm * 64 + i * 16, lane);
      else af[i] = *reinterpret_cast<const bf16x8*>(sa + (wm * 64 + i * 16 + (lane & 15)) * ROW + 8 * (lane >> 4));
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if constexpr (BKO) bfr[j] = frag_kout(sb, wn * (TN / 2) + j * 16, lane);
      else bfr[j] = *reinterpret_cast<const bf16x8*>(sb + (wn * (TN / 2) + j * 16 + (lane & 15)) * ROW + 8 * (lane >> 4));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    __syncthreads();
  }
  float csum[NJ], csq[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) csum[j] = csq[j] = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wn * (TN / 2) + j * 16 + (lane & 15);
      if (n >= p.N) continue;
      float bv = 0.f;
      if constexpr (EPI == 0)
        if (p.bias) bv = p.bias[n];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * 64 + i * 16 + 4 * (lane >> 4) + e;
        if (m >= p.M) continue;
        float v = acc[i][j][e];
        if constexpr (EPI == 0) {
          v += bv;
          if (p.R) v += bf2f(p.R[(long)m * p.ldr + n]);
          if (p.bnbwd) {
            const long go = (long)(m0 / p.stat_rows) * p.N + n;
            const float x = bf2f(p.bn.X[(long)m * p.bn.ldx + n]);
            const float mu = p.bn.mean[go], rs = p.bn.rstd[go];
            bool live;
            if (p.bn.Y) {
              live = bf2f(p.bn.Y[(long)m * p.bn.ldx + n]) > 0.f;
            } else {
              const float sc = p.bn.gamma[n] * rs;
              live = fmaf(x, sc, p.bn.beta[n] - mu * sc) > 0.f;
            }
            const bf16_t o = live ? f2bf(v) : (bf16_t)0;
            Cp[(long)m * p.ldc + n] = o;
            const float g = bf2f(o);
            csum[j] += g;
            csq[j] = fmaf(g, (x - mu) * rs, csq[j]);
          } else {
            const bf16_t o = f2bf(v);
            Cp[(long)m * p.ldc + n] = o;
            const float r = bf2f(o);
            csum[j] += r;
            csq[j] = fmaf(r, r, csq[j]);
          }
        } else {
          float* dst = p.Cf + (long)blockIdx.z * p.slab + (long)m * p.ldcf + n;
          *dst = p.accumulate ? *dst + v : v;
        }
      }
    }
  if constexpr (EPI == 0) {
    if (p.stats) {
      // lanes l, l^16, l^32, l^48 hold the same columns: fold them, then lane l adds column block
      // j = l >> 4, column l & 15 — one wave-instruction per moment (atomics are issue-bound)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        csum[j] += __shfl_xor(csum[j], 16, 64);
        csq[j] += __shfl_xor(csq[j], 16, 64);
        csum[j] += __shfl_xor(csum[j], 32, 64);
        csq[j] += __shfl_xor(csq[j], 32, 64);
      }
      const int jl = lane >> 4;
      float s = csum[0], q = csq[0];
#pragma unroll
      for (int j = 1; j < NJ; ++j) {
        s = jl == j ? csum[j] : s;
        q = jl == j ? csq[j] : q;
      }
      const int n = n0 + wn * (TN / 2) + jl * 16 + (lane & 15);
      if (jl < NJ && n < p.N) {
        float* st = p.stats + (m0 / p.stat_rows) * 2L * p.N;
        atomicAdd(st + n, s);
        atomicAdd(st + p.N + n, q);
      }
    }
  }
}

// out = finish(sum_z ws[z][m, n]): bf16 (+ bias)(+ R) or fp32 (+)=
template <bool TO_BF16>
__global__ __launch_bounds__(256) void slab_finish_kernel(const float* __restrict__ ws, int S, int M, int N,
                                                          bf16_t* C, long ldc, const float* bias, const bf16_t* R,
                                                          long ldr, float* Cf, long ldcf, int accumulate) {
  const long total = (long)M * N;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int m = (int)(idx / N), n = (int)(idx % N);
    float s = 0.f;
    for (int z = 0; z < S; ++z) s += ws[(long)z * total + idx];
    if constexpr (TO_BF16) {
      if (bias) s += bias[n];
      if (R) s += bf2f(R[(long)m * ldr + n]);
      C[(long)m * ldc + n] = f2bf(s);
    } else {
      float* dst = Cf + (long)m * ldcf + n;
      *dst = accumulate ? *dst + s : s;
    }
  }
}

template <int EPI, int TN, int LA, bool VA>
void launch_b(const SmallArgs& a, int LB, bool VB, dim3 grid, hipStream_t st) {
  if (LB == L_KIN) {
    if (VB) gemm_small_kernel<EPI, TN, LA, VA, L_KIN, true><<<grid, NTH, 0, st>>>(a);
    else gemm_small_kernel<EPI, TN, LA, VA, L_KIN, false><<<grid, NTH, 0, st>>>(a);
  } else {
    if (VB) gemm_small_kernel<EPI, TN, LA, VA, L_RIN, true><<<grid, NTH, 0, st>>>(a);
    else gemm_small_kernel<EPI, TN, LA, VA, L_RIN, false><<<grid, NTH, 0, st>>>(a);
  }
}

template <int EPI, int TN>
void launch(const SmallArgs& a, int LA, bool VA, int LB, bool VB, dim3 grid, hipStream_t st) {
  if (LA == L_KIN) {
    if (VA) launch_b<EPI, TN, L_KIN, true>(a, LB, VB, grid, st);
    else launch_b<EPI, TN, L_KIN, false>(a, LB, VB, grid, st);
  } else {
    if (VA) launch_b<EPI, TN, L_RIN, true>(a, LB, VB, grid, st);
    else launch_b<EPI, TN, L_RIN, false>(a, LB, VB, grid, st);
  }
}

template <int EPI>
void launch_tn(const SmallArgs& a, int LA, bool VA, int LB, bool VB, int tn, int S, hipStream_t st) {
  const dim3 grid((a.N + tn - 1) / tn, (a.M + TM - 1) / TM, S);
  if (tn == 64) launch<EPI, 64>(a, LA, VA, LB, VB, grid, st);
  else launch<EPI, 128>(a, LA, VA, LB, VB, grid, st);
}

// walk layout of an operand and whether its 8-chunks can be read as 16-byte vectors
void walk(const bf16_t* p, long srow, long sk, int* L, bool* vec) {
  const bool aligned = ((uintptr_t)p & 15) == 0;
  if (sk == 1) {
    *L = L_KIN;
    *vec = aligned && srow % 8 == 0;
  } else if (srow == 1) {
    *L = L_RIN;
    *vec = aligned && sk % 8 == 0;
  } else {
    *L = L_KIN;
    *vec = false;
  }
}

}  // namespace

// batch independent GEMMs C_b = A_b B_b^T (same strides in every entry; entry b at A + b*sab,
// B + b*sbb, and C + b*scb (epi 0) or Cf + b*scb (epi 1)): one launch, gridDim.z = batch
int dl_gemm_small_batched(int epi, const bf16_t* A, long sam, long sak, long sab, const bf16_t* B, long sbn, long sbk,
                          long sbb, int M, int N, int K, bf16_t* C, long ldc, float* Cf, long ldcf, long scb,
                          int batch, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0 || batch < 1 || batch > 65535) return -1;
  if ((epi == 0 && !C) || (epi == 1 && !Cf) || (M + TM - 1) / TM > 65535) return -1;
  int LA, LB;
  bool VA, VB;
  walk(A, sam, sak, &LA, &VA);
  walk(B, sbn, sbk, &LB, &VB);
  // the 16-byte vector walk also needs every batch entry's base aligned
  VA = VA && sab % 8 == 0;
  VB = VB && sbb % 8 == 0;
  SmallArgs a{A, sam, sak, B, sbn, sbk, M, N, K, K, C, ldc, Cf, ldcf, scb, 0, nullptr, nullptr, 0,
              nullptr, 0, DlBnBwdEpi{}, 0, sab, sbb, scb, 1};
  const int tn = N <= 64 ? 64 : 128;
  if (epi == 0) launch_tn<0>(a, LA, VA, LB, VB, tn, batch, st);
  else launch_tn<1>(a, LA, VA, LB, VB, tn, batch, st);
  return 0;
}

int dl_gemm_small_splits(int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0) return 1;
  const int tn = N <= 64 ? 64 : 128;
  const long tiles = (long)((M + TM - 1) / TM) * ((N + tn - 1) / tn);
  // ~4 workgroups per CU (40 KiB of LDS each), at least 512 reduction rows per slice, and at most
  // 256 MiB of fp32 slabs
  long S = std::min<long>((1024 + tiles - 1) / tiles, std::max(1, K / 512));
  while (S > 1 && S * (long)M * N > (64L << 20)) --S;
  if (S <= 1) return 1;
  const int kchunk = ((K + S - 1) / S + TK - 1) / TK * TK;
  return (K + kchunk - 1) / kchunk;
}

int dl_gemm_small(int epi, const bf16_t* A, long sam, long sak, const bf16_t* B, long sbn, long sbk, int M, int N,
                  int K, bf16_t* C, long ldc, float* Cf, long ldcf, int accumulate, const float* bias, const bf16_t* R,
                  long ldr, int splits, float* ws, hipStream_t st, float* stats, long stat_rows,
                  const DlBnBwdEpi* bn) {
  if (M <= 0 || N <= 0 || K <= 0 || splits < 1) return -1;
  if (stats && (epi != 0 || splits != 1 || stat_rows < TM || stat_rows % TM || M % stat_rows)) return -1;
  if (bn && (!stats || !bn->X || (!bn->Y && (!bn->gamma || !bn->beta)))) return -1;
  if (epi == 0 && !C) return -1;
  if (epi == 1 && !Cf) return -1;
  if (splits > 1 && !ws) return -1;
  const int kchunk = splits > 1 ? ((K + splits - 1) / splits + TK - 1) / TK * TK : K;
  const int S = (K + kchunk - 1) / kchunk;
  const int tn = N <= 64 ? 64 : 128;
  if ((M + TM - 1) / TM > 65535 || S > 65535) return -1;
  int LA, LB;
  bool VA, VB;
  walk(A, sam, sak, &LA, &VA);
  walk(B, sbn, sbk, &LB, &VB);
  if (S == 1) {
    SmallArgs a{A, sam, sak, B, sbn, sbk, M, N, K, kchunk, C, ldc, Cf, ldcf, 0, accumulate, bias, R, ldr, stats,
                stat_rows, bn ? *bn : DlBnBwdEpi{}, bn ? 1 : 0, 0, 0, 0, 0};
    if (epi == 0) launch_tn<0>(a, LA, VA, LB, VB, tn, 1, st);
    else launch_tn<1>(a, LA, VA, LB, VB, tn, 1, st);
    return 0;
  }
  if (bn) return -1;  // the BN preparation needs the single-pass (unsplit) epilogue
  SmallArgs a{A, sam, sak, B, sbn, sbk, M, N, K, kchunk, nullptr, 0, ws, N, (long)M * N, 0, nullptr, nullptr, 0,
              nullptr, 0, DlBnBwdEpi{}, 0, 0, 0, 0, 0};
  launch_tn<1>(a, LA, VA, LB, VB, tn, S, st);
  const long total = (long)M * N;
  const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
  if (epi == 0)
    slab_finish_kernel<true><<<blocks, 256, 0, st>>>(ws, S, M, N, C, ldc, bias, R, ldr, nullptr, 0, 0);
  else
    slab_finish_kernel<false><<<blocks, 256, 0, st>>>(ws, S, M, N, nullptr, 0, nullptr, nullptr, 0, Cf, ldcf,
                                                      accumulate);
  return 0;
}

// bf16 MFMA GEMM with fused epilogues for the ALBERT layer.
//
//   C[M,N] = sum_k A(m,k) B(k,n)     fp32 accumulation, v_mfma_f32_16x16x32_bf16
//
// Operand storage (template flags):
//   K-inner ("row") : element (r, k) at p[r * ld + k]   -> LDS [256 rows][64 k], ds_read_b128 frags
//   K-outer ("col") : element (r, k) at p[k * ld + r]   -> LDS [64 k][256 rows], ds_read_b64_tr_b16
// so one kernel covers forward (A row, B=W row), dgrad (A=dY row, B=W col) and wgrad
// (A=dY col, B=X col) with no transposed copies anywhere.
//
// Tiling (cdna_hip_programming.md §5): 256x256x64 workgroup tile, 8 waves (2 x 4), 128x64 per wave
// = 8x4 MFMA tiles; register-staged double-buffered LDS (T14: issue tile t+1's global loads before
// the MFMAs of tile t, write them to the other LDS buffer after, one barrier per k-step);
// XOR-swizzled LDS images conflict-free for both read kinds (derivation in docs/KERNELS.md);
// XCD-aware tile order (T1).  Split-K over gridDim.z for the fp32-accumulating (wgrad) form.
//
// Epilogues:  EPI_STORE   C = acc (+ bias[n]) (+ R[m,n])                     bf16
//             EPI_GELU    H = acc + bias (pre-activation), C = gelu_new(H)     bf16 x2
//             EPI_DGELU   C = acc * gelu_new'(F[m,n]);  dbias[n] += sum_m C   bf16 (+fp32 atomics)
//             EPI_ACC32   Cf[m,n] += acc                                      fp32 (atomics if split-K)
#include "dl_common.h"
#include "dl_kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s4_t __attribute__((ext_vector_type(4)));
typedef short s8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s4_t lds_s4;

enum { EPI_STORE = 0, EPI_GELU = 1, EPI_DGELU = 2, EPI_ACC32 = 3 };

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NTHREADS = 512;
constexpr int TILE_BYTES = BM * BK * 2;  // 32 KiB per operand per stage

// ---- LDS image addressing --------------------------------------------------------------------
// K-inner image: [256 rows][8 chunks of 16 B]; chunk c of row r stored at c ^ ((r >> 1) & 7)
__device__ __forceinline__ int kin_off(int row, int c) { return row * 128 + ((c ^ ((row >> 1) & 7)) << 4); }
// K-outer image: [64 k-rows][32 chunks of 16 B]; chunk c of k-row r stored at c ^ h(r),
// h(r) = 2 * ((r & 3) | ((r >> 1) & 4))
__device__ __forceinline__ int kout_off(int row, int c) {
  return row * 512 + ((c ^ (((row & 3) | ((row >> 1) & 4)) << 1)) << 4);
}

__device__ __forceinline__ floatx4 mfma16(bf16x8 a, bf16x8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// fragment of 16 rows x 32 k (rows r0.., k-chunk base kc = 4*ksub): lane l -> row r0 + (l&15),
// k = 8*(l>>4) + j
template <bool KOUTER>
__device__ __forceinline__ bf16x8 load_frag(const uint8_t* img, int r0, int ksub, int lane) {
  if constexpr (!KOUTER) {
    return *reinterpret_cast<const bf16x8*>(img + kin_off(r0 + (lane & 15), 4 * ksub + (lane >> 4)));
  } else {
    // two ds_read_b64_tr_b16: k-rows 8g..8g+3 and 8g+4..8g+7 of this ksub, columns r0..r0+15
    const int g = lane >> 4, i = lane & 15;
    const int krow = 32 * ksub + 8 * g + (i >> 2);
    const int col = r0 + 4 * (i & 3);
    const int o1 = kout_off(krow, col >> 3) + ((col & 7) << 1);
    const int o2 = kout_off(krow + 4, col >> 3) + ((col & 7) << 1);
    const s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + o1));
    const s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + o2));
    const s8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
  }
}

struct Stage { uint4 v0, v1, v2, v3; };

template <bool KOUTER>
__device__ __forceinline__ uint4 g_ld1(const bf16_t* p, long ld, int r0, int k0, int rows_valid, int u) {
  const int idx = threadIdx.x + NTHREADS * u;
  if constexpr (!KOUTER) {
    const int row = min(r0 + (idx >> 3), rows_valid - 1);
    return *reinterpret_cast<const uint4*>(p + (long)row * ld + k0 + (idx & 7) * 8);
  } else {
    return *reinterpret_cast<const uint4*>(p + (long)(k0 + (idx >> 5)) * ld + r0 + (idx & 31) * 8);
  }
}

// global -> registers for one operand tile (4 x 16 B per thread)
template <bool KOUTER>
__device__ __forceinline__ void g_load(Stage& s, const bf16_t* p, long ld, int r0, int k0, int rows_valid) {
  s.v0 = g_ld1<KOUTER>(p, ld, r0, k0, rows_valid, 0);
  s.v1 = g_ld1<KOUTER>(p, ld, r0, k0, rows_valid, 1);
  s.v2 = g_ld1<KOUTER>(p, ld, r0, k0, rows_valid, 2);
  s.v3 = g_ld1<KOUTER>(p, ld, r0, k0, rows_valid, 3);
}

template <bool KOUTER>
__device__ __forceinline__ void s_st1(uint8_t* img, int u, const uint4& v) {
  const int idx = threadIdx.x + NTHREADS * u;
  const int off = KOUTER ? kout_off(idx >> 5, idx & 31) : kin_off(idx >> 3, idx & 7);
  *reinterpret_cast<uint4*>(img + off) = v;
}

template <bool KOUTER>
__device__ __forceinline__ void s_store(const Stage& s, uint8_t* img) {
  s_st1<KOUTER>(img, 0, s.v0);
  s_st1<KOUTER>(img, 1, s.v1);
  s_st1<KOUTER>(img, 2, s.v2);
  s_st1<KOUTER>(img, 3, s.v3);
}

struct GemmArgs {
  const bf16_t* A; long lda;
  const bf16_t* B; long ldb;
  int M, N, K;
  bf16_t* C; long ldc;          // bf16 output (EPI_STORE/GELU/DGELU)
  float* Cf; long ldcf;         // fp32 output (EPI_ACC32)
  const float* bias;            // fp32 [N] (STORE/GELU)
  const bf16_t* R; long ldr;    // residual (STORE) or pre-activation F (DGELU)
  bf16_t* H; long ldh;          // pre-activation out (GELU)
  float* dbias;                 // column-sum out (DGELU)
  int k_per_split;
};

template <bool AKO, bool BKO, int EPI>
__global__ __launch_bounds__(NTHREADS, 1) void gemm_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 2, wn = w & 3;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles_m = (p.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.z * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nk = (kend - kbeg) / BK;

  floatx4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  Stage sa, sb;
  g_load<AKO>(sa, p.A, p.lda, m0, kbeg, p.M);
  g_load<BKO>(sb, p.B, p.ldb, n0, kbeg, p.N);
  s_store<AKO>(sa, smem);
  s_store<BKO>(sb, smem + TILE_BYTES);
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    const uint8_t* Ai = smem + cur * 2 * TILE_BYTES;
    const uint8_t* Bi = Ai + TILE_BYTES;
    if (t + 1 < nk) {
      g_load<AKO>(sa, p.A, p.lda, m0, kbeg + (t + 1) * BK, p.M);
      g_load<BKO>(sb, p.B, p.ldb, n0, kbeg + (t + 1) * BK, p.N);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 bf[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bf[ni] = load_frag<BKO>(Bi, wn * 64 + ni * 16, ks, lane);
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        const bf16x8 af = load_frag<AKO>(Ai, wm * 128 + mi * 16, ks, lane);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = mfma16(af, bf[ni], acc[mi][ni]);
      }
    }
    if (t + 1 < nk) {
      uint8_t* An = smem + (cur ^ 1) * 2 * TILE_BYTES;
      s_store<AKO>(sa, An);
      s_store<BKO>(sb, An + TILE_BYTES);
    }
    __syncthreads();
  }

  // ---- epilogue: lane holds C[row 4*(lane>>4) + i][col lane&15] of each 16x16 tile
  const int rq = 4 * (lane >> 4), cl = lane & 15;
  if constexpr (EPI == EPI_STORE) {
    if (p.R == nullptr && p.ldc % 8 == 0 && (reinterpret_cast<uintptr_t>(p.C) & 15) == 0) {
      // bf16 tile staged through the (now free) 128 KiB of LDS and written as 16-byte row chunks:
      // the per-element stores (4 rows x 32 bytes per wave instruction) made the ALBERT decoder's
      // 39424 x 30000 logits GEMM (K = 128) store-bound at ~1.3 TB/s.  Row r's 16-byte chunk c sits
      // at chunk c ^ (r & 31) of its 512-byte LDS row.
      uint8_t* st = smem;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int col = wn * 64 + ni * 16 + cl;
        const float bv = (p.bias && n0 + col < p.N) ? p.bias[n0 + col] : 0.f;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = wm * 128 + mi * 16 + rq + i;
            const int off = row * 512 + ((((col >> 3) ^ (row & 31)) << 4) | ((col & 7) << 1));
            *reinterpret_cast<bf16_t*>(st + off) = f2bf(acc[mi][ni][i] + bv);
          }
      }
      __syncthreads();
      const int ch = threadIdx.x & 31;
#pragma unroll 4
      for (int pass = 0; pass < 16; ++pass) {
        const int row = pass * 16 + (threadIdx.x >> 5);
        const int m = m0 + row, n = n0 + ch * 8;
        if (m >= p.M || n >= p.N) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(st + row * 512 + ((ch ^ (row & 31)) << 4));
        bf16_t* dst = p.C + (long)m * p.ldc + n;
        if (n + 8 <= p.N) {
          *reinterpret_cast<uint4*>(dst) = v;
        } else {
          const bf16_t* e = reinterpret_cast<const bf16_t*>(&v);
          for (int j = 0; j < p.N - n; ++j) dst[j] = e[j];
        }
      }
      return;
    }
  }
  float colsum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = n0 + wn * 64 + ni * 16 + cl;
    const bool nok = n < p.N;
    float bv = 0.f;
    if constexpr (EPI == EPI_STORE || EPI == EPI_GELU)
      if (p.bias && nok) bv = p.bias[n];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 128 + mi * 16 + rq + i;
        if (!nok || m >= p.M) continue;
        float v = acc[mi][ni][i];
        if constexpr (EPI == EPI_STORE) {
          v += bv;
          if (p.R) v += bf2f(p.R[(long)m * p.ldr + n]);
          p.C[(long)m * p.ldc + n] = f2bf(v);
        } else if constexpr (EPI == EPI_GELU) {
          const bf16_t hb = f2bf(v + bv);
          p.H[(long)m * p.ldh + n] = hb;
          p.C[(long)m * p.ldc + n] = f2bf(gelu_tanh_sig(bf2f(hb)));
        } else if constexpr (EPI == EPI_DGELU) {
          const bf16_t cb = f2bf(v * gelu_tanh_grad_sig(bf2f(p.R[(long)m * p.ldr + n])));
          p.C[(long)m * p.ldc + n] = cb;
          colsum[ni] += bf2f(cb);
        } else {
          float* dst = p.Cf + (long)m * p.ldcf + n;
          if (gridDim.z > 1) atomicAdd(dst, v);
          else *dst += v;
        }
      }
    }
  }
  if constexpr (EPI == EPI_DGELU) {
    if (p.dbias) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        float s = colsum[ni];
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        const int n = n0 + wn * 64 + ni * 16 + cl;
        if (lane < 16 && n < p.N) atomicAdd(&p.dbias[n], s);
      }
    }
  }
}

template <bool AKO, bool BKO, int EPI>
int launch(const GemmArgs& a, int splits, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles, 1, splits);
  const size_t lds = 4 * TILE_BYTES;  // 2 stages x (A + B)
  static bool attr = false;
  if (!attr) {
    DL_HIP_CHECK(hipFuncSetAttribute((const void*)gemm_kernel<AKO, BKO, EPI>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  gemm_kernel<AKO, BKO, EPI><<<grid, NTHREADS, lds, st>>>(a);
  return 0;
}

}  // namespace

// Returns -1 when the shape is not supported by the MFMA kernel (caller falls back to the library):
// the reduction extent must be a multiple of 64 (per split), K-outer operands need their row extent
// (M or N) to be a multiple of 256 and ld a multiple of 8.
int dl_gemm(int a_kouter, int b_kouter, int epi, const bf16_t* A, long lda, const bf16_t* B, long ldb, int M, int N,
            int K, bf16_t* C, long ldc, float* Cf, long ldcf, const float* bias, const bf16_t* R, long ldr, bf16_t* H,
            long ldh, float* dbias, int splits, hipStream_t st) {
  if (K % BK || M <= 0 || N <= 0) return -1;
  if (lda % 8 || ldb % 8) return -1;
  if (a_kouter && M % BM) return -1;
  if (b_kouter && N % BN) return -1;
  if (splits < 1) splits = 1;
  while (splits > 1 && (K / splits) % BK) --splits;
  GemmArgs a{A, lda, B, ldb, M, N, K, C, ldc, Cf, ldcf, bias, R, ldr, H, ldh, dbias, K / splits};
#define DL_GEMM_CASE(AK, BK_, E) \
  if (a_kouter == AK && b_kouter == BK_ && epi == E) return launch<AK, BK_, E>(a, splits, st);
  DL_GEMM_CASE(0, 0, EPI_STORE)
  DL_GEMM_CASE(0, 0, EPI_GELU)
  DL_GEMM_CASE(0, 1, EPI_STORE)
  DL_GEMM_CASE(0, 1, EPI_DGELU)
  DL_GEMM_CASE(1, 1, EPI_ACC32)
  DL_GEMM_CASE(0, 0, EPI_ACC32)
#undef DL_GEMM_CASE
  return -1;
}

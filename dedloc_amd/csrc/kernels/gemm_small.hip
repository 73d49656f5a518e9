// General-shape bf16 MFMA GEMM for the shapes outside the tiled kernels' contracts (SURVEY.md
// §2.7 K20/K23 and the small ALBERT heads): any M, N, K and any element strides — the SwAV
// prototypes (N = 3000, and K = 3000 in their gradient GEMMs), the 512-row SwAV head, the SOP /
// pooler heads, the conv stem's column matrix.  Correctness-first and simple: the big GEMMs of
// both models go to gemm8.hip / gemm.hip; what lands here is a few GFLOP per step at most.
//
//   C[m, n] = sum_k A(m, k) B(n, k)    A(m, k) = A[m*sam + k*sak], B(n, k) = B[n*sbn + k*sbk]
//
// Tile 64 x 64 x 32, 256 threads = 4 waves (2 x 2), 32 x 32 outputs per wave = 2 x 2
// v_mfma_f32_16x16x32_bf16.  Operands are staged element-wise with bounds checks (zero fill) into
// LDS rows of 32 k (+8 pad, keeps the 16-byte fragment reads aligned and bank-spread); the global
// walk follows whichever operand stride is unit (k or row), so either layout coalesces.
//
// Epilogues: EPI_STORE C = acc (+ bias[n]) (+ R[m, n])  bf16 (row stride ldc)
//            EPI_F32   Cf[m, n] = acc  or  += acc        fp32 (row stride ldcf)
#include "dl_common.h"
#include "dl_kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int TM = 64, TN = 64, TK = 32, ROW = TK + 8;

struct SmallArgs {
  const bf16_t* A; long sam, sak;
  const bf16_t* B; long sbn, sbk;
  int M, N, K;
  bf16_t* C; long ldc;
  float* Cf; long ldcf; int accumulate;
  const float* bias;
  const bf16_t* R; long ldr;
};

__device__ __forceinline__ void stage(const bf16_t* __restrict__ p, long srow, long sk, int r0, int k0, int rows,
                                      int K, bf16_t* img) {
  // 64 rows x 32 k = 2048 elements, 8 per thread
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int idx = threadIdx.x + 256 * u;
    int r, k;
    if (sk == 1) {
      r = idx >> 5;
      k = idx & 31;
    } else {
      k = idx >> 6;
      r = idx & 63;
    }
    const int gr = r0 + r, gk = k0 + k;
    bf16_t v = 0;
    if (gr < rows && gk < K) v = p[(long)gr * srow + (long)gk * sk];
    img[r * ROW + k] = v;
  }
}

template <int EPI>
__global__ __launch_bounds__(256) void gemm_small_kernel(SmallArgs p) {
  __shared__ __attribute__((aligned(16))) bf16_t sa[TM * ROW];
  __shared__ __attribute__((aligned(16))) bf16_t sb[TN * ROW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
  floatx4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < p.K; k0 += TK) {
    stage(p.A, p.sam, p.sak, m0, k0, p.M, p.K, sa);
    stage(p.B, p.sbn, p.sbk, n0, k0, p.N, p.K, sb);
    __syncthreads();
    bf16x8 af[2], bfr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      af[i] = *reinterpret_cast<const bf16x8*>(sa + (wm * 32 + i * 16 + (lane & 15)) * ROW + 8 * (lane >> 4));
      bfr[i] = *reinterpret_cast<const bf16x8*>(sb + (wn * 32 + i * 16 + (lane & 15)) * ROW + 8 * (lane >> 4));
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * 32 + i * 16 + 4 * (lane >> 4) + e;
        const int n = n0 + wn * 32 + j * 16 + (lane & 15);
        if (m >= p.M || n >= p.N) continue;
        float v = acc[i][j][e];
        if constexpr (EPI == 0) {
          if (p.bias) v += p.bias[n];
          if (p.R) v += bf2f(p.R[(long)m * p.ldr + n]);
          p.C[(long)m * p.ldc + n] = f2bf(v);
        } else {
          float* dst = p.Cf + (long)m * p.ldcf + n;
          *dst = p.accumulate ? *dst + v : v;
        }
      }
}

}  // namespace

int dl_gemm_small(int epi, const bf16_t* A, long sam, long sak, const bf16_t* B, long sbn, long sbk, int M, int N,
                  int K, bf16_t* C, long ldc, float* Cf, long ldcf, int accumulate, const float* bias, const bf16_t* R,
                  long ldr, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0) return -1;
  if (epi == 0 && !C) return -1;
  if (epi == 1 && !Cf) return -1;
  SmallArgs a{A, sam, sak, B, sbn, sbk, M, N, K, C, ldc, Cf, ldcf, accumulate, bias, R, ldr};
  dim3 grid((N + TN - 1) / TN, (M + TM - 1) / TM);
  if (grid.y > 65535) return -1;
  if (epi == 0)
    gemm_small_kernel<0><<<grid, 256, 0, st>>>(a);
  else
    gemm_small_kernel<1><<<grid, 256, 0, st>>>(a);
  return 0;
}

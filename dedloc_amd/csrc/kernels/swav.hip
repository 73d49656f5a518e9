// SwAV loss kernels (reference: vissl/losses/swav_loss.py:177-326,
// vissl/hooks/swav_hooks.py:63-92).
//
// Sinkhorn-Knopp over P[n, K] (n = batch + queue rows, K = prototypes), vissl semantics:
//   P = exp((S - max S) / eps)                       (log-sum-exp stabilised, never overflows)
//   repeat iters:  P *= (1/K) / colsum_k(P)          (prototype marginal)
//                  P *= (1/n) / rowsum_b(P)          (sample marginal)
//   Q = P / rowsum_b(P)   for the last `bs` rows      (assignments of the current crop)
// Each pass is one row-block kernel: a block owns `rpb` rows, keeps its per-prototype partial
// column sums in registers across those rows and adds them with one lane-contiguous atomic per
// prototype per block, so the [3904 x 3000] fp32 matrix is streamed once per iteration.
//
// Swapped-prediction loss: loss = -mean_b sum_k q_bk log_softmax(s_b / T)_k with its gradient
// ds = (softmax(s/T) * sum(q) - q) / T * scale accumulated in place (one block per row).
#include "dl_common.h"
#include "dl_kernels.h"

namespace {

constexpr int MAXK_PER_THREAD = 16;  // K <= 4096 prototypes with 256 threads

__device__ __forceinline__ unsigned f2ord(float f) {
  unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__global__ __launch_bounds__(256) void max_kernel(const float* __restrict__ s, size_t n, unsigned* __restrict__ out) {
  float m = -INFINITY;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    m = fmaxf(m, s[i]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) atomicMax(out, f2ord(m));
}

// P = exp((S - M)/eps) and colsum += column partials
__global__ __launch_bounds__(256) void exp_colsum_kernel(const float* __restrict__ s, float* __restrict__ P,
                                                         const unsigned* __restrict__ mx, float inv_eps,
                                                         float* __restrict__ colsum, int n, int K, int rpb) {
  const float M = ord2f(*mx);
  float acc[MAXK_PER_THREAD];
#pragma unroll
  for (int j = 0; j < MAXK_PER_THREAD; ++j) acc[j] = 0.f;
  const int r0 = blockIdx.x * rpb, r1 = min(n, r0 + rpb);
  for (int r = r0; r < r1; ++r) {
#pragma unroll
    for (int j = 0; j < MAXK_PER_THREAD; ++j) {
      const int k = threadIdx.x + 256 * j;
      if (k < K) {
        const float p = __expf((s[(size_t)r * K + k] - M) * inv_eps);
        P[(size_t)r * K + k] = p;
        acc[j] += p;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < MAXK_PER_THREAD; ++j) {
    const int k = threadIdx.x + 256 * j;
    if (k < K) atomicAdd(&colsum[k], acc[j]);
  }
}

// one Sinkhorn iteration; `last` writes the normalised assignments of rows >= n - bs into Q
__global__ __launch_bounds__(256) void sinkhorn_iter_kernel(float* __restrict__ P, const float* __restrict__ colsum_in,
                                                            float* __restrict__ colsum_out, float* __restrict__ Q,
                                                            int n, int K, int rpb, int bs, int last) {
  __shared__ float red[8];
  float cs[MAXK_PER_THREAD], acc[MAXK_PER_THREAD];
  const float rK = 1.f / K, cn = 1.f / n;
#pragma unroll
  for (int j = 0; j < MAXK_PER_THREAD; ++j) {
    const int k = threadIdx.x + 256 * j;
    cs[j] = (k < K) ? rK / colsum_in[k] : 0.f;
    acc[j] = 0.f;
  }
  const int r0 = blockIdx.x * rpb, r1 = min(n, r0 + rpb);
  for (int r = r0; r < r1; ++r) {
    float v[MAXK_PER_THREAD];
    float rs = 0.f;
#pragma unroll
    for (int j = 0; j < MAXK_PER_THREAD; ++j) {
      const int k = threadIdx.x + 256 * j;
      v[j] = (k < K) ? P[(size_t)r * K + k] * cs[j] : 0.f;
      rs += v[j];
    }
    rs = wave_sum(rs);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = rs;
    __syncthreads();
    const float tot = red[0] + red[1] + red[2] + red[3];
    const float sc = cn / tot;
    const bool emit = last && r >= n - bs;
#pragma unroll
    for (int j = 0; j < MAXK_PER_THREAD; ++j) {
      const int k = threadIdx.x + 256 * j;
      if (k < K) {
        const float p = v[j] * sc;
        if (!last) {
          P[(size_t)r * K + k] = p;
          acc[j] += p;
        } else if (emit) {
          Q[(size_t)(r - (n - bs)) * K + k] = v[j] / tot;  // == p * n: final per-sample normalisation
        }
      }
    }
  }
  if (!last) {
#pragma unroll
    for (int j = 0; j < MAXK_PER_THREAD; ++j) {
      const int k = threadIdx.x + 256 * j;
      if (k < K) atomicAdd(&colsum_out[k], acc[j]);
    }
  }
}

// swapped-prediction cross-entropy of one crop's scores against assignments q (one block per row)
template <typename T>
__global__ __launch_bounds__(256) void swav_ce_kernel(const T* __restrict__ s, const float* __restrict__ q,
                                                      float* __restrict__ ds, float* __restrict__ loss, int K,
                                                      float inv_temp, float scale) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const T* x = s + (size_t)row * K;
  const float* qr = q + (size_t)row * K;
  float m = -INFINITY;
  for (int k = threadIdx.x; k < K; k += blockDim.x) m = fmaxf(m, (float)x[k] * inv_temp);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float se = 0.f, qx = 0.f, qs = 0.f;
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const float xv = (float)x[k] * inv_temp;
    se += __expf(xv - m);
    qx += qr[k] * xv;
    qs += qr[k];
  }
  se = wave_sum(se);
  qx = wave_sum(qx);
  qs = wave_sum(qs);
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = se;
    red[4 + (threadIdx.x >> 6)] = qx;
    red[8 + (threadIdx.x >> 6)] = qs;
  }
  __syncthreads();
  se = red[0] + red[1] + red[2] + red[3];
  qx = red[4] + red[5] + red[6] + red[7];
  qs = red[8] + red[9] + red[10] + red[11];
  const float lse = m + __logf(se);
  if (threadIdx.x == 0) atomicAdd(loss, (qs * lse - qx) * scale);
  const float inv_se = 1.f / se;
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const float sm = __expf((float)x[k] * inv_temp - m) * inv_se;
    ds[(size_t)row * K + k] += (sm * qs - qr[k]) * inv_temp * scale;
  }
}

__global__ __launch_bounds__(128) void row_normalize_kernel(float* __restrict__ w, int rows, int d) {
  const int row = blockIdx.x * 2 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float ss = 0.f;
  for (int c = lane; c < d; c += 64) ss += w[(size_t)row * d + c] * w[(size_t)row * d + c];
  ss = wave_sum(ss);
  const float inv = 1.f / fmaxf(sqrtf(ss), 1e-12f);
  for (int c = lane; c < d; c += 64) w[(size_t)row * d + c] *= inv;
}

}  // namespace

// scores [n, K] fp32 -> Q [bs, K] fp32 (assignments of the last bs rows); ws: float[2K + 1]
int dl_sinkhorn(const float* scores, float* P, float* Q, float* ws, int n, int K, int bs, float eps, int iters,
                hipStream_t st) {
  if (K > 256 * MAXK_PER_THREAD || iters < 1) return -1;
  unsigned* mx = reinterpret_cast<unsigned*>(ws);
  float* cs0 = ws + 1;
  float* cs1 = ws + 1 + K;
  DL_HIP_CHECK(hipMemsetAsync(ws, 0, sizeof(float) * (2 * K + 1), st));
  const size_t total = (size_t)n * K;
  const int mgrid = (int)(((total + 255) / 256) < 1024 ? (total + 255) / 256 : 1024);
  max_kernel<<<mgrid, 256, 0, st>>>(scores, total, mx);
  const int rpb = 16;
  const int nb = (n + rpb - 1) / rpb;
  exp_colsum_kernel<<<nb, 256, 0, st>>>(scores, P, mx, 1.f / eps, cs0, n, K, rpb);
  for (int it = 0; it < iters; ++it) {
    float* cin = (it & 1) ? cs1 : cs0;
    float* cout = (it & 1) ? cs0 : cs1;
    const int last = it + 1 == iters;
    if (!last) DL_HIP_CHECK(hipMemsetAsync(cout, 0, sizeof(float) * K, st));
    // the last iteration's sample normalisation coincides with the final Q / rowsum(Q): it writes Q
    sinkhorn_iter_kernel<<<nb, 256, 0, st>>>(P, cin, cout, Q, n, K, rpb, bs, last);
  }
  return 0;
}

int dl_swav_ce(const void* scores, int scores_bf16, const float* q, float* dscores, float* loss, int rows, int K,
               float temperature, float scale, hipStream_t st) {
  if (scores_bf16)
    swav_ce_kernel<__bf16><<<rows, 256, 0, st>>>(reinterpret_cast<const __bf16*>(scores), q, dscores, loss, K,
                                                 1.f / temperature, scale);
  else
    swav_ce_kernel<float><<<rows, 256, 0, st>>>(reinterpret_cast<const float*>(scores), q, dscores, loss, K,
                                                1.f / temperature, scale);
  return 0;
}

int dl_row_normalize(float* w, int rows, int d, hipStream_t st) {
  row_normalize_kernel<<<(rows + 1) / 2, 128, 0, st>>>(w, rows, d);
  return 0;
}

// SwAV loss kernels (reference: vissl/losses/swav_loss.py:177-326,
// vissl/hooks/swav_hooks.py:63-92).
//
// Sinkhorn-Knopp over the scores S[n, K] (n = batch + queue rows, K = prototypes), vissl semantics
// (swav_loss.py:177-244): Q = exp(S / eps), then `iters` x (prototype marginal, sample marginal), then
// each sample's row normalised.  Kept as two scale vectors instead of a rewritten matrix:
//   P[b,k] = E[b,k] a[k] c[b],   E[b,k] = exp((S[b,k] - m[k]) / eps)
// with m[k] the column maximum (any per-column constant is absorbed by a[k], and it keeps every
// column's largest entry at 1: no overflow, no empty column).  An iteration is
//   a[k] = (1/K) / sum_b E[b,k] c[b]        (c = 1 before the first)
//   c[b] = (1/n) / sum_k E[b,k] a[k]
// and the assignments are Q[b,k] = E[b,k] a[k] / sum_k E[b,k] a[k] for the last `bs` rows.
// Workgroups own 16 prototype columns each (K = 3000: 188 workgroups at any n — the row-block form
// launched 4 at n = 64): the column sums are local to a workgroup; the row sums are per-workgroup
// partials reduced by a small row kernel.  S (fp32, 0.8-15 MB) is re-read from L2 each pass; E is
// recomputed, never stored.
// Swapped-prediction loss: loss = -mean_b sum_k q_bk log_softmax(s_b / T)_k with its gradient
// ds = (softmax(s/T) * sum(q) - q) / T * scale accumulated in place (one block per row).
#include "dl_common.h"
#include "dl_kernels.h"

namespace {

constexpr int SK_COLS = 16;  // prototype columns per workgroup (256 threads = 16 columns x 16 row groups)

// One Sinkhorn iteration over this workgroup's columns: (first) column maxima; a[k] from the column
// sums weighted by c; the per-row partial sums sum_{k in block} E[b,k] a[k] into part[blockIdx.x][b].
__global__ __launch_bounds__(256) void sk_col_kernel(const float* __restrict__ S, float* __restrict__ colmax,
                                                     float* __restrict__ a, const float* __restrict__ c,
                                                     float* __restrict__ part, int n, int K, float inv_eps,
                                                     int first) {
  __shared__ float red[16][SK_COLS];
  const int cl = threadIdx.x & (SK_COLS - 1), rg = threadIdx.x >> 4;
  const int k = blockIdx.x * SK_COLS + cl;
  const bool kv = k < K;
  float m;
  if (first) {
    m = -INFINITY;
    if (kv)
      for (int b = rg; b < n; b += 16) m = fmaxf(m, S[(size_t)b * K + k]);
    red[rg][cl] = m;
    __syncthreads();
    m = red[0][cl];
#pragma unroll
    for (int g = 1; g < 16; ++g) m = fmaxf(m, red[g][cl]);
    __syncthreads();
    if (rg == 0 && kv) colmax[k] = m;
  } else {
    m = kv ? colmax[k] : 0.f;
  }
  float cs = 0.f;
  if (kv)
    for (int b = rg; b < n; b += 16) cs += __expf((S[(size_t)b * K + k] - m) * inv_eps) * (c ? c[b] : 1.f);
  red[rg][cl] = cs;
  __syncthreads();
  cs = 0.f;
#pragma unroll
  for (int g = 0; g < 16; ++g) cs += red[g][cl];
  const float ak = kv ? (1.f / K) / cs : 0.f;
  if (rg == 0 && kv) a[k] = ak;
  // row partials: the 16 lanes of a row group hold the block's 16 columns of row b
  for (int b = rg; b < n; b += 16) {
    float v = kv ? __expf((S[(size_t)b * K + k] - m) * inv_eps) * ak : 0.f;
    v += __shfl_xor(v, 1, 16);
    v += __shfl_xor(v, 2, 16);
    v += __shfl_xor(v, 4, 16);
    v += __shfl_xor(v, 8, 16);
    if (cl == 0) part[(size_t)b * gridDim.x + blockIdx.x] = v;
  }
}

// row sums s[b] = sum over the column blocks' partials (part[b][0..nblk), one wave per row: a
// serial loop of 188 dependent loads in one lane took 45 us at n = 64); c[b] = (1/n) / s[b],
// rinv[b] = 1 / s[b]
__global__ __launch_bounds__(256) void sk_row_kernel(const float* __restrict__ part, int nblk, int n,
                                                     float* __restrict__ c, float* __restrict__ rinv) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= n) return;
  float s = 0.f;
  for (int j = lane; j < nblk; j += 64) s += part[(size_t)b * nblk + j];
  s = wave_sum(s);
  if (lane == 0) {
    c[b] = (1.f / n) / s;
    rinv[b] = 1.f / s;
  }
}

// Q[r, k] = E[n - bs + r, k] a[k] / s[n - bs + r]
__global__ __launch_bounds__(256) void sk_emit_kernel(const float* __restrict__ S, const float* __restrict__ colmax,
                                                      const float* __restrict__ a, const float* __restrict__ rinv,
                                                      float* __restrict__ Q, int n, int K, int bs, float inv_eps) {
  const int r = blockIdx.y;
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  const int b = n - bs + r;
  Q[(size_t)r * K + k] = __expf((S[(size_t)b * K + k] - colmax[k]) * inv_eps) * a[k] * rinv[b];
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

// All swapped predictions of one iteration in one launch: block (v, row) reads crop v's score row
// once, its log-sum-exp once, and pairs it with every assignment i of another crop:
//   loss += scale * sum_i (sum(q_i) lse - <q_i, x>),  ds[v, row] = scale / T * sum_i (softmax(x) sum(q_i) - q_i)
// (x = s / T).  ds is written, not accumulated.  Up to 4 assignment crops.
struct SwavAssign {
  int crop[4];
  int n;
};

template <typename T>
__global__ __launch_bounds__(256) void swav_ce_multi_kernel(const T* __restrict__ s, const float* __restrict__ q,
                                                            float* __restrict__ ds, float* __restrict__ loss, int bs,
                                                            int K, SwavAssign as, float inv_temp, float scale) {
  __shared__ float red[4][4 + 8];
  const int v = blockIdx.y, row = blockIdx.x;
  const T* x = s + ((size_t)v * bs + row) * K;
  float m = -INFINITY;
  for (int k = threadIdx.x; k < K; k += 256) m = fmaxf(m, (float)x[k] * inv_temp);
  m = wave_max(m);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w][0] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0][0], red[1][0]), fmaxf(red[2][0], red[3][0]));
  __syncthreads();
  float se = 0.f, qx[4] = {0.f, 0.f, 0.f, 0.f}, qs[4] = {0.f, 0.f, 0.f, 0.f};
  for (int k = threadIdx.x; k < K; k += 256) {
    const float xv = (float)x[k] * inv_temp;
    se += __expf(xv - m);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i < as.n && as.crop[i] != v) {
        const float qv = q[((size_t)i * bs + row) * K + k];
        qx[i] += qv * xv;
        qs[i] += qv;
      }
    }
  }
  se = wave_sum(se);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    qx[i] = wave_sum(qx[i]);
    qs[i] = wave_sum(qs[i]);
  }
  if ((threadIdx.x & 63) == 0) {
    red[w][0] = se;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      red[w][4 + i] = qx[i];
      red[w][8 + i] = qs[i];
    }
  }
  __syncthreads();
  se = red[0][0] + red[1][0] + red[2][0] + red[3][0];
  float qst = 0.f, lterm = 0.f;
  const float lse = m + __logf(se);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float qsi = red[0][8 + i] + red[1][8 + i] + red[2][8 + i] + red[3][8 + i];
    const float qxi = red[0][4 + i] + red[1][4 + i] + red[2][4 + i] + red[3][4 + i];
    qst += qsi;
    lterm += qsi * lse - qxi;
  }
  if (threadIdx.x == 0) atomicAdd(loss, lterm * scale);
  const float inv_se = 1.f / se, g = inv_temp * scale;
  for (int k = threadIdx.x; k < K; k += 256) {
    float qsum = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < as.n && as.crop[i] != v) qsum += q[((size_t)i * bs + row) * K + k];
    const float sm = __expf((float)x[k] * inv_temp - m) * inv_se;
    ds[((size_t)v * bs + row) * K + k] = (sm * qst - qsum) * g;
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

// scores [n, K] fp32 -> Q [bs, K] fp32 (assignments of the last bs rows); ws: dl_sinkhorn_ws(n, K) floats
int dl_sinkhorn_ws(int n, int K) {
  const int nblk = (K + SK_COLS - 1) / SK_COLS;
  return 2 * K + 2 * n + nblk * n;
}

int dl_sinkhorn(const float* scores, float* Q, float* ws, int n, int K, int bs, float eps, int iters,
                hipStream_t st) {
  if (iters < 1 || n < 1 || K < 1 || bs > n) return -1;
  const int nblk = (K + SK_COLS - 1) / SK_COLS;
  float* colmax = ws;
  float* a = ws + K;
  float* c = ws + 2 * K;
  float* rinv = c + n;
  float* part = rinv + n;
  const float inv_eps = 1.f / eps;
  for (int it = 0; it < iters; ++it) {
    sk_col_kernel<<<nblk, 256, 0, st>>>(scores, colmax, a, it ? c : nullptr, part, n, K, inv_eps, it == 0);
    sk_row_kernel<<<(n + 3) / 4, 256, 0, st>>>(part, nblk, n, c, rinv);
  }
  sk_emit_kernel<<<dim3((K + 255) / 256, bs), 256, 0, st>>>(scores, colmax, a, rinv, Q, n, K, bs, inv_eps);
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

int dl_swav_ce_multi(const void* scores, int scores_bf16, const float* q, const int* crops, int n_assign,
                     float* dscores, float* loss, int num_crops, int bs, int K, float temperature, float scale,
                     hipStream_t st) {
  if (n_assign < 1 || n_assign > 4) return -1;
  SwavAssign as{};
  as.n = n_assign;
  for (int i = 0; i < n_assign; ++i) as.crop[i] = crops[i];
  const dim3 grid(bs, num_crops);
  if (scores_bf16)
    swav_ce_multi_kernel<__bf16><<<grid, 256, 0, st>>>(reinterpret_cast<const __bf16*>(scores), q, dscores, loss, bs,
                                                       K, as, 1.f / temperature, scale);
  else
    swav_ce_multi_kernel<float><<<grid, 256, 0, st>>>(reinterpret_cast<const float*>(scores), q, dscores, loss, bs,
                                                      K, as, 1.f / temperature, scale);
  return 0;
}

int dl_row_normalize(float* w, int rows, int d, hipStream_t st) {
  row_normalize_kernel<<<(rows + 1) / 2, 128, 0, st>>>(w, rows, d);
  return 0;
}

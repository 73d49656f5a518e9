// SwAV ResNet-50 pooling and head kernels on channels-last bf16 (SURVEY.md §2.7 K17 max-pool, K19
// global average pool, K20 L2 normalisation; reference vissl/models/trunks/resnext.py:48-172 (the
// torchvision stem's MaxPool2d(3, 2, 1) and AdaptiveAvgPool2d(1)) and
// vissl/models/heads/swav_prototypes_head.py:93-112 (nn.functional.normalize(p=2, dim=1))).
//
// Every thread owns 8 consecutive channels of one pixel: 16-byte loads and stores of the NHWC rows.
//
//   maxpool_fwd : y[n,p,q,c] = max over the 3x3 window at (2p-1, 2q-1) (padding = -inf), and the
//                 window slot (0..8) of the maximum per element (uint8, the backward's routing)
//   maxpool_bwd : dx[n,h,w,c] = sum of dy over the (at most 4) windows whose recorded maximum is
//                 (h, w) — a gather, so no atomics and a deterministic result
//   avgpool_fwd : y[n,c] = mean_{h,w} x[n,h,w,c]   (bf16 out; one block per (n, 256-channel chunk))
//   avgpool_bwd : dx[n,h,w,c] = dy[n,c] / (H W)
//   l2norm_fwd  : y = x / max(||x||, eps) per row (rows of D <= 1024 bf16), inverse norm kept (fp32)
//   l2norm_bwd  : dx = (dy - y <y, dy>) / max(||x||, eps)
#include <algorithm>

#include "dl_common.h"
#include "dl_kernels.h"

namespace {

__device__ __forceinline__ void load8(const bf16_t* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
}

__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                          uint8_t* __restrict__ arg, int N, int H, int W, int C,
                                                          int P, int Q) {
  const int C8 = C / 8;
  const long total = (long)N * P * Q * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    long t = i / C8;
    const int q = (int)(t % Q);
    t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float best[8];
    uint8_t slot[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      slot[j] = 0;
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int h = 2 * p - 1 + r;
      if (h < 0 || h >= H) continue;
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int w = 2 * q - 1 + s;
        if (w < 0 || w >= W) continue;
        float v[8];
        load8(x + (((long)n * H + h) * W + w) * C + c8 * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (v[j] > best[j] || (v[j] != v[j] && best[j] == best[j])) {  // first maximum in window order wins (torch's tie rule); the first NaN wins over numbers, as in torch
            best[j] = v[j];
            slot[j] = (uint8_t)(r * 3 + s);
          }
      }
    }
    *reinterpret_cast<uint4*>(y + i * 8) = pack8_bf16(best);
    uint2 packed;
    packed.x = slot[0] | (slot[1] << 8) | (slot[2] << 16) | ((uint32_t)slot[3] << 24);
    packed.y = slot[4] | (slot[5] << 8) | (slot[6] << 16) | ((uint32_t)slot[7] << 24);
    *reinterpret_cast<uint2*>(arg + i * 8) = packed;
  }
}

__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                          bf16_t* __restrict__ dx, int N, int H, int W, int C, int P,
                                                          int Q) {
  const int C8 = C / 8;
  const long total = (long)N * H * W * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    long t = i / C8;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    // windows p with 2p - 1 <= h <= 2p + 1  ->  p in [(h - 1) / 2, (h + 1) / 2]
    const int p0 = h / 2, p1 = min(P - 1, (h + 1) / 2);  // ceil((h - 1) / 2) == h / 2 for h >= 0
    const int q0 = w / 2, q1 = min(Q - 1, (w + 1) / 2);
    for (int p = p0; p <= p1; ++p) {
      const int r = h - (2 * p - 1);
      if (r < 0 || r > 2) continue;
      for (int q = q0; q <= q1; ++q) {
        const int s = w - (2 * q - 1);
        if (s < 0 || s > 2) continue;
        const long o = (((long)n * P + p) * Q + q) * C + c8 * 8;
        const uint2 packed = *reinterpret_cast<const uint2*>(arg + o);
        float g[8];
        load8(dy + o, g);
        const uint8_t want = (uint8_t)(r * 3 + s);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t word = j < 4 ? packed.x : packed.y;
          if (((word >> (8 * (j & 3))) & 0xff) == want) acc[j] += g[j];
        }
      }
    }
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8_bf16(acc);
  }
}

// one block = 32 channel-groups (256 channels) x 8 pixel lanes of one image; fp32 sums
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                          int HW, int C, float inv) {
  __shared__ float part[8][256 + 4];
  const int n = blockIdx.y;
  const int cg = threadIdx.x & 31, pl = threadIdx.x >> 5;  // 32 channel groups of 8, 8 pixel lanes
  const int c0 = blockIdx.x * 256 + cg * 8;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (c0 < C) {
    for (int px = pl; px < HW; px += 8) {
      float v[8];
      load8(x + ((long)n * HW + px) * C + c0, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[pl][cg * 8 + j] = acc[j];
  __syncthreads();
  if (threadIdx.x < 256) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += part[k][threadIdx.x];
    if (c < C) y[(long)n * C + c] = f2bf(s * inv);
  }
}

__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx,
                                                          int N, int HW, int C, float inv) {
  const int C8 = C / 8;
  const long total = (long)N * HW * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    const int n = (int)(i / ((long)HW * C8));
    float g[8];
    load8(dy + (long)n * C + c8 * 8, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] *= inv;
    *reinterpret_cast<uint4*>(dx + i * 8) = pack8_bf16(g);
  }
}

// one wave per row, D <= 1024 (16 values per lane)
__global__ __launch_bounds__(256) void l2norm_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                         float* __restrict__ rinv, int rows, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float v[16];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int d = lane + 64 * j;
    v[j] = d < D ? bf2f(x[(long)row * D + d]) : 0.f;
    ss += v[j] * v[j];
  }
  ss = wave_sum(ss);
  const float r = 1.f / fmaxf(sqrtf(ss), eps);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int d = lane + 64 * j;
    if (d < D) y[(long)row * D + d] = f2bf(v[j] * r);
  }
  if (lane == 0) rinv[row] = r;
}

__global__ __launch_bounds__(256) void l2norm_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                         const float* __restrict__ rinv, bf16_t* __restrict__ dx,
                                                         int rows, int D) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float g[16], yy[16];
  float dot = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int d = lane + 64 * j;
    g[j] = d < D ? bf2f(dy[(long)row * D + d]) : 0.f;
    yy[j] = d < D ? bf2f(y[(long)row * D + d]) : 0.f;
    dot += g[j] * yy[j];
  }
  dot = wave_sum(dot);
  const float r = rinv[row];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int d = lane + 64 * j;
    if (d < D) dx[(long)row * D + d] = f2bf((g[j] - yy[j] * dot) * r);
  }
}

inline int grid_for(long work) { return (int)std::min<long>(std::max<long>(1, (work + 255) / 256), 8192); }

}  // namespace

int dl_maxpool_fwd(const bf16_t* x, bf16_t* y, uint8_t* arg, int N, int H, int W, int C, int P, int Q, hipStream_t st) {
  if (C % 8 || P != (H - 1) / 2 + 1 || Q != (W - 1) / 2 + 1) return -1;
  maxpool_fwd_kernel<<<grid_for((long)N * P * Q * (C / 8)), 256, 0, st>>>(x, y, arg, N, H, W, C, P, Q);
  return 0;
}

int dl_maxpool_bwd(const bf16_t* dy, const uint8_t* arg, bf16_t* dx, int N, int H, int W, int C, int P, int Q,
                   hipStream_t st) {
  if (C % 8 || P != (H - 1) / 2 + 1 || Q != (W - 1) / 2 + 1) return -1;
  maxpool_bwd_kernel<<<grid_for((long)N * H * W * (C / 8)), 256, 0, st>>>(dy, arg, dx, N, H, W, C, P, Q);
  return 0;
}

int dl_avgpool_fwd(const bf16_t* x, bf16_t* y, int N, int HW, int C, hipStream_t st) {
  if (C % 8 || HW <= 0) return -1;
  avgpool_fwd_kernel<<<dim3((C + 255) / 256, N), 256, 0, st>>>(x, y, HW, C, 1.f / HW);
  return 0;
}

int dl_avgpool_bwd(const bf16_t* dy, bf16_t* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8 || HW <= 0) return -1;
  avgpool_bwd_kernel<<<grid_for((long)N * HW * (C / 8)), 256, 0, st>>>(dy, dx, N, HW, C, 1.f / HW);
  return 0;
}

int dl_l2norm_fwd(const bf16_t* x, bf16_t* y, float* rinv, int rows, int D, float eps, hipStream_t st) {
  if (D > 1024 || rows <= 0) return -1;
  l2norm_fwd_kernel<<<(rows + 3) / 4, 256, 0, st>>>(x, y, rinv, rows, D, eps);
  return 0;
}

int dl_l2norm_bwd(const bf16_t* dy, const bf16_t* y, const float* rinv, bf16_t* dx, int rows, int D, hipStream_t st) {
  if (D > 1024 || rows <= 0) return -1;
  l2norm_bwd_kernel<<<(rows + 3) / 4, 256, 0, st>>>(dy, y, rinv, dx, rows, D);
  return 0;
}

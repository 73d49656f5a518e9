// Memory-bound elementwise / reduction kernels: gelu_new fwd/bwd, bias-gradient column sums,
// fp32<->bf16 casts of the flat parameter buffer, tanh for the SOP pooler.
// All bf16 traffic is 16 B per lane (Guideline 13); grids are capped at 256 CUs x 8 blocks and
// grid-strided (Guideline 11).
#include <cstdlib>

#include "dl_common.h"
#include "dl_kernels.h"

namespace {

constexpr int kMaxGrid = 2048;

inline int grid_for(size_t nvec, int block) {
  size_t g = (nvec + block - 1) / block;
  return (int)(g < (size_t)kMaxGrid ? (g == 0 ? 1 : g) : kMaxGrid);
}

// No grid stride: each thread owns VPT vectors of a 1024-vector block chunk and issues all their
// loads before any math (LayerNorm's access shape, which streams at ~6.3 TB/s), branch-free
// hardware bf16 conversion: 498 -> 389 us at T=131072 x 4096 against the grid-strided form (4.3 ->
// 5.5 TB/s, bench/ew_bench.py), sigmoid-form GELU (one exp2 + one rcp).
constexpr int VPT = 4;
__global__ __launch_bounds__(256) void gelu_fwd_v2_kernel(const bf16_t* __restrict__ h, bf16_t* __restrict__ y,
                                                          size_t nvec) {
  const size_t base = (size_t)blockIdx.x * (256 * VPT) + threadIdx.x;
  uint4 raw[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const size_t i = base + (size_t)k * 256;
    if (i < nvec) raw[k] = reinterpret_cast<const uint4*>(h)[i];
  }
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const size_t i = base + (size_t)k * 256;
    if (i < nvec) {
      float v[8];
      load_bf16<8>(reinterpret_cast<const bf16_t*>(&raw[k]), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = gelu_tanh_sig(v[j]);
      reinterpret_cast<uint4*>(y)[i] = pack8_bf16(v);
    }
  }
}


// y = gelu_new(h), d = gelu_new'(h) (the unfused form of gemm8's EPI_GELUD)
__global__ __launch_bounds__(256) void gelu_fwd_d_kernel(const bf16_t* __restrict__ h, bf16_t* __restrict__ y,
                                                         bf16_t* __restrict__ d, size_t nvec) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    float v[8], g[8], dv[8];
    load_bf16<8>(h + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) gelu_and_grad_sig(v[j], g[j], dv[j]);
    store_bf16<8>(y + i * 8, g);
    store_bf16<8>(d + i * 8, dv);
  }
}

__global__ __launch_bounds__(256) void gelu_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ h,
                                                       bf16_t* __restrict__ dh, size_t nvec) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    float g[8], v[8];
    load_bf16<8>(dy + i * 8, g);
    load_bf16<8>(h + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] *= gelu_tanh_grad(v[j]);
    store_bf16<8>(dh + i * 8, g);
  }
}


// v2 of the fused GELU backward + bias-gradient column sums: straight-line per wave (no row loop):
// each of the 8 waves of a block issues the loads of its 8 rows x 8 columns-per-lane at once, then
// computes and stores them, so no row's loads queue behind another row's stores in the in-order
// vmcnt (the v1 row loop waits for its own previous stores every iteration).  Block = 512 columns
// x 64 rows; the 8 wave partials meet in LDS, one fp32 atomic per column per block.
// GELU = 1: dh = x * gelu_new'(h); GELU = 2: dh = x * h (h already gelu_new', EPI_GELUD's output)
template <int GELU>
__global__ __launch_bounds__(512) void colsum_rows_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ h,
                                                          bf16_t* __restrict__ dh, float* __restrict__ out, int rows,
                                                          int N) {
  constexpr int RW = 8;  // rows per wave
  __shared__ float red[8][512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cb = blockIdx.x * 512;
  const int c0 = cb + lane * 8;
  const bool active = c0 < N;
  const int rbase = blockIdx.y * (8 * RW) + w * RW;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (active) {
    uint4 xr[RW], hr[RW];
#pragma unroll
    for (int u = 0; u < RW; ++u) {
      const int r = min(rbase + u, rows - 1);
      xr[u] = *reinterpret_cast<const uint4*>(x + (size_t)r * N + c0);
      if (GELU) hr[u] = *reinterpret_cast<const uint4*>(h + (size_t)r * N + c0);
    }
#pragma unroll
    for (int u = 0; u < RW; ++u) {
      if (rbase + u >= rows) break;
      float g[8];
      load_bf16<8>(reinterpret_cast<const bf16_t*>(&xr[u]), g);
      if (GELU) {
        float v[8];
        load_bf16<8>(reinterpret_cast<const bf16_t*>(&hr[u]), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = bf2f(f2bf(g[j] * (GELU == 2 ? v[j] : gelu_tanh_grad_sig(v[j]))));
        store_bf16<8>(dh + (size_t)(rbase + u) * N + c0, g);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += g[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[w][lane * 8 + j] = acc[j];
  __syncthreads();
  const int c = threadIdx.x;  // 512 threads = 512 columns
  if (cb + c < N) {
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) sum += red[k][c];
    atomicAdd(&out[cb + c], sum);
  }
}

__global__ __launch_bounds__(256) void tanh_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = f2bf(tanhf(bf2f(x[i])));
}

__global__ __launch_bounds__(256) void tanh_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                       bf16_t* __restrict__ dx, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float t = bf2f(y[i]);
    dx[i] = f2bf(bf2f(dy[i]) * (1.f - t * t));
  }
}

// Column partial sums of a bf16 [rows, N] matrix: block (px, py) sums rows [py*rpb, ...) of the
// 8*256 = 2048 columns starting at px*2048 -> part[py][col] (fp32).
__global__ __launch_bounds__(256) void colsum_bf16_kernel(const bf16_t* __restrict__ x, float* __restrict__ part,
                                                          int rows, int N, int rpb) {
  const int c0 = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (c0 >= N) return;
  const int r0 = blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int r = r0;
  // 8 independent 16-byte loads in flight per thread (the plain loop was HBM-latency bound)
  for (; r + 8 <= r1; r += 8) {
    uint4 raw[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) raw[u] = *reinterpret_cast<const uint4*>(x + (size_t)(r + u) * N + c0);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      float v[8];
      load_bf16<8>(reinterpret_cast<const bf16_t*>(&raw[u]), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
  }
  for (; r < r1; ++r) {
    float v[8];
    load_bf16<8>(x + (size_t)r * N + c0, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) atomicAdd(&part[c0 + j], acc[j]);
}

// scalar variant for N % 8 != 0 (e.g. the 2-way SOP classifier bias)
__global__ __launch_bounds__(256) void colsum_bf16_scalar_kernel(const bf16_t* __restrict__ x, float* __restrict__ part,
                                                                 int rows, int N, int rpb) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N) return;
  const int r0 = blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
  float acc = 0.f;
  for (int r = r0; r < r1; ++r) acc += bf2f(x[(size_t)r * N + c]);
  atomicAdd(&part[c], acc);
}

// out[c] (+)= sum_p part[p][c]
__global__ __launch_bounds__(256) void colsum_f32_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                         int nparts, int N, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N) return;
  float s = 0.f;
  for (int p = 0; p < nparts; ++p) s += part[(size_t)p * N + c];
  out[c] = accumulate ? out[c] + s : s;
}

__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, size_t n) {
  const size_t nvec = n / 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    float4 v = reinterpret_cast<const float4*>(x)[i];
    uint2 o;
    o.x = (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
    o.y = (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16);
    reinterpret_cast<uint2*>(y)[i] = o;
  }
  for (size_t i = nvec * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}

// y (fp32) (+)= bf16 x   -- used to fold bf16 partial gradients into fp32 accumulators
__global__ __launch_bounds__(256) void add_bf16_to_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y,
                                                              size_t n, float alpha) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] += alpha * bf2f(x[i]);
}

}  // namespace

int dl_gelu_fwd(const bf16_t* h, bf16_t* y, size_t n, hipStream_t st) {
  if (n % 8) return -1;
  const size_t nvec = n / 8;
  gelu_fwd_v2_kernel<<<(unsigned)((nvec + 256 * VPT - 1) / (256 * VPT)), 256, 0, st>>>(h, y, nvec);
  return 0;
}

int dl_gelu_bwd(const bf16_t* dy, const bf16_t* h, bf16_t* dh, size_t n, hipStream_t st) {
  if (n % 8) return -1;
  gelu_bwd_kernel<<<grid_for(n / 8, 256), 256, 0, st>>>(dy, h, dh, n / 8);
  return 0;
}

int dl_gelu_bwd_colsum(const bf16_t* dy, const bf16_t* h, bf16_t* dh, float* dbias, int rows, int N, hipStream_t st) {
  if (N % 8) return -1;
  dim3 grid((N + 511) / 512, (rows + 63) / 64);
  colsum_rows_kernel<1><<<grid, 512, 0, st>>>(dy, h, dh, dbias, rows, N);
  return 0;
}

int dl_mul_colsum(const bf16_t* dy, const bf16_t* d, bf16_t* dh, float* dbias, int rows, int N, hipStream_t st) {
  if (N % 8) return -1;
  dim3 grid((N + 511) / 512, (rows + 63) / 64);
  colsum_rows_kernel<2><<<grid, 512, 0, st>>>(dy, d, dh, dbias, rows, N);
  return 0;
}

int dl_gelu_fwd_d(const bf16_t* h, bf16_t* y, bf16_t* d, size_t n, hipStream_t st) {
  if (n % 8) return -1;
  gelu_fwd_d_kernel<<<grid_for(n / 8, 256), 256, 0, st>>>(h, y, d, n / 8);
  return 0;
}

int dl_tanh_fwd(const bf16_t* x, bf16_t* y, size_t n, hipStream_t st) {
  tanh_fwd_kernel<<<grid_for(n, 256), 256, 0, st>>>(x, y, n);
  return 0;
}

int dl_tanh_bwd(const bf16_t* dy, const bf16_t* y, bf16_t* dx, size_t n, hipStream_t st) {
  tanh_bwd_kernel<<<grid_for(n, 256), 256, 0, st>>>(dy, y, dx, n);
  return 0;
}

int dl_colsum_bf16(const bf16_t* x, float* part, int rows, int N, int nparts, hipStream_t st) {
  const int rpb = (rows + nparts - 1) / nparts;
  // `part` is the fp32 [N] destination: every block adds its row-chunk sums atomically
  if (N % 8) {
    colsum_bf16_scalar_kernel<<<dim3((N + 255) / 256, nparts), 256, 0, st>>>(x, part, rows, N, rpb);
    return 0;
  }
  dim3 grid((N + 511) / 512, (rows + 63) / 64);
  colsum_rows_kernel<0><<<grid, 512, 0, st>>>(x, nullptr, nullptr, part, rows, N);
  (void)rpb;
  return 0;
}

int dl_colsum_f32(const float* part, float* out, int nparts, int N, int accumulate, hipStream_t st) {
  colsum_f32_kernel<<<(N + 255) / 256, 256, 0, st>>>(part, out, nparts, N, accumulate);
  return 0;
}

int dl_cast_f32_bf16(const float* x, bf16_t* y, size_t n, hipStream_t st) {
  cast_f32_bf16_kernel<<<grid_for(n / 4 + 1, 256), 256, 0, st>>>(x, y, n);
  return 0;
}

int dl_add_bf16_to_f32(const bf16_t* x, float* y, size_t n, float alpha, hipStream_t st) {
  add_bf16_to_f32_kernel<<<grid_for(n, 256), 256, 0, st>>>(x, y, n, alpha);
  return 0;
}

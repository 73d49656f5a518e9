// Streaming-bandwidth probe for the LayerNorm shape ([262144, 1024] bf16 = 512 MiB in, 512 MiB out):
// which copy pattern reaches the HBM roof on this box, so the LN kernels can follow it.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/bw_probe bench/hip/bw_probe.hip && /tmp/bw_probe
//
// Variants (one JSON line each, median of 20 cold-cache runs, bytes = read + write):
//   rowwave  one 2 KiB row per wave, R rows per wave, a grid over all rows (the LN forward's layout)
//   stride   a fixed grid of waves looping over rows, the next row's loads issued before this row's
//            stores (register double buffer)
//   *_nt     the same with nontemporal stores (and loads)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));    \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

constexpr int D = 1024;       // bf16 per row: 2 KiB, 2 x 16 B per lane
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int NV = D / 8 / 64;

template <int R, bool NT>
__global__ __launch_bounds__(256) void rowwave(const u32x4* __restrict__ x, u32x4* __restrict__ y, int rows) {
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (row0 >= rows) return;
  u32x4 v[R][NV];
#pragma unroll
  for (int u = 0; u < R; ++u)
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const size_t o = (size_t)min(row0 + u, rows - 1) * (D / 8) + i * 64 + lane;
      v[u][i] = NT ? __builtin_nontemporal_load(x + o) : x[o];
    }
#pragma unroll
  for (int u = 0; u < R; ++u)
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (row0 + u >= rows) break;
      const size_t o = (size_t)(row0 + u) * (D / 8) + i * 64 + lane;
      if (NT) __builtin_nontemporal_store(v[u][i], y + o);
      else y[o] = v[u][i];
    }
}

// a fixed grid; wave w handles rows w, w + W, w + 2W, ... two rows per step, the next step's loads
// issued before this step's stores
template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void stride(const u32x4* __restrict__ x, u32x4* __restrict__ y, int rows) {
  const int lane = threadIdx.x & 63;
  const int W = gridDim.x * 4;
  int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  constexpr int R = 2;
  auto ld = [&](const u32x4* p) { return NTL ? __builtin_nontemporal_load(p) : *p; };
  u32x4 cur[R][NV];
#pragma unroll
  for (int u = 0; u < R; ++u)
#pragma unroll
    for (int i = 0; i < NV; ++i) cur[u][i] = ld(x + (size_t)min(row + u * W, rows - 1) * (D / 8) + i * 64 + lane);
  for (; row < rows; row += R * W) {
    u32x4 nxt[R][NV];
#pragma unroll
    for (int u = 0; u < R; ++u)
#pragma unroll
      for (int i = 0; i < NV; ++i)
        nxt[u][i] = ld(x + (size_t)min(row + (R + u) * W, rows - 1) * (D / 8) + i * 64 + lane);
#pragma unroll
    for (int u = 0; u < R; ++u)
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int rr = row + u * W;
        if (rr < rows) {
          u32x4* p = y + (size_t)rr * (D / 8) + i * 64 + lane;
          if (NTS) __builtin_nontemporal_store(cur[u][i], p);
          else *p = cur[u][i];
        }
      }
#pragma unroll
    for (int u = 0; u < R; ++u)
#pragma unroll
      for (int i = 0; i < NV; ++i) cur[u][i] = nxt[u][i];
  }
}

template <typename F>
float timed(F f, uint8_t* flush, size_t flush_bytes) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> ts;
  f();
  CK(hipDeviceSynchronize());
  for (int it = 0; it < 20; ++it) {
    CK(hipMemsetAsync(flush, it, flush_bytes, 0));  // evict the 256 MiB MALL
    CK(hipEventRecord(a, 0));
    f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms * 1000.f);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main() {
  const int rows = 262144;
  const size_t bytes = (size_t)rows * D * 2;
  u32x4 *x, *y;
  uint8_t* flush;
  const size_t flush_bytes = 1ull << 29;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&y, bytes));
  CK(hipMalloc(&flush, flush_bytes));
  CK(hipMemset(x, 1, bytes));
  auto report = [&](const char* name, int grid, float us) {
    std::printf("{\"variant\": \"%s\", \"grid\": %d, \"us\": %.1f, \"TBps\": %.3f}\n", name, grid, us,
                2.0 * bytes / us / 1e6);
    std::fflush(stdout);
  };
  {
    const int g = rows / 4 / 2;
    report("rowwave_r2", g, timed([&] { rowwave<2, false><<<g, 256>>>(x, y, rows); }, flush, flush_bytes));
    report("rowwave_r2_nt", g, timed([&] { rowwave<2, true><<<g, 256>>>(x, y, rows); }, flush, flush_bytes));
    const int g4 = rows / 4 / 4;
    report("rowwave_r4", g4, timed([&] { rowwave<4, false><<<g4, 256>>>(x, y, rows); }, flush, flush_bytes));
    report("rowwave_r4_nt", g4, timed([&] { rowwave<4, true><<<g4, 256>>>(x, y, rows); }, flush, flush_bytes));
  }
  for (int g : {512, 1024, 2048, 4096}) {
    report("stride", g, timed([&] { stride<false, false><<<g, 256>>>(x, y, rows); }, flush, flush_bytes));
    report("stride_nts", g, timed([&] { stride<false, true><<<g, 256>>>(x, y, rows); }, flush, flush_bytes));
    report("stride_ntls", g, timed([&] { stride<true, true><<<g, 256>>>(x, y, rows); }, flush, flush_bytes));
  }
  CK(hipMemcpy(x, y, 64, hipMemcpyDeviceToDevice));
  std::printf("{\"done\": true}\n");
  return 0;
}

// Averaging data-plane kernels: everything stays in HBM.
//
// pack      : wire = compress(local * weight)                 (FLOAT16 clamps to +-65504)
// reduce    : avg  = sum_k decompress(part_k) * inv_total     (fp32 accumulation, k <= 64 peers)
// unpack    : local = decompress(avg)            (mode 0, synchronous averaging)
//             local += decompress(avg) - snap    (mode 1, delta rule for delayed averaging)
// dtype codes: 0 = fp32, 1 = fp16, 2 = bf16.
#include "dl_common.h"
#include "dl_kernels.h"

namespace {

__device__ __forceinline__ float load_any(const void* p, size_t i, int dt) {
  if (dt == 0) return reinterpret_cast<const float*>(p)[i];
  if (dt == 1) return h2f(reinterpret_cast<const uint16_t*>(p)[i]);
  return bf2f(reinterpret_cast<const uint16_t*>(p)[i]);
}

__device__ __forceinline__ void store_any(void* p, size_t i, float v, int dt) {
  if (dt == 0) reinterpret_cast<float*>(p)[i] = v;
  else if (dt == 1) reinterpret_cast<uint16_t*>(p)[i] = f2h(fminf(fmaxf(v, -65504.f), 65504.f));
  else reinterpret_cast<uint16_t*>(p)[i] = f2bf(v);
}

template <int DT>
__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ src, void* __restrict__ dst, size_t n,
                                                   float weight) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    store_any(dst, i, src[i] * weight, DT);
}

template <int DT>
__global__ __launch_bounds__(256) void reduce_kernel(const void* __restrict__ parts, size_t part_stride, int nparts,
                                                     void* __restrict__ out, int out_dt, size_t n, float inv_total) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < nparts; ++k) s += load_any(parts, (size_t)k * part_stride + i, DT);
    store_any(out, i, s * inv_total, out_dt);
  }
}

template <int DT>
__global__ __launch_bounds__(256) void unpack_kernel(const void* __restrict__ src, float* __restrict__ dst,
                                                     const float* __restrict__ snap, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float a = load_any(src, i, DT);
    dst[i] = snap ? dst[i] + (a - snap[i]) : a;
  }
}

inline int grid_for(size_t n) {
  size_t g = (n + 255) / 256;
  return (int)(g < 4096 ? (g == 0 ? 1 : g) : 4096);
}

}  // namespace

int dl_pack(const float* src, void* dst, int dst_dt, size_t n, float weight, hipStream_t st) {
  switch (dst_dt) {
    case 0: pack_kernel<0><<<grid_for(n), 256, 0, st>>>(src, dst, n, weight); break;
    case 1: pack_kernel<1><<<grid_for(n), 256, 0, st>>>(src, dst, n, weight); break;
    case 2: pack_kernel<2><<<grid_for(n), 256, 0, st>>>(src, dst, n, weight); break;
    default: return -1;
  }
  return 0;
}

int dl_reduce_parts(const void* parts, int part_dt, size_t part_stride, int nparts, void* out, int out_dt, size_t n,
                    float inv_total, hipStream_t st) {
  switch (part_dt) {
    case 0: reduce_kernel<0><<<grid_for(n), 256, 0, st>>>(parts, part_stride, nparts, out, out_dt, n, inv_total); break;
    case 1: reduce_kernel<1><<<grid_for(n), 256, 0, st>>>(parts, part_stride, nparts, out, out_dt, n, inv_total); break;
    case 2: reduce_kernel<2><<<grid_for(n), 256, 0, st>>>(parts, part_stride, nparts, out, out_dt, n, inv_total); break;
    default: return -1;
  }
  return 0;
}

int dl_unpack(const void* src, int src_dt, float* dst, const float* snap, size_t n, hipStream_t st) {
  switch (src_dt) {
    case 0: unpack_kernel<0><<<grid_for(n), 256, 0, st>>>(src, dst, snap, n); break;
    case 1: unpack_kernel<1><<<grid_for(n), 256, 0, st>>>(src, dst, snap, n); break;
    case 2: unpack_kernel<2><<<grid_for(n), 256, 0, st>>>(src, dst, snap, n); break;
    default: return -1;
  }
  return 0;
}

// Averaging data-plane kernels: everything stays in HBM.
//
// pack      : wire = compress(local * weight)                 (FLOAT16 clamps to +-65504)
// reduce    : avg  = sum_k decompress(part_k) * inv_total     (fp32 accumulation, k <= 64 peers)
// reduce_delta (the averaging path): avg = sum_k w_k decompress(part_k) / sum_k w_k in fp32, and
//             per sender delta_k = compress(avg - decompress(part_k)).  Returning deltas instead of
//             the average (hivemind's averaged-part deltas) keeps every peer's fp32 master tensor:
//             the sender adds delta_k, so the quantisation residual of its own contribution is
//             never written back and updates below half a wire ulp survive averaging.
// unpack    : local = decompress(avg)            (mode 0)
//             local += decompress(avg) - snap    (mode 1, snapshot delta rule)
//             local += decompress(delta)         (mode 2, averaged-part delta)
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
__global__ __launch_bounds__(256) void reduce_delta_kernel(const void* __restrict__ parts, size_t part_stride,
                                                           int nparts, const float* __restrict__ weights,
                                                           void* __restrict__ deltas, size_t n) {
  float wsum = 0.f;
  for (int k = 0; k < nparts; ++k) wsum += weights[k];
  // no weight at all (every contributor's micro-steps were dropped as non-finite): the round is a
  // no-op — zero deltas, every member keeps its own tensor — instead of adopting member 0's values
  const bool none = !(wsum > 0.f);
  const float inv = none ? 0.f : 1.f / wsum;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if (none) {
      for (int k = 0; k < nparts; ++k) store_any(deltas, (size_t)k * part_stride + i, 0.f, DT);
      continue;
    }
    // avg = v_0 + sum_k w_k (v_k - v_0) / sum_k w_k: identical contributions give exactly v_0 (zero
    // deltas, the fp32 masters untouched) and the differences keep the sum well conditioned
    float v[16];
    v[0] = load_any(parts, i, DT);
    float s = 0.f;
#pragma unroll
    for (int k = 1; k < 16; ++k) {
      if (k < nparts) {
        v[k] = load_any(parts, (size_t)k * part_stride + i, DT);
        s += weights[k] * (v[k] - v[0]);
      }
    }
    for (int k = 16; k < nparts; ++k) s += weights[k] * (load_any(parts, (size_t)k * part_stride + i, DT) - v[0]);
    const float avg = v[0] + s * inv;
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < nparts) store_any(deltas, (size_t)k * part_stride + i, avg - v[k], DT);
    for (int k = 16; k < nparts; ++k)
      store_any(deltas, (size_t)k * part_stride + i, avg - load_any(parts, (size_t)k * part_stride + i, DT), DT);
  }
}

template <int DT>
__global__ __launch_bounds__(256) void unpack_kernel(const void* __restrict__ src, float* __restrict__ dst,
                                                     const float* __restrict__ snap, int add, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float a = load_any(src, i, DT);
    dst[i] = add ? dst[i] + a : (snap ? dst[i] + (a - snap[i]) : a);
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

int dl_reduce_delta(const void* parts, void* deltas, int dt, size_t part_stride, int nparts, const float* weights,
                    size_t n, hipStream_t st) {
  if (nparts < 1 || nparts > 64) return -1;
  switch (dt) {
    case 0: reduce_delta_kernel<0><<<grid_for(n), 256, 0, st>>>(parts, part_stride, nparts, weights, deltas, n); break;
    case 1: reduce_delta_kernel<1><<<grid_for(n), 256, 0, st>>>(parts, part_stride, nparts, weights, deltas, n); break;
    case 2: reduce_delta_kernel<2><<<grid_for(n), 256, 0, st>>>(parts, part_stride, nparts, weights, deltas, n); break;
    default: return -1;
  }
  return 0;
}

int dl_unpack(const void* src, int src_dt, float* dst, const float* snap, int add, size_t n, hipStream_t st) {
  switch (src_dt) {
    case 0: unpack_kernel<0><<<grid_for(n), 256, 0, st>>>(src, dst, snap, add, n); break;
    case 1: unpack_kernel<1><<<grid_for(n), 256, 0, st>>>(src, dst, snap, add, n); break;
    case 2: unpack_kernel<2><<<grid_for(n), 256, 0, st>>>(src, dst, snap, add, n); break;
    default: return -1;
  }
  return 0;
}

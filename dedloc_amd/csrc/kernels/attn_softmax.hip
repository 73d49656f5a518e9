// Row softmax of the composed attention path (head sizes the flash kernels in attention.hip do not
// take, e.g. albert-xlarge's 128): the [B*H, S, S] fp32 scores come from a batched GEMM, and these
// two kernels replace the chain of PyTorch elementwise passes over them.
//   fwd: scale (log2 units) + key bias + max / sum-exp2 in one wave per row -> bf16 P and lse
//        (one fp32 read + one bf16 write of the scores, second row read L2-resident)
//   bwd: P recomputed from lse, dS = P * (dP - delta) * scale -> bf16 P (for dV) and bf16 dS in one
//        elementwise pass over the scores and dP.
#include "dl_common.h"
#include "dl_kernels.h"

namespace {

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__device__ __forceinline__ void st4_bf16(bf16_t* p, float a, float b, float c, float d) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack2_bf16(a, b), pack2_bf16(c, d));
}

// one wave per row, 4 rows per 256-thread block; lanes own 4 adjacent columns per 256-column chunk
__global__ __launch_bounds__(256) void attn_softmax_fwd_kernel(const float* __restrict__ s,
                                                               const float* __restrict__ mbias,
                                                               bf16_t* __restrict__ p, float* __restrict__ lse,
                                                               long rows, long rows_per_batch, int S, float c) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;  // whole waves leave; no block-level synchronisation below
  const int lane = threadIdx.x & 63;
  const float* sr = s + row * S;
  const float* mb = mbias ? mbias + (row / rows_per_batch) * S : nullptr;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  float m = -INFINITY;
  for (int j = lane * 4; j < S; j += 256) {
    const float4 v = ld4(sr + j), b = mb ? ld4(mb + j) : z;
    m = fmaxf(m, fmaxf(fmaxf(fmaf(v.x, c, b.x), fmaf(v.y, c, b.y)), fmaxf(fmaf(v.z, c, b.z), fmaf(v.w, c, b.w))));
  }
  m = wave_max(m);
  float l = 0.f;
  for (int j = lane * 4; j < S; j += 256) {
    const float4 v = ld4(sr + j), b = mb ? ld4(mb + j) : z;
    l += exp2f(fmaf(v.x, c, b.x) - m) + exp2f(fmaf(v.y, c, b.y) - m) + exp2f(fmaf(v.z, c, b.z) - m) +
         exp2f(fmaf(v.w, c, b.w) - m);
  }
  l = wave_sum(l);
  const float mm = m + log2f(l);  // p = exp2(x - lse) = exp2(x - m) / l
  bf16_t* pr = p + row * S;
  for (int j = lane * 4; j < S; j += 256) {
    const float4 v = ld4(sr + j), b = mb ? ld4(mb + j) : z;
    st4_bf16(pr + j, exp2f(fmaf(v.x, c, b.x) - mm), exp2f(fmaf(v.y, c, b.y) - mm), exp2f(fmaf(v.z, c, b.z) - mm),
             exp2f(fmaf(v.w, c, b.w) - mm));
  }
  if (lane == 0) lse[row] = mm;
}

__global__ __launch_bounds__(256) void attn_softmax_bwd_kernel(
    const float* __restrict__ s, const float* __restrict__ dp, const float* __restrict__ mbias,
    const float* __restrict__ lse, const float* __restrict__ delta, bf16_t* __restrict__ p, bf16_t* __restrict__ ds,
    long n4, long rows_per_batch, int S, float c, float scale) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const long e = i * 4, row = e / S;
  const int j = (int)(e - row * S);
  const float4 v = ld4(s + e), g = ld4(dp + e);
  const float4 b = mbias ? ld4(mbias + (row / rows_per_batch) * S + j) : make_float4(0.f, 0.f, 0.f, 0.f);
  const float L = lse[row], d = delta[row];
  const float p0 = exp2f(fmaf(v.x, c, b.x) - L), p1 = exp2f(fmaf(v.y, c, b.y) - L);
  const float p2 = exp2f(fmaf(v.z, c, b.z) - L), p3 = exp2f(fmaf(v.w, c, b.w) - L);
  st4_bf16(p + e, p0, p1, p2, p3);
  st4_bf16(ds + e, p0 * (g.x - d) * scale, p1 * (g.y - d) * scale, p2 * (g.z - d) * scale, p3 * (g.w - d) * scale);
}

}  // namespace

int dl_attn_softmax_fwd(const float* s, const float* mbias, bf16_t* p, float* lse, long rows, int H, int S, float c,
                        hipStream_t st) {
  if (S % 4 != 0 || rows % ((long)H * S) != 0) return -1;
  const long blocks = (rows + 3) / 4;
  attn_softmax_fwd_kernel<<<dim3((unsigned)blocks), 256, 0, st>>>(s, mbias, p, lse, rows, (long)H * S, S, c);
  return 0;
}

int dl_attn_softmax_bwd(const float* s, const float* dp, const float* mbias, const float* lse, const float* delta,
                        bf16_t* p, bf16_t* ds, long rows, int H, int S, float c, float scale, hipStream_t st) {
  if (S % 4 != 0 || rows % ((long)H * S) != 0) return -1;
  const long n4 = rows * S / 4;
  attn_softmax_bwd_kernel<<<dim3((unsigned)((n4 + 255) / 256)), 256, 0, st>>>(s, dp, mbias, lse, delta, p, ds, n4,
                                                                               (long)H * S, S, c, scale);
  return 0;
}

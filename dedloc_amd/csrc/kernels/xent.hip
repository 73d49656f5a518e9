// Fused softmax cross-entropy forward+backward over bf16 logits.
// One 256-thread block per row: pass 1 online max/sum-exp (fp32), pass 2 writes
// dlogits = (softmax - onehot) * scale in place of (or beside) the logits, so the [M, V] logits
// are read twice (second read mostly L2-resident) and written once; no fp32 copy is made.
// Rows with label == ignore_index contribute 0 loss and 0 gradient.
// scale = 1 / #valid rows is computed on device (graph-capturable, no host sync).
#include "dl_common.h"
#include "dl_kernels.h"

namespace {

__global__ void count_valid_kernel(const long* __restrict__ labels, int M, int ignore_index, float* __restrict__ scale,
                                   float* __restrict__ loss_out) {
  __shared__ float scratch[16];
  float c = 0.f;
  for (int i = threadIdx.x; i < M; i += blockDim.x) c += (labels[i] != ignore_index) ? 1.f : 0.f;
  c = block_sum(c, scratch);
  if (threadIdx.x == 0) {
    scale[0] = c > 0.f ? 1.f / c : 0.f;
    scale[1] = c;
    loss_out[0] = 0.f;
  }
}

template <bool VEC>
__global__ __launch_bounds__(256) void xent_kernel(const bf16_t* logits, const long* __restrict__ labels,
                                                   bf16_t* dlogits, float* __restrict__ row_loss,
                                                   float* __restrict__ loss_out, const float* __restrict__ scale_p,
                                                   int V, long ld, int ignore_index) {
  __shared__ float red[32];
  const int row = blockIdx.x;
  const long lab = labels[row];
  const bf16_t* x = logits + row * ld;
  bf16_t* dx = dlogits + row * ld;
  const float scale = scale_p[0];
  if (lab == ignore_index) {
    if (VEC) {
      for (int i = threadIdx.x * 8; i < V; i += blockDim.x * 8) *reinterpret_cast<uint4*>(dx + i) = make_uint4(0, 0, 0, 0);
    } else {
      for (int i = threadIdx.x; i < V; i += blockDim.x) dx[i] = 0;
    }
    if (threadIdx.x == 0 && row_loss) row_loss[row] = 0.f;
    return;
  }
  // the label logit is read before any thread starts overwriting the row (dlogits may alias logits)
  const float xl = threadIdx.x == 0 ? bf2f(x[lab]) : 0.f;
  // pass 1: online max / sum
  float m = -INFINITY, s = 0.f;
  if (VEC) {
    for (int i = threadIdx.x * 8; i < V; i += blockDim.x * 8) {
      float v[8];
      load_bf16<8>(x + i, v);
      float mx = v[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) mx = fmaxf(mx, v[j]);
      const float mn = fmaxf(m, mx);
      float acc = s * __expf(m - mn);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += __expf(v[j] - mn);
      m = mn;
      s = acc;
    }
  } else {
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      const float v = bf2f(x[i]);
      const float mn = fmaxf(m, v);
      s = s * __expf(m - mn) + __expf(v - mn);
      m = mn;
    }
  }
  // combine (m, s) across the block
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float mo = __shfl_xor(m, o, 64), so = __shfl_xor(s, o, 64);
    const float mn = fmaxf(m, mo);
    s = (mn == -INFINITY) ? 0.f : s * __expf(m - mn) + so * __expf(mo - mn);
    m = mn;
  }
  if (lane == 0) { red[wid] = m; red[16 + wid] = s; }
  __syncthreads();
  float M = -INFINITY;
  for (int w = 0; w < nw; ++w) M = fmaxf(M, red[w]);
  float Ssum = 0.f;
  for (int w = 0; w < nw; ++w) Ssum += red[16 + w] * __expf(red[w] - M);
  const float lse = M + __logf(Ssum);
  const float inv = 1.f / Ssum;
  if (threadIdx.x == 0) {
    const float l = lse - xl;
    if (row_loss) row_loss[row] = l;
    atomicAdd(loss_out, l * scale);
  }
  // pass 2: gradient
  if (VEC) {
    for (int i = threadIdx.x * 8; i < V; i += blockDim.x * 8) {
      float v[8];
      load_bf16<8>(x + i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__expf(v[j] - M) * inv - ((i + j) == lab ? 1.f : 0.f)) * scale;
      store_bf16<8>(dx + i, v);
    }
  } else {
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      const float v = bf2f(x[i]);
      dx[i] = f2bf((__expf(v - M) * inv - (i == lab ? 1.f : 0.f)) * scale);
    }
  }
}

}  // namespace

// scale_buf: float[2] workspace (1/count, count); loss_out: float[1] mean loss over valid rows.
int dl_xent_fwd_bwd(const bf16_t* logits, const long* labels, bf16_t* dlogits, float* row_loss, float* loss_out,
                    float* scale_buf, int M, int V, long ld, int ignore_index, hipStream_t st) {
  count_valid_kernel<<<1, 256, 0, st>>>(labels, M, ignore_index, scale_buf, loss_out);
  if (M == 0) return 0;
  const bool vec = (V % 8 == 0) && (ld % 8 == 0);
  if (vec) xent_kernel<true><<<M, 256, 0, st>>>(logits, labels, dlogits, row_loss, loss_out, scale_buf, V, ld, ignore_index);
  else xent_kernel<false><<<M, 256, 0, st>>>(logits, labels, dlogits, row_loss, loss_out, scale_buf, V, ld, ignore_index);
  return 0;
}

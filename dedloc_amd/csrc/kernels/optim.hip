// Fused multi-tensor optimizer kernels over flat fp32 buffers.
//
// * LAMB (torch_optimizer.Lamb semantics as configured at albert/run_trainer.py:86-94, spec in
//   SURVEY.md App. F): 2 launches per optimizer step instead of ~10 torch kernels per tensor.
//   phase 1: m,v update + per-tensor partial ||p||^2 and ||u||^2 (u = m/(sqrt(v)+eps) + wd*p)
//   phase 2: trust = clamp(||p||,0,clamp)/||u|| (1 if either is 0);  p -= lr*bc*trust*u
// * LARC + SGD-momentum (apex LARC around torch SGD, sgd_collaborative.py:135-144): per-tensor
//   ||p||,||g|| in phase 1, adaptive lr + momentum update in phase 2.
// * grad-norm / clip / finite flag / accumulate — all on device, no
//   host synchronisation, so they can sit inside a captured graph.
//
// Work is split into chunks (tensor id, start, len) built once on the host for the flat layout.
#include "dl_common.h"
#include "dl_kernels.h"

namespace {

constexpr int kBlock = 256;

// ---------------------------------------------------------------- LAMB
__global__ __launch_bounds__(kBlock) void lamb_phase1(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ m, float* __restrict__ v,
                                                      const int* __restrict__ chunk_tensor, const long* __restrict__ chunk_start,
                                                      const int* __restrict__ chunk_len, const float* __restrict__ tensor_wd,
                                                      float* __restrict__ norms,  // [T][2]: ||p||^2, ||u||^2
                                                      float beta1, float beta2, float eps, float grad_scale) {
  __shared__ float scratch[16];
  const int c = blockIdx.x;
  const int t = chunk_tensor[c];
  const long s0 = chunk_start[c];
  const int len = chunk_len[c];
  const float wd = tensor_wd[t];
  float pp = 0.f, uu = 0.f;
  for (int i = threadIdx.x; i < len; i += blockDim.x) {
    const long k = s0 + i;
    const float gi = g[k] * grad_scale;
    const float mi = beta1 * m[k] + (1.f - beta1) * gi;
    const float vi = beta2 * v[k] + (1.f - beta2) * gi * gi;
    m[k] = mi;
    v[k] = vi;
    const float pi = p[k];
    const float u = mi / (sqrtf(vi) + eps) + wd * pi;
    pp += pi * pi;
    uu += u * u;
  }
  pp = block_sum(pp, scratch);
  uu = block_sum(uu, scratch + 8);
  if (threadIdx.x == 0) {
    atomicAdd(&norms[2 * t], pp);
    atomicAdd(&norms[2 * t + 1], uu);
  }
}

__global__ __launch_bounds__(kBlock) void lamb_phase2(float* __restrict__ p, const float* __restrict__ m,
                                                      const float* __restrict__ v, const int* __restrict__ chunk_tensor,
                                                      const long* __restrict__ chunk_start, const int* __restrict__ chunk_len,
                                                      const float* __restrict__ tensor_wd, const float* __restrict__ norms,
                                                      float step_size, float eps, float clamp_value,
                                                      float* __restrict__ trust_out) {
  const int c = blockIdx.x;
  const int t = chunk_tensor[c];
  const long s0 = chunk_start[c];
  const int len = chunk_len[c];
  const float wd = tensor_wd[t];
  const float wn = fminf(fmaxf(sqrtf(norms[2 * t]), 0.f), clamp_value);
  const float un = sqrtf(norms[2 * t + 1]);
  const float trust = (wn == 0.f || un == 0.f) ? 1.f : wn / un;
  if (trust_out && threadIdx.x == 0) trust_out[t] = trust;  // same value from every chunk
  const float a = step_size * trust;
  for (int i = threadIdx.x; i < len; i += blockDim.x) {
    const long k = s0 + i;
    const float pi = p[k];
    const float u = m[k] / (sqrtf(v[k]) + eps) + wd * pi;
    p[k] = pi - a * u;
  }
}

// ---------------------------------------------------------------- LARC + SGD
__global__ __launch_bounds__(kBlock) void larc_phase1(const float* __restrict__ p, const float* __restrict__ g,
                                                      const int* __restrict__ chunk_tensor, const long* __restrict__ chunk_start,
                                                      const int* __restrict__ chunk_len, float* __restrict__ norms,
                                                      float grad_scale) {
  __shared__ float scratch[16];
  const int c = blockIdx.x;
  const int t = chunk_tensor[c];
  const long s0 = chunk_start[c];
  const int len = chunk_len[c];
  float pp = 0.f, gg = 0.f;
  for (int i = threadIdx.x; i < len; i += blockDim.x) {
    const float pi = p[s0 + i], gi = g[s0 + i] * grad_scale;
    pp += pi * pi;
    gg += gi * gi;
  }
  pp = block_sum(pp, scratch);
  gg = block_sum(gg, scratch + 8);
  if (threadIdx.x == 0) {
    atomicAdd(&norms[2 * t], pp);
    atomicAdd(&norms[2 * t + 1], gg);
  }
}

__global__ __launch_bounds__(kBlock) void larc_phase2(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ buf, const int* __restrict__ chunk_tensor,
                                                      const long* __restrict__ chunk_start, const int* __restrict__ chunk_len,
                                                      const float* __restrict__ tensor_wd, const float* __restrict__ norms,
                                                      float lr, float momentum, float trust_coef, float eps, int clip,
                                                      int first_step, float grad_scale) {
  const int c = blockIdx.x;
  const int t = chunk_tensor[c];
  const long s0 = chunk_start[c];
  const int len = chunk_len[c];
  const float wd = tensor_wd[t];
  const float pn = sqrtf(norms[2 * t]), gn = sqrtf(norms[2 * t + 1]);
  float a = 1.f;
  if (pn != 0.f && gn != 0.f) {
    a = trust_coef * pn / (gn + pn * wd + eps);
    if (clip) a = fminf(a / lr, 1.f);
  }
  for (int i = threadIdx.x; i < len; i += blockDim.x) {
    const long k = s0 + i;
    const float pi = p[k];
    const float d = (g[k] * grad_scale + wd * pi) * a;
    const float b = first_step ? d : momentum * buf[k] + d;
    buf[k] = b;
    p[k] = pi - lr * b;
  }
}

// ---------------------------------------------------------------- norms / clip / accumulate
__global__ __launch_bounds__(kBlock) void sumsq_kernel(const float* __restrict__ x, size_t n, float* __restrict__ part) {
  __shared__ float scratch[16];
  float s = 0.f;
  const size_t nvec = n / 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    float4 v = reinterpret_cast<const float4*>(x)[i];
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (size_t i = nvec * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s += x[i] * x[i];
  s = block_sum(s, scratch);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// Reads the partials, computes the global norm on every block (cheap) and scales x in place by
// min(1, max_norm / (norm + 1e-6)).  out[0] = norm, out[1] = finite flag (1.0 if finite).
__global__ __launch_bounds__(kBlock) void clip_kernel(float* __restrict__ x, size_t n, const float* __restrict__ part,
                                                      int nparts, float max_norm, float* __restrict__ out,
                                                      int nout) {
  __shared__ float scratch[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) s += part[i];
  s = block_sum(s, scratch);
  const float norm = sqrtf(s);
  const bool finite = isfinite(norm);
  if (blockIdx.x == 0 && threadIdx.x == 0 && out) {
    out[0] = norm;
    out[1] = finite ? 1.f : 0.f;
    if (nout > 2) out[2] = finite ? 0.f : 1.f;  // the "drop this step" flag for axpby(flag=...)
  }
  if (max_norm <= 0.f || !finite) return;
  const float coef = max_norm / (norm + 1e-6f);
  if (coef >= 1.f) return;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) x[i] *= coef;
}

// y = a*y + b*x  (fp32).  With `flag` (device scalar, e.g. the finite flag of dl_grad_norm_clip)
// the update is skipped entirely when *flag == 0, so a non-finite step never reaches y.
__global__ __launch_bounds__(kBlock) void axpby_kernel(float* __restrict__ y, const float* __restrict__ x, size_t n,
                                                       float a, float b, const float* __restrict__ flag,
                                                       const float* __restrict__ bdiv) {
  if (flag != nullptr && flag[0] == 0.f) return;
  if (bdiv != nullptr) b /= fmaxf(1.f, bdiv[0]);  // a device-side count (finite micro-steps)
  const size_t nvec = n / 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    float4 yv = reinterpret_cast<float4*>(y)[i];
    const float4 xv = reinterpret_cast<const float4*>(x)[i];
    // a == 0 / b == 0 drop the term entirely (so NaN * 0 never leaks: used to clear bad grads)
    yv.x = (a != 0.f ? a * yv.x : 0.f) + (b != 0.f ? b * xv.x : 0.f);
    yv.y = (a != 0.f ? a * yv.y : 0.f) + (b != 0.f ? b * xv.y : 0.f);
    yv.z = (a != 0.f ? a * yv.z : 0.f) + (b != 0.f ? b * xv.z : 0.f);
    yv.w = (a != 0.f ? a * yv.w : 0.f) + (b != 0.f ? b * xv.w : 0.f);
    reinterpret_cast<float4*>(y)[i] = yv;
  }
  for (size_t i = nvec * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = (a != 0.f ? a * y[i] : 0.f) + (b != 0.f ? b * x[i] : 0.f);
}

// x *= *s (bf16, in place) — skipped entirely when the device scalar is exactly 1 (the gradient of a
// loss that is backpropagated with the default ones seed: the cross-entropy's saved d(loss)/d(logits)
// needs no 2.4 GB read-modify-write pass then)
__global__ __launch_bounds__(kBlock) void scale_by_kernel(bf16_t* __restrict__ x, size_t n, const float* __restrict__ s) {
  const float f = s[0];
  if (f == 1.f) return;
  const size_t nvec = n / 8;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    float v[8];
    load_bf16<8>(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= f;
    store_bf16<8>(x + i * 8, v);
  }
  for (size_t i = nvec * 8 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    x[i] = f2bf(bf2f(x[i]) * f);
}

// out += sum_j slabs[j * n : (j + 1) * n]   (split-K partial reduction, fp32, float4 lanes); ZERO:
// each slab element is cleared once read (gradient buffers that are accumulated into again)
template <bool ZERO>
__global__ __launch_bounds__(kBlock) void sum_slabs_kernel(float* __restrict__ out, float* __restrict__ slabs,
                                                           int s, size_t n) {
  const size_t nvec = n / 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    float4 acc = reinterpret_cast<float4*>(out)[i];
    for (int j = 0; j < s; ++j) {
      float4* sp = reinterpret_cast<float4*>(slabs + (size_t)j * n) + i;
      const float4 v = *sp;
      if (ZERO) *sp = float4{0.f, 0.f, 0.f, 0.f};
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    reinterpret_cast<float4*>(out)[i] = acc;
  }
  for (size_t i = nvec * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    for (int j = 0; j < s; ++j) {
      out[i] += slabs[(size_t)j * n + i];
      if (ZERO) slabs[(size_t)j * n + i] = 0.f;
    }
}

inline int grid_for(size_t n) {
  size_t g = (n / 4 + kBlock - 1) / kBlock;
  return (int)(g < 2048 ? (g == 0 ? 1 : g) : 2048);
}

}  // namespace

int dl_lamb_step(float* p, const float* g, float* m, float* v, const int* chunk_tensor, const long* chunk_start,
                 const int* chunk_len, int nchunks, const float* tensor_wd, float* norms, int ntensors, float beta1,
                 float beta2, float eps, float step_size, float clamp_value, float grad_scale, float* trust_out,
                 hipStream_t st) {
  DL_HIP_CHECK(hipMemsetAsync(norms, 0, sizeof(float) * 2 * ntensors, st));
  lamb_phase1<<<nchunks, kBlock, 0, st>>>(p, g, m, v, chunk_tensor, chunk_start, chunk_len, tensor_wd, norms, beta1,
                                          beta2, eps, grad_scale);
  lamb_phase2<<<nchunks, kBlock, 0, st>>>(p, m, v, chunk_tensor, chunk_start, chunk_len, tensor_wd, norms, step_size,
                                          eps, clamp_value, trust_out);
  return 0;
}

int dl_larc_sgd_step(float* p, const float* g, float* buf, const int* chunk_tensor, const long* chunk_start,
                     const int* chunk_len, int nchunks, const float* tensor_wd, float* norms, int ntensors, float lr,
                     float momentum, float trust_coef, float eps, int clip, int first_step, float grad_scale,
                     hipStream_t st) {
  DL_HIP_CHECK(hipMemsetAsync(norms, 0, sizeof(float) * 2 * ntensors, st));
  larc_phase1<<<nchunks, kBlock, 0, st>>>(p, g, chunk_tensor, chunk_start, chunk_len, norms, grad_scale);
  larc_phase2<<<nchunks, kBlock, 0, st>>>(p, g, buf, chunk_tensor, chunk_start, chunk_len, tensor_wd, norms, lr,
                                          momentum, trust_coef, eps, clip, first_step, grad_scale);
  return 0;
}

int dl_grad_norm_clip(float* x, size_t n, float max_norm, float* part, int nparts, float* out, int nout,
                      hipStream_t st) {
  sumsq_kernel<<<nparts, kBlock, 0, st>>>(x, n, part);
  // no clipping: one block publishes the norm and flags
  clip_kernel<<<max_norm > 0.f ? grid_for(n) : 1, kBlock, 0, st>>>(x, n, part, nparts, max_norm, out, nout);
  return 0;
}

int dl_sum_slabs(float* out, const float* slabs, int s, size_t n, hipStream_t st) {
  sum_slabs_kernel<false><<<grid_for(n), kBlock, 0, st>>>(out, const_cast<float*>(slabs), s, n);
  return 0;
}

int dl_add_slabs_zero(float* out, float* slabs, int s, size_t n, hipStream_t st) {
  sum_slabs_kernel<true><<<grid_for(n), kBlock, 0, st>>>(out, slabs, s, n);
  return 0;
}

int dl_scale_by(bf16_t* x, size_t n, const float* s, hipStream_t st) {
  if (n == 0) return 0;
  scale_by_kernel<<<grid_for(n / 8 + 1), kBlock, 0, st>>>(x, n, s);
  return 0;
}

int dl_axpby(float* y, const float* x, size_t n, float a, float b, const float* flag, const float* bdiv,
             hipStream_t st) {
  axpby_kernel<<<grid_for(n), kBlock, 0, st>>>(y, x, n, a, b, flag, bdiv);
  return 0;
}

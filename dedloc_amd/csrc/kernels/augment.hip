// SwAV multi-crop augmentation on the GPU (reference: vissl ssl_transforms img_pil_to_multicrop.py,
// img_pil_color_distortion.py, img_pil_gaussian_blur.py).  The reference runs
// PIL transforms in DataLoader worker processes; here the whole pipeline is four launches per crop
// resolution over a device-resident image pool, with every random draw made on the host into a
// [nb, 20] parameter table (data/multicrop.py:sample_params):
//
//   sample   RandomResizedCrop + flip as a bilinear resample (grid_sample semantics: align_corners
//            false, border padding) of the planar fp32 source, plus a per-image luminance sum
//   color    brightness, contrast (mean luminance), saturation, hue (one 3x3 YIQ rotation matrix),
//            clamp, p-applied, then p-grayscale — in place
//   hblur    per-image Gaussian (sigma, identity when 0) along x, reflect padding
//   vblur    the same along y, then Normalize(mean, std) and the bf16 NHWC (channels-last) store
//
// Parameter row: 0 src image, 1-4 affine (ax, cx, ay, cy), 5 brightness, 6 contrast, 7 saturation,
// 8 colour applied, 9 grayscale, 10-18 hue matrix (row-major), 19 blur sigma.
#include "dl_common.h"
#include "dl_kernels.h"

namespace {

constexpr int NP = 20;
constexpr int MAX_RAD = 16;

__device__ __forceinline__ float lum(float r, float g, float b) { return 0.299f * r + 0.587f * g + 0.114f * b; }

__global__ __launch_bounds__(256) void mc_sample_kernel(const float* __restrict__ pool, int P, int Hp, int Wp,
                                                         const float* __restrict__ prm, int S,
                                                         float* __restrict__ out, float* __restrict__ lumsum) {
  __shared__ float red[16];
  const int i = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const float* pr = prm + (size_t)i * NP;
  const long plane = (long)Hp * Wp;
  const int si = min(max((int)pr[0], 0), P - 1);  // clamped: a bad table row can never read out of bounds
  const float* src = pool + (long)si * 3 * plane;
  float l = 0.f;
  if (p < S * S) {
    const int yy = p / S, xx = p - yy * S;
    const float xn = (2.f * xx + 1.f) / S - 1.f, yn = (2.f * yy + 1.f) / S - 1.f;
    const float xs = pr[1] * xn + pr[2], ys = pr[3] * yn + pr[4];
    float ix = ((xs + 1.f) * Wp - 1.f) * 0.5f, iy = ((ys + 1.f) * Hp - 1.f) * 0.5f;
    ix = fminf(fmaxf(ix, 0.f), (float)(Wp - 1));
    iy = fminf(fmaxf(iy, 0.f), (float)(Hp - 1));
    const int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
    const int x1 = min(x0 + 1, Wp - 1), y1 = min(y0 + 1, Hp - 1);
    const float fx = ix - x0, fy = iy - y0;
    const float w00 = (1.f - fx) * (1.f - fy), w01 = fx * (1.f - fy), w10 = (1.f - fx) * fy, w11 = fx * fy;
    float v[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float* s = src + c * plane;
      v[c] = w00 * s[y0 * Wp + x0] + w01 * s[y0 * Wp + x1] + w10 * s[y1 * Wp + x0] + w11 * s[y1 * Wp + x1];
      out[((size_t)i * 3 + c) * S * S + p] = v[c];
    }
    l = lum(v[0], v[1], v[2]);
  }
  l = block_sum(l, red);
  if (threadIdx.x == 0) atomicAdd(lumsum + i, l);
}

__global__ __launch_bounds__(256) void mc_color_kernel(float* __restrict__ x, int S, const float* __restrict__ prm,
                                                        const float* __restrict__ lumsum) {
  const int i = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= S * S) return;
  const float* pr = prm + (size_t)i * NP;
  const size_t HW = (size_t)S * S;
  float* px = x + (size_t)i * 3 * HW + p;
  float r = px[0], g = px[HW], b = px[2 * HW];
  if (pr[8] != 0.f) {
    const float br = pr[5], ct = pr[6], sat = pr[7];
    const float gm = br * lumsum[i] / (float)HW;
    float y0 = (r * br - gm) * ct + gm, y1 = (g * br - gm) * ct + gm, y2 = (b * br - gm) * ct + gm;
    const float l = lum(y0, y1, y2);
    y0 = (y0 - l) * sat + l;
    y1 = (y1 - l) * sat + l;
    y2 = (y2 - l) * sat + l;
    const float* M = pr + 10;
    r = fminf(fmaxf(M[0] * y0 + M[1] * y1 + M[2] * y2, 0.f), 1.f);
    g = fminf(fmaxf(M[3] * y0 + M[4] * y1 + M[5] * y2, 0.f), 1.f);
    b = fminf(fmaxf(M[6] * y0 + M[7] * y1 + M[8] * y2, 0.f), 1.f);
  }
  if (pr[9] != 0.f) r = g = b = lum(r, g, b);
  px[0] = r;
  px[HW] = g;
  px[2 * HW] = b;
}

__device__ __forceinline__ int reflect(int j, int n) { return j < 0 ? -j : (j >= n ? 2 * (n - 1) - j : j); }

// Gaussian taps for one image: w[k] = exp(-k^2 / 2 sigma^2) normalised over [-rad, rad]; sigma <= 0
// is the identity kernel (the p=0.5 "no blur" draw; the blur kernels copy those images directly)
__device__ __forceinline__ void blur_taps(float sigma, int rad, float* w) {
  if (sigma <= 0.f) {
    for (int k = 0; k <= 2 * rad; ++k) w[k] = k == rad ? 1.f : 0.f;
    return;
  }
  const float a = -0.5f / (sigma * sigma);
  float s = 0.f;
  for (int k = 0; k <= 2 * rad; ++k) {
    const float d = (float)(k - rad);
    w[k] = __expf(a * d * d);
    s += w[k];
  }
  const float inv = 1.f / s;
  for (int k = 0; k <= 2 * rad; ++k) w[k] *= inv;
}

__global__ __launch_bounds__(256) void mc_hblur_kernel(const float* __restrict__ x, float* __restrict__ y, int S,
                                                        const float* __restrict__ prm, int rad) {
  __shared__ float w[2 * MAX_RAD + 1];
  const int i = blockIdx.y;
  const bool blur = prm[(size_t)i * NP + 19] > 0.f;  // uniform per block: the p=0.5 "no blur" draw copies
  if (blur && threadIdx.x == 0) blur_taps(prm[(size_t)i * NP + 19], rad, w);
  __syncthreads();
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= S * S) return;
  const int yy = p / S, xx = p - yy * S;
  const size_t HW = (size_t)S * S;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float* row = x + ((size_t)i * 3 + c) * HW + (size_t)yy * S;
    float acc = 0.f;
    if (blur) {
      for (int k = -rad; k <= rad; ++k) acc += w[k + rad] * row[reflect(xx + k, S)];
    } else {
      acc = row[xx];
    }
    y[((size_t)i * 3 + c) * HW + p] = acc;
  }
}

__global__ __launch_bounds__(256) void mc_vblur_norm_kernel(const float* __restrict__ x, bf16_t* __restrict__ out,
                                                             int S, const float* __restrict__ prm, int rad,
                                                             float m0, float m1, float m2, float is0, float is1,
                                                             float is2) {
  __shared__ float w[2 * MAX_RAD + 1];
  const int i = blockIdx.y;
  const bool blur = prm[(size_t)i * NP + 19] > 0.f;
  if (blur && threadIdx.x == 0) blur_taps(prm[(size_t)i * NP + 19], rad, w);
  __syncthreads();
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= S * S) return;
  const int yy = p / S, xx = p - yy * S;
  const size_t HW = (size_t)S * S;
  const float mean[3] = {m0, m1, m2}, istd[3] = {is0, is1, is2};
  bf16_t* o = out + ((size_t)i * HW + p) * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float* col = x + ((size_t)i * 3 + c) * HW + xx;
    float acc = 0.f;
    if (blur) {
      for (int k = -rad; k <= rad; ++k) acc += w[k + rad] * col[(size_t)reflect(yy + k, S) * S];
    } else {
      acc = col[(size_t)yy * S];
    }
    o[c] = f2bf((acc - mean[c]) * istd[c]);
  }
}

}  // namespace

int dl_multicrop(const float* pool, int P, int Hp, int Wp, const float* params, int nb, int S, int rad, const float* mean,
                 const float* stdv, float* ws, bf16_t* out, hipStream_t st) {
  if (rad < 0 || rad > MAX_RAD || rad >= S || nb <= 0) return -1;
  const size_t img = (size_t)nb * 3 * S * S;
  float* a = ws;
  float* b = ws + img;
  float* lumsum = ws + 2 * img;
  DL_HIP_CHECK(hipMemsetAsync(lumsum, 0, sizeof(float) * nb, st));
  const dim3 grid((S * S + 255) / 256, nb);
  mc_sample_kernel<<<grid, 256, 0, st>>>(pool, P, Hp, Wp, params, S, a, lumsum);
  mc_color_kernel<<<grid, 256, 0, st>>>(a, S, params, lumsum);
  mc_hblur_kernel<<<grid, 256, 0, st>>>(a, b, S, params, rad);
  mc_vblur_norm_kernel<<<grid, 256, 0, st>>>(b, out, S, params, rad, mean[0], mean[1], mean[2], 1.f / stdv[0],
                                             1.f / stdv[1], 1.f / stdv[2]);
  return 0;
}

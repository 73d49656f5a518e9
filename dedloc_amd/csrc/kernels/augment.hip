// SwAV multi-crop augmentation on the GPU (reference: vissl ssl_transforms img_pil_to_multicrop.py,
// img_pil_color_distortion.py, img_pil_gaussian_blur.py).  The reference runs
// PIL transforms in DataLoader worker processes; here the whole pipeline is two launches per crop
// resolution over a device-resident image pool, with every random draw made on the host into a
// [nb, 20] parameter table (data/multicrop.py:sample_params):
//
//   sample   RandomResizedCrop + flip as a bilinear resample (grid_sample semantics: align_corners
//            false, border padding) of the planar fp32 source, plus a per-image luminance sum
//   color_blur_norm  per band of output rows, through LDS: brightness, contrast (mean luminance),
//            saturation, hue (one 3x3 YIQ rotation matrix), clamp, p-applied, then p-grayscale;
//            the per-image Gaussian (sigma, none when 0) along x and along y, reflect padding; then
//            Normalize(mean, std) and the bf16 NHWC (channels-last) store
//
// Parameter row: 0 src image, 1-4 affine (ax, cx, ay, cy), 5 brightness, 6 contrast, 7 saturation,
// 8 colour applied, 9 grayscale, 10-18 hue matrix (row-major), 19 blur sigma.
#include "dl_common.h"
#include "dl_kernels.h"

namespace {

constexpr int NP = 20;
constexpr int MAX_RAD = 16;

__device__ __forceinline__ float lum(float r, float g, float b) { return 0.299f * r + 0.587f * g + 0.114f * b; }

// a / b for 0 <= a < 2^24 through the float reciprocal rb = 1 / b (+-1 correction): ~6 VALU against
// ~20 for an integer division by a run-time divisor
__device__ __forceinline__ int fdiv(int a, int b, float rb) {
  int q = (int)((float)a * rb);
  const int r = a - q * b;
  q += (r >= b) - (r < 0);
  return q;
}

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
    const float rS = 1.f / (float)S;
    const int yy = fdiv(p, S, rS), xx = p - yy * S;
    const float xn = (2.f * xx + 1.f) * rS - 1.f, yn = (2.f * yy + 1.f) * rS - 1.f;
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

__device__ __forceinline__ int reflect(int j, int n) { return j < 0 ? -j : (j >= n ? 2 * (n - 1) - j : j); }

// Colour distortion + separable Gaussian blur + Normalize + the bf16 NHWC store, for a band of T
// output rows of one image (grid: bands x images).  The band and its 2*rad halo rows (reflected at
// the image edges) are read once from the sampled fp32 planes, colour-transformed and kept in LDS as
// fp16 (values in [0, 1], 11-bit precision, far below the bf16 output's); the horizontal pass goes
// into a second LDS image, the vertical pass and the normalisation write the output.  Replaces four
// launches (colour in place, hblur and vblur through HBM, one global tap read per weight).
// `sigma` <= 0 (the p=0.5 "no blur" draw): no halo, no taps.
__global__ __launch_bounds__(256) void mc_color_blur_norm_kernel(const float* __restrict__ a, bf16_t* __restrict__ out,
                                                                  int S, int T, const float* __restrict__ prm,
                                                                  const float* __restrict__ lumsum, int rad, float m0,
                                                                  float m1, float m2, float is0, float is1,
                                                                  float is2) {
  extern __shared__ __align__(16) _Float16 img[];  // [2][3][T + 2 rad][S]
  __shared__ float w[2 * MAX_RAD + 1];
  const int i = blockIdx.y;
  const int y0 = blockIdx.x * T;
  const int nout = min(T, S - y0);
  const float* pr = prm + (size_t)i * NP;
  const float sigma = pr[19];
  const bool blur = sigma > 0.f;  // uniform per block
  const int hr = blur ? rad : 0;
  const int rows = nout + 2 * hr;
  const int plane = (T + 2 * rad) * S;
  _Float16* b1 = img;
  _Float16* b2 = img + 3 * plane;
  if (blur && threadIdx.x <= 2 * rad) {
    const float d = (float)((int)threadIdx.x - rad);
    w[threadIdx.x] = __expf(-0.5f / (sigma * sigma) * d * d);
  }
  // colour: brightness / contrast (about the brightness-scaled mean luminance) / saturation / hue,
  // clamp, p-applied; then p-grayscale
  const bool col = pr[8] != 0.f, gray = pr[9] != 0.f;
  const float br = pr[5], ct = pr[6], sat = pr[7];
  const size_t HW = (size_t)S * S;
  const float gm = br * lumsum[i] / (float)HW;
  const float* M = pr + 10;
  const float* src = a + (size_t)i * 3 * HW;
  const float rS = 1.f / (float)S;
  for (int idx = threadIdx.x; idx < rows * S; idx += blockDim.x) {
    const int r = fdiv(idx, S, rS), x = idx - r * S;
    const size_t o = (size_t)reflect(y0 - hr + r, S) * S + x;
    float R = src[o], G = src[HW + o], B = src[2 * HW + o];
    if (col) {
      float c0 = (R * br - gm) * ct + gm, c1 = (G * br - gm) * ct + gm, c2 = (B * br - gm) * ct + gm;
      const float l = lum(c0, c1, c2);
      c0 = (c0 - l) * sat + l;
      c1 = (c1 - l) * sat + l;
      c2 = (c2 - l) * sat + l;
      R = fminf(fmaxf(M[0] * c0 + M[1] * c1 + M[2] * c2, 0.f), 1.f);
      G = fminf(fmaxf(M[3] * c0 + M[4] * c1 + M[5] * c2, 0.f), 1.f);
      B = fminf(fmaxf(M[6] * c0 + M[7] * c1 + M[8] * c2, 0.f), 1.f);
    }
    if (gray) R = G = B = lum(R, G, B);
    b1[r * S + x] = (_Float16)R;
    b1[plane + r * S + x] = (_Float16)G;
    b1[2 * plane + r * S + x] = (_Float16)B;
  }
  __syncthreads();
  const float mean[3] = {m0, m1, m2}, istd[3] = {is0, is1, is2};
  bf16_t* dst = out + ((size_t)i * HW + (size_t)y0 * S) * 3;
  if (!blur) {
    for (int idx = threadIdx.x; idx < nout * S; idx += blockDim.x) {
#pragma unroll
      for (int c = 0; c < 3; ++c) dst[(size_t)idx * 3 + c] = f2bf(((float)b1[c * plane + idx] - mean[c]) * istd[c]);
    }
    return;
  }
  float ws = 0.f;
  for (int k = 0; k <= 2 * rad; ++k) ws += w[k];
  const float inv = 1.f / ws;
  // horizontal pass (reflect at the row ends) into the second image
  for (int idx = threadIdx.x; idx < rows * S; idx += blockDim.x) {
    const int r = fdiv(idx, S, rS), x = idx - r * S;
    float acc[3] = {0.f, 0.f, 0.f};
    for (int k = 0; k <= 2 * rad; ++k) {
      const int xs = r * S + reflect(x + k - rad, S);
#pragma unroll
      for (int c = 0; c < 3; ++c) acc[c] += w[k] * (float)b1[c * plane + xs];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) b2[c * plane + idx] = (_Float16)(acc[c] * inv);
  }
  __syncthreads();
  // vertical pass over the halo'd rows (already reflected), Normalize, NHWC bf16 store
  for (int idx = threadIdx.x; idx < nout * S; idx += blockDim.x) {
    float acc[3] = {0.f, 0.f, 0.f};
    for (int k = 0; k <= 2 * rad; ++k) {
#pragma unroll
      for (int c = 0; c < 3; ++c) acc[c] += w[k] * (float)b2[c * plane + idx + k * S];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) dst[(size_t)idx * 3 + c] = f2bf((acc[c] * inv - mean[c]) * istd[c]);
  }
}

}  // namespace

int dl_multicrop(const float* pool, int P, int Hp, int Wp, const float* params, int nb, int S, int rad, const float* mean,
                 const float* stdv, float* ws, bf16_t* out, hipStream_t st) {
  if (rad < 0 || rad > MAX_RAD || rad >= S || nb <= 0) return -1;
  const size_t img = (size_t)nb * 3 * S * S;
  float* a = ws;
  float* lumsum = ws + img;
  // band height: the two fp16 band images within ~56 KiB of LDS (a light co-tenant of the trunk's
  // kernels, which run concurrently with the data prefetch)
  const int T = std::max(1, std::min(32, (56 * 1024) / (12 * S) - 2 * rad));
  const size_t lds = sizeof(_Float16) * 2 * 3 * (size_t)(T + 2 * rad) * S;
  if (lds > 150 * 1024) return -1;
  DL_HIP_CHECK(hipMemsetAsync(lumsum, 0, sizeof(float) * nb, st));
  mc_sample_kernel<<<dim3((S * S + 255) / 256, nb), 256, 0, st>>>(pool, P, Hp, Wp, params, S, a, lumsum);
  static bool attr = false;
  if (!attr) {
    DL_HIP_CHECK(hipFuncSetAttribute((const void*)mc_color_blur_norm_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
    attr = true;
  }
  mc_color_blur_norm_kernel<<<dim3((S + T - 1) / T, nb), 256, lds, st>>>(
      a, out, S, T, params, lumsum, rad, mean[0], mean[1], mean[2], 1.f / stdv[0], 1.f / stdv[1], 1.f / stdv[2]);
  return 0;
}

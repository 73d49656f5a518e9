// Training-mode BatchNorm for channels-last bf16 activations, with the ResNet epilogues fused:
//   y = act(BN(x) [+ residual]),  act in {identity, ReLU}
// (SwAV ResNet-50 Bottleneck bn1+relu, bn2+relu, bn3+residual+relu, downsample bn).
//
// Layout: x is [R, C] with C contiguous (NHWC, R = N*H*W).  A thread owns 8 consecutive channels
// (one 16-byte vector); CV = C/8 vectors per row must divide 256 (C in {64,...,2048}, all ResNet-50
// widths), so a 256-thread block covers 256/CV rows per iteration with fully coalesced loads.
//
// forward : (memset) stats  -> per-channel sum / sum of squares (block partials in LDS, one
//           lane-contiguous atomic per channel per block), normalize -> every block rebuilds
//           scale/shift for all C channels in LDS from the sums, block 0 also writes mean/rstd and
//           updates the running statistics (momentum, unbiased variance like torch).
// backward: (memset) stats  -> sum g and sum g*xhat (g = dy masked by y > 0 when ReLU was fused),
//           dx       -> dx = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)); d(residual) = g;
//                       block 0 writes dgamma = sum g*xhat and dbeta = sum g.
// MIOpen's path for the same work is 4 kernels forward + 3 backward + separate ReLU / add kernels.
//
// Statistics groups: the rows may be G equal consecutive groups with SEPARATE batch statistics
// (gridDim.y = group).  SwAV runs all crops of one resolution through the trunk as one batch but
// normalises every crop with its own statistics — exactly the reference's SINGLE_PASS_EVERY_CROP
// semantics (one trunk pass per crop) with 8x fewer, 6x larger kernels; the running statistics
// take the G momentum updates in crop order.
#include <cstdlib>

#include "dl_common.h"
#include "dl_kernels.h"

namespace {

constexpr int kThreads = 256;
// 16-byte vectors (rows) in flight per thread in the streaming passes (apply, backward statistics,
// dx): template parameter BN_U = 2.  4 needed 116-190 VGPRs and halved the resident waves: SwAV
// iteration 2186-2191 vs 2202-2212 samples/s with 2 (same box; the 4 form was removed in round 4)

__device__ __forceinline__ void ld8(const bf16_t* p, float (&v)[8]) { load_bf16<8>(p, v); }

// ---------------------------------------------------------------------------------- forward stats
__global__ __launch_bounds__(kThreads) void bn_stats_kernel(const bf16_t* __restrict__ x, float* __restrict__ sums,
                                                            long R, int C, long rpb) {
  __shared__ float red[kThreads * 16];
  const int CV = C >> 3, rpi = kThreads / CV;
  const int cv = threadIdx.x % CV, rsub = threadIdx.x / CV;
  x += (long)blockIdx.y * R * C;  // R = rows per statistics group
  sums += (long)blockIdx.y * 2 * C;
  const long r0 = blockIdx.x * rpb, r1 = min(R, r0 + rpb);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  long r = r0 + rsub;
  for (; r + 3 * rpi < r1; r += 4 * rpi) {  // four 16-byte loads in flight per thread
    float v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) ld8(x + (r + u * rpi) * C + cv * 8, v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += v[u][j];
        q[j] = fmaf(v[u][j], v[u][j], q[j]);
      }
  }
  for (; r < r1; r += rpi) {
    float v[8];
    ld8(x + r * C + cv * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] += v[j];
      q[j] = fmaf(v[j], v[j], q[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[threadIdx.x * 16 + j] = s[j];
    red[threadIdx.x * 16 + 8 + j] = q[j];
  }
  __syncthreads();
  // threads [0, 2C) each sum one (channel, moment) over the rpi row-lanes, then one atomic
  for (int i = threadIdx.x; i < 2 * C; i += kThreads) {
    const int moment = i / C, c = i % C, v = c >> 3, j = c & 7;
    float a = 0.f;
    for (int k = 0; k < rpi; ++k) a += red[(k * CV + v) * 16 + moment * 8 + j];
    atomicAdd(&sums[i], a);
  }
}

// ---------------------------------------------------------------------------------- forward apply
// HR / RL: residual input / ReLU, template flags (as run-time flags they were per-element selects)
template <int BN_U, bool HR, bool RL>
__global__ __launch_bounds__(kThreads) void bn_apply_kernel(const bf16_t* __restrict__ x,
                                                            const bf16_t* __restrict__ res, bf16_t* __restrict__ y,
                                                            const float* __restrict__ sums,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float* __restrict__ mean_out,
                                                            float* __restrict__ rstd_out, float* __restrict__ run_mean,
                                                            float* __restrict__ run_var, long R, int C, float eps,
                                                            float momentum, int relu) {
  __shared__ float sc[2048], sh[2048];
  const int grp = blockIdx.y, G = gridDim.y;
  const float invR = 1.f / (float)R;
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const float* sg = sums + (long)grp * 2 * C;
    const float mean = sg[c] * invR;
    const float var = fmaxf(sg[C + c] * invR - mean * mean, 0.f);
    const float rstd = rsqrtf(var + eps);
    const float g = gamma[c] * rstd;
    sc[c] = g;
    sh[c] = beta[c] - mean * g;
    if (blockIdx.x == 0) {
      mean_out[(long)grp * C + c] = mean;
      rstd_out[(long)grp * C + c] = rstd;
    }
    if (blockIdx.x == 0 && grp == 0 && run_mean != nullptr) {  // G momentum updates, in group order
      float rm = run_mean[c], rv = run_var[c];
      for (int k = 0; k < G; ++k) {
        const float* sk = sums + (long)k * 2 * C;
        const float mk = sk[c] * invR;
        const float vk = fmaxf(sk[C + c] * invR - mk * mk, 0.f);
        rm = (1.f - momentum) * rm + momentum * mk;
        rv = (1.f - momentum) * rv + momentum * vk * ((float)R / (float)max(R - 1, 1L));
      }
      run_mean[c] = rm;
      run_var[c] = rv;
    }
  }
  __syncthreads();
  const int CV = C >> 3;
  const long nvec = R * CV, base = (long)grp * R * C;
  x += base;
  y += base;
  if (HR) res += base;
  // CV is a power of two (bn_shape_ok), so the channel of vector i is i & (CV - 1); two vectors per
  // iteration keep two independent load chains in flight per thread
  const long stride = (long)gridDim.x * kThreads;
  long i = blockIdx.x * (long)kThreads + threadIdx.x;
  for (; i + (BN_U - 1) * stride < nvec; i += BN_U * stride) {
    float v[BN_U][8], rr[BN_U][8];
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      ld8(x + (i + u * stride) * 8, v[u]);
      if (HR) ld8(res + (i + u * stride) * 8, rr[u]);
    }
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const int c0 = ((int)(i + u * stride) & (CV - 1)) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float o = fmaf(v[u][j], sc[c0 + j], sh[c0 + j]);
        if (HR) o += rr[u][j];
        v[u][j] = RL && o < 0.f ? 0.f : o;  // NaN passes, as torch.relu
      }
      store_bf16<8>(y + (i + u * stride) * 8, v[u]);
    }
  }
  for (; i < nvec; i += stride) {
    const int c0 = ((int)i & (CV - 1)) * 8;
    float v[8];
    ld8(x + i * 8, v);
    float rr[8];
    if (HR) ld8(res + i * 8, rr);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float o = fmaf(v[j], sc[c0 + j], sh[c0 + j]);
      if (HR) o += rr[j];
      v[j] = RL && o < 0.f ? 0.f : o;
    }
    store_bf16<8>(y + i * 8, v);
  }
}

// ---------------------------------------------------------------------------------- backward stats
// ReLU mask without reading y: for a BatchNorm+ReLU with no residual branch, y > 0 exactly when the
// pre-activation fmaf(x, gamma*rstd, beta - mean*gamma*rstd) > 0 — the forward's own expression over
// the saved mean / rstd — so with `beta` given the backward passes read dy and x only (2 of 3
// streams; with a residual the mask depends on it and y is read).
// MK: ReLU mask source, template flag — 0 none, 1 from x (beta given), 2 from y
template <int BN_U, int MK>
__global__ __launch_bounds__(kThreads) void bn_bwd_stats_kernel(const bf16_t* __restrict__ dy,
                                                                const bf16_t* __restrict__ y,
                                                                const bf16_t* __restrict__ x,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ rstd, float* __restrict__ sums,
                                                                long R, int C, long rpb, int relu,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta,
                                                                bf16_t* gout) {
  __shared__ float red[kThreads * 16];
  const int CV = C >> 3, rpi = kThreads / CV;
  const int cv = threadIdx.x % CV, rsub = threadIdx.x / CV;
  const long base = (long)blockIdx.y * R * C;
  dy += base;
  x += base;
  if (y != nullptr) y += base;
  if (gout != nullptr) gout += base;  // optional: the masked gradient written back (may alias dy)
  mean += (long)blockIdx.y * C;
  rstd += (long)blockIdx.y * C;
  sums += (long)blockIdx.y * 2 * C;
  const long r0 = blockIdx.x * rpb, r1 = min(R, r0 + rpb);
  float mu[8], rs[8], sc[8], sh[8];  // mu: -mean * rstd (xhat = x * rs + mu)
  constexpr bool xmask = MK == 1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float m = mean[cv * 8 + j];
    rs[j] = rstd[cv * 8 + j];
    mu[j] = -m * rs[j];
    if (xmask) {
      sc[j] = gamma[cv * 8 + j] * rs[j];
      sh[j] = beta[cv * 8 + j] - m * sc[j];
    }
  }
  float sg[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, sgx[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  long r = r0 + rsub;
  for (; r + (BN_U - 1) * rpi < r1; r += BN_U * rpi) {  // BN_U rows (2-3 loads each) in flight per thread
    float g[BN_U][8], xv[BN_U][8], yv[BN_U][8];
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const long off = (r + u * rpi) * C + cv * 8;
      ld8(dy + off, g[u]);
      ld8(x + off, xv[u]);
      if (MK == 2) ld8(y + off, yv[u]);
    }
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool live = MK == 0 || (MK == 1 ? fmaf(xv[u][j], sc[j], sh[j]) > 0.f : yv[u][j] > 0.f);
        const float gg = live ? g[u][j] : 0.f;
        g[u][j] = gg;
        sg[j] += gg;
        sgx[j] = fmaf(gg, fmaf(xv[u][j], rs[j], mu[j]), sgx[j]);
      }
      if (gout != nullptr) store_bf16<8>(gout + (r + u * rpi) * C + cv * 8, g[u]);
    }
  }
  for (; r < r1; r += rpi) {
    const long off = r * C + cv * 8;
    float g[8], xv[8];
    ld8(dy + off, g);
    ld8(x + off, xv);
    if (MK == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = fmaf(xv[j], sc[j], sh[j]) > 0.f ? g[j] : 0.f;
    } else if (MK == 2) {
      float yv[8];
      ld8(y + off, yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sg[j] += g[j];
      sgx[j] = fmaf(g[j], fmaf(xv[j], rs[j], mu[j]), sgx[j]);
    }
    if (gout != nullptr) store_bf16<8>(gout + off, g);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[threadIdx.x * 16 + j] = sg[j];
    red[threadIdx.x * 16 + 8 + j] = sgx[j];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * C; i += kThreads) {
    const int moment = i / C, c = i % C, v = c >> 3, j = c & 7;
    float a = 0.f;
    for (int k = 0; k < rpi; ++k) a += red[(k * CV + v) * 16 + moment * 8 + j];
    atomicAdd(&sums[i], a);
  }
}

// ---------------------------------------------------------------------------------- backward dx
// MK: ReLU mask source (0 none, 1 from x, 2 from y); HD: the residual gradient dres is stored
template <int BN_U, int MK, bool HD>
__global__ __launch_bounds__(kThreads) void bn_bwd_dx_kernel(const bf16_t* __restrict__ dy,
                                                             const bf16_t* __restrict__ y,
                                                             const bf16_t* __restrict__ x,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ sums, bf16_t* __restrict__ dx,
                                                             bf16_t* __restrict__ dres, float* __restrict__ dgamma,
                                                             float* __restrict__ dbeta, long R, int C, int relu,
                                                             int accumulate, const float* __restrict__ beta) {
  // dx = k1 (g - mg - xhat mgx), xhat = (x - mu) rs, folded per channel into dx = ca g + cb x + cc
  // (two FMAs and three table reads per element instead of five reads and ~6 VALU).  The LDS
  // footprint stays 6 x 2048 floats on purpose: BN blocks that take less of the CU crowd out the
  // concurrent trunk pass's conv workgroups (round 4, r4_ab_bn_dynamic_lds_folded.jsonl).
  __shared__ float tab[6 * 2048];
  float* ca = tab;
  float* cb = tab + 2048;
  float* cc = tab + 2 * 2048;
  float* k1 = tab + 3 * 2048;
  float* sh_s = tab + 4 * 2048;
  constexpr bool xmask = MK == 1;  // ReLU mask from x (see bn_bwd_stats_kernel)
  const int grp = blockIdx.y, G = gridDim.y;
  const float invR = 1.f / (float)R;
  for (int c = threadIdx.x; c < C; c += kThreads) {
    const float* sg = sums + (long)grp * 2 * C;
    const float rs = rstd[(long)grp * C + c], mu = mean[(long)grp * C + c];
    const float kk = gamma[c] * rs, mg = sg[c] * invR, mgx = sg[C + c] * invR;
    k1[c] = kk;
    if (xmask) sh_s[c] = beta[c] - mu * kk;
    ca[c] = kk;
    cb[c] = -kk * rs * mgx;
    cc[c] = kk * (rs * mgx * mu - mg);
    tab[5 * 2048 + c] = 0.f;  // keeps the sixth table (and the block's LDS size) live
    if (blockIdx.x == 0 && grp == 0) {  // parameter grads: sum over the statistics groups
      float db = 0.f, dg = 0.f;
      for (int k = 0; k < G; ++k) {
        db += sums[(long)k * 2 * C + c];
        dg += sums[(long)k * 2 * C + C + c];
      }
      if (accumulate) {  // straight into the parameters' (flat) gradient buffers
        dbeta[c] += db;
        dgamma[c] += dg;
      } else {
        dbeta[c] = db;
        dgamma[c] = dg;
      }
    }
  }
  __syncthreads();
  const long base = (long)grp * R * C;
  dy += base;
  x += base;
  dx += base;
  if (MK == 2) y += base;
  if (HD) dres += base;
  const int CV = C >> 3;
  const long nvec = R * CV;
  const long stride = (long)gridDim.x * kThreads;
  long i = blockIdx.x * (long)kThreads + threadIdx.x;
  for (; i + (BN_U - 1) * stride < nvec; i += BN_U * stride) {
    float g[BN_U][8], xv[BN_U][8], yv[BN_U][8];
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      ld8(dy + (i + u * stride) * 8, g[u]);
      ld8(x + (i + u * stride) * 8, xv[u]);
      if (MK == 2) ld8(y + (i + u * stride) * 8, yv[u]);
    }
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const long iv = i + u * stride;
      const int c0 = ((int)iv & (CV - 1)) * 8;
      if (MK == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) g[u][j] = fmaf(xv[u][j], k1[c0 + j], sh_s[c0 + j]) > 0.f ? g[u][j] : 0.f;
      } else if (MK == 2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) g[u][j] = yv[u][j] > 0.f ? g[u][j] : 0.f;
      }
      if (HD) store_bf16<8>(dres + iv * 8, g[u]);
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        o[j] = fmaf(ca[c], g[u][j], fmaf(cb[c], xv[u][j], cc[c]));
      }
      store_bf16<8>(dx + iv * 8, o);
    }
  }
  for (; i < nvec; i += stride) {
    const int c0 = ((int)i & (CV - 1)) * 8;
    float g[8], xv[8];
    ld8(dy + i * 8, g);
    ld8(x + i * 8, xv);
    if (MK == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = fmaf(xv[j], k1[c0 + j], sh_s[c0 + j]) > 0.f ? g[j] : 0.f;
    } else if (MK == 2) {
      float yv[8];
      ld8(y + i * 8, yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
    }
    if (HD) store_bf16<8>(dres + i * 8, g);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      o[j] = fmaf(ca[c], g[j], fmaf(cb[c], xv[j], cc[c]));
    }
    store_bf16<8>(dx + i * 8, o);
  }
}

// the streaming kernels run with BN_U = 2 rows in flight per thread (4 measured slower in round 3:
// 2186 / 2191 vs 2212 / 2203 samples/s)

inline bool bn_shape_ok(int C) {
  if (C % 8 || C > 2048) return false;
  const int CV = C / 8;
  return (kThreads % CV) == 0;
}

// Rows per block: enough for ~8 row-iterations per thread (a block covers rpi = 256 / (C/8) rows per
// iteration), at most 1024 blocks per statistics group.  Sizing by rows alone gave the 2048-channel
// layers (rpi = 1) 64 serial iterations per thread on fewer blocks than CUs (profiles/README.md).
// (cap: SwAV's concurrent passes, as DL_BN_APPLY_MAXB: 256 +0.5% / +1.1% over 1024 in two same-box
// A/Bs, 512 +0.3%, 2048 -0.4%; profiles/r5_swav_grid_caps_ab.jsonl)
#ifndef DL_BN_STATS_MAXB
#define DL_BN_STATS_MAXB 256  // (a measurement build may override)
#endif
// Deterministic statistics (DEDLOC_DETERMINISTIC_BN=1, read at every launch so a process can switch
// it around one parity run): ONE block per statistics group, so every channel's sum is one fixed-order
// block reduction added to a zeroed slot — bitwise reproducible, and slow (parity runs only).  The
// model side also stops accumulating statistics in conv / GEMM epilogues (models/resnet_swav.py).
inline bool bn_deterministic() {
  const char* e = std::getenv("DEDLOC_DETERMINISTIC_BN");
  return e != nullptr && e[0] == '1';
}

inline int stats_blocks(long R, int C, long& rpb) {
  const long rpi = kThreads / (C / 8);
  long nb = (R + 8 * rpi - 1) / (8 * rpi);
  if (nb > DL_BN_STATS_MAXB) nb = DL_BN_STATS_MAXB;
  if (bn_deterministic()) nb = 1;
  if (nb < 1) nb = 1;
  rpb = (R + nb - 1) / nb;
  return (int)((R + rpb - 1) / rpb);
}

// Grid cap of the streaming apply / dx kernels.  SwAV runs its resolution passes concurrently, and
// every BN block beyond what saturates HBM takes CU slots from the other pass's convs: SwAV b=64
// iteration +1.8% at 768 vs 2048 (512: +0.1%, 1024: +1.1%, 4096: -1.7%; same-box A/Bs,
// profiles/r5_swav_grid_caps_ab.jsonl)
#ifndef DL_BN_APPLY_MAXB
#define DL_BN_APPLY_MAXB 768  // (a measurement build may override)
#endif
inline int apply_blocks(long nvec) {
  constexpr long cap = DL_BN_APPLY_MAXB;
  long g = (nvec + kThreads - 1) / kThreads;
  return (int)(g < cap ? (g < 1 ? 1 : g) : cap);
}

}  // namespace

// sums: fp32 [2C] workspace; mean/rstd: fp32 [C] outputs; run_mean/run_var may be null
// R = rows per statistics group, G groups (the tensor holds G*R rows); sums [G, 2C], mean/rstd [G, C]
// sums_zeroed: the caller hands a pre-zeroed sums slice (one memset per trunk pass covers every
// BatchNorm's workspace instead of one hipMemsetAsync — a ~5 us launch — per call)
int dl_bn_fwd(const bf16_t* x, const bf16_t* res, bf16_t* y, const float* gamma, const float* beta, float* sums,
              float* mean, float* rstd, float* run_mean, float* run_var, long R, int C, int G, float eps,
              float momentum, int relu, hipStream_t st, int sums_zeroed, int stats_ready) {
  if (!bn_shape_ok(C) || R < 1 || G < 1) return -1;
  if (!stats_ready) {  // else: the producing conv / GEMM epilogue already accumulated them
    if (!sums_zeroed) DL_HIP_CHECK(hipMemsetAsync(sums, 0, sizeof(float) * 2 * C * G, st));
    long rpb;
    const int nb = stats_blocks(R, C, rpb);
    bn_stats_kernel<<<dim3(nb, G), kThreads, 0, st>>>(x, sums, R, C, rpb);
  }
  const int na = (apply_blocks(R * (C / 8) * G) + G - 1) / G;
#define DL_BN_APPLY(HR_, RL_)                                                                             \
  bn_apply_kernel<2, HR_, RL_><<<dim3(na, G), kThreads, 0, st>>>(x, res, y, sums, gamma, beta, mean, rstd, run_mean, \
                                                                 run_var, R, C, eps, momentum, relu)
  if (res) {
    if (relu) DL_BN_APPLY(true, true);
    else DL_BN_APPLY(true, false);
  } else {
    if (relu) DL_BN_APPLY(false, true);
    else DL_BN_APPLY(false, false);
  }
#undef DL_BN_APPLY
  return 0;
}

int dl_bn_stats(const bf16_t* x, float* sums, long R, int C, int G, hipStream_t st) {
  if (!bn_shape_ok(C) || R < 1 || G < 1) return -1;
  long rpb;
  const int nb = stats_blocks(R, C, rpb);
  bn_stats_kernel<<<dim3(nb, G), kThreads, 0, st>>>(x, sums, R, C, rpb);
  return 0;
}

// BatchNorm+ReLU backward preparation as a separate pass (the fallback of the fused data-gradient
// epilogues): dy (in place) <- dy masked by the ReLU (y > 0, or from x with beta), sums += the two
// backward column sums; then dl_bn_bwd(..., relu = 0, stats_ready = 1)
int dl_bn_bwd_prep(bf16_t* dy, const bf16_t* y, const bf16_t* x, const float* mean, const float* rstd,
                   const float* gamma, const float* beta, float* sums, long R, int C, int G, hipStream_t st) {
  if (!bn_shape_ok(C) || R < 1 || G < 1 || (!y && !beta)) return -1;
  long rpb;
  const int nb = stats_blocks(R, C, rpb);
  if (y) bn_bwd_stats_kernel<2, 2><<<dim3(nb, G), kThreads, 0, st>>>(dy, y, x, mean, rstd, sums, R, C, rpb, 1, gamma,
                                                                     nullptr, dy);
  else bn_bwd_stats_kernel<2, 1><<<dim3(nb, G), kThreads, 0, st>>>(dy, y, x, mean, rstd, sums, R, C, rpb, 1, gamma,
                                                                   beta, dy);
  return 0;
}

// accumulate: dgamma / dbeta += (the parameters' gradient buffers) instead of =
// beta: non-null -> the ReLU mask is recomputed from x (BatchNorm+ReLU without a residual branch;
// y is then not read at all)
int dl_bn_bwd(const bf16_t* dy, const bf16_t* y, const bf16_t* x, const float* mean, const float* rstd,
              const float* gamma, float* sums, bf16_t* dx, bf16_t* dres, float* dgamma, float* dbeta, long R, int C,
              int G, int relu, hipStream_t st, int sums_zeroed, int accumulate, const float* beta, int stats_ready) {
  if (!bn_shape_ok(C) || R < 1 || G < 1) return -1;
  long rpb;
  const int nb = stats_blocks(R, C, rpb);
  if (!stats_ready) {  // else: a data-gradient epilogue (or dl_bn_bwd_prep) accumulated the sums and
                       // already masked dy by the ReLU (the caller then passes relu = 0)
    if (!sums_zeroed) DL_HIP_CHECK(hipMemsetAsync(sums, 0, sizeof(float) * 2 * C * G, st));
    const int mk = !relu ? 0 : beta != nullptr ? 1 : 2;
#define DL_BN_BSTATS(MK_)                                                                                    \
  bn_bwd_stats_kernel<2, MK_><<<dim3(nb, G), kThreads, 0, st>>>(dy, y, x, mean, rstd, sums, R, C, rpb, relu, gamma, \
                                                                beta, nullptr)
    if (mk == 0) DL_BN_BSTATS(0);
    else if (mk == 1) DL_BN_BSTATS(1);
    else DL_BN_BSTATS(2);
#undef DL_BN_BSTATS
  }
  const int na = (apply_blocks(R * (C / 8) * G) + G - 1) / G;
  const int mkd = !relu ? 0 : beta != nullptr ? 1 : 2;
#define DL_BN_DX(MK_, HD_)                                                                                   \
  bn_bwd_dx_kernel<2, MK_, HD_><<<dim3(na, G), kThreads, 0, st>>>(dy, y, x, mean, rstd, gamma, sums, dx, dres,    \
                                                                  dgamma, dbeta, R, C, relu, accumulate, beta)
  if (dres) {
    if (mkd == 0) DL_BN_DX(0, true);
    else if (mkd == 1) DL_BN_DX(1, true);
    else DL_BN_DX(2, true);
  } else {
    if (mkd == 0) DL_BN_DX(0, false);
    else if (mkd == 1) DL_BN_DX(1, false);
    else DL_BN_DX(2, false);
  }
#undef DL_BN_DX
  return 0;
}

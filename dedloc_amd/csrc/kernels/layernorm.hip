// Fused (residual-add +) LayerNorm forward/backward for gfx950.
//
// Replaces the reference's torch LayerNorm calls inside HF ALBERT (SURVEY.md §2.7 K1/K5/K6/K7:
// attention `LayerNorm(ctx_out + x)`, `full_layer_layer_norm(ffn_out + attn_out)`, embedding LN,
// MLM-head LN).  One 64-lane wave owns one row; each lane keeps D/64 elements in registers, so the
// row is read once and written once (HBM-bound by design: 2 bf16 reads + 1-2 bf16 writes per elem).
//
// fwd:  s = x (+ r);  y = (s - mean) * rstd * gamma + beta;  saves mean/rstd (fp32) and s (bf16)
// bwd:  ds = rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat)),  dgamma/dbeta column partials
#include <algorithm>
#include <cstdlib>

#include "dl_common.h"
#include "dl_kernels.h"

namespace {

template <int D>
struct RowCfg {
  static constexpr int EPL = D / 64;                  // elements per lane
  // vector width (elements) per load: the widest of 8 / 4 / 2 / 1 that divides EPL (D = 768 has 12
  // elements per lane: three 4-wide vectors; 8-wide would leave a third of the row untouched)
  static constexpr int VW = EPL % 8 == 0 ? 8 : EPL % 4 == 0 ? 4 : EPL % 2 == 0 ? 2 : 1;
  static constexpr int NV = EPL / VW;                 // vector loads per lane
};

// Column index of vector v of lane `lane`: vectors are interleaved across lanes so that one
// wave-instruction covers 64*VW contiguous elements (fully coalesced).
template <int D>
__device__ __forceinline__ int col_of(int lane, int v) {
  return (v * 64 + lane) * RowCfg<D>::VW;
}

// R rows per wave: gamma / beta are read once per wave (before the rows: they are L2 hits, and
// issued after the first reduction they put an L2 round trip on every row's critical path), all R
// rows' loads are issued before the first is used, and the row sums go through DPP / lane swaps
// (wave_sum_dpp) instead of six LDS-crossbar round trips each.
template <int D, bool HAS_RES, bool SAVE_SUM, int R>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ r,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     bf16_t* __restrict__ y, bf16_t* __restrict__ s_out,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int rows, float eps) {
  using C = RowCfg<D>;
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * R;
  if (row0 >= rows) return;
  static_assert(C::VW == 8 || R == 1, "several rows per wave need 8-wide row vectors");
  // every load of the wave first (the rows raw, gamma / beta), then a scheduling fence: left alone
  // the compiler sinks the later rows' loads behind the first row's math to save registers
  uint4 xr[R][C::NV], rr[HAS_RES ? R : 1][C::NV];
  if constexpr (C::VW == 8) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const size_t base = (size_t)min(row0 + u, rows - 1) * D;  // a tail row repeats the last one (never stored)
#pragma unroll
      for (int i = 0; i < C::NV; ++i) {
        xr[u][i] = *reinterpret_cast<const uint4*>(x + base + col_of<D>(lane, i));
        if constexpr (HAS_RES) rr[u][i] = *reinterpret_cast<const uint4*>(r + base + col_of<D>(lane, i));
      }
    }
  }
  float g[C::EPL], b[C::EPL];
#pragma unroll
  for (int i = 0; i < C::NV; ++i)
#pragma unroll
    for (int j = 0; j < C::VW; ++j) {
      g[i * C::VW + j] = gamma[col_of<D>(lane, i) + j];
      b[i * C::VW + j] = beta[col_of<D>(lane, i) + j];
    }
  __builtin_amdgcn_sched_barrier(0);
  float v[R][C::EPL];
#pragma unroll
  for (int u = 0; u < R; ++u) {
    const size_t base = (size_t)min(row0 + u, rows - 1) * D;
#pragma unroll
    for (int i = 0; i < C::NV; ++i) {
      if constexpr (C::VW == 8) unpack8_bf16(xr[u][i], v[u] + i * C::VW);
      else load_bf16<C::VW>(x + base + col_of<D>(lane, i), v[u] + i * C::VW);
    }
    if constexpr (HAS_RES) {
      float t[C::EPL];
#pragma unroll
      for (int i = 0; i < C::NV; ++i) {
        if constexpr (C::VW == 8) unpack8_bf16(rr[u][i], t + i * C::VW);
        else load_bf16<C::VW>(r + base + col_of<D>(lane, i), t + i * C::VW);
      }
#pragma unroll
      for (int i = 0; i < C::EPL; ++i) v[u][i] += t[i];
    }
  }
#pragma unroll
  for (int u = 0; u < R; ++u) {
    const int row = row0 + u;
    if (R > 1 && row >= rows) break;
    const size_t base = (size_t)row * D;
    if constexpr (SAVE_SUM) {
      // round the residual sum to bf16 first so that bwd sees exactly the normalised values
#pragma unroll
      for (int i = 0; i < C::EPL; ++i) v[u][i] = round_bf16(v[u][i]);
#pragma unroll
      for (int i = 0; i < C::NV; ++i) store_bf16<C::VW>(s_out + base + col_of<D>(lane, i), v[u] + i * C::VW);
    }
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < C::EPL; ++i) sum += v[u][i];
    const float mean = wave_sum_dpp(sum) * (1.f / D);
    float sq = 0.f;
#pragma unroll
    for (int i = 0; i < C::EPL; ++i) { const float d = v[u][i] - mean; sq = fmaf(d, d, sq); }
    const float rstd = rsqrtf(wave_sum_dpp(sq) * (1.f / D) + eps);
    float o[C::EPL];
#pragma unroll
    for (int i = 0; i < C::EPL; ++i) o[i] = fmaf((v[u][i] - mean) * rstd, g[i], b[i]);
#pragma unroll
    for (int i = 0; i < C::NV; ++i) store_bf16<C::VW>(y + base + col_of<D>(lane, i), o + i * C::VW);
    if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
  }
}

// Each block handles a contiguous chunk of rows (one wave per row, grid-strided inside the
// block) and writes one fp32 partial row of dgamma/dbeta; dl_colsum_f32 reduces the partials.
template <int D, int R>
__global__ __launch_bounds__(512) void ln_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ s,
                                                     const float* __restrict__ gamma, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, bf16_t* __restrict__ ds,
                                                     float* __restrict__ dgamma_part, float* __restrict__ dbeta_part,
                                                     float* __restrict__ dsum, int rows, int rows_per_block) {
  using C = RowCfg<D>;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  float g[C::EPL], dg[C::EPL], db[C::EPL], dx[C::EPL];
#pragma unroll
  for (int i = 0; i < C::NV; ++i)
#pragma unroll
    for (int j = 0; j < C::VW; ++j) {
      g[i * C::VW + j] = gamma[col_of<D>(lane, i) + j];
      dg[i * C::VW + j] = 0.f;
      db[i * C::VW + j] = 0.f;
      dx[i * C::VW + j] = 0.f;
    }
  // R rows per wave iteration, all R rows' loads issued before any is used: with one row in flight
  // per wave (2 waves/SIMD) the kernel is bound by loads in flight, not by bandwidth.  (Prefetching
  // row i+1 behind row i's stores measured slower: the stores sit ahead of the prefetch in the
  // in-order vmcnt queue.)
  for (int row = r0 + wid; row < r1; row += R * nw) {
    int rr[R];
    bool live[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      live[u] = row + u * nw < r1;
      rr[u] = live[u] ? row + u * nw : row;
    }
    float gy[R][C::EPL], xh[R][C::EPL];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const size_t base = (size_t)rr[u] * D;
#pragma unroll
      for (int i = 0; i < C::NV; ++i) {
        load_bf16<C::VW>(dy + base + col_of<D>(lane, i), gy[u] + i * C::VW);
        load_bf16<C::VW>(s + base + col_of<D>(lane, i), xh[u] + i * C::VW);
      }
    }
    float a[R], b[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const float mean = mean_in[rr[u]], rstd = rstd_in[rr[u]];
      const float keep = live[u] ? 1.f : 0.f;  // a duplicated row adds nothing to the column sums
      a[u] = 0.f;
      b[u] = 0.f;
#pragma unroll
      for (int i = 0; i < C::EPL; ++i) {
        xh[u][i] = (xh[u][i] - mean) * rstd;
        dg[i] += keep * gy[u][i] * xh[u][i];
        db[i] += keep * gy[u][i];
        gy[u][i] *= g[i];
        a[u] += gy[u][i];
        b[u] += gy[u][i] * xh[u][i];
      }
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      a[u] = wave_sum_dpp(a[u]) * (1.f / D);
      b[u] = wave_sum_dpp(b[u]) * (1.f / D);
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      if (!live[u]) break;
      const float rstd = rstd_in[rr[u]];
#pragma unroll
      for (int i = 0; i < C::EPL; ++i) {
        gy[u][i] = bf2f(f2bf(rstd * (gy[u][i] - a[u] - xh[u][i] * b[u])));
        dx[i] += gy[u][i];
      }
      const size_t base = (size_t)rr[u] * D;
#pragma unroll
      for (int i = 0; i < C::NV; ++i) store_bf16<C::VW>(ds + base + col_of<D>(lane, i), gy[u] + i * C::VW);
    }
  }
  // reduce the per-wave column partials through LDS, one quantity at a time through one nw x D
  // buffer (so an 8-wave block needs 32 KiB, not 96), then one fp32 atomic per column per block
  // straight into the (accumulating) gradient buffers; dsum = column sum of ds = the bias gradient
  // of the Linear that produced the LN input
  extern __shared__ __attribute__((aligned(16))) float lds[];
#pragma unroll
  for (int which = 0; which < 3; ++which) {
    float* dst = which == 0 ? dgamma_part : which == 1 ? dbeta_part : dsum;
    if (dst == nullptr) break;  // block-uniform
    const float* v = which == 0 ? dg : which == 1 ? db : dx;
    if (which) __syncthreads();  // the previous round's column reads are done
#pragma unroll
    for (int i = 0; i < C::NV; ++i)
#pragma unroll
      for (int j = 0; j < C::VW; ++j) lds[wid * D + col_of<D>(lane, i) + j] = v[i * C::VW + j];
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += blockDim.x) {
      float sum = 0.f;
      for (int w = 0; w < nw; ++w) sum += lds[w * D + c];
      atomicAdd(&dst[c], sum);
    }
  }
}

// Wide rows (D = 2048 / 4096, e.g. albert-xxlarge's 4096): one 256-thread block per row (each thread
// D / 256 elements, 8-wide vectors interleaved over the block so every load instruction covers
// 4 KiB contiguous), the two row sums reduced through LDS; the block walks its chunk of rows and
// keeps per-thread column partials of dgamma / dbeta / colsum(ds), added with one fp32 atomic per
// column at the end.  (The one-wave-per-row kernel above would need 6 x D / 64 floats per lane.)
template <int D>
__global__ __launch_bounds__(256) void ln_bwd_wide_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ s,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ mean_in,
                                                         const float* __restrict__ rstd_in, bf16_t* __restrict__ ds,
                                                         float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                         float* __restrict__ dsum, int rows, int rows_per_block) {
  constexpr int EPT = D / 256, NV = EPT / 8;
  static_assert(EPT % 8 == 0, "wide LayerNorm rows: D must be a multiple of 2048");
  __shared__ float red[2][4];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  float g[EPT], dg[EPT], db[EPT], dx[EPT];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      g[v * 8 + j] = gamma[(v * 256 + t) * 8 + j];
      dg[v * 8 + j] = db[v * 8 + j] = dx[v * 8 + j] = 0.f;
    }
  for (int row = r0; row < r1; ++row) {
    const size_t base = (size_t)row * D;
    float gy[EPT], xh[EPT];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      load_bf16<8>(dy + base + (v * 256 + t) * 8, gy + v * 8);
      load_bf16<8>(s + base + (v * 256 + t) * 8, xh + v * 8);
    }
    const float mean = mean_in[row], rstd = rstd_in[row];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      xh[i] = (xh[i] - mean) * rstd;
      dg[i] += gy[i] * xh[i];
      db[i] += gy[i];
      gy[i] *= g[i];
      a += gy[i];
      b += gy[i] * xh[i];
    }
    a = wave_sum_dpp(a);
    b = wave_sum_dpp(b);
    if (lane == 0) {
      red[0][wid] = a;
      red[1][wid] = b;
    }
    __syncthreads();
    a = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) * (1.f / D);
    b = (red[1][0] + red[1][1] + red[1][2] + red[1][3]) * (1.f / D);
    __syncthreads();  // red is rewritten by the next row
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      gy[i] = bf2f(f2bf(rstd * (gy[i] - a - xh[i] * b)));
      dx[i] += gy[i];
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) store_bf16<8>(ds + base + (v * 256 + t) * 8, gy + v * 8);
  }
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = (v * 256 + t) * 8 + j;
      if (dgamma) atomicAdd(&dgamma[c], dg[v * 8 + j]);
      if (dbeta) atomicAdd(&dbeta[c], db[v * 8 + j]);
      if (dsum) atomicAdd(&dsum[c], dx[v * 8 + j]);
    }
}

// rows per wave of the forward (tuning knob DEDLOC_LN_FWD_R = 1 / 2 / 4, read once)
static int ln_fwd_rows_per_wave() {
  static const int r = [] {
    const char* e = std::getenv("DEDLOC_LN_FWD_R");
    const int v = e ? std::atoi(e) : 2;
    return v == 1 || v == 4 ? v : 2;
  }();
  return r;
}

template <int D, int R>
void launch_fwd_r(const bf16_t* x, const bf16_t* r, const float* gamma, const float* beta, bf16_t* y, bf16_t* s_out,
                  float* mean, float* rstd, int rows, float eps, hipStream_t st) {
  const int wpb = 4;
  dim3 grid((rows + wpb * R - 1) / (wpb * R)), block(64 * wpb);
  if (r) {
    if (s_out) ln_fwd_kernel<D, true, true, R><<<grid, block, 0, st>>>(x, r, gamma, beta, y, s_out, mean, rstd, rows, eps);
    else ln_fwd_kernel<D, true, false, R><<<grid, block, 0, st>>>(x, r, gamma, beta, y, s_out, mean, rstd, rows, eps);
  } else {
    ln_fwd_kernel<D, false, false, R><<<grid, block, 0, st>>>(x, r, gamma, beta, y, s_out, mean, rstd, rows, eps);
  }
}

template <int D>
void launch_fwd(const bf16_t* x, const bf16_t* r, const float* gamma, const float* beta, bf16_t* y, bf16_t* s_out,
                float* mean, float* rstd, int rows, float eps, hipStream_t st) {
  // several rows per wave for 8-wide row vectors (D = 512 / 1024); wide rows (their EPL floats per
  // lane already fill the registers) and narrow ones keep one row per wave
  constexpr bool multi = RowCfg<D>::VW == 8 && D <= 1024;
  const int R = multi ? ln_fwd_rows_per_wave() : 1;
  if (R == 4) launch_fwd_r<D, multi ? 4 : 1>(x, r, gamma, beta, y, s_out, mean, rstd, rows, eps, st);
  else if (R == 2) launch_fwd_r<D, multi ? 2 : 1>(x, r, gamma, beta, y, s_out, mean, rstd, rows, eps, st);
  else launch_fwd_r<D, 1>(x, r, gamma, beta, y, s_out, mean, rstd, rows, eps, st);
}

template <int D>
void launch_bwd(const bf16_t* dy, const bf16_t* s, const float* gamma, const float* mean, const float* rstd,
                bf16_t* ds, float* dg_part, float* db_part, float* dsum, int rows, int nparts, hipStream_t st) {
  // 4 waves per block (8 measured equal: the two-row form's 202 VGPRs cap the kernel at 2 waves per
  // SIMD either way) and 2 rows in flight per wave (the round-2 A/B winner over 1 and 4)
  constexpr int wpb = 4;
  const int rpb = (rows + nparts - 1) / nparts;
  const size_t lds = (size_t)wpb * D * sizeof(float);
  ln_bwd_kernel<D, 2><<<nparts, 64 * wpb, lds, st>>>(dy, s, gamma, mean, rstd, ds, dg_part, db_part, dsum, rows, rpb);
}

}  // namespace

int dl_layernorm_fwd(const bf16_t* x, const bf16_t* r, const float* gamma, const float* beta, bf16_t* y,
                     bf16_t* s_out, float* mean, float* rstd, int rows, int D, float eps, hipStream_t st) {
  switch (D) {
    case 64: launch_fwd<64>(x, r, gamma, beta, y, s_out, mean, rstd, rows, eps, st); break;
    case 128: launch_fwd<128>(x, r, gamma, beta, y, s_out, mean, rstd, rows, eps, st); break;
    case 256: launch_fwd<256>(x, r, gamma, beta, y, s_out, mean, rstd, rows, eps, st); break;
    case 512: launch_fwd<512>(x, r, gamma, beta, y, s_out, mean, rstd, rows, eps, st); break;
    case 768: launch_fwd<768>(x, r, gamma, beta, y, s_out, mean, rstd, rows, eps, st); break;
    case 1024: launch_fwd<1024>(x, r, gamma, beta, y, s_out, mean, rstd, rows, eps, st); break;
    case 2048: launch_fwd<2048>(x, r, gamma, beta, y, s_out, mean, rstd, rows, eps, st); break;
    case 4096: launch_fwd<4096>(x, r, gamma, beta, y, s_out, mean, rstd, rows, eps, st); break;
    default: return -1;
  }
  return 0;
}

int dl_layernorm_bwd(const bf16_t* dy, const bf16_t* s, const float* gamma, const float* mean, const float* rstd,
                     bf16_t* ds, float* dg_part, float* db_part, float* dsum, int rows, int D, int nparts,
                     hipStream_t st) {
  switch (D) {
    case 64: launch_bwd<64>(dy, s, gamma, mean, rstd, ds, dg_part, db_part, dsum, rows, nparts, st); break;
    case 128: launch_bwd<128>(dy, s, gamma, mean, rstd, ds, dg_part, db_part, dsum, rows, nparts, st); break;
    case 256: launch_bwd<256>(dy, s, gamma, mean, rstd, ds, dg_part, db_part, dsum, rows, nparts, st); break;
    case 512: launch_bwd<512>(dy, s, gamma, mean, rstd, ds, dg_part, db_part, dsum, rows, nparts, st); break;
    case 768: launch_bwd<768>(dy, s, gamma, mean, rstd, ds, dg_part, db_part, dsum, rows, nparts, st); break;
    case 1024: launch_bwd<1024>(dy, s, gamma, mean, rstd, ds, dg_part, db_part, dsum, rows, nparts, st); break;
    case 2048:
      ln_bwd_wide_kernel<2048><<<nparts, 256, 0, st>>>(dy, s, gamma, mean, rstd, ds, dg_part, db_part, dsum, rows,
                                                      (rows + nparts - 1) / nparts);
      break;
    case 4096:
      ln_bwd_wide_kernel<4096><<<nparts, 256, 0, st>>>(dy, s, gamma, mean, rstd, ds, dg_part, db_part, dsum, rows,
                                                      (rows + nparts - 1) / nparts);
      break;
    default: return -1;
  }
  return 0;
}

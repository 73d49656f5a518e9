// ALBERT embeddings: word + position + token-type gather, sum, LayerNorm(E)
// fused into one pass that reads the fp32 master tables directly (no bf16 copy of the 30000x128
// table is ever materialised).  Backward scatters into the fp32 gradient tables: word rows by
// atomics (low contention, rows are spread over the vocabulary), position/type rows by a
// per-position reduction (one block per position, no atomics for position rows).
#include "dl_common.h"
#include "dl_kernels.h"

namespace {

template <int E>
__global__ __launch_bounds__(256) void embed_ln_fwd_kernel(const long* __restrict__ ids, const long* __restrict__ tt,
                                                           const float* __restrict__ wemb, const float* __restrict__ pemb,
                                                           const float* __restrict__ temb, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, bf16_t* __restrict__ y,
                                                           bf16_t* __restrict__ s_out, float* __restrict__ mean_out,
                                                           float* __restrict__ rstd_out, int T, int S, float eps) {
  constexpr int EPL = E / 64;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= T) return;
  const long id = ids[row];
  const long ty = tt ? tt[row] : 0;
  const int pos = row % S;
  float v[EPL];
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    const int c = i * 64 + lane;
    v[i] = bf2f(f2bf(wemb[id * E + c] + pemb[(long)pos * E + c] + temb[ty * E + c]));
  }
#pragma unroll
  for (int i = 0; i < EPL; ++i) s_out[(size_t)row * E + i * 64 + lane] = f2bf(v[i]);
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) sum += v[i];
  const float mean = wave_sum(sum) * (1.f / E);
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) { const float d = v[i] - mean; sq += d * d; }
  const float rstd = rsqrtf(wave_sum(sq) * (1.f / E) + eps);
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    const int c = i * 64 + lane;
    y[(size_t)row * E + c] = f2bf((v[i] - mean) * rstd * gamma[c] + beta[c]);
  }
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

template <int E>
__global__ __launch_bounds__(256) void embed_word_bwd_kernel(const bf16_t* __restrict__ ds, const long* __restrict__ ids,
                                                             float* __restrict__ dwemb, int T) {
  constexpr int EPL = E / 64;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= T) return;
  const long id = ids[row];
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    const int c = i * 64 + lane;
    atomicAdd(&dwemb[id * E + c], bf2f(ds[(size_t)row * E + c]));
  }
}

// one block per position p, E threads: dpos[p] += sum_b ds[b, p];  dtype[t] += per-block sums
__global__ void embed_pos_type_bwd_kernel(const bf16_t* __restrict__ ds, const long* __restrict__ tt,
                                          float* __restrict__ dpemb, float* __restrict__ dtemb, int B, int S, int E,
                                          int ntypes) {
  const int p = blockIdx.x;
  for (int c = threadIdx.x; c < E; c += blockDim.x) {
    float acc = 0.f, t0 = 0.f, t1 = 0.f;
    for (int b = 0; b < B; ++b) {
      const size_t row = (size_t)b * S + p;
      const float g = bf2f(ds[row * E + c]);
      acc += g;
      const long ty = tt ? tt[row] : 0;
      if (ty == 0) t0 += g;
      else if (ty == 1) t1 += g;
      else atomicAdd(&dtemb[ty * E + c], g);
    }
    dpemb[(size_t)p * E + c] += acc;
    if (dtemb) {
      atomicAdd(&dtemb[c], t0);
      if (ntypes > 1) atomicAdd(&dtemb[E + c], t1);
    }
  }
}

}  // namespace

int dl_embed_ln_fwd(const long* ids, const long* tt, const float* wemb, const float* pemb, const float* temb,
                    const float* gamma, const float* beta, bf16_t* y, bf16_t* s_out, float* mean, float* rstd, int T,
                    int S, int E, float eps, hipStream_t st) {
  const int wpb = 4;
  dim3 grid((T + wpb - 1) / wpb), block(64 * wpb);
  switch (E) {
    case 64: embed_ln_fwd_kernel<64><<<grid, block, 0, st>>>(ids, tt, wemb, pemb, temb, gamma, beta, y, s_out, mean, rstd, T, S, eps); break;
    case 128: embed_ln_fwd_kernel<128><<<grid, block, 0, st>>>(ids, tt, wemb, pemb, temb, gamma, beta, y, s_out, mean, rstd, T, S, eps); break;
    case 256: embed_ln_fwd_kernel<256><<<grid, block, 0, st>>>(ids, tt, wemb, pemb, temb, gamma, beta, y, s_out, mean, rstd, T, S, eps); break;
    case 512: embed_ln_fwd_kernel<512><<<grid, block, 0, st>>>(ids, tt, wemb, pemb, temb, gamma, beta, y, s_out, mean, rstd, T, S, eps); break;
    default: return -1;
  }
  return 0;
}

int dl_embed_bwd(const bf16_t* ds, const long* ids, const long* tt, float* dwemb, float* dpemb, float* dtemb, int B,
                 int S, int E, int ntypes, hipStream_t st) {
  const int T = B * S;
  const int wpb = 4;
  dim3 grid((T + wpb - 1) / wpb), block(64 * wpb);
  switch (E) {
    case 64: embed_word_bwd_kernel<64><<<grid, block, 0, st>>>(ds, ids, dwemb, T); break;
    case 128: embed_word_bwd_kernel<128><<<grid, block, 0, st>>>(ds, ids, dwemb, T); break;
    case 256: embed_word_bwd_kernel<256><<<grid, block, 0, st>>>(ds, ids, dwemb, T); break;
    case 512: embed_word_bwd_kernel<512><<<grid, block, 0, st>>>(ds, ids, dwemb, T); break;
    default: return -1;
  }
  embed_pos_type_bwd_kernel<<<S, E < 256 ? E : 256, 0, st>>>(ds, tt, dpemb, dtemb, B, S, E, ntypes);
  return 0;
}

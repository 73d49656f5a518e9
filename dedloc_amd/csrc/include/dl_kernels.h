// Host-side launcher ABI of the dedloc_amd HIP kernels (all gfx950).  Every launcher enqueues on
// the given stream, never allocates and never synchronises, and returns 0 on success or -1 when
// the shape is unsupported (the binding layer turns that into a Python exception).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

typedef uint16_t bf16_t;

// layernorm.hip
int dl_layernorm_fwd(const bf16_t* x, const bf16_t* r, const float* gamma, const float* beta, bf16_t* y,
                     bf16_t* s_out, float* mean, float* rstd, int rows, int D, float eps, hipStream_t st);
int dl_layernorm_bwd(const bf16_t* dy, const bf16_t* s, const float* gamma, const float* mean, const float* rstd,
                     bf16_t* ds, float* dg_part, float* db_part, float* dsum, int rows, int D, int nparts,
                     hipStream_t st);

// elementwise.hip
int dl_gelu_fwd(const bf16_t* h, bf16_t* y, size_t n, hipStream_t st);
int dl_gelu_bwd(const bf16_t* dy, const bf16_t* h, bf16_t* dh, size_t n, hipStream_t st);
int dl_gelu_bwd_colsum(const bf16_t* dy, const bf16_t* h, bf16_t* dh, float* dbias, int rows, int N, hipStream_t st);
// y = gelu_new(h), d = gelu_new'(h); dh = dy * d with dbias += colsum(dh)
int dl_gelu_fwd_d(const bf16_t* h, bf16_t* y, bf16_t* d, size_t n, hipStream_t st);
int dl_mul_colsum(const bf16_t* dy, const bf16_t* d, bf16_t* dh, float* dbias, int rows, int N, hipStream_t st);
int dl_tanh_fwd(const bf16_t* x, bf16_t* y, size_t n, hipStream_t st);
int dl_tanh_bwd(const bf16_t* dy, const bf16_t* y, bf16_t* dx, size_t n, hipStream_t st);
int dl_colsum_bf16(const bf16_t* x, float* part, int rows, int N, int nparts, hipStream_t st);
int dl_colsum_f32(const float* part, float* out, int nparts, int N, int accumulate, hipStream_t st);
int dl_cast_f32_bf16(const float* x, bf16_t* y, size_t n, hipStream_t st);
int dl_add_bf16_to_f32(const bf16_t* x, float* y, size_t n, float alpha, hipStream_t st);

// optim.hip
int dl_lamb_step(float* p, const float* g, float* m, float* v, const int* chunk_tensor, const long* chunk_start,
                 const int* chunk_len, int nchunks, const float* tensor_wd, float* norms, int ntensors, float beta1,
                 float beta2, float eps, float step_size, float clamp_value, float grad_scale, float* trust_out,
                 hipStream_t st);
int dl_larc_sgd_step(float* p, const float* g, float* buf, const int* chunk_tensor, const long* chunk_start,
                     const int* chunk_len, int nchunks, const float* tensor_wd, float* norms, int ntensors, float lr,
                     float momentum, float trust_coef, float eps, int clip, int first_step, float grad_scale,
                     hipStream_t st);
// out[0] = ||x||, out[1] = finite flag, out[2] (if nout > 2) = 1 - finite; clips x to max_norm if > 0
int dl_grad_norm_clip(float* x, size_t n, float max_norm, float* part, int nparts, float* out, int nout,
                      hipStream_t st);
// y = a*y + (b / max(1, *bdiv))*x; skipped when *flag == 0; bdiv/flag may be null
int dl_axpby(float* y, const float* x, size_t n, float a, float b, const float* flag, const float* bdiv,
             hipStream_t st);
// x *= s[0] in place (bf16; a device scalar, no pass at all when it is exactly 1)
int dl_scale_by(bf16_t* x, size_t n, const float* s, hipStream_t st);
int dl_sum_slabs(float* out, const float* slabs, int s, size_t n, hipStream_t st);
int dl_add_slabs_zero(float* out, float* slabs, int s, size_t n, hipStream_t st);

// comm.hip
int dl_pack(const float* src, void* dst, int dst_dt, size_t n, float weight, hipStream_t st);
int dl_reduce_parts(const void* parts, int part_dt, size_t part_stride, int nparts, void* out, int out_dt, size_t n,
                    float inv_total, hipStream_t st);
int dl_unpack(const void* src, int src_dt, float* dst, const float* snap, int add, size_t n, hipStream_t st);
int dl_reduce_delta(const void* parts, void* deltas, int dt, size_t part_stride, int nparts, const float* weights,
                    size_t n, hipStream_t st);

// embedding.hip
int dl_embed_ln_fwd(const long* ids, const long* tt, const float* wemb, const float* pemb, const float* temb,
                    const float* gamma, const float* beta, bf16_t* y, bf16_t* s_out, float* mean, float* rstd, int T,
                    int S, int E, float eps, hipStream_t st);
int dl_embed_bwd(const bf16_t* ds, const long* ids, const long* tt, float* dwemb, float* dpemb, float* dtemb, int B,
                 int S, int E, int ntypes, hipStream_t st);

// xent.hip
int dl_xent_fwd_bwd(const bf16_t* logits, const long* labels, bf16_t* dlogits, float* row_loss, float* loss_out,
                    float* scale_buf, int M, int V, long ld, int ignore_index, hipStream_t st);

// gemm.hip  (epi: 0 store(+bias,+residual), 1 bias+gelu (H and gelu(H)), 2 dgelu(+colsum), 3 fp32 +=)
int dl_gemm(int a_kouter, int b_kouter, int epi, const bf16_t* A, long lda, const bf16_t* B, long ldb, int M, int N,
            int K, bf16_t* C, long ldc, float* Cf, long ldcf, const float* bias, const bf16_t* R, long ldr, bf16_t* H,
            long ldh, float* dbias, int splits, hipStream_t st);

// BatchNorm+ReLU backward preparation fused into a data-gradient GEMM epilogue (gemm8 EPI 5,
// gemm_small): the GEMM's output is dY of the BN's output; the epilogue masks it by the ReLU
// (Y > 0, or the forward's pre-activation X*gamma*rstd + beta - mean*gamma*rstd > 0 when Y is null),
// stores the masked g and accumulates stats[m / stat_rows][n] += g and [N + n] += g*(X - mean)*rstd.
struct DlBnBwdEpi {
  const bf16_t* X;      // BN input [M, N], row stride ldx
  const bf16_t* Y;      // optional BN output (ReLU mask source when the BN had a residual), stride ldx
  long ldx;
  const float* mean;    // [G][N]
  const float* rstd;    // [G][N]
  const float* gamma;   // [N] (mask from X)
  const float* beta;    // [N]
};

// gemm8.hip (LDS-DMA 8-phase MFMA GEMM; epi as dl_gemm; EPI 3 writes fp32 slab blockIdx.y of
// Cf (+= when accumulate); splits > 1 only for EPI 3; EPI 4 = EPI 0 plus BatchNorm statistics of
// the stored values: stats[m / stat_rows][0..N) += column sums, [N..2N) += sums of squares)
int dl_gemm8(int a_kouter, int b_kouter, int epi, const bf16_t* A, long lda, const bf16_t* B, long ldb, int M, int N,
             int K, bf16_t* C, long ldc, float* Cf, long ldcf, long slab, int accumulate, const float* bias,
             const bf16_t* R, long ldr, bf16_t* H, long ldh, float* dbias, int splits, hipStream_t st,
             float* stats = nullptr, long stat_rows = 0, const DlBnBwdEpi* bn = nullptr);

// swav.hip
int dl_sinkhorn_ws(int n, int K);
int dl_sinkhorn(const float* scores, float* Q, float* ws, int n, int K, int bs, float eps, int iters,
                hipStream_t st);
int dl_swav_ce(const void* scores, int scores_bf16, const float* q, float* dscores, float* loss, int rows, int K,
               float temperature, float scale, hipStream_t st);
int dl_swav_ce_multi(const void* scores, int scores_bf16, const float* q, const int* crops, int n_assign,
                     float* dscores, float* loss, int num_crops, int bs, int K, float temperature, float scale,
                     hipStream_t st);
int dl_row_normalize(float* w, int rows, int d, hipStream_t st);
// SwAV multi-crop augmentation (augment.hip): pool [P, 3, Hp, Wp] fp32, params [nb, 20] fp32,
// ws >= 2 * nb*3*S*S + nb floats, out [nb, S, S, 3] bf16 (channels-last [nb, 3, S, S])
int dl_multicrop(const float* pool, int P, int Hp, int Wp, const float* params, int nb, int S, int rad, const float* mean,
                 const float* stdv, float* ws, bf16_t* out, hipStream_t st);
int dl_bn_fwd(const bf16_t* x, const bf16_t* res, bf16_t* y, const float* gamma, const float* beta, float* sums,
              float* mean, float* rstd, float* run_mean, float* run_var, long R, int C, int G, float eps,
              float momentum, int relu, hipStream_t st, int sums_zeroed = 0, int stats_ready = 0);
// BatchNorm forward statistics alone (sums [G][2C] += per-group channel sums / sums of squares of
// x [G*R, C]); dl_bn_fwd with stats_ready = 1 then skips its own statistics pass
int dl_bn_stats(const bf16_t* x, float* sums, long R, int C, int G, hipStream_t st);
int dl_bn_bwd(const bf16_t* dy, const bf16_t* y, const bf16_t* x, const float* mean, const float* rstd,
              const float* gamma, float* sums, bf16_t* dx, bf16_t* dres, float* dgamma, float* dbeta, long R, int C,
              int G, int relu, hipStream_t st, int sums_zeroed = 0, int accumulate = 0, const float* beta = nullptr,
              int stats_ready = 0);
int dl_bn_bwd_prep(bf16_t* dy, const bf16_t* y, const bf16_t* x, const float* mean, const float* rstd,
                   const float* gamma, const float* beta, float* sums, long R, int C, int G, hipStream_t st);

// conv.hip — implicit-GEMM NHWC convolutions.  The gathered operand is an NHWC image
// [Nimg, H, W, C]; GEMM rows m = (n, i, j) over [Nimg, I, J]; tap t = (tr < TR, ts < TS) reads
// pixel (i*sh + dh0 + tr*dhs, j*sw + dw0 + ts*dws) (zero outside the image).
struct DlConvGeom {
  const bf16_t* img;
  int Nimg, H, W, C;
  int I, J, sh, sw;
  int TR, TS, dh0, dhs, dw0, dws;
};
// out[(n, i*osh+oh0, j*osw+ow0), 0..N) (NHWC, row stride ldo) = sum_{t,c} img(pixel(m,t), c) * w[n][t*C + c]
// stats (optional): BatchNorm statistics of the stored output as in dl_gemm8 EPI 4 (stat_rows a
// multiple of 128 dividing M; -1 otherwise)
int dl_conv_fwd(const DlConvGeom& g, const bf16_t* w, long ldw, int N, bf16_t* out, int OH, int OW, int osh, int osw,
                int oh0, int ow0, long ldo, hipStream_t st, float* stats = nullptr, long stat_rows = 0,
                const DlBnBwdEpi* bn = nullptr);  // bn (needs stats): BN-backward preparation epilogue
// several independent forward jobs (same output tensor / channel count / epilogue, e.g. the parity
// classes of a strided data gradient) in ONE launch; at most 4 jobs, all of one kernel variant
// (-1 and nothing launched otherwise)
struct DlConvFwdJob {
  DlConvGeom g;
  const bf16_t* w;
  long ldw;
  int oh0, ow0;
  long stat_rows;
};
int dl_conv_fwd_multi(const DlConvFwdJob* jobs, int njobs, int N, bf16_t* out, int OH, int OW, int osh, int osw,
                      long ldo, hipStream_t st, float* stats = nullptr, const DlBnBwdEpi* bn = nullptr);
// dw[k][col] += sum_m dy[m][k] * img(pixel(m, col / C), col % C)    (fp32; col < Ncols; the pixel
// reduction is split over workgroups that add their partial tiles with fp32 atomics)
// dst[c][tr][ts][k] = src[k][r0 + tr*st][s0 + ts*st][c] for many (src KRSC bf16, K and C multiples of
// 64): the tap-transposed data-gradient weights of several convs and parity classes in one launch
struct DlWtJob {
  const bf16_t* src;
  bf16_t* dst;
  int K, C, R, S;
  int r0, s0, st, TR, TS;
};
int dl_conv_dgrad_weights_batched(const DlWtJob* jobs, int njobs, hipStream_t st);
int dl_conv_wgrad(const DlConvGeom& g, const bf16_t* dy, long ldy, int Cout, float* dw, long lddw, int Ncols,
                  hipStream_t st);
// stem im2col: col[m][r*SCp + s*C + c] (filter rows padded to SCp columns), zero columns up to Kp
// space-to-depth of the 3-channel stem input: x NHWC [N, H, W, 3] -> [N, H/2, W/2, 16] (H, W even)
int dl_stem_s2d(const bf16_t* x, int N, int H, int W, bf16_t* xs, hipStream_t st);
int dl_im2col(const bf16_t* x, int N, int H, int W, int C, int R, int S, int stride, int pad, int P, int Q, int SCp,
              int Kp, bf16_t* col, hipStream_t st);

// attn_softmax.hip (composed attention for head sizes other than 64): scores s [rows = B*H*S, S]
// fp32, mbias [B, S] log2 units (optional), c = scale * log2(e); lse / delta [rows]
int dl_attn_softmax_fwd(const float* s, const float* mbias, bf16_t* p, float* lse, long rows, int H, int S, float c,
                        hipStream_t st);
int dl_attn_softmax_bwd(const float* s, const float* dp, const float* mbias, const float* lse, const float* delta,
                        bf16_t* p, bf16_t* ds, long rows, int H, int S, float c, float scale, hipStream_t st);

// attention.hip
int dl_attn_fwd(const bf16_t* qkv, long ld, const float* mbias, const int* kvinfo, bf16_t* out, long ldo, float* lse,
                int B, int H, int S, int D, float scale, hipStream_t st);
// dbias (optional, fp32 [3 H D], accumulated): the QKV projection's bias gradient (query: column
// sums of dQ; key: zero; value: column sums of dout)
int dl_attn_bwd(const bf16_t* qkv, long ld, const float* mbias, const int* kvinfo, const bf16_t* out,
                const bf16_t* dout, long ldo, const float* lse, float* delta, bf16_t* dqkv, float* dbias, int B, int H,
                int S, int D, float scale, hipStream_t st);

// pool.hip (SwAV trunk pools and head normalisation; channels-last bf16, C % 8 == 0)
int dl_maxpool_fwd(const bf16_t* x, bf16_t* y, uint8_t* arg, int N, int H, int W, int C, int P, int Q, hipStream_t st);
int dl_maxpool_bwd(const bf16_t* dy, const uint8_t* arg, bf16_t* dx, int N, int H, int W, int C, int P, int Q,
                   hipStream_t st);
int dl_avgpool_fwd(const bf16_t* x, bf16_t* y, int N, int HW, int C, hipStream_t st);
int dl_avgpool_bwd(const bf16_t* dy, bf16_t* dx, int N, int HW, int C, hipStream_t st);
int dl_l2norm_fwd(const bf16_t* x, bf16_t* y, float* rinv, int rows, int D, float eps, hipStream_t st);
int dl_l2norm_bwd(const bf16_t* dy, const bf16_t* y, const float* rinv, bf16_t* dx, int rows, int D, hipStream_t st);

// gemm_small.hip: any-shape / any-stride bf16 MFMA GEMM (epi 0: bf16 C (+bias)(+R); 1: fp32 Cf (+)=).
// splits > 1 splits the reduction into fp32 slabs: ws must hold splits * M * N floats.
int dl_gemm_small_splits(int M, int N, int K);
// batch GEMMs in one launch (entry b: A + b*sab, B + b*sbb, C / Cf + b*scb); epi 0 bf16, 1 fp32 (=)
int dl_gemm_small_batched(int epi, const bf16_t* A, long sam, long sak, long sab, const bf16_t* B, long sbn, long sbk,
                          long sbb, int M, int N, int K, bf16_t* C, long ldc, float* Cf, long ldcf, long scb,
                          int batch, hipStream_t st);
// stats (epi 0, splits 1 only): BatchNorm statistics of the stored values as in dl_gemm8 EPI 4
// (stat_rows a multiple of 128 dividing M)
int dl_gemm_small(int epi, const bf16_t* A, long sam, long sak, const bf16_t* B, long sbn, long sbk, int M, int N,
                  int K, bf16_t* C, long ldc, float* Cf, long ldcf, int accumulate, const float* bias, const bf16_t* R,
                  long ldr, int splits, float* ws, hipStream_t st, float* stats = nullptr, long stat_rows = 0,
                  const DlBnBwdEpi* bn = nullptr);

// Implicit-GEMM convolutions on MFMA for the SwAV ResNet-50 trunk.
//
// Activations are NHWC bf16 (torch channels_last), weights KRSC (the flat fp32 master buffer stores
// every conv weight channels-last, utils/flat.py), so one gathered-operand GEMM covers all three
// passes with no im2col buffer and no layout transposes (the 3-channel stem is the one exception:
// it is lowered to an explicit im2col matrix, then runs as a 1x1 conv over it):
//
//   forward  Y[m=(n,p,q), k]     = sum_{t=(r,s), c} X[n, p*st+r-pad, q*st+s-pad, c] * W[k, t, c]
//   dgrad    dX[(n,h,w), c]      = same kernel over dY with the tap-transposed weights; a stride-2
//                                  conv splits into stride^2 parity classes (h = i*st + a), each a
//                                  dense stride-1 sub-convolution over only its contributing taps
//   wgrad    dW[k, (t, c)]      += sum_m dY[m, k] * X[pixel(m, t), c]     (fp32, split-K atomics)
//
// A "geometry" (DlConvGeom) describes the gathered operand: an NHWC image [Nimg, H, W, C], a grid
// of GEMM rows m = (n, i, j) over [Nimg, I, J], and a tap lattice t = (tr, ts) whose pixel is
// (i*sh + dh0 + tr*dhs, j*sw + dw0 + ts*dws); out-of-image taps read as zero (padding).
//
// Tiling (cdna_hip_programming.md §5): 128x128x64 workgroup tile, 4 waves (2 x 2) of 64x64 =
// 4x4 v_mfma_f32_16x16x32_bf16 tiles, register-staged double-buffered LDS (T14: tile t+1's global
// loads are issued before tile t's MFMAs and written to the other buffer after them), XOR-swizzled
// LDS images (K-inner rows read with ds_read_b128, K-outer rows with ds_read_b64_tr_b16), 64 KiB
// LDS and <=256 VGPRs so two workgroups share a CU, XCD-aware tile order (T1).  Gathered loads are
// unconditional 16-byte buffer loads whose padding taps read zeros through the descriptor's range
// check, so the compiler never branches around a load (§5 item 4(c)) and never waits early; two
// register stage sets keep two k-tiles of loads in flight.  The forward kernel swaps the MFMA
// operand roles so each lane owns 4 consecutive output channels of one pixel (8-byte NHWC stores).
#include <algorithm>
#include <cstdlib>

#include "dl_common.h"
#include "dl_kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s4_t __attribute__((ext_vector_type(4)));
typedef short s8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s4_t lds_s4;

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int NT = 256;
constexpr int TILE = BM * BK * 2;  // 16 KiB per operand per stage
constexpr int LDS_BYTES = 4 * TILE;

// K-inner image [128 rows][64 k] (128-B rows, 8 chunks of 16 B): chunk c of row r at c ^ ((r>>1)&7)
__device__ __forceinline__ int kin_off(int row, int c) { return row * 128 + ((c ^ ((row >> 1) & 7)) << 4); }
// K-outer image [64 k][128 rows] (256-B rows, 16 chunks): chunk c of k-row r at c ^ 2((r&3)|((r>>1)&4)),
// so the four k-rows of one ds_read_b64_tr_b16 land on distinct bank groups
__device__ __forceinline__ int kout_off(int krow, int c) {
  return krow * 256 + ((c ^ (((krow & 3) | ((krow >> 1) & 4)) << 1)) << 4);
}

__device__ __forceinline__ floatx4 mfma16(bf16x8 a, bf16x8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// 16 rows x 32 k fragment: lane l -> row r0 + (l&15), k = 8*(l>>4) + j  (either image kind)
template <bool KOUTER>
__device__ __forceinline__ bf16x8 load_frag(const uint8_t* img, int r0, int ksub, int lane) {
  if constexpr (!KOUTER) {
    return *reinterpret_cast<const bf16x8*>(img + kin_off(r0 + (lane & 15), 4 * ksub + (lane >> 4)));
  } else {
    const int g = lane >> 4, i = lane & 15;
    const int krow = 32 * ksub + 8 * g + (i >> 2);
    const int col = r0 + 4 * (i & 3);
    const int o1 = kout_off(krow, col >> 3) + ((col & 7) << 1);
    const int o2 = kout_off(krow + 4, col >> 3) + ((col & 7) << 1);
    const s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + o1));
    const s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + o2));
    const s8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
  }
}

struct Stage { uint4 v[4]; };

// thread `tid`, slot u: K-inner tiles put chunk (tid&7) of row (tid>>3)+32u; K-outer tiles put
// chunk (tid&15) of k-row (tid>>4)+16u
__device__ __forceinline__ void st_kin(const Stage& s, uint8_t* img) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int idx = threadIdx.x + NT * u;
    *reinterpret_cast<uint4*>(img + kin_off(idx >> 3, idx & 7)) = s.v[u];
  }
}
__device__ __forceinline__ void st_kout(const Stage& s, uint8_t* img) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int idx = threadIdx.x + NT * u;
    *reinterpret_cast<uint4*>(img + kout_off(idx >> 4, idx & 15)) = s.v[u];
  }
}

// Gathered operands are read with raw buffer loads (SRSRC descriptor, 32-bit byte offsets): a padding
// tap or a row past the end gets an offset beyond num_records and the hardware returns zeros, so no
// select consumes the loaded value early (a select right after the load forces a vmcnt wait there and
// serialises the prefetch pipeline).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr unsigned OOB = 0xFFFFFFF0u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 bload(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0);
  return uint4{v.x, v.y, v.z, v.w};
}

// exact a / b for 0 <= a < 2^24 through one float reciprocal (+-1 correction)
__device__ __forceinline__ int fdiv(int a, int b, float rb) {
  int q = (int)((float)a * rb);
  const int r = a - q * b;
  q += (r >= b) - (r < 0);
  return q;
}

// =============================================================================================
// forward / dgrad:  out[pixel(m), n] = sum_k A(m, k) W[n, k],  A gathered K-inner
// =============================================================================================
struct FwdArgs {
  DlConvGeom g;
  const bf16_t* w;
  long ldw;
  int N;  // output channels
  bf16_t* out;
  int OH, OW, osh, osw, oh0, ow0;
  long ldo;
  int M, K;
  unsigned img_bytes, w_bytes;
  int tpw;  // output tiles per workgroup
  float* stats;    // optional BatchNorm statistics [M / stat_rows][2N] of the stored output
  long stat_rows;
  DlBnBwdEpi bn;   // bnbwd: the stored output is the data gradient of a BatchNorm+ReLU's output,
  int bnbwd;       // prepared for that BN's backward (as gemm8's EPI_BNBWD): ReLU-masked, and
                   // `stats` receives its two column sums (sum g, sum g * xhat)
};

// One launch over up to MAXJ independent jobs of the same kernel variant (the stride^2 parity
// classes of a strided data gradient: four quarter-size grids launched back to back left the GPU
// three-quarters idle in each).  Dispatch-order workgroups [wg_begin[c], wg_begin[c+1]) run job c,
// each job's range a multiple of 8 long so that the XCD remap applies inside it (a remap over the
// whole grid would put each job on a contiguous quarter of the XCDs); the job index is
// wave-uniform, so its arguments stay scalar loads.
constexpr int MAXJ = 4;
struct FwdMulti {
  FwdArgs a[MAXJ];
  int wg_begin[MAXJ + 1];
  int n;
};

// Tile shapes: TM_ x TN_ = 128 x 128 (four 64 x 64 waves as 2 x 2) or 256 x 64 (4 x 1) for
// outputs of at most 64 channels — the 64-channel 3x3 convs of the first stage would leave half of
// a 128-wide channel tile empty.  The per-wave MFMA work is the same 64 x 64 in both.
template <int U>
struct StageN {
  uint4 v[U];
};
// thread `tid`, slot u: K-inner tiles put chunk (tid&7) of row (tid>>3)+32u
template <int U>
__device__ __forceinline__ void st_kin_n(const StageN<U>& s, uint8_t* img) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int idx = threadIdx.x + NT * u;
    *reinterpret_cast<uint4*>(img + kin_off(idx >> 3, idx & 7)) = s.v[u];
  }
}

// SUB: C < 64 (a divisor of 64, multiple of 8): a 64-deep k-step spans 64 / C taps, so each thread
// decodes the tap of its own 8-channel chunk (the space-to-depth stem: C = 16, 4 x 4 taps)
// MULTI: the launch holds several jobs (FwdMulti); otherwise a[0] only, with static argument
// offsets (a run-time job index in every launch cost the forward 3-4%)
template <int TM_, int TN_, bool SUB = false, bool MULTI = false>
__global__ __launch_bounds__(NT, 2) void conv_fwd_kernel(const FwdMulti P) {
  constexpr int WN = TN_ / 64, UA = TM_ / 32, UB = TN_ / 32;
  int job = 0, bid;
  if constexpr (MULTI) {
    const int b = blockIdx.x;
#pragma unroll
    for (int q = 1; q < MAXJ; ++q) job += (q < P.n && b >= P.wg_begin[q]);
    bid = xcd_remap(b - P.wg_begin[job], P.wg_begin[job + 1] - P.wg_begin[job]);
  } else {
    bid = xcd_remap(blockIdx.x, gridDim.x);
  }
  const FwdArgs& p = P.a[MULTI ? job : 0];
  constexpr int CPR = TN_ / 8;            // 16-byte chunks per staged output row
  constexpr int AIMG = TM_ * 128;         // A image bytes (64 k per row)
  constexpr int SBYTES = (TM_ + TN_) * 128;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const DlConvGeom& g = p.g;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv / WN, wn = wv % WN;
  const int tiles_n = (p.N + TN_ - 1) / TN_;
  const int tiles_m = (p.M + TM_ - 1) / TM_;
  const int ntiles = tiles_m * tiles_n;
  // persistent over `tpw` consecutive output tiles (same pixel rows, successive channel blocks
  // first): the load stream runs on across tile boundaries, so short-K convs (1x1 over 64-256
  // channels: 1-4 k-steps per tile) keep loads in flight under the previous tile's MFMAs/epilogue
  const int tile0 = bid * p.tpw;
  const int mytiles = min(p.tpw, ntiles - tile0);
  if (mytiles <= 0) return;
  const int nk = p.K / BK;
  const int IJ = g.I * g.J;
  const int cofs = (tid & 7) * 8;
  // float reciprocals for the per-lane pixel decodes (fdiv: exact below 2^24, checked on the host);
  // an integer division by a run-time divisor is ~20 VALU, fdiv ~6
  const float rIJ = 1.f / (float)IJ, rJ = 1.f / (float)g.J, rC = 1.f / (float)g.C, rTS = 1.f / (float)g.TS;

  // load cursor: per-thread decoded gathered rows of the tile being loaded
  int dec_tile = -1;
  int hb[UA], wb[UA], nb[UA], brow[UB];
  auto decode = [&](int tile) {
    dec_tile = tile;
    const int m0 = (tile / tiles_n) * TM_, n0 = (tile % tiles_n) * TN_;
#pragma unroll
    for (int u = 0; u < UA; ++u) {
      const int m = m0 + (tid >> 3) + 32 * u;
      if (m < p.M) {
        const int n = fdiv(m, IJ, rIJ), r = m - n * IJ;
        const int i = fdiv(r, g.J, rJ), j = r - i * g.J;
        hb[u] = i * g.sh;
        wb[u] = j * g.sw;
        nb[u] = n * g.H;
      } else {
        hb[u] = -(1 << 29);  // never inside the image -> zero row
        wb[u] = 0;
        nb[u] = 0;
      }
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) brow[u] = min(n0 + (tid >> 3) + 32 * u, p.N - 1);
  };

  const __amdgpu_buffer_rsrc_t rimg = make_rsrc(g.img, p.img_bytes);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w, p.w_bytes);
  const int nsteps = mytiles * nk;
  // Step cursor: load_step is called for s = 0, 1, 2, ... in order, so the step's tile, its k0 and
  // (non-SUB) the tap (tr, ts) and channel offset of k0 advance incrementally — the K loop divides
  // by nothing (four run-time divisions per step were ~100 VALU beside 32 MFMAs per wave).
  int cur_s = -1, cur_tile = tile0, cur_kk = 0, cur_c0 = 0, cur_t = 0, cur_tr = 0, cur_ts = 0;
  auto advance = [&]() {
    if (cur_s < 0) {
      cur_s = 0;
      return;
    }
    ++cur_s;
    if (++cur_kk == nk) {
      cur_kk = 0;
      ++cur_tile;
      cur_c0 = cur_t = cur_tr = cur_ts = 0;
    } else if (!SUB) {
      cur_c0 += BK;  // C is a multiple of BK: one tap per C / BK steps
      if (cur_c0 == g.C) {
        cur_c0 = 0;
        ++cur_t;
        if (++cur_ts == g.TS) {
          cur_ts = 0;
          ++cur_tr;
        }
      }
    }
  };
  // stage step s (clamped: steps past the end reload the last one; staged, never computed)
  auto load_step = [&](StageN<UA>& sa, StageN<UB>& sb, int s) {
    if (cur_s < min(s, nsteps - 1)) advance();
    const int tile = cur_tile, k0 = cur_kk * BK;
    if (tile != dec_tile) decode(tile);
    int t, cc, tr, ts;  // tap and channel offset of this thread's chunk
    if constexpr (SUB) {
      const int kk = k0 + cofs;
      t = fdiv(kk, g.C, rC);
      cc = kk - t * g.C;
      tr = fdiv(t, g.TS, rTS);
      ts = t - tr * g.TS;
    } else {
      t = cur_t;
      cc = cur_c0 + cofs;
      tr = cur_tr;
      ts = cur_ts;
    }
    const int dh = g.dh0 + tr * g.dhs, dw = g.dw0 + ts * g.dws;
#pragma unroll
    for (int u = 0; u < UA; ++u) {
      const int h = hb[u] + dh, w = wb[u] + dw;
      const bool ok = (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
      const unsigned off = 2u * ((unsigned)((nb[u] + h) * g.W + w) * (unsigned)g.C + (unsigned)cc);
      sa.v[u] = bload(rimg, ok ? off : OOB);
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) sb.v[u] = bload(rw, 2u * ((unsigned)brow[u] * (unsigned)p.ldw + (unsigned)(k0 + cofs)));
  };

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const uint8_t* Ai) {
    const uint8_t* Bi = Ai + AIMG;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) af[mi] = load_frag<false>(Ai, wm * 64 + mi * 16, ks, lane);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const bf16x8 bfr = load_frag<false>(Bi, wn * 64 + ni * 16, ks, lane);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) acc[ni][mi] = mfma16(bfr, af[mi], acc[ni][mi]);
      }
    }
  };

  // acc[ni][mi][i] = out[pixel m0+wm*64+mi*16+(lane&15)][channel n0+wn*64+ni*16+4*(lane>>4)+i].
  // The TM_ x TN_ bf16 tile (32 KiB) is staged through the LDS buffer the pipeline is not using
  // (`stage`: [TM_ pixels][CPR chunks of 16 B], chunk c of row r at c ^ (r & (CPR-1))) and written
  // back as whole pixel rows (16 B per lane), instead of 8-byte pieces scattered over 16 rows.
  auto epilogue = [&](int tile, uint8_t* stage) {
    const int m0 = (tile / tiles_n) * TM_, n0 = (tile % tiles_n) * TN_;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int row = wm * 64 + mi * 16 + (lane & 15);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int col = wn * 64 + ni * 16 + 4 * (lane >> 4);  // channel within the tile
        uint2 v;
        v.x = (uint32_t)f2bf(acc[ni][mi][0]) | ((uint32_t)f2bf(acc[ni][mi][1]) << 16);
        v.y = (uint32_t)f2bf(acc[ni][mi][2]) | ((uint32_t)f2bf(acc[ni][mi][3]) << 16);
        *reinterpret_cast<uint2*>(stage + row * (CPR * 16) + (((col >> 3) ^ (row & (CPR - 1))) << 4) +
                                  ((col & 7) << 1)) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    // thread tid always writes channel chunk tid % CPR (8 channels) of rows tid / CPR + (NT / CPR) u
    float csum[8], csq[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] = csq[e] = 0.f;
    // bnbwd: this thread's 8 channels of the tile's statistics group (mean / rstd, and the ReLU
    // mask's scale / shift when it comes from the BN input X)
    float bmu[8], brs[8], bsc[8], bsh[8];
    if (p.bnbwd) {
      const int ch0 = min(n0 + (tid % CPR) * 8, p.N - 8);
      const long go = (long)(m0 / p.stat_rows) * p.N + ch0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float mu = p.bn.mean[go + e];
        brs[e] = p.bn.rstd[go + e];
        bmu[e] = -mu * brs[e];  // xhat = x * rstd + bmu
        bsc[e] = p.bn.Y ? 0.f : p.bn.gamma[ch0 + e] * brs[e];
        bsh[e] = p.bn.Y ? 0.f : p.bn.beta[ch0 + e] - mu * bsc[e];
      }
    }
#pragma unroll
    for (int u = 0; u < TM_ * CPR / NT; ++u) {
      const int idx = tid + NT * u, row = idx / CPR, c = idx % CPR;
      const int m = m0 + row, ch = n0 + c * 8;
      uint4 v = *reinterpret_cast<const uint4*>(stage + row * (CPR * 16) + ((c ^ (row & (CPR - 1))) << 4));
      if (m < p.M && ch < p.N) {
        const int n = fdiv(m, IJ, rIJ), r = m - n * IJ;
        const int i = fdiv(r, g.J, rJ), j = r - i * g.J;
        const long pix = (long)(n * p.OH + i * p.osh + p.oh0) * p.OW + j * p.osw + p.ow0;
        bf16_t* orow = p.out + pix * p.ldo;
        if (p.bnbwd) {  // g = dY masked by the BN's ReLU; the BN backward's two sums
          float f[8], xv[8], yv[8];
          unpack8_bf16(v, f);
          load_bf16<8>(p.bn.X + pix * p.bn.ldx + ch, xv);
          bool live[8];
          if (p.bn.Y) {  // uniform: the mask source is chosen once, not per element
            load_bf16<8>(p.bn.Y + pix * p.bn.ldx + ch, yv);
#pragma unroll
            for (int e = 0; e < 8; ++e) live[e] = yv[e] > 0.f;
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) live[e] = fmaf(xv[e], bsc[e], bsh[e]) > 0.f;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float gg = live[e] ? f[e] : 0.f;  // f is bf16 already: the masked store is exact
            f[e] = gg;
            csum[e] += gg;
            csq[e] = fmaf(gg, fmaf(xv[e], brs[e], bmu[e]), csq[e]);
          }
          v = pack8_bf16(f);
          *reinterpret_cast<uint4*>(orow + ch) = v;
        } else {
          *reinterpret_cast<uint4*>(orow + ch) = v;
        }
        if (p.stats && !p.bnbwd) {
          float f[8];
          unpack8_bf16(v, f);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            csum[e] += f[e];
            csq[e] = fmaf(f[e], f[e], csq[e]);
          }
        }
      }
    }
    if (p.stats) {
      // Atomics are issue-bound (one wave-instruction per ~50 ns per CU, MI355X_MICROARCH.md), so
      // the tile's 2 x TN_ statistics are folded before they leave: the lanes of a wave that share
      // a chunk (shuffles), then the 4 waves in the (drained) staging buffer, and one thread per
      // value adds it — 2-4 wave-instructions per tile.
#pragma unroll
      for (int e = 0; e < 8; ++e) {
#pragma unroll
        for (int d = CPR; d < 64; d *= 2) {
          csum[e] += __shfl_xor(csum[e], d, 64);
          csq[e] += __shfl_xor(csq[e], d, 64);
        }
      }
      __syncthreads();  // every staged row has been read: the buffer is free
      float* red = reinterpret_cast<float*>(stage);  // [wave][moment][TN_ channels]
      if (lane < CPR) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          red[wv * 2 * TN_ + lane * 8 + e] = csum[e];
          red[wv * 2 * TN_ + TN_ + lane * 8 + e] = csq[e];
        }
      }
      __syncthreads();
      if (tid < 2 * TN_) {
        const float v = red[tid] + red[2 * TN_ + tid] + red[4 * TN_ + tid] + red[6 * TN_ + tid];
        const int chl = tid % TN_, mom = tid / TN_;
        if (n0 + chl < p.N) atomicAdd(p.stats + (m0 / p.stat_rows) * 2L * p.N + (long)mom * p.N + n0 + chl, v);
      }
    }
    __syncthreads();  // the staging buffer is restaged by the pipeline right after
  };

  if (nk == 0) {  // no contributing tap (a dgrad parity class): the tiles are zero
    for (int t = 0; t < mytiles; ++t) epilogue(tile0 + t, smem);
    return;
  }

  // Two register stage sets (x: even steps, y: odd steps) keep the global loads of steps s+1 AND
  // s+2 in flight while step s computes.  The loop body is branch-free around the loads and LDS
  // stores, so the compiler's wait counting sees the true issue order and waits only for the set
  // it is about to store.
  uint8_t* buf0 = smem;
  uint8_t* buf1 = smem + SBYTES;
  StageN<UA> xa, ya;
  StageN<UB> xb, yb;
  load_step(xa, xb, 0);
  load_step(ya, yb, 1);
  st_kin_n(xa, buf0);
  st_kin_n(xb, buf0 + AIMG);
  load_step(xa, xb, 2);
  __syncthreads();
  int ekk = 0, etile = tile0;  // k-step and tile of the step being computed
  for (int s = 0; s < nsteps; s += 2) {
    compute(buf0);  // step s
    if (++ekk == nk) {
      epilogue(etile++, buf1);  // buf1: drained, not yet restaged
      ekk = 0;
    }
    st_kin_n(ya, buf1);
    st_kin_n(yb, buf1 + AIMG);
    load_step(ya, yb, s + 3);
    __syncthreads();
    if (s + 1 < nsteps) {
      compute(buf1);  // step s + 1
      if (++ekk == nk) {
        epilogue(etile++, buf0);
        ekk = 0;
      }
    }
    st_kin_n(xa, buf0);
    st_kin_n(xb, buf0 + AIMG);
    load_step(xa, xb, s + 4);
    __syncthreads();
  }
}

// =============================================================================================
// wgrad:  dW[k, col] += sum_m dY[m, k] * B(col, m),  col = (t, c), both operands K-outer
// =============================================================================================
// Gathered-operand k-row of thread quad q (the wgrad kernels' register-staged B images): quads 2j and
// 2j + 1 take rows b and b + 2, so the two k-rows of each 8-lane ds_write_b128 group have kout
// swizzles that differ in chunk bit 2 and fill 32 distinct banks (rows b, b + 1 hit 16 banks twice)
__device__ __forceinline__ int gather_row(int q) { return (q & ~3) | ((q & 1) << 1) | ((q >> 1) & 1); }

struct WgradArgs {
  DlConvGeom g;
  const bf16_t* dy;
  long ldy;
  int Cout;
  float* dw;
  long lddw;
  int Ncols;   // stored gradient columns (<= gathered rows)
  int Brows;   // gathered operand extent TR*TS*C (load clamp)
  int M;       // reduction extent Nimg*I*J
  int m_per_split;
  float rIJ, rJ;
  unsigned img_bytes, dy_bytes;
};

__global__ __launch_bounds__(NT, 2) void conv_wgrad_kernel(WgradArgs p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const DlConvGeom& g = p.g;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int tiles_n = (p.Ncols + BN - 1) / BN;
  const int tiles_m = (p.Cout + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (bid / tiles_n) * BM, n0 = (bid % tiles_n) * BN;
  const int kbeg = blockIdx.z * p.m_per_split;
  const int kend = min(p.M, kbeg + p.m_per_split);
  if (kbeg >= kend) return;
  const int nk = (kend - kbeg + BK - 1) / BK;
  const int IJ = g.I * g.J;

  const int chunk = tid & 15, krow0 = tid >> 4;
  const int acol = min(m0 + chunk * 8, p.Cout - 8);
  // gathered operand: thread = one pixel row (tid >> 2) x chunks (tid & 3) + 4u, so the pixel
  // decode (two divisions) runs once per thread and k-step instead of once per chunk; the chunks'
  // tap offsets and channels are fixed per workgroup
  const int brow = gather_row(tid >> 2);
  int bdh[4], bdw[4], bc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int kk = min(n0 + ((tid & 3) + 4 * u) * 8, p.Brows - 8);
    const int t = kk / g.C;
    bc[u] = kk - t * g.C;
    const int tr = t / g.TS, ts = t - tr * g.TS;
    bdh[u] = g.dh0 + tr * g.dhs;
    bdw[u] = g.dw0 + ts * g.dws;
  }

  const __amdgpu_buffer_rsrc_t rimg = make_rsrc(g.img, p.img_bytes);
  const __amdgpu_buffer_rsrc_t rdy = make_rsrc(p.dy, p.dy_bytes);
  auto load_a = [&](Stage& s, int k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int m = kbeg + k0 + krow0 + 16 * u;
      const unsigned off = 2u * ((unsigned)m * (unsigned)p.ldy + (unsigned)acol);
      s.v[u] = bload(rdy, m < kend ? off : OOB);
    }
  };
  auto load_b = [&](Stage& s, int k0) {
    const int m = kbeg + k0 + brow;
    const int n = fdiv(m, IJ, p.rIJ), r = m - n * IJ;
    const int i = fdiv(r, g.J, p.rJ), j = r - i * g.J;
    const int h0 = i * g.sh, w0 = j * g.sw, nh = n * g.H;
    const bool mok = m < kend;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int h = h0 + bdh[u], w = w0 + bdw[u];
      const bool ok = mok && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
      const unsigned off = 2u * ((unsigned)((nh + h) * g.W + w) * (unsigned)g.C + (unsigned)bc[u]);
      s.v[u] = bload(rimg, ok ? off : OOB);
    }
  };
  auto st_b = [&](const Stage& s, uint8_t* img) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      *reinterpret_cast<uint4*>(img + kout_off(brow, (tid & 3) + 4 * u)) = s.v[u];
  };

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const uint8_t* Ai) {
    const uint8_t* Bi = Ai + TILE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 bfr[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bfr[ni] = load_frag<true>(Bi, wn * 64 + ni * 16, ks, lane);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const bf16x8 af = load_frag<true>(Ai, wm * 64 + mi * 16, ks, lane);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = mfma16(af, bfr[ni], acc[mi][ni]);
      }
    }
  };

  // 2-deep register prefetch (see the forward kernel)
  uint8_t* buf0 = smem;
  uint8_t* buf1 = smem + 2 * TILE;
  Stage xa, xb, ya, yb;
  const int last = (nk - 1) * BK;  // branch-free loop body, clamped tile indices (forward kernel)
  load_a(xa, 0);
  load_b(xb, 0);
  load_a(ya, min(BK, last));
  load_b(yb, min(BK, last));
  st_kout(xa, buf0);
  st_b(xb, buf0 + TILE);
  load_a(xa, min(2 * BK, last));
  load_b(xb, min(2 * BK, last));
  __syncthreads();
  for (int s = 0; s < nk; s += 2) {
    compute(buf0);
    st_kout(ya, buf1);
    st_b(yb, buf1 + TILE);
    load_a(ya, min((s + 3) * BK, last));
    load_b(yb, min((s + 3) * BK, last));
    __syncthreads();
    if (s + 1 < nk) compute(buf1);
    st_kout(xa, buf0);
    st_b(xb, buf0 + TILE);
    load_a(xa, min((s + 4) * BK, last));
    load_b(xb, min((s + 4) * BK, last));
    __syncthreads();
  }

  // acc[mi][ni][i] = dW[channel m0+wm*64+mi*16+4*(lane>>4)+i][col n0+wn*64+ni*16+(lane&15)]
  const bool split = gridDim.z > 1;
  float* out = p.dw;
  const long ld = p.lddw;
  const bool atomics = split;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ch = m0 + wm * 64 + mi * 16 + 4 * (lane >> 4) + i;
      if (ch >= p.Cout) continue;
      float* drow = out + (long)ch * ld;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int col = n0 + wn * 64 + ni * 16 + (lane & 15);
        if (col >= p.Ncols) continue;
        if (atomics) atomicAdd(drow + col, acc[mi][ni][i]);
        else if (split) drow[col] = acc[mi][ni][i];
        else drow[col] += acc[mi][ni][i];
      }
    }
  }
}

// =============================================================================================
// im2col for the 3-channel stem: col[m=(n,p,q)][r*SCp + s*C + c], each filter row (r) padded from
// S*C (21) to SCp (24) columns so every 16-byte chunk belongs to one filter row; columns
// [R*SCp, Kp) are zero.
// =============================================================================================
template <int C>
__global__ __launch_bounds__(256) void im2col_kernel(const bf16_t* __restrict__ x, int H, int W, int R, int stride,
                                                     int pad, int P, int Q, int SCp, int Kp, bf16_t* __restrict__ col,
                                                     int chunks, int SC) {
  // one thread per 16-byte chunk (8 columns) of the matrix, so a wave writes 1 KiB contiguously.
  // Within filter row r the columns s*C + c of pixel (p, q) are x[n, h, w0*C + k] for k = s*C + c:
  // a contiguous run of the NHWC row, valid while w0 + k/C lies inside the image.  32-bit index
  // math throughout (the launcher checks the chunk count) and a compile-time C: 64-bit and
  // run-time divisions made the first version 2.5x slower than its store bandwidth.
  const int cpr = Kp >> 3, cpf = SCp >> 3;  // chunks per matrix row / per filter row
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < chunks; idx += gridDim.x * blockDim.x) {
    const int m = idx / cpr;
    const int j = idx - m * cpr;
    const int r = j / cpf, k0 = (j - r * cpf) * 8;
    uint32_t w32[4] = {0u, 0u, 0u, 0u};
    if (r < R) {
      const int t = m / Q, q = m - t * Q;
      const int n = t / P, pp = t - n * P;
      const int h = pp * stride - pad + r, w0 = q * stride - pad;
      if ((unsigned)h < (unsigned)H) {
        const bf16_t* row = x + (((long)n * H + h) * W + w0) * C;  // may point before the row: guarded below
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = k0 + e;
          const int w = w0 + k / C;
          const bf16_t v = (k < SC && (unsigned)w < (unsigned)W) ? row[k] : (bf16_t)0;
          w32[e >> 1] |= (uint32_t)v << (16 * (e & 1));
        }
      }
    }
    *reinterpret_cast<uint4*>(col + (long)m * Kp + j * 8) = uint4{w32[0], w32[1], w32[2], w32[3]};
  }
}

// Weight gradient for Cout <= 64 (the stem and the first stage's convs): the 128 x 128 tile above
// would compute 64 duplicate output rows.  Here a workgroup owns 64 output channels x 256 gathered
// columns, its four waves side by side along the columns (64 x 64 each, the same MFMA work per wave
// and k-step as the wide kernel).  The dY image holds 64-column k-rows (128 B) with its own swizzle:
// 32-byte segment s of k-row r at s ^ f(r), f(r) = ((r >> 1) & 1) | (((r >> 3) & 1) << 1), so the
// eight k-rows of one ds_read_b64_tr_b16 lane group (r, r+1, r+2, r+3, r+8 ... r+11; segment fixed)
// fall on eight distinct 32-byte bank groups.  The gathered operand is two standard 128-column
// images.  LDS: 2 stages x (8 + 32) KiB = 80 KiB, two workgroups per CU.
constexpr int NW_AIMG = 64 * 128;           // dY image: 64 k-rows x 64 channels
constexpr int NW_STAGE = NW_AIMG + 2 * TILE;  // + two 128-column gathered images
constexpr int NW_LDS = 2 * NW_STAGE;

__device__ __forceinline__ int kout64_off(int krow, int c) {  // c: 16-byte chunk 0..7 of the k-row
  const int f = ((krow >> 1) & 1) | (((krow >> 3) & 1) << 1);
  return krow * 128 + (((((c >> 1) ^ f) << 1) | (c & 1)) << 4);
}
__device__ __forceinline__ bf16x8 load_frag64(const uint8_t* img, int r0, int ksub, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int krow = 32 * ksub + 8 * g + (i >> 2);
  const int col = r0 + 4 * (i & 3);
  const int o1 = kout64_off(krow, col >> 3) + ((col & 7) << 1);
  const int o2 = kout64_off(krow + 4, col >> 3) + ((col & 7) << 1);
  const s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + o1));
  const s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + o2));
  const s8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

struct NarrowStage {
  uint4 a[2];  // dY: chunk (tid & 7) of k-rows (tid >> 3) + 32u
  uint4 b[8];  // gathered: chunks (tid & 3) + 4u of k-row (tid >> 2)
};

__global__ __launch_bounds__(NT, 2) void conv_wgrad_narrow_kernel(WgradArgs p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const DlConvGeom& g = p.g;
  const int tid = threadIdx.x, lane = tid & 63, wn = tid >> 6;
  const int tiles_n = (p.Ncols + 255) / 256;
  const int bid = xcd_remap(blockIdx.x, tiles_n);
  const int n0 = bid * 256;
  const int kbeg = blockIdx.z * p.m_per_split;
  const int kend = min(p.M, kbeg + p.m_per_split);
  if (kbeg >= kend) return;
  const int nk = (kend - kbeg + BK - 1) / BK;
  const int IJ = g.I * g.J;

  const int achunk = tid & 7, akrow = tid >> 3;
  const int acol = min(achunk * 8, p.Cout - 8);
  // gathered operand: thread = one pixel row (tid >> 2) x chunks (tid & 3) + 4u (see the wide kernel)
  const int brow = gather_row(tid >> 2);
  int bdh[8], bdw[8], bc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int kk = min(n0 + ((tid & 3) + 4 * u) * 8, p.Brows - 8);
    const int t = kk / g.C;
    bc[u] = kk - t * g.C;
    const int tr = t / g.TS, ts = t - tr * g.TS;
    bdh[u] = g.dh0 + tr * g.dhs;
    bdw[u] = g.dw0 + ts * g.dws;
  }

  const __amdgpu_buffer_rsrc_t rimg = make_rsrc(g.img, p.img_bytes);
  const __amdgpu_buffer_rsrc_t rdy = make_rsrc(p.dy, p.dy_bytes);
  auto load = [&](NarrowStage& s, int k0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int m = kbeg + k0 + akrow + 32 * u;
      const unsigned off = 2u * ((unsigned)m * (unsigned)p.ldy + (unsigned)acol);
      s.a[u] = bload(rdy, m < kend ? off : OOB);
    }
    const int m = kbeg + k0 + brow;
    const int n = fdiv(m, IJ, p.rIJ), r = m - n * IJ;
    const int i = fdiv(r, g.J, p.rJ), j = r - i * g.J;
    const int h0 = i * g.sh, w0 = j * g.sw, nh = n * g.H;
    const bool mok = m < kend;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int h = h0 + bdh[u], w = w0 + bdw[u];
      const bool ok = mok && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
      const unsigned off = 2u * ((unsigned)((nh + h) * g.W + w) * (unsigned)g.C + (unsigned)bc[u]);
      s.b[u] = bload(rimg, ok ? off : OOB);
    }
  };
  auto store = [&](const NarrowStage& s, uint8_t* st) {
#pragma unroll
    for (int u = 0; u < 2; ++u) *reinterpret_cast<uint4*>(st + kout64_off(akrow + 32 * u, achunk)) = s.a[u];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int ch = (tid & 3) + 4 * u;  // chunk 0..31 of the 256 columns: image ch >> 4
      *reinterpret_cast<uint4*>(st + NW_AIMG + (ch >> 4) * TILE + kout_off(brow, ch & 15)) = s.b[u];
    }
  };

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const uint8_t* st) {
    const uint8_t* Bi = st + NW_AIMG + (wn >> 1) * TILE;
    const int cb = (wn & 1) * 64;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 bfr[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bfr[ni] = load_frag<true>(Bi, cb + ni * 16, ks, lane);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const bf16x8 af = load_frag64(st, mi * 16, ks, lane);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = mfma16(af, bfr[ni], acc[mi][ni]);
      }
    }
  };

  // 2-deep register prefetch, as the wide kernel
  uint8_t* buf0 = smem;
  uint8_t* buf1 = smem + NW_STAGE;
  NarrowStage x, y;
  const int last = (nk - 1) * BK;
  load(x, 0);
  load(y, min(BK, last));
  store(x, buf0);
  load(x, min(2 * BK, last));
  __syncthreads();
  for (int s = 0; s < nk; s += 2) {
    compute(buf0);
    store(y, buf1);
    load(y, min((s + 3) * BK, last));
    __syncthreads();
    if (s + 1 < nk) compute(buf1);
    store(x, buf0);
    load(x, min((s + 4) * BK, last));
    __syncthreads();
  }

  // acc[mi][ni][i] = dW[channel mi*16+4*(lane>>4)+i][col n0+wn*64+ni*16+(lane&15)]
  const bool split = gridDim.z > 1;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ch = mi * 16 + 4 * (lane >> 4) + i;
      if (ch >= p.Cout) continue;
      float* drow = p.dw + (long)ch * p.lddw;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int col = n0 + wn * 64 + ni * 16 + (lane & 15);
        if (col >= p.Ncols) continue;
        if (split) atomicAdd(drow + col, acc[mi][ni][i]);
        else drow[col] += acc[mi][ni][i];
      }
    }
  }
}

// Space-to-depth of the stem's input: x NHWC [N, H, W, 3] -> xs [N, H/2, W/2, 16], channel
// (2a + b) * 3 + c = x[2i + a, 2j + b, c], channels 12-15 zero.  The 7x7 stride-2 pad-3 stem conv
// over x is then a 4x4 stride-1 conv over xs (taps i - 2 .. i + 1, weights remapped by the caller):
// one implicit GEMM with K = 256 on conv.hip instead of an im2col matrix of 1.6 G bf16 elements.
__global__ __launch_bounds__(256) void stem_s2d_kernel(const bf16_t* __restrict__ x, int N, int H, int W,
                                                       bf16_t* __restrict__ xs) {
  const int H2 = H >> 1, W2 = W >> 1;
  const long total = (long)N * H2 * W2;
  for (long o = blockIdx.x * 256L + threadIdx.x; o < total; o += (long)gridDim.x * 256) {
    const int j = (int)(o % W2);
    const long r = o / W2;
    const int i = (int)(r % H2), n = (int)(r / H2);
    uint32_t w32[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const bf16_t* row = x + (((long)n * H + 2 * i + a) * W + 2 * j) * 3;  // 2 pixels x 3 channels
#pragma unroll
      for (int e = 0; e < 6; ++e) {
        const int ch = a * 6 + e;  // (2a + b) * 3 + c with b = e / 3, c = e % 3
        w32[ch >> 1] |= (uint32_t)row[e] << (16 * (ch & 1));
      }
    }
    uint4* dst = reinterpret_cast<uint4*>(xs + o * 16);
    dst[0] = uint4{w32[0], w32[1], w32[2], w32[3]};
    dst[1] = uint4{w32[4], w32[5], w32[6], w32[7]};
  }
}

template <typename Kern>
void set_lds(Kern k) {
  DL_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
}


// =============================================================================================
// tap-transposed data-gradient weights of many convs in one launch
// =============================================================================================
// One 64 (k) x 64 (c) tile of one tap of one job per workgroup: read as 64 rows of 64 input
// channels (128 B each, KRSC), transposed through LDS, written as 64 rows of 64 output channels
// ([C][TR][TS][K]).  Replaces one strided-permute copy kernel per conv and parity class (41 per
// SwAV iteration, ~270 us on the side stream, 4-15 us each for 0.05-4.7 MB).
constexpr int MAXWJ = 40;
struct WtJobs {
  DlWtJob j[MAXWJ];
  int begin[MAXWJ + 1];  // first tile of each job; begin[n] = the launch's tile count
  int n;
};

__global__ __launch_bounds__(256) void wt_transpose_kernel(const WtJobs P) {
  __shared__ uint16_t tile[64][66];  // +2: a column read walks 33 banks apart
  const int u = blockIdx.x;
  int jb = 0;
  for (int q = 1; q < P.n; ++q) jb += u >= P.begin[q];  // wave-uniform
  const DlWtJob& J = P.j[jb];
  const int local = u - P.begin[jb];
  const int kt = J.K / 64, ct = J.C / 64;
  const int tap = local / (kt * ct), rem = local - tap * (kt * ct);
  const int kb = rem / ct, cb = rem - kb * ct;
  const int tr = tap / J.TS, ts = tap - tr * J.TS;
  const int r = J.r0 + tr * J.st, sc = J.s0 + ts * J.st;
  const int t = threadIdx.x;
#pragma unroll
  for (int h = 0; h < 2; ++h) {  // 512 chunks of 8 channels: row = chunk / 8, 8-channel group = chunk % 8
    const int chunk = t + 256 * h, row = chunk >> 3, g = chunk & 7;
    const long src = (((long)(kb * 64 + row) * J.R + r) * J.S + sc) * J.C + cb * 64 + g * 8;
    const uint4 v = *reinterpret_cast<const uint4*>(J.src + src);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      tile[row][g * 8 + 2 * e] = (uint16_t)(w[e] & 0xffffu);
      tile[row][g * 8 + 2 * e + 1] = (uint16_t)(w[e] >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {  // output row = input channel c, 8 consecutive k per thread
    const int chunk = t + 256 * h, c = chunk >> 3, g = chunk & 7;
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w[e] = (uint32_t)tile[g * 8 + 2 * e][c] | ((uint32_t)tile[g * 8 + 2 * e + 1][c] << 16);
    const long dst = (((long)(cb * 64 + c) * J.TR + tr) * J.TS + ts) * J.K + kb * 64 + g * 8;
    *reinterpret_cast<uint4*>(J.dst + dst) = uint4{w[0], w[1], w[2], w[3]};
  }
}

}  // namespace

#ifndef DL_CONV_FWD_WG
#define DL_CONV_FWD_WG 1024  // (a measurement build may override)
#endif
int dl_conv_fwd_multi(const DlConvFwdJob* jobs, int njobs, int N, bf16_t* out, int OH, int OW, int osh, int osw,
                      long ldo, hipStream_t st, float* stats, const DlBnBwdEpi* bn) {
  if (njobs < 1 || njobs > MAXJ || N % 4 || ldo % 4) return -1;
  if (bn && (!stats || !bn->X || bn->ldx % 8 || (!bn->Y && (!bn->gamma || !bn->beta)))) return -1;
  // validate every job before anything launches (-1: nothing ran); all jobs must take one variant
  int variant = -1;
  long tiles[MAXJ];
  long total = 0;
  for (int c = 0; c < njobs; ++c) {
    const DlConvGeom& g = jobs[c].g;
    const long stat_rows = jobs[c].stat_rows;
    const bool sub = g.C < BK;  // C in {8, 16, 32}: several taps per k-step (SUB kernels)
    if ((sub ? (BK % g.C || g.C % 8) : g.C % BK) || jobs[c].ldw % 8 || g.I < 0 || g.J < 0) return -1;
    if (sub && (bn || (g.TR * g.TS * g.C) % BK)) return -1;
    const long M = (long)g.Nimg * g.I * g.J;
    // statistics: every 128-row tile inside one group, whole 8-channel chunks
    if (stats && M > 0 && (stat_rows < BM || stat_rows % BM || M % stat_rows || N % 8)) return -1;
    if (M >= (1L << 24)) return -1;  // fdiv exactness bound (pixel decodes)
    const long img_bytes = 2L * g.Nimg * g.H * g.W * g.C, w_bytes = 2L * N * jobs[c].ldw;
    if (img_bytes >= (1L << 31) || w_bytes >= (1L << 31)) return -1;  // 32-bit buffer offsets
    // outputs of at most 64 channels: 256 x 64 tiles (the 128-wide channel tile would be half
    // empty; SwAV b=64 2015 / 2037 -> 2058 / 2055 samples/s in round 3)
    const bool narrow = N <= 64 && (!stats || stat_rows % 256 == 0);
    const int v = 2 * sub + narrow;
    tiles[c] = 0;
    if (M == 0 || N == 0) continue;
    if (variant >= 0 && v != variant) return -1;
    variant = v;
    const int TMv = narrow ? 256 : BM, TNv = narrow ? 64 : BN;
    tiles[c] = ((M + TMv - 1) / TMv) * ((N + TNv - 1) / TNv);
    total += tiles[c];
  }
  if (total == 0) return 0;
  if (total >= (1L << 31)) return -1;
  // several jobs: one launch (stride-2 data gradients, SwAV b=64 shapes: 1022 -> 799 us per
  // iteration over the 12 strided convs, every shape faster; profiles/r5_conv_dgrad_merged_classes.jsonl)
  const bool multi = njobs > 1;
  FwdMulti P{};
  int wg = 0;
  auto launch = [&]() {
    const bool sub = variant & 2, narrow = variant & 1;
    const int lds = 2 * ((narrow ? 256 : BM) + (narrow ? 64 : BN)) * 128;
    const dim3 grid(wg);
    if (multi) {
      if (narrow) conv_fwd_kernel<256, 64, false, true><<<grid, NT, lds, st>>>(P);
      else conv_fwd_kernel<BM, BN, false, true><<<grid, NT, lds, st>>>(P);
    } else if (sub) {
      if (narrow) conv_fwd_kernel<256, 64, true><<<grid, NT, lds, st>>>(P);
      else conv_fwd_kernel<BM, BN, true><<<grid, NT, lds, st>>>(P);
    } else {
      if (narrow) conv_fwd_kernel<256, 64><<<grid, NT, lds, st>>>(P);
      else conv_fwd_kernel<BM, BN><<<grid, NT, lds, st>>>(P);
    }
  };
  static bool attr = false;
  if (!attr) {
    DL_HIP_CHECK(hipFuncSetAttribute((const void*)conv_fwd_kernel<BM, BN>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 2 * (BM + BN) * 128));
    DL_HIP_CHECK(hipFuncSetAttribute((const void*)conv_fwd_kernel<256, 64>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 2 * (256 + 64) * 128));
    DL_HIP_CHECK(hipFuncSetAttribute((const void*)conv_fwd_kernel<BM, BN, true>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 2 * (BM + BN) * 128));
    DL_HIP_CHECK(hipFuncSetAttribute((const void*)conv_fwd_kernel<256, 64, true>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 2 * (256 + 64) * 128));
    DL_HIP_CHECK(hipFuncSetAttribute((const void*)conv_fwd_kernel<BM, BN, false, true>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 2 * (BM + BN) * 128));
    DL_HIP_CHECK(hipFuncSetAttribute((const void*)conv_fwd_kernel<256, 64, false, true>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 2 * (256 + 64) * 128));
    attr = true;
  }
  if (multi && (variant & 2)) return -1;  // no SUB job-indexed kernel (data gradients have C >= 64)
  for (int c = 0; c < njobs; ++c) {
    if (tiles[c] == 0) continue;
    const DlConvFwdJob& jb = jobs[c];
    // ~1024 workgroups (two per CU, two rounds); short-K shapes get several tiles per workgroup
    const int tpw = (int)std::max<long>(1, tiles[c] / DL_CONV_FWD_WG);
    const DlConvGeom& g = jb.g;
    FwdArgs& a = P.a[P.n];
    a = FwdArgs{g, jb.w, jb.ldw, N, out, OH, OW, osh, osw, jb.oh0, jb.ow0, ldo, g.Nimg * g.I * g.J, g.TR * g.TS * g.C,
                (unsigned)(2L * g.Nimg * g.H * g.W * g.C), (unsigned)(2L * N * jb.ldw), tpw, stats, jb.stat_rows,
                bn ? *bn : DlBnBwdEpi{}, bn ? 1 : 0};
    P.wg_begin[P.n++] = wg;
    const int jw = (int)((tiles[c] + tpw - 1) / tpw);
    wg += multi ? (jw + 7) / 8 * 8 : jw;  // surplus workgroups find no tile and return
    P.wg_begin[P.n] = wg;
    if (!multi) {  // this job alone
      launch();
      P = FwdMulti{};
      wg = 0;
    }
  }
  if (multi) launch();
  return 0;
}

int dl_conv_fwd(const DlConvGeom& g, const bf16_t* w, long ldw, int N, bf16_t* out, int OH, int OW, int osh, int osw,
                int oh0, int ow0, long ldo, hipStream_t st, float* stats, long stat_rows, const DlBnBwdEpi* bn) {
  const DlConvFwdJob job{g, w, ldw, oh0, ow0, stat_rows};
  return dl_conv_fwd_multi(&job, 1, N, out, OH, OW, osh, osw, ldo, st, stats, bn);
}

// Split count of dl_conv_wgrad: the (long) pixel reduction is split so that ~`target` workgroups
// exist, each split a multiple of the 64-deep k-step and at least 8 k-steps long.  Fewer than one per
// CU leaves slots to the concurrent pass: SwAV b=64 iteration, round 3: 1990-1997 samples/s at 1024,
// 2051-2061 at 256, 2041 at 512; round 5 (same-box A/Bs, profiles/r5_swav_grid_caps_ab.jsonl): 192
// +0.6-0.8% over 256, 128 = 256, 512 -2.8%, 1024 -6.2%
#ifndef DL_CONV_WGRAD_TARGET
#define DL_CONV_WGRAD_TARGET 192  // (a measurement build may override)
#endif
static long wgrad_splits(const DlConvGeom& g, int tiles) {
  const long M = (long)g.Nimg * g.I * g.J;
  constexpr long target = DL_CONV_WGRAD_TARGET;
  const long ksteps = (M + BK - 1) / BK;
  long splits = std::max(1L, std::min<long>((target + tiles - 1) / tiles, ksteps / 8));
  const long steps_per = (ksteps + splits - 1) / splits;
  return (ksteps + steps_per - 1) / steps_per;
}

int dl_conv_wgrad(const DlConvGeom& g, const bf16_t* dy, long ldy, int Cout, float* dw, long lddw, int Ncols,
                  hipStream_t st) {
  const int Brows = g.TR * g.TS * g.C;
  if (g.C % 8 || Cout % 8 || Cout < 8 || ldy % 8 || Brows < 8 || Ncols > Brows) return -1;
  const long M = (long)g.Nimg * g.I * g.J;
  if (M >= (1L << 24)) return -1;  // fdiv exactness bound
  if (M == 0 || Ncols == 0) return 0;
  const bool narrow = Cout <= 64;  // conv_wgrad_narrow_kernel: 64 x 256 tiles
  const int tiles = narrow ? (Ncols + 255) / 256 : ((Cout + BM - 1) / BM) * ((Ncols + BN - 1) / BN);
  const long ksteps = (M + BK - 1) / BK;
  const long splits = wgrad_splits(g, tiles);
  const long steps_per = (ksteps + splits - 1) / splits;
  const long img_bytes = 2L * g.Nimg * g.H * g.W * g.C, dy_bytes = 2L * M * ldy;
  if (img_bytes >= (1L << 31) || dy_bytes >= (1L << 31)) return -1;  // 32-bit buffer offsets
  WgradArgs a{g, dy, ldy, Cout, dw, lddw, Ncols, Brows, (int)M, (int)(steps_per * BK),
              1.f / (float)(g.I * g.J), 1.f / (float)g.J, (unsigned)img_bytes, (unsigned)dy_bytes};
  static bool attr = false;
  if (!attr) {
    set_lds(conv_wgrad_kernel);
    DL_HIP_CHECK(hipFuncSetAttribute((const void*)conv_wgrad_narrow_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, NW_LDS));
    attr = true;
  }
  if (narrow) conv_wgrad_narrow_kernel<<<dim3(tiles, 1, (unsigned)splits), NT, NW_LDS, st>>>(a);
  else conv_wgrad_kernel<<<dim3(tiles, 1, (unsigned)splits), NT, LDS_BYTES, st>>>(a);
  return 0;
}

int dl_conv_dgrad_weights_batched(const DlWtJob* jobs, int njobs, hipStream_t st) {
  for (int c = 0; c < njobs; ++c) {
    const DlWtJob& j = jobs[c];
    if (j.K % 64 || j.C % 64 || j.K <= 0 || j.C <= 0 || j.TR < 1 || j.TS < 1 || j.st < 1 ||
        j.r0 + (j.TR - 1) * j.st >= j.R || j.s0 + (j.TS - 1) * j.st >= j.S)
      return -1;
  }
  for (int c0 = 0; c0 < njobs; c0 += MAXWJ) {
    WtJobs P{};
    P.n = std::min(MAXWJ, njobs - c0);
    long units = 0;
    for (int c = 0; c < P.n; ++c) {
      const DlWtJob& j = jobs[c0 + c];
      P.j[c] = j;
      P.begin[c] = (int)units;
      units += (long)j.TR * j.TS * (j.K / 64) * (j.C / 64);
    }
    if (units >= (1L << 30)) return -1;
    P.begin[P.n] = (int)units;
    if (units) wt_transpose_kernel<<<dim3((unsigned)units), 256, 0, st>>>(P);
  }
  return 0;
}

int dl_stem_s2d(const bf16_t* x, int N, int H, int W, bf16_t* xs, hipStream_t st) {
  if (H % 2 || W % 2 || N < 0) return -1;
  const long total = (long)N * (H / 2) * (W / 2);
  if (total == 0) return 0;
  const int blocks = (int)std::min<long>((total + 255) / 256, 256L * 64);
  stem_s2d_kernel<<<blocks, 256, 0, st>>>(x, N, H, W, xs);
  return 0;
}

int dl_im2col(const bf16_t* x, int N, int H, int W, int C, int R, int S, int stride, int pad, int P, int Q, int SCp,
              int Kp, bf16_t* col, hipStream_t st) {
  if (SCp % 8 || SCp < S * C || Kp % 8 || Kp < R * SCp) return -1;
  const long chunks = (long)N * P * Q * (Kp / 8);
  if (chunks == 0) return 0;
  if (chunks >= (1L << 30) || (C != 3 && C != 4 && C != 1)) return -1;  // int grid-stride loop stays < 2^31
  const int threads = 256;
  const int blocks = (int)std::min<long>((chunks + threads - 1) / threads, 256L * 256);
  auto kern = C == 3 ? im2col_kernel<3> : (C == 4 ? im2col_kernel<4> : im2col_kernel<1>);
  kern<<<dim3(blocks), threads, 0, st>>>(x, H, W, R, stride, pad, P, Q, SCp, Kp, col, (int)chunks, S * C);
  return 0;
}

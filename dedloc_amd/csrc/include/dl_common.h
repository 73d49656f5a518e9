// dedloc_amd — shared device helpers for the gfx950 (CDNA4) kernels.
//
// Conventions used by every kernel in csrc/kernels:
//   * bf16 tensors are passed as raw `uint16_t*` (bit patterns); conversion is done with the
//     round-to-nearest-even helpers below so results are bit-identical to torch's bf16 casts.
//   * a wave is 64 lanes; all reductions use 64-wide xor shuffles (never warp-32 idioms).
//   * every launcher takes an explicit hipStream_t and never allocates or synchronises, so the
//     whole training micro-step can be captured into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DL_WAVE 64

#define DL_HIP_CHECK(expr)                                                              \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__, __LINE__); \
      abort();                                                                          \
    }                                                                                   \
  } while (0)

typedef uint16_t bf16_t;
typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// f32 -> bf16, round-to-nearest-even, by the hardware converter (v_cvt_pk_bf16_f32): bit-identical
// to torch's cast for every finite value and infinity, NaN stays NaN, and branch-free — the integer
// rounding sequence with its NaN test cost VALU-bound kernels up to ~25% (bench/ew_bench.py).
__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}

// Hardware f32 -> bf16 (v_cvt_pk_bf16_f32: round-to-nearest-even, NaN stays NaN), branch-free:
// same results as f2bf for every input except the NaN payload bits.
typedef float dl_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 dl_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2_bf16(float a, float b) {
  // one two-source v_cvt_pk_bf16_f32 (two scalar casts became two cvts and a v_or_b32_sdwa)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((dl_f32x2){a, b}, dl_bf16x2));
}
__device__ __forceinline__ float round_bf16(float a) { return (float)(__bf16)a; }
__device__ __forceinline__ uint4 pack8_bf16(const float* v) {
  return uint4{pack2_bf16(v[0], v[1]), pack2_bf16(v[2], v[3]), pack2_bf16(v[4], v[5]), pack2_bf16(v[6], v[7])};
}

// fp16 (IEEE half) conversions for the FLOAT16 wire format.
__device__ __forceinline__ uint16_t f2h(float f) {
  _Float16 h = (_Float16)f;
  return *reinterpret_cast<uint16_t*>(&h);
}
__device__ __forceinline__ float h2f(uint16_t v) {
  _Float16 h = *reinterpret_cast<_Float16*>(&v);
  return (float)h;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Wave-wide f32 sum without the LDS crossbar: DPP within each 16-lane row (xor 1, xor 2, half-row
// mirror, row mirror), then the gfx950 row-pair and half-wave swaps.  Every lane gets the total.
// (__shfl_xor lowers to a chain of six ds_bpermute_b32 round trips, ~1 us of latency per row
// reduction in the LayerNorm kernels.)
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f32<0xB1>(v);   // quad_perm(1,0,3,2): lane ^ 1
  v += dpp_f32<0x4E>(v);   // quad_perm(2,3,0,1): lane ^ 2
  v += dpp_f32<0x141>(v);  // row_half_mirror: the other quad of each 8 lanes
  v += dpp_f32<0x140>(v);  // row_mirror: the other 8 lanes of each row of 16
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);  // rows 0+1, 2+3
  r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);  // halves
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `scratch` must hold >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  return r;
}

// tanh through one v_exp_f32 (libm tanhf is a long VALU sequence): 1 - 2 / (1 + e^{2u});
// saturates correctly at +-inf and is accurate to ~1e-7 relative, far below bf16 resolution.
__device__ __forceinline__ float fast_tanh(float u) {
  return 1.f - 2.f / (1.f + __builtin_amdgcn_exp2f(2.8853900817779268f * u));
}

__device__ __forceinline__ float gelu_tanh(float x) {
  // gelu_new (HF ALBERT): 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3)))
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float u = k0 * (x + k1 * x * x * x);
  return 0.5f * x * (1.f + fast_tanh(u));
}

__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float x2 = x * x;
  float u = k0 * (x + k1 * x2 * x);
  float t = fast_tanh(u);
  float du = k0 * (1.f + 3.f * k1 * x2);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * du;
}

// gelu_new(x) = x * sigma(2u) = x / (1 + 2^(-2 u log2 e)), u = k0 (x + k1 x^3): one exp2 + one rcp.
// The constants are folded: -2 u log2(e) = x (G0 + G1 x^2) with G0 = -2 log2(e) k0, G1 = G0 k1, and
// 2 u' = D0 + D1 x^2 with D0 = 2 k0, D1 = 6 k0 k1 (three fewer VALU per value than the unfolded
// products, which the compiler may not reassociate).
constexpr float kGeluG0 = -2.302208198144325f, kGeluG1 = -0.1029432395800235f;
constexpr float kGeluD0 = 1.5957691216057308f, kGeluD1 = 0.21406444881780076f;

__device__ __forceinline__ float gelu_sig_s(float x, float x2) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * fmaf(kGeluG1, x2, kGeluG0)));
}

__device__ __forceinline__ float gelu_tanh_sig(float x) { return x * gelu_sig_s(x, x * x); }

// gelu_new'(x) in the sigmoid form: gelu_new(x) = x * sigma(2u), so
// gelu_new'(x) = s + 2 x s (1 - s) u',  s = sigma(2u) = 1 / (1 + 2^(-2 u log2 e)):
// one exp2 + one rcp and ~6 FMAs (the tanh form above needs ~15); same value to ~1e-7 relative.
__device__ __forceinline__ float gelu_tanh_grad_sig(float x) {
  const float x2 = x * x;
  const float s = gelu_sig_s(x, x2);
  return fmaf(x * fmaf(kGeluD1, x2, kGeluD0), fmaf(-s, s, s), s);
}

// gelu_new and gelu_new' of one value sharing the exp2 / rcp (the FFN-up epilogue that stores the
// derivative for the backward instead of the pre-activation)
__device__ __forceinline__ void gelu_and_grad_sig(float x, float& g, float& d) {
  const float x2 = x * x;
  const float s = gelu_sig_s(x, x2);
  g = x * s;
  d = fmaf(x * fmaf(kGeluD1, x2, kGeluD0), fmaf(-s, s, s), s);
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5, T1):
// consecutive logical tiles land on the same XCD so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// Vectorised bf16 <-> fp32 row fragments (cdna_hip_programming.md Guideline 13: never scalar bf16).
template <int VW>
__device__ __forceinline__ void load_bf16(const bf16_t* p, float* out) {
  if constexpr (VW == 8) {
    uint4 v = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      out[2 * i] = __uint_as_float(w[i] << 16);
      out[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  } else if constexpr (VW == 4) {
    uint2 v = *reinterpret_cast<const uint2*>(p);
    out[0] = __uint_as_float(v.x << 16); out[1] = __uint_as_float(v.x & 0xffff0000u);
    out[2] = __uint_as_float(v.y << 16); out[3] = __uint_as_float(v.y & 0xffff0000u);
  } else if constexpr (VW == 2) {
    uint32_t v = *reinterpret_cast<const uint32_t*>(p);
    out[0] = __uint_as_float(v << 16); out[1] = __uint_as_float(v & 0xffff0000u);
  } else {
#pragma unroll
    for (int i = 0; i < VW; ++i) out[i] = bf2f(p[i]);
  }
}

// 8 bf16 already in registers (a prefetched 16-byte row chunk) -> fp32
__device__ __forceinline__ void unpack8_bf16(const uint4& v, float* out) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    out[2 * i] = __uint_as_float(w[i] << 16);
    out[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

template <int VW>
__device__ __forceinline__ void store_bf16(bf16_t* p, const float* in) {
  if constexpr (VW == 8) {
    *reinterpret_cast<uint4*>(p) = pack8_bf16(in);
  } else if constexpr (VW == 4) {
    *reinterpret_cast<uint2*>(p) = uint2{pack2_bf16(in[0], in[1]), pack2_bf16(in[2], in[3])};
  } else if constexpr (VW == 2) {
    *reinterpret_cast<uint32_t*>(p) = pack2_bf16(in[0], in[1]);
  } else {
#pragma unroll
    for (int i = 0; i < VW; ++i) p[i] = f2bf(in[i]);
  }
}


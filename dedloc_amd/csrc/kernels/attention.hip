// Flash-style multi-head self-attention for ALBERT: head_dim 64, S % 64 == 0,
// additive key-padding bias, bf16 in/out, fp32 softmax state, never materialises [B,H,S,S].
//
// Inputs come straight from the fused QKV projection: qkv is [B*S, 3*H*64] (Q | K | V, head h at
// columns h*64 of each third) and the context is written as [B*S, H*64] — exactly the layout the
// output projection consumes, so no transposes exist anywhere in the attention path.
//
// MFMA: v_mfma_f32_32x32x16_bf16 (cdna_hip_programming.md §3).  Every product is arranged so that
// the "reduction-side" operand comes out of the previous MFMA's accumulator with no lane movement
// (§3 "An accumulator tile as the next MFMA's operand"), and the other operand is read from LDS
// either by rows (ds_read_b128) or transposed (ds_read_b64_tr_b16, T10):
//   fwd   : S^T = K Q^T (query on the lane -> softmax row state is per-lane)
//           O^T += V^T P^T (P^T accumulator is the B operand; V^T via tr-reads)
//   bwd dq: S^T, dP^T = V dO^T, dQ^T += K^T dS^T        (query on the lane)
//   bwd dkdv: S = Q K^T, dP = dO V^T (key on the lane), dV^T += dO^T P, dK^T += Q^T dS
// One LDS image per 64x64 bf16 tile serves both the row reads and the transposed reads: 16-byte
// chunk c of row r lives at chunk c ^ f((r>>1)&7), f(x) = x ^ ((x&1)<<2) — conflict-free for the
// ds_read_b128 lane groups and for the 4-row tr-read blocks (derivation in docs/KERNELS.md).
#include <cstdlib>
#include <type_traits>

#include "dl_common.h"
#include "dl_kernels.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s4_t __attribute__((ext_vector_type(4)));
typedef short s8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s4_t lds_s4;

constexpr int HD = 64;          // head dim
constexpr int TILE_BYTES = 64 * 128;
constexpr float NEG_BIG = -1.0e30f;

__device__ __forceinline__ int swzf(int x) { return x ^ ((x & 1) << 2); }
__device__ __forceinline__ int chunk_off(int row, int c) { return row * 128 + ((c ^ swzf((row >> 1) & 7)) << 4); }
__device__ __forceinline__ int crow(int i, int hh) { return (i & 3) + 8 * (i >> 2) + 4 * hh; }

__device__ __forceinline__ floatx16 mfma32(bf16x8 a, bf16x8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// 16-byte row fragment: row `row`, chunk `c` of a swizzled tile
__device__ __forceinline__ bf16x8 lds_row_frag(const uint8_t* tile, int row, int c) {
  return *reinterpret_cast<const bf16x8*>(tile + chunk_off(row, c));
}

// ds_read_b64_tr_b16 on a swizzled tile: the calling lane (index i within its 16-lane group)
// supplies row row0 + (i>>2), columns col0 + 4*(i&3) .. +3; it receives column col0 + i of the
// four rows row0..row0+3.
__device__ __forceinline__ s4_t lds_tr(const uint8_t* tile, int row0, int col0, int i) {
  const int row = row0 + (i >> 2);
  const int col = col0 + 4 * (i & 3);
  const int off = chunk_off(row, col >> 3) + ((col & 7) << 1);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(tile + off));
}

// A-operand fragment whose element e is taken from k-row 16*s + 8*(e>>2) + 4*hh + (e&3) of the
// tile (matching the permuted k order of an accumulator used as B operand), column = 32*t + r.
__device__ __forceinline__ bf16x8 tr_operand(const uint8_t* tile, int kbase, int hh, int t, int lane) {
  const int col0 = 32 * t + 16 * ((lane >> 4) & 1);
  const s4_t lo = lds_tr(tile, kbase + 4 * hh, col0, lane & 15);
  const s4_t hi = lds_tr(tile, kbase + 8 + 4 * hh, col0, lane & 15);
  // whole-vector shuffle + bit_cast: per-element __bf16 bit_casts of an s4 vector miscompile
  // (hipcc 7.2 broadcast element 0) — see tests/hip/primitives_test.hip
  const s8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// accumulator registers 8s..8s+7 -> bf16 B-operand fragment
__device__ __forceinline__ bf16x8 pack_acc(const floatx16& x, int s) {
  bf16x8 b;
#pragma unroll
  for (int e = 0; e < 8; ++e) b[e] = (__bf16)x[8 * s + e];
  return b;
}

__device__ __forceinline__ bf16x8 gload8(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

// cooperative 64-row x 64-col tile stage: 256 threads, 2 x 16 B each (two named registers —
// an indexed array of uint4 was demoted to scratch by hipcc)
struct TileRegs { uint4 a, b; };

__device__ __forceinline__ uint4 tile_ld1(const bf16_t* g, long ld, int row0, int rows_valid, int idx) {
  const int row = min(row0 + (idx >> 3), rows_valid - 1);
  return *reinterpret_cast<const uint4*>(g + (long)row * ld + (idx & 7) * 8);
}

__device__ __forceinline__ void tile_load(TileRegs& t, const bf16_t* g, long ld, int row0, int rows_valid) {
  t.a = tile_ld1(g, ld, row0, rows_valid, threadIdx.x);
  t.b = tile_ld1(g, ld, row0, rows_valid, threadIdx.x + 256);
}

__device__ __forceinline__ void tile_store(const TileRegs& t, uint8_t* tile) {
  const int i0 = threadIdx.x, i1 = threadIdx.x + 256;
  *reinterpret_cast<uint4*>(tile + chunk_off(i0 >> 3, i0 & 7)) = t.a;
  *reinterpret_cast<uint4*>(tile + chunk_off(i1 >> 3, i1 & 7)) = t.b;
}

// ---- LDS-DMA staging ring (RING kernels) ---------------------------------------------------------
// Each pipeline stage holds the two 64x64 tiles of one key (or query) block plus 64-128 floats of
// per-row data, written by global_load_lds (no VGPR round trip, no ds_write).  NBUF stages: the
// loads of stage s + NBUF - 1 are issued while stage s computes, and a counted vmcnt waits for
// stage s only (PMC on the register-staged form: 26-43% of wave cycles parked in s_waitcnt /
// barrier, scripts/gpu_r2_pmc.sh).  LDS-DMA writes lane-linearly (lane i -> base + 16 i), so the
// XOR swizzle of chunk_off is applied to the SOURCE: lane i of 1-KiB piece p loads row 8p + i/8,
// chunk (i & 7) ^ swz(row).
typedef __attribute__((address_space(3))) void lds_void;
// Two stages: the next tile's DMA is issued at the top of the current tile and has a whole tile of
// MFMA / softmax work to land (4 stages measured 1.3% slower forward, 0.5% slower dQ at B=512:
// profiles/r5_attn_ring_depth_occupancy.jsonl); the dQ epilogue's column-sum scratch (33 KiB)
// still fits the ring.
constexpr int NBUF = 2;
constexpr int STAGE = 2 * TILE_BYTES + 512;

// The DMA instructions are issued from inline asm.  With __builtin_amdgcn_global_load_lds the
// compiler's wait-count pass, which cannot tell ring slots apart, puts s_waitcnt vmcnt(0) in front
// of the first LDS read after any in-flight DMA (seen in the ISA: before the V tr-reads), which
// drains the whole prefetch every tile.  Hidden in asm, the DMAs are covered by the ring's own
// counted waits; the compiler's waits for its own loads stay correct (they only get stricter).
// M0 (the LDS base of the DMA) is written here and used by nothing else in these kernels.
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(const lds_void*)p);
}
__device__ __forceinline__ void dma16(const void* g, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds), "v"(g) : "memory", "m0");
}
__device__ __forceinline__ void dma4(const void* g, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, off" ::"s"(lds), "v"(g) : "memory", "m0");
}

// Prologue order in the RING kernels: issue the first NBUF-1 stages, THEN the block's compiler-visible
// register loads (Q / dO / K / V rows, lse ...), then this real s_waitcnt vmcnt(0) (the builtin, so
// the compiler's wait-count pass sees it): the asm DMAs are invisible to that pass, and a
// compiler-placed partial vmcnt for those register loads inside the tile loop would drain the ring.
// (the empty asm keeps the scheduler from sinking those loads below the wait; loads from const
// __restrict__ arguments may still move, so values the tile loop reads are also passed through
// `settle`, which makes the compiler complete the load before the asm and treat the register as
// the asm's output)
__device__ __forceinline__ void wait_vm_all() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
}
template <typename T>
__device__ __forceinline__ void settle(T& v) { asm volatile("" : "+v"(v)); }

// this wave's 1-KiB pieces (p = w, w + NW, ...) of a 64-row tile starting at global row row0
template <int NW = 4>
__device__ __forceinline__ void dma_tile(const bf16_t* g, long ld, int row0, uint8_t* tile, int w, int lane) {
#pragma unroll
  for (int j = 0; j < 8 / NW; ++j) {
    const int p = w + NW * j;
    const int row = 8 * p + (lane >> 3);
    const int c = (lane & 7) ^ swzf((row >> 1) & 7);
    dma16(g + (long)(row0 + row) * ld + c * 8, lds_u32(tile + p * 1024));
  }
}

// 64 consecutive floats -> 256 B of LDS (one dword per lane)
__device__ __forceinline__ void dma_f32x64(const float* g, uint8_t* dst, int lane) {
  dma4(g + lane, lds_u32(dst));
}

// Wait until this wave's pieces of the oldest in-flight stage have landed, leaving `ahead` later
// stages (0..NBUF-2) in flight; N = vector-memory ops this wave issues per stage.
template <int N>
__device__ __forceinline__ void wait_cnt(int ahead) {
  if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * N) : "memory");
  else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// PIECES = K + V tile pieces per wave per stage; the optional mask-bias piece adds one
template <int PIECES = 4>
__device__ __forceinline__ void wait_stages(int ahead, bool bias) {
  if (bias) wait_cnt<PIECES + 1>(ahead);
  else wait_cnt<PIECES>(ahead);
}

// store 4 consecutive bf16 (8 bytes)
__device__ __forceinline__ void store4(bf16_t* p, float a, float b, float c, float d) {
  uint2 v;
  v.x = (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
  v.y = (uint32_t)f2bf(c) | ((uint32_t)f2bf(d) << 16);
  *reinterpret_cast<uint2*>(p) = v;
}

// ------------------------------------------------------------------------------------------ fwd
// Key masking comes in two forms.  kvinfo = int32[B + 1] (lengths of right-padded key masks plus a
// device-side "every mask is a prefix" flag in kvinfo[B], computed by the model without a host
// sync): then tiles past the batch's length are skipped and only the boundary tile is masked.
// Otherwise (or when kvinfo[B] == 0) the generic additive bias mbias[B, S] (log2 units) is used.
// Interior tiles run the lean softmax: one FMA (scale, -max) + exp2 + add per score, row max via
// max3, and the online-softmax rescale of O is deferred until a row's max grows by more than
// 2^RESCALE_THR (cdna_hip_programming.md T13: P <= 2^8 is exact enough in bf16 for P.V; the
// rescale decision precedes the tile's exponentiation, so nothing is ever scaled twice).
constexpr float RESCALE_THR = 8.f;

// XCD-aware block order (T1): the hardware deals consecutive workgroups round-robin to the 8 XCDs,
// which would put the S/128 query (or key) blocks of one head on different XCDs, each re-reading
// that head's K/V (Q/dO) into its own L2.  Renumber so each XCD gets a contiguous run of logical
// blocks: all blocks of a head then share one L2.
struct BlockId {
  int x, h, b;
};
__device__ __forceinline__ BlockId block_id(int xcd) {
  const int gx = gridDim.x, gy = gridDim.y;
  const int n = gx * gy * gridDim.z;
  int p = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  if (xcd && (n & 7) == 0) p = (p & 7) * (n >> 3) + (p >> 3);
  return BlockId{p % gx, (p / gx) % gy, p / (gx * gy)};
}


__device__ __forceinline__ int kv_end_of(const int* kvinfo, int B, int b, int S, bool& use_len) {
  use_len = false;
  if (kvinfo == nullptr || kvinfo[B] == 0) return S;
  const int len = kvinfo[b];
  if (len <= 0 || len > S) return S;  // empty / malformed rows take the generic path
  use_len = true;
  return len;
}

// v_max3_f32 without the canonicalising v_max the compiler inserts in front of fmaxf on MFMA results
// (MI355X_MICROARCH.md pitfalls): one instruction per two new scores
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// Cross-half (lane L <-> L ^ 32) max / sum through v_permlane32_swap (a VALU op; __shfl_xor(x, 32)
// is an LDS round trip on the softmax's critical path, T12).  After the swap r[0] holds, in lanes
// 32..63, the value of lane L - 32 and r[1], in lanes 0..31, the value of lane L + 32, so one op
// over r[0], r[1] combines the pair in every lane.
__device__ __forceinline__ float half_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  float m;
  asm("v_max_f32 %0, %1, %2" : "=v"(m) : "v"(__uint_as_float(r[0])), "v"(__uint_as_float(r[1])));
  return m;
}
__device__ __forceinline__ float half_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Forward tile loop over key tiles [kt0, kt1) of nt, with the next tile's K/V (and per-key bias)
// prefetched through registers while this tile computes (T14).  Tile kt0 must already be staged.
// LEAN: unmasked tiles — raw scores, the softmax scale rides in the exp FMA, no bias reads.
// !LEAN: s = s*sl2 + bias[key] with the bias staged in LDS (additive mask or 0/-1e30 from the
// key length).  The two instantiations run as consecutive loops (lean body, then the boundary
// tile), never in one loop body, so they do not add register pressure to each other.
struct FwdCtx {
  const bf16_t* Kg;
  const bf16_t* Vg;
  long ld;
  int S, kv_end;
  const float* mb_g;
  float sl2;
  uint8_t* smem;
  float* mbs;
  int w, lane;
  // RING: issue stage s (key tile s) into ring slot s % NBUF (NW waves share the tile pieces)
  template <int NW = 4>
  __device__ __forceinline__ void issue(int s) const {
    uint8_t* slot = smem + (s % NBUF) * STAGE;
    dma_tile<NW>(Kg, ld, s * 64, slot, w, lane);
    dma_tile<NW>(Vg, ld, s * 64, slot + TILE_BYTES, w, lane);
    if (mb_g) dma_f32x64(mb_g + s * 64, slot + 2 * TILE_BYTES, lane);
  }
};

__device__ __forceinline__ float key_bias(const FwdCtx& c, int key) {
  return c.mb_g ? c.mb_g[key] : (key < c.kv_end ? 0.f : NEG_BIG);
}

// QS = 32-row query sub-blocks per wave (1 or 2).  With QS = 2 every K fragment (row reads) and V
// fragment (tr-reads) read from LDS feeds two MFMAs, and each wave carries two independent softmax
// chains the scheduler can interleave (the loop is latency-bound: PMC, profiles/README.md).
template <bool LEAN, bool RING, int QS, int NW>
__device__ __forceinline__ void fwd_tiles(const FwdCtx& c, int kt0, int kt1, int nt, const bf16x8 (&qf)[QS][4],
                                          floatx16 (&o)[QS][2], float (&m)[QS], float (&l)[QS], int r, int hh,
                                          int lane) {
  TileRegs kr, vr;
  float mbr = 0.f;
  for (int kt = kt0; kt < kt1; ++kt) {
    const uint8_t* Ks;
    const float* mb;
    bool more = false;
    if constexpr (RING) {
      // stage kt landed (this wave) -> barrier: every wave's pieces landed and every wave is done
      // with slot (kt - 1) % NBUF, which the stage issued next overwrites
      wait_stages<16 / NW>(min(nt - 1 - kt, NBUF - 2), c.mb_g != nullptr);
      __syncthreads();
      if (kt + NBUF - 1 < nt) c.template issue<NW>(kt + NBUF - 1);
      Ks = c.smem + (kt % NBUF) * STAGE;
      mb = reinterpret_cast<const float*>(Ks + 2 * TILE_BYTES);
    } else {
      const int cur = kt & 1;
      Ks = c.smem + cur * 2 * TILE_BYTES;
      mb = c.mbs + cur * 64;
      more = kt + 1 < nt;
      if (more) {  // issue next tile's loads early; they land under the MFMAs below
        tile_load(kr, c.Kg, c.ld, (kt + 1) * 64, c.S);
        tile_load(vr, c.Vg, c.ld, (kt + 1) * 64, c.S);
        if (threadIdx.x < 64) mbr = key_bias(c, (kt + 1) * 64 + threadIdx.x);
      }
    }
    const uint8_t* Vs = Ks + TILE_BYTES;
    floatx16 s[QS][2];
#pragma unroll
    for (int u = 0; u < QS; ++u)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) s[u][j][i] = 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 kfr = lds_row_frag(Ks, 32 * j + r, 2 * ks + hh);
#pragma unroll
        for (int u = 0; u < QS; ++u) s[u][j] = mfma32(kfr, qf[u][ks], s[u][j]);
      }
#pragma unroll
    for (int u = 0; u < QS; ++u) {
      if (!LEAN) {
        if (!RING || c.mb_g) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) s[u][j][i] = fmaf(s[u][j][i], c.sl2, mb[32 * j + crow(i, hh)]);
        } else {  // RING stages carry the generic additive bias only; the length mask is computed here
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i)
              s[u][j][i] = fmaf(s[u][j][i], c.sl2, kt * 64 + 32 * j + crow(i, hh) < c.kv_end ? 0.f : NEG_BIG);
        }
      }
      // row max as four independent max3 chains of 8 scores (depth 6 instead of 16), then the halves
      float mc[4];
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const floatx16& sv = s[u][q4 >> 1];
        const int o8 = (q4 & 1) * 8;
        float v = vmax3(sv[o8], sv[o8 + 1], sv[o8 + 2]);
        v = vmax3(v, sv[o8 + 3], sv[o8 + 4]);
        v = vmax3(v, sv[o8 + 5], sv[o8 + 6]);
        mc[q4] = v;
      }
      float mx = vmax3(vmax3(mc[0], mc[1], s[u][0][7]), vmax3(mc[2], mc[3], s[u][0][15]),
                       vmax3(s[u][1][7], s[u][1][15], mc[0]));
      mx = half_max(mx);
      if (LEAN) mx *= c.sl2;
      const bool grow = mx > m[u] + RESCALE_THR;
      if (__ballot(grow) != 0) {  // rare after the first tile: rescale O and l to the new max
        const float mn = grow ? mx : m[u];
        const float alpha = __builtin_amdgcn_exp2f(m[u] - mn);
        l[u] *= alpha;
        m[u] = mn;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[u][t][i] *= alpha;
      }
      const float nm = -m[u];
      float rsa[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // 8 independent add chains (latency bound)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float pv = __builtin_amdgcn_exp2f(LEAN ? fmaf(s[u][j][i], c.sl2, nm) : s[u][j][i] + nm);
          s[u][j][i] = pv;
          rsa[i & 7] += pv;
        }
      float rs = ((rsa[0] + rsa[1]) + (rsa[2] + rsa[3])) + ((rsa[4] + rsa[5]) + (rsa[6] + rsa[7]));
      l[u] += half_sum(rs);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        bf16x8 pb[QS];
#pragma unroll
        for (int u = 0; u < QS; ++u) pb[u] = pack_acc(s[u][j], ss);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const bf16x8 vfr = tr_operand(Vs, 32 * j + 16 * ss, hh, t, lane);
#pragma unroll
          for (int u = 0; u < QS; ++u) o[u][t] = mfma32(vfr, pb[u], o[u][t]);
        }
      }
    if constexpr (!RING) {
      if (more) {
        uint8_t* Kn = c.smem + ((kt & 1) ^ 1) * 2 * TILE_BYTES;
        tile_store(kr, Kn);
        tile_store(vr, Kn + TILE_BYTES);
        if (threadIdx.x < 64) c.mbs[((kt & 1) ^ 1) * 64 + threadIdx.x] = mbr;
      }
      __syncthreads();
    }
  }
}

// Block = NW waves x QS x 32 query rows of one (batch, head).  NW = 8 (ring only): one 512-query
// block per head at S = 512, so K / V are staged once per head, and each SIMD's two waves belong
// to one block.
template <bool RING, int QS, int NW = 4>
__global__ __launch_bounds__(64 * NW, NW == 8 ? 1 : 2) void attn_fwd_kernel(const bf16_t* __restrict__ qkv, long ld,
                                                          const float* __restrict__ mbias,
                                                          const int* __restrict__ kvinfo, bf16_t* __restrict__ out,
                                                          long ldo, float* __restrict__ lse, int B, int H, int S,
                                                          float sl2, int xcd) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[RING ? NBUF * STAGE : 4 * TILE_BYTES + 2 * 64 * 4];
  const BlockId bid = block_id(xcd);
  const int b = bid.b, h = bid.h;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, hh = lane >> 5;
  const long rb = (long)b * S;
  const bf16_t* Qg = qkv + rb * ld + h * HD;
  bool use_len;
  FwdCtx c;
  c.Kg = qkv + rb * ld + (long)H * HD + h * HD;
  c.Vg = qkv + rb * ld + 2L * H * HD + h * HD;
  c.ld = ld;
  c.S = S;
  c.kv_end = kv_end_of(kvinfo, B, b, S, use_len);
  c.mb_g = (!use_len && mbias) ? mbias + rb : nullptr;
  c.sl2 = sl2;
  c.smem = smem;
  c.mbs = reinterpret_cast<float*>(smem + 4 * TILE_BYTES);
  c.w = w;
  c.lane = lane;

  static_assert(NW == 4 || (NW == 8 && RING), "8-wave blocks stage through the ring");
  const int nt = (c.kv_end + 63) / 64;
  if constexpr (RING) {
    for (int s0 = 0; s0 < NBUF - 1 && s0 < nt; ++s0) c.template issue<NW>(s0);
  }
  int q[QS];
  bf16x8 qf[QS][4];
#pragma unroll
  for (int u = 0; u < QS; ++u) {
    q[u] = bid.x * (32 * QS * NW) + w * (32 * QS) + 32 * u + r;
    const int qc = min(q[u], S - 1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qf[u][ks] = gload8(Qg + (long)qc * ld + ks * 16 + 8 * hh);
    if constexpr (RING) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) settle(qf[u][ks]);
    }
  }

  floatx16 o[QS][2];
  float m[QS], l[QS];
#pragma unroll
  for (int u = 0; u < QS; ++u) {
    m[u] = NEG_BIG;
    l[u] = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[u][t][i] = 0.f;
  }

  if constexpr (RING) {
    wait_vm_all();
  } else {
    TileRegs kr, vr;
    tile_load(kr, c.Kg, ld, 0, S);
    tile_load(vr, c.Vg, ld, 0, S);
    const float mbr = threadIdx.x < 64 ? key_bias(c, threadIdx.x) : 0.f;
    tile_store(kr, smem);
    tile_store(vr, smem + TILE_BYTES);
    if (threadIdx.x < 64) c.mbs[threadIdx.x] = mbr;
    __syncthreads();
  }
  // lean tiles first (every tile when there is no mask), then the masked remainder: the boundary
  // tile of a length mask, or all tiles of a generic additive mask
  const int nlean = c.mb_g ? 0 : c.kv_end / 64;
  fwd_tiles<true, RING, QS, NW>(c, 0, nlean, nt, qf, o, m, l, r, hh, lane);
  fwd_tiles<false, RING, QS, NW>(c, nlean, nt, nt, qf, o, m, l, r, hh, lane);

#pragma unroll
  for (int u = 0; u < QS; ++u) {
    if (q[u] < S) {
      const float inv = 1.f / l[u];
      bf16_t* op = out + (rb + q[u]) * ldo + h * HD;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int v = 0; v < 4; ++v)
          store4(op + 32 * t + 8 * v + 4 * hh, o[u][t][4 * v] * inv, o[u][t][4 * v + 1] * inv,
                 o[u][t][4 * v + 2] * inv, o[u][t][4 * v + 3] * inv);
      if (hh == 0) lse[((long)b * H + h) * S + q[u]] = m[u] + log2f(l[u]);
    }
  }
}

// ------------------------------------------------------------------------------------------ bwd dq
// Also computes delta = rowsum(dO * O) for its queries and publishes it for the dkdv kernel.
// QS = 32-row query sub-blocks per wave (as in the forward: every K / V fragment read from LDS
// feeds QS MFMAs, and each wave carries QS independent chains).
template <bool RING, int QS>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(const bf16_t* __restrict__ qkv, long ld,
                                                             const float* __restrict__ mbias,
                                                             const int* __restrict__ kvinfo,
                                                             const bf16_t* __restrict__ out, const bf16_t* __restrict__ dout,
                                                             long ldo, const float* __restrict__ lse,
                                                             float* __restrict__ delta, bf16_t* __restrict__ dqkv,
                                                             float* __restrict__ dbias, int B, int H, int S, float sl2,
                                                             float scale, int xcd) {
  // tail: mask bias / bias-grad partials (the epilogue reuses the first 33 KiB for its column sums)
  __shared__ __attribute__((aligned(16))) uint8_t smem[RING ? NBUF * STAGE : 4 * TILE_BYTES + 4 * 64 * 4];
  const BlockId bid = block_id(xcd);
  const int b = bid.b, h = bid.h;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, hh = lane >> 5;
  const long rb = (long)b * S;
  const bf16_t* Qg = qkv + rb * ld + h * HD;
  const bf16_t* Kg = qkv + rb * ld + (long)H * HD + h * HD;
  const bf16_t* Vg = qkv + rb * ld + 2L * H * HD + h * HD;
  bool use_len;
  const int kv_end = kv_end_of(kvinfo, B, b, S, use_len);
  const float* mb_g = (!use_len && mbias) ? mbias + rb : nullptr;
  float* mbs = reinterpret_cast<float*>(smem + 4 * TILE_BYTES);
  const int nt = (kv_end + 63) / 64;
  auto issue = [&](int st) {  // RING: key tile st -> slot st % NBUF
    uint8_t* slot = smem + (st % NBUF) * STAGE;
    dma_tile(Kg, ld, st * 64, slot, w, lane);
    dma_tile(Vg, ld, st * 64, slot + TILE_BYTES, w, lane);
    if (mb_g) dma_f32x64(mb_g + st * 64, slot + 2 * TILE_BYTES, lane);
  };
  if constexpr (RING) {
    for (int s0 = 0; s0 < NBUF - 1 && s0 < nt; ++s0) issue(s0);
  }

  int q[QS];
  bf16x8 qf[QS][4], df[QS][4];
  float dl[QS], l2[QS];
#pragma unroll
  for (int u = 0; u < QS; ++u) {
    q[u] = bid.x * (128 * QS) + w * (32 * QS) + 32 * u + r;
    const int qc = min(q[u], S - 1);
    dl[u] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      qf[u][ks] = gload8(Qg + (long)qc * ld + ks * 16 + 8 * hh);
      const long oo = (rb + qc) * ldo + h * HD + ks * 16 + 8 * hh;
      df[u][ks] = gload8(dout + oo);
      const bf16x8 of = gload8(out + oo);
#pragma unroll
      for (int e = 0; e < 8; ++e) dl[u] += (float)df[u][ks][e] * (float)of[e];
    }
    dl[u] += __shfl_xor(dl[u], 32, 64);
    l2[u] = lse[((long)b * H + h) * S + qc];
    if constexpr (RING) {
      settle(l2[u]);
      settle(dl[u]);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        settle(qf[u][ks]);
        settle(df[u][ks]);
      }
    }
  }
  // (delta is stored after the tile loop: a store issued here would sit in the vmcnt queue ahead of
  // the ring's loads, and CDNA4 counts stores in vmcnt too)

  floatx16 dq[QS][2];
#pragma unroll
  for (int u = 0; u < QS; ++u)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) dq[u][t][i] = 0.f;

  TileRegs kr, vr;
  float mbr = 0.f;
  if constexpr (RING) {
    wait_vm_all();
  } else {
    tile_load(kr, Kg, ld, 0, S);
    tile_load(vr, Vg, ld, 0, S);
    if (threadIdx.x < 64) mbr = mb_g ? mb_g[threadIdx.x] : 0.f;
    tile_store(kr, smem);
    tile_store(vr, smem + TILE_BYTES);
    if (threadIdx.x < 64) mbs[threadIdx.x] = mbr;
    __syncthreads();
  }

  for (int kt = 0; kt < nt; ++kt) {
    const uint8_t* Ks;
    const float* mb;
    if constexpr (RING) {
      wait_stages(min(nt - 1 - kt, NBUF - 2), mb_g != nullptr);
      __syncthreads();
      if (kt + NBUF - 1 < nt) issue(kt + NBUF - 1);
      Ks = smem + (kt % NBUF) * STAGE;
      mb = reinterpret_cast<const float*>(Ks + 2 * TILE_BYTES);
    } else {
      Ks = smem + (kt & 1) * 2 * TILE_BYTES;
      mb = mbs + (kt & 1) * 64;
      if (kt + 1 < nt) {
        tile_load(kr, Kg, ld, (kt + 1) * 64, S);
        tile_load(vr, Vg, ld, (kt + 1) * 64, S);
        if (threadIdx.x < 64) mbr = mb_g ? mb_g[(kt + 1) * 64 + threadIdx.x] : 0.f;
      }
    }
    const uint8_t* Vs = Ks + TILE_BYTES;
    const bool interior = mb_g == nullptr && (kt + 1) * 64 <= kv_end;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      floatx16 st[QS], dp[QS];
#pragma unroll
      for (int u = 0; u < QS; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) { st[u][i] = 0.f; dp[u][i] = 0.f; }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 kfr = lds_row_frag(Ks, 32 * j + r, 2 * ks + hh);
        const bf16x8 vfr = lds_row_frag(Vs, 32 * j + r, 2 * ks + hh);
#pragma unroll
        for (int u = 0; u < QS; ++u) {
          st[u] = mfma32(kfr, qf[u][ks], st[u]);
          dp[u] = mfma32(vfr, df[u][ks], dp[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < QS; ++u) {
        if (interior) {  // interior tile: no mask
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float p = __builtin_amdgcn_exp2f(fmaf(st[u][i], sl2, -l2[u]));
            st[u][i] = p * (dp[u][i] - dl[u]);
          }
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int key = kt * 64 + 32 * j + crow(i, hh);
            const float bias = mb_g ? mb[32 * j + crow(i, hh)] : (key < kv_end ? 0.f : NEG_BIG);
            const float p = __builtin_amdgcn_exp2f(st[u][i] * sl2 + bias - l2[u]);
            st[u][i] = p * (dp[u][i] - dl[u]);
          }
        }
      }
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        bf16x8 pb[QS];
#pragma unroll
        for (int u = 0; u < QS; ++u) pb[u] = pack_acc(st[u], ss);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const bf16x8 ktr = tr_operand(Ks, 32 * j + 16 * ss, hh, t, lane);
#pragma unroll
          for (int u = 0; u < QS; ++u) dq[u][t] = mfma32(ktr, pb[u], dq[u][t]);
        }
      }
    }
    if constexpr (!RING) {
      if (kt + 1 < nt) {
        uint8_t* Kn = smem + ((kt & 1) ^ 1) * 2 * TILE_BYTES;
        tile_store(kr, Kn);
        tile_store(vr, Kn + TILE_BYTES);
        if (threadIdx.x < 64) mbs[((kt & 1) ^ 1) * 64 + threadIdx.x] = mbr;
      }
      __syncthreads();
    }
  }
  if constexpr (RING) __syncthreads();  // every wave is done with the ring before the epilogue reuses it
#pragma unroll
  for (int u = 0; u < QS; ++u) {
    if (q[u] < S && hh == 0) delta[((long)b * H + h) * S + q[u]] = dl[u];
    if (q[u] < S) {
      bf16_t* dp_ = dqkv + (rb + q[u]) * ld + h * HD;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int v = 0; v < 4; ++v)
          store4(dp_ + 32 * t + 8 * v + 4 * hh, dq[u][t][4 * v] * scale, dq[u][t][4 * v + 1] * scale,
                 dq[u][t][4 * v + 2] * scale, dq[u][t][4 * v + 3] * scale);
    }
  }
  if (dbias) {
    // Fused bias gradient of the QKV projection (replaces a [T, 3H*64] column-sum pass):
    //   query bias: column sums of the dQ just stored (bf16-rounded, as stored);
    //   value bias: sum_k dV[k] = sum_q dO[q] (softmax rows sum to one), from the dO this block loaded;
    //   key bias:   sum_k dK[k] = 0 exactly (sum_k dS[q,k] = delta - delta), so nothing is added.
    // Column sums through LDS (cross-lane shuffles of 64 values per lane cost more than the
    // column-sum pass they replace): per sub-block, each wave writes its [32 queries][64 columns]
    // fp32 block (16-B chunk c of row r at c ^ (r & 15): conflict-free writes and column reads),
    // then thread (wave w', column c) sums the 32 rows of wave w' and the four partials meet in
    // the last 1 KiB.
    float* red = reinterpret_cast<float*>(smem);          // [4 waves][32 rows][64 columns]
    float* part = red + 4 * 32 * 64;                       // [4 waves][64 columns]
    auto chunk_addr = [&](int row, int ch) { return red + (w * 32 + row) * 64 + ((ch ^ (row & 15)) << 2); };
#pragma unroll
    for (int u = 0; u < QS; ++u) {
      const bool live = q[u] < S;
#pragma unroll
      for (int which = 0; which < 2; ++which) {
        if (which == 0) {
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int v4 = 0; v4 < 4; ++v4) {  // dQ columns 32 t + 8 v4 + 4 hh + (0..3), as stored above
              float4 v = float4{0.f, 0.f, 0.f, 0.f};
              if (live)
                v = float4{round_bf16(dq[u][t][4 * v4] * scale), round_bf16(dq[u][t][4 * v4 + 1] * scale),
                           round_bf16(dq[u][t][4 * v4 + 2] * scale), round_bf16(dq[u][t][4 * v4 + 3] * scale)};
              *reinterpret_cast<float4*>(chunk_addr(r, 8 * t + 2 * v4 + hh)) = v;
            }
        } else {
#pragma unroll
          for (int ks = 0; ks < 4; ++ks)
#pragma unroll
            for (int g = 0; g < 2; ++g) {  // dO columns 16 ks + 8 hh + 4 g + (0..3), as loaded above
              float4 v = float4{0.f, 0.f, 0.f, 0.f};
              if (live)
                v = float4{(float)df[u][ks][4 * g], (float)df[u][ks][4 * g + 1], (float)df[u][ks][4 * g + 2],
                           (float)df[u][ks][4 * g + 3]};
              *reinterpret_cast<float4*>(chunk_addr(r, 4 * ks + 2 * hh + g)) = v;
            }
        }
        __syncthreads();
        {
          const int c = lane;  // this thread: column c of wave w's 32 rows
          float sum = 0.f;
#pragma unroll 8
          for (int row = 0; row < 32; ++row)
            sum += red[(w * 32 + row) * 64 + (((c >> 2) ^ (row & 15)) << 2) + (c & 3)];
          part[w * 64 + c] = sum;
        }
        __syncthreads();
        if (threadIdx.x < 64) {
          const int c = threadIdx.x;
          atomicAdd(&dbias[(which ? 2L * H * HD : 0L) + h * HD + c],
                    part[c] + part[64 + c] + part[128 + c] + part[192 + c]);
        }
        __syncthreads();
      }
    }
  }
}

// ------------------------------------------------------------------------------------------ bwd dkdv
// KS = 32-key sub-blocks per wave: with KS = 2 every Q / dO fragment read from LDS feeds two
// MFMAs; the dK/dV accumulators (128 registers) need the whole 512-entry register file, so that
// form runs one wave per SIMD (launch bound 256 x 1) and hides latency by ILP instead of waves.
template <bool RING, int KS>
__global__ __launch_bounds__(256, KS == 2 ? 1 : 2) void attn_bwd_dkdv_kernel(
    const bf16_t* __restrict__ qkv, long ld, const float* __restrict__ mbias, const int* __restrict__ kvinfo,
    const bf16_t* __restrict__ dout, long ldo, const float* __restrict__ lse, const float* __restrict__ delta,
    bf16_t* __restrict__ dqkv, int B, int H, int S, float sl2, float scale, int xcd) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[RING ? NBUF * STAGE : 4 * TILE_BYTES + 2 * 2 * 64 * 4];
  const BlockId bid = block_id(xcd);
  const int b = bid.b, h = bid.h;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, hh = lane >> 5;
  const long rb = (long)b * S;
  const bf16_t* Qg = qkv + rb * ld + h * HD;
  const bf16_t* Kg = qkv + rb * ld + (long)H * HD + h * HD;
  const bf16_t* Vg = qkv + rb * ld + 2L * H * HD + h * HD;
  const bf16_t* dOg = dout + rb * ldo + h * HD;
  const float* lse_g = lse + ((long)b * H + h) * S;
  const float* del_g = delta + ((long)b * H + h) * S;
  float* rowv = reinterpret_cast<float*>(smem + 4 * TILE_BYTES);  // [2 buf][lse 64 | delta 64]

  int k[KS];
#pragma unroll
  for (int u = 0; u < KS; ++u) k[u] = bid.x * (128 * KS) + w * (32 * KS) + 32 * u + r;
  bool use_len;
  const int kv_end = kv_end_of(kvinfo, B, b, S, use_len);
  if (use_len && bid.x * (128 * KS) >= kv_end) {  // every key of this block is padding: dK = dV = 0
#pragma unroll
    for (int u = 0; u < KS; ++u) {
      if (k[u] < S) {
        bf16_t* dkp = dqkv + (rb + k[u]) * ld + (long)H * HD + h * HD;
        bf16_t* dvp = dqkv + (rb + k[u]) * ld + 2L * H * HD + h * HD;
#pragma unroll
        for (int v = 0; v < 8; ++v) {  // the same 64 columns the regular epilogue covers (32t + 8v' + 4hh)
          store4(dkp + 8 * v + 4 * hh, 0.f, 0.f, 0.f, 0.f);
          store4(dvp + 8 * v + 4 * hh, 0.f, 0.f, 0.f, 0.f);
        }
      }
    }
    return;
  }
  const int nt = S / 64;
  auto issue = [&](int st) {  // RING: query tile st -> slot st % NBUF; waves 0-1 fetch lse, 2-3 delta
    uint8_t* slot = smem + (st % NBUF) * STAGE;
    dma_tile(Qg, ld, st * 64, slot, w, lane);
    dma_tile(dOg, ldo, st * 64, slot + TILE_BYTES, w, lane);
    dma_f32x64((w < 2 ? lse_g : del_g) + st * 64, slot + 2 * TILE_BYTES + (w < 2 ? 0 : 256), lane);
  };
  if constexpr (RING) {
    for (int s0 = 0; s0 < NBUF - 1 && s0 < nt; ++s0) issue(s0);
  }
  bf16x8 kf[KS][4], vf[KS][4];
  float mbk[KS];
#pragma unroll
  for (int u = 0; u < KS; ++u) {
    const int kc = min(k[u], S - 1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      kf[u][ks] = gload8(Kg + (long)kc * ld + ks * 16 + 8 * hh);
      vf[u][ks] = gload8(Vg + (long)kc * ld + ks * 16 + 8 * hh);
    }
    mbk[u] = use_len ? (k[u] < kv_end ? 0.f : NEG_BIG) : (mbias ? mbias[rb + kc] : 0.f);
    if constexpr (RING) {
      settle(mbk[u]);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        settle(kf[u][ks]);
        settle(vf[u][ks]);
      }
    }
  }

  floatx16 dk[KS][2], dv[KS][2];
#pragma unroll
  for (int u = 0; u < KS; ++u)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) { dk[u][t][i] = 0.f; dv[u][t][i] = 0.f; }

  TileRegs qr, dr;
  float rv = 0.f;
  if constexpr (RING) {
    wait_vm_all();
  } else {
    tile_load(qr, Qg, ld, 0, S);
    tile_load(dr, dOg, ldo, 0, S);
    if (threadIdx.x < 128) rv = threadIdx.x < 64 ? lse_g[threadIdx.x] : del_g[threadIdx.x - 64];
    tile_store(qr, smem);
    tile_store(dr, smem + TILE_BYTES);
    if (threadIdx.x < 128) rowv[threadIdx.x] = rv;
    __syncthreads();
  }

  // LEAN (a key-length mask, the model's case): the mask term leaves the loop — a masked key's P
  // is computed as if it were live and its dK / dV rows are zeroed once at the end (dK / dV of a
  // key depend on that key's P and dS only); the generic additive mask keeps the bias in the
  // exponent.
  auto qloop = [&](auto lean_tag) {
  constexpr bool LEAN = decltype(lean_tag)::value;
  for (int qt = 0; qt < nt; ++qt) {
    const uint8_t* Qs;
    const float* lse_s;
    if constexpr (RING) {
      wait_stages(min(nt - 1 - qt, NBUF - 2), true);
      __syncthreads();
      if (qt + NBUF - 1 < nt) issue(qt + NBUF - 1);
      Qs = smem + (qt % NBUF) * STAGE;
      lse_s = reinterpret_cast<const float*>(Qs + 2 * TILE_BYTES);
    } else {
      Qs = smem + (qt & 1) * 2 * TILE_BYTES;
      lse_s = rowv + (qt & 1) * 128;
      if (qt + 1 < nt) {
        tile_load(qr, Qg, ld, (qt + 1) * 64, S);
        tile_load(dr, dOg, ldo, (qt + 1) * 64, S);
        if (threadIdx.x < 128)
          rv = threadIdx.x < 64 ? lse_g[(qt + 1) * 64 + threadIdx.x] : del_g[(qt + 1) * 64 + threadIdx.x - 64];
      }
    }
    const uint8_t* Ds = Qs + TILE_BYTES;
    const float* del_s = lse_s + 64;
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2) {
      floatx16 sc[KS], dp[KS];
#pragma unroll
      for (int u = 0; u < KS; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) { sc[u][i] = 0.f; dp[u][i] = 0.f; }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 qfr = lds_row_frag(Qs, 32 * i2 + r, 2 * ks + hh);
        const bf16x8 dfr = lds_row_frag(Ds, 32 * i2 + r, 2 * ks + hh);
#pragma unroll
        for (int u = 0; u < KS; ++u) {
          sc[u] = mfma32(qfr, kf[u][ks], sc[u]);
          dp[u] = mfma32(dfr, vf[u][ks], dp[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < KS; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int qq = 32 * i2 + crow(i, hh);
          // LEAN: one FMA per score (-lse is a free operand modifier)
          const float p = __builtin_amdgcn_exp2f(LEAN ? fmaf(sc[u][i], sl2, -lse_s[qq])
                                                      : sc[u][i] * sl2 + mbk[u] - lse_s[qq]);
          sc[u][i] = p;
          dp[u][i] = p * (dp[u][i] - del_s[qq]);
        }
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        bf16x8 pb[KS], db[KS];
#pragma unroll
        for (int u = 0; u < KS; ++u) {
          pb[u] = pack_acc(sc[u], ss);
          db[u] = pack_acc(dp[u], ss);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const bf16x8 dtr = tr_operand(Ds, 32 * i2 + 16 * ss, hh, t, lane);
          const bf16x8 qtr = tr_operand(Qs, 32 * i2 + 16 * ss, hh, t, lane);
#pragma unroll
          for (int u = 0; u < KS; ++u) {
            dv[u][t] = mfma32(dtr, pb[u], dv[u][t]);
            dk[u][t] = mfma32(qtr, db[u], dk[u][t]);
          }
        }
      }
    }
    if constexpr (!RING) {
      if (qt + 1 < nt) {
        uint8_t* Qn = smem + ((qt & 1) ^ 1) * 2 * TILE_BYTES;
        tile_store(qr, Qn);
        tile_store(dr, Qn + TILE_BYTES);
        if (threadIdx.x < 128) rowv[((qt & 1) ^ 1) * 128 + threadIdx.x] = rv;
      }
      __syncthreads();
    }
  }
  };
  if (use_len) {
    qloop(std::true_type{});
#pragma unroll
    for (int u = 0; u < KS; ++u)
      if (k[u] >= kv_end)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) dk[u][t][i] = dv[u][t][i] = 0.f;
  } else {
    qloop(std::false_type{});
  }
#pragma unroll
  for (int u = 0; u < KS; ++u) {
    if (k[u] < S) {
      bf16_t* dkp = dqkv + (rb + k[u]) * ld + (long)H * HD + h * HD;
      bf16_t* dvp = dqkv + (rb + k[u]) * ld + 2L * H * HD + h * HD;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          store4(dkp + 32 * t + 8 * v + 4 * hh, dk[u][t][4 * v] * scale, dk[u][t][4 * v + 1] * scale,
                 dk[u][t][4 * v + 2] * scale, dk[u][t][4 * v + 3] * scale);
          store4(dvp + 32 * t + 8 * v + 4 * hh, dv[u][t][4 * v], dv[u][t][4 * v + 1], dv[u][t][4 * v + 2],
                 dv[u][t][4 * v + 3]);
        }
    }
  }
}

// Block order remapped so that the query blocks of one (batch, head) share an XCD's L2 (their K/V
// tiles are read by every one of them).
constexpr int kAttnXcd = 1;

}  // namespace

int dl_attn_fwd(const bf16_t* qkv, long ld, const float* mbias, const int* kvinfo, bf16_t* out, long ldo, float* lse,
                int B, int H, int S, int D, float scale, hipStream_t st) {
  if (D != HD || S % 64 != 0 || ld % 8 != 0 || ldo % 8 != 0) return -1;
  const float sl2 = scale * 1.4426950408889634f;
  // 4 waves x 2 query sub-blocks of 32 rows per wave, K/V staged by the LDS-DMA ring (it frees the
  // 16 staging VGPRs the second sub-block needs); 8-wave blocks measured 5% slower (round 2)
  dim3 grid((S + 255) / 256, H, B);
  attn_fwd_kernel<true, 2><<<grid, 256, 0, st>>>(qkv, ld, mbias, kvinfo, out, ldo, lse, B, H, S, sl2, kAttnXcd);
  return 0;
}

int dl_attn_bwd(const bf16_t* qkv, long ld, const float* mbias, const int* kvinfo, const bf16_t* out,
                const bf16_t* dout, long ldo, const float* lse, float* delta, bf16_t* dqkv, float* dbias, int B, int H,
                int S, int D, float scale, hipStream_t st) {
  if (D != HD || S % 64 != 0 || ld % 8 != 0 || ldo % 8 != 0) return -1;
  const float sl2 = scale * 1.4426950408889634f;
  // dQ: 2 query sub-blocks per wave with the LDS-DMA ring; dK/dV: one key sub-block per wave with
  // register staging (the one-wave-per-SIMD 2-sub-block form measured 8% slower, profiles/README.md)
  dim3 grid_dq((S + 255) / 256, H, B);
  attn_bwd_dq_kernel<true, 2><<<grid_dq, 256, 0, st>>>(qkv, ld, mbias, kvinfo, out, dout, ldo, lse, delta, dqkv,
                                                       dbias, B, H, S, sl2, scale, kAttnXcd);
  dim3 grid_kv((S + 127) / 128, H, B);
  attn_bwd_dkdv_kernel<false, 1><<<grid_kv, 256, 0, st>>>(qkv, ld, mbias, kvinfo, dout, ldo, lse, delta, dqkv, B, H,
                                                          S, sl2, scale, kAttnXcd);
  return 0;
}

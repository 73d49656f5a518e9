// Round-5 experiment, NOT built: the 8-wave ping-pong attention forward (measured 13% slower than
// the shipped 4-wave kernel at B=512, S=512, d=64: profiles/r5_attn_fwd_pingpong_negative.jsonl).
// It was compiled inside dedloc_amd/csrc/kernels/attention.hip (helpers FwdCtx, vmax3, half_max,
// tr_operand, lds_row_frag, wait_stages, STAGE, ... live there) and dispatched from dl_attn_fwd with
//   dim3 gp((S + PP_Q - 1) / PP_Q, H, B);
//   attn_fwd_pp_kernel<0><<<gp, 512, 0, st>>>(qkv, ld, mbias, kvinfo, out, ldo, lse, B, H, S, sl2, 1);
// Template PRIO: 0 = groups w >> 2 (waves w and w + 4 share a SIMD), 1 = groups w & 1 (slower
// still: 1183 us, which confirms the w / w + 4 pairing), 2 = group 1 at s_setprio 1 (no change).

// ------------------------------------------------------------------------------------ fwd, ping-pong
// 8-wave blocks of 512 queries (QS = 2 per wave) in which the two waves of each SIMD (w and w + 4,
// cdna_hip_programming.md T16 / MI355X_MICROARCH.md "Two waves per SIMD") alternate between a
// matrix segment and a softmax segment, separated by block barriers:
//   X(t): O += V(t-1)^T P(t-1)^T, then S(t) = K(t) Q^T                  (32 MFMAs, LDS reads)
//   Y(t): row max / rescale / exp2 / row sum / bf16 pack of S(t) -> P(t) (VALU only)
// Group 1 (waves 4-7) runs one segment behind group 0, so in every segment one wave of each SIMD
// feeds the matrix pipe while its partner runs the softmax.  In the 4-wave kernel both waves of a
// SIMD drift through S MFMAs, softmax and PV MFMAs at random phase, and PMC shows the SIMD time
// close to the SUM of VALU and MFMA time (profiles/README.md, round 5).
// Ring: tiles t-1 (V) and t (K) are read in segments 2t, 2t+1; X(t) issues tile t+2 into the slot
// of tile t-2, and every wave waits for its pieces of tile t+1 before the barrier that ends
// segment 2t+1.
constexpr int PP_NB = 4;
constexpr int PP_Q = 512;  // queries per block

template <bool LEAN>
__device__ __forceinline__ void pp_softmax(floatx16 (&s)[2][2], float (&m)[2], float (&l)[2], floatx16 (&o)[2][2],
                                           bf16x8 (&pk)[2][2][2], const float* mb, int kbase, int kv_end,
                                           float sl2, int hh) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (!LEAN) {
      if (mb) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int i = 0; i < 16; ++i) s[u][j][i] = fmaf(s[u][j][i], sl2, mb[32 * j + crow(i, hh)]);
      } else {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            s[u][j][i] = fmaf(s[u][j][i], sl2, kbase + 32 * j + crow(i, hh) < kv_end ? 0.f : NEG_BIG);
      }
    }
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
    if (LEAN) mx *= sl2;
    const bool grow = mx > m[u] + RESCALE_THR;
    if (__ballot(grow) != 0) {  // O already holds every P before this tile (PV(t-1) ran in X(t))
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
    float rsa[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float pv = __builtin_amdgcn_exp2f(LEAN ? fmaf(s[u][j][i], sl2, nm) : s[u][j][i] + nm);
        s[u][j][i] = pv;
        rsa[i & 7] += pv;
      }
    const float rs = ((rsa[0] + rsa[1]) + (rsa[2] + rsa[3])) + ((rsa[4] + rsa[5]) + (rsa[6] + rsa[7]));
    l[u] += half_sum(rs);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) pk[u][j][ss] = pack_acc(s[u][j], ss);
  }
}

__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int PRIO>
__global__ __launch_bounds__(512, 1) void attn_fwd_pp_kernel(const bf16_t* __restrict__ qkv, long ld,
                                                             const float* __restrict__ mbias,
                                                             const int* __restrict__ kvinfo, bf16_t* __restrict__ out,
                                                             long ldo, float* __restrict__ lse, int B, int H, int S,
                                                             float sl2, int xcd) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[PP_NB * STAGE];
  const BlockId bid = block_id(xcd);
  const int b = bid.b, h = bid.h;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, hh = lane >> 5;
  const int grp = PRIO == 1 ? (__builtin_amdgcn_readfirstlane(w) & 1) : (__builtin_amdgcn_readfirstlane(w) >> 2);
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
  c.mbs = nullptr;
  c.w = w;
  c.lane = lane;
  const int nt = (c.kv_end + 63) / 64;
  const bool has_mb = c.mb_g != nullptr;
  for (int s0 = 0; s0 < PP_NB - 2 && s0 < nt; ++s0) c.template issue<8, PP_NB>(s0);

  int q[2];
  bf16x8 qf[2][4];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    q[u] = bid.x * PP_Q + w * 64 + 32 * u + r;
    const int qc = min(q[u], S - 1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      qf[u][ks] = gload8(Qg + (long)qc * ld + ks * 16 + 8 * hh);
      settle(qf[u][ks]);
    }
  }
  floatx16 o[2][2], s[2][2];
  bf16x8 pk[2][2][2];
  float m[2], l[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    m[u] = NEG_BIG;
    l[u] = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[u][t][i] = 0.f;
  }
  wait_vm_all();
  __syncthreads();
  if (grp == 1) pp_barrier();  // group 1 runs one segment behind
  if (PRIO == 2 && grp == 1) __builtin_amdgcn_s_setprio(1);

  // waits for this wave's pieces of tile t + 1 with tile t + 2 possibly still in flight
  auto wait_next = [&](int t) {
    if (t + 2 < nt) wait_stages<2>(1, has_mb);
    else if (t + 1 < nt) wait_stages<2>(0, has_mb);
  };
  auto pv = [&](int t) {  // O += V(t)^T P(t)^T
    const uint8_t* Vs = smem + (t % PP_NB) * STAGE + TILE_BYTES;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const bf16x8 vfr = tr_operand(Vs, 32 * j + 16 * ss, hh, tt, lane);
#pragma unroll
          for (int u = 0; u < 2; ++u) o[u][tt] = mfma32(vfr, pk[u][j][ss], o[u][tt]);
        }
  };
  auto qk = [&](int t) {  // S(t) = K(t) Q^T; issues tile t + 2
    if (t + 2 < nt) c.template issue<8, PP_NB>(t + 2);
    const uint8_t* Ks = smem + (t % PP_NB) * STAGE;
#pragma unroll
    for (int u = 0; u < 2; ++u)
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
        for (int u = 0; u < 2; ++u) s[u][j] = mfma32(kfr, qf[u][ks], s[u][j]);
      }
  };
  auto mb_of = [&](int t) {
    return has_mb ? reinterpret_cast<const float*>(smem + (t % PP_NB) * STAGE + 2 * TILE_BYTES) : nullptr;
  };
  // Y(t) then X(t + 1) for t in [t0, t1); LEAN: tiles without any mask (separate loops, so the
  // two softmax bodies never share a loop body's registers)
  auto run = [&](auto lean_tag, int t0, int t1) {
    constexpr bool LEAN = decltype(lean_tag)::value;
    for (int t = t0; t < t1; ++t) {
      pp_softmax<LEAN>(s, m, l, o, pk, mb_of(t), t * 64, c.kv_end, sl2, hh);
      if (grp == 0) wait_next(t);
      pp_barrier();
      pv(t);
      __builtin_amdgcn_sched_barrier(0);
      qk(t + 1);
      if (grp == 1) wait_next(t + 1);
      pp_barrier();
    }
  };
  auto tail = [&](auto lean_tag) {  // Y(nt - 1), X(nt) = PV(nt - 1)
    constexpr bool LEAN = decltype(lean_tag)::value;
    pp_softmax<LEAN>(s, m, l, o, pk, mb_of(nt - 1), (nt - 1) * 64, c.kv_end, sl2, hh);
    pp_barrier();
    pv(nt - 1);
    pp_barrier();
  };
  // tiles [0, nlean) need no mask: every tile without the generic bias that ends inside kv_end
  const int nlean = has_mb ? 0 : c.kv_end / 64;
  // segment 0: X(0) = S(0)
  qk(0);
  if (grp == 1) wait_next(0);
  pp_barrier();
  run(std::true_type{}, 0, min(nlean, nt - 1));
  run(std::false_type{}, min(nlean, nt - 1), nt - 1);
  tail(std::false_type{});  // (a lean/masked branch here costs ~10 spilled registers)
  if (grp == 0) pp_barrier();

#pragma unroll
  for (int u = 0; u < 2; ++u) {
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


// hipBLASLt GELU-family epilogue probe (gfx950, ROCm 7.2): which of GELU_AUX(_BIAS) / DGELU(_BGRAD)
// have solutions for bf16 in / bf16 out / fp32 compute, and what exactly do they compute?
// The FFN of ALBERT would drop one HBM-bound kernel per direction if one of them is usable
// (profiles/README.md: GELU forward 3.1%, GELU backward + bias sums 5.0% of the micro-step).
//
// Column-major, our forward's form: D[m x n] = op(A)^T... with opA = T (A stored [k x m], ld k),
// opB = N (B stored [k x n], ld k), D / aux stored [m x n] (ld m), bias [m] (m = features, n = tokens).
// Every result is compared against host references of several interpretations, so a layout or
// formula mismatch shows up as "matches hypothesis X" instead of a bare relative error.
//
//   hipcc --offload-arch=gfx950 -O2 bench/hip/lt_epilogue_probe.cpp -lhipblaslt -o bench/hip/lt_epilogue_probe
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hipblaslt/hipblaslt.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

static float bf2f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
static uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float gelu_tanh(float x) {
  const float u = 0.7978845608f * (x + 0.044715f * x * x * x);
  return 0.5f * x * (1.f + std::tanh(u));
}
static float dgelu_tanh(float x) {
  const float u = 0.7978845608f * (x + 0.044715f * x * x * x);
  const float t = std::tanh(u);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * 0.7978845608f * (1.f + 3.f * 0.044715f * x * x);
}
static float dgelu_erf(float x) {
  return 0.5f * (1.f + std::erf(x / std::sqrt(2.f))) + x * std::exp(-0.5f * x * x) / std::sqrt(2.f * (float)M_PI);
}
static double rel(const std::vector<float>& a, const std::vector<float>& b) {
  double num = 0, den = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    num += (double)(a[i] - b[i]) * (a[i] - b[i]);
    den += (double)b[i] * b[i];
  }
  return std::sqrt(num / (den + 1e-30));
}

#define CK(x)                                                                  \
  do {                                                                         \
    auto _s = (x);                                                             \
    if (_s != 0) std::printf("  %s -> status %d\n", #x, (int)_s);              \
  } while (0)

int main(int argc, char** argv) {
  const int m = argc > 1 ? std::atoi(argv[1]) : 1024;  // features
  const int n = argc > 2 ? std::atoi(argv[2]) : 2048;  // tokens
  const int k = argc > 3 ? std::atoi(argv[3]) : 512;
  std::mt19937 rng(0);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<uint16_t> hA((size_t)k * m), hB((size_t)k * n), hAux((size_t)m * n);
  std::vector<float> fA(hA.size()), fB(hB.size()), fAux(hAux.size()), bias(m);
  for (size_t i = 0; i < hA.size(); ++i) { hA[i] = f2bf(nd(rng) / std::sqrt((float)k)); fA[i] = bf2f(hA[i]); }
  for (size_t i = 0; i < hB.size(); ++i) { hB[i] = f2bf(nd(rng)); fB[i] = bf2f(hB[i]); }
  for (size_t i = 0; i < hAux.size(); ++i) { hAux[i] = f2bf(1.5f * nd(rng)); fAux[i] = bf2f(hAux[i]); }
  for (int i = 0; i < m; ++i) bias[i] = 0.5f * nd(rng);
  // host GEMM: G[i + j*m] = sum_l A[l + i*k] * B[l + j*k]
  std::vector<float> G((size_t)m * n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) {
      double s = 0;
      for (int l = 0; l < k; ++l) s += (double)fA[l + (size_t)i * k] * fB[l + (size_t)j * k];
      G[i + (size_t)j * m] = (float)s;
    }

  void *dA, *dB, *dD, *dAux, *dBias, *dWs;
  const size_t ws = 64ull << 20;
  hipMalloc(&dA, hA.size() * 2);
  hipMalloc(&dB, hB.size() * 2);
  hipMalloc(&dD, (size_t)m * n * 2);
  hipMalloc(&dAux, hAux.size() * 4);  // room for an fp32 aux
  hipMalloc(&dBias, m * 4);
  hipMalloc(&dWs, ws);
  hipMemcpy(dA, hA.data(), hA.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB.data(), hB.size() * 2, hipMemcpyHostToDevice);
  hipblasLtHandle_t h;
  hipblasLtCreate(&h);

  struct Case { const char* name; hipblasLtEpilogue_t epi; bool aux_in; bool has_bias; bool bias_out; };
  const Case cases[] = {
      {"GELU_AUX_BIAS", HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, false, true, false},
      {"GELU_AUX", HIPBLASLT_EPILOGUE_GELU_AUX, false, false, false},
      {"GELU_BIAS", HIPBLASLT_EPILOGUE_GELU_BIAS, false, true, false},
      {"DGELU", HIPBLASLT_EPILOGUE_DGELU, true, false, false},
      {"DGELU_BGRAD", HIPBLASLT_EPILOGUE_DGELU_BGRAD, true, false, true},
  };
  for (const Case& c : cases) {
    // aux type variants: 0 = bf16, 1 = attribute left unset (library default), 2 = fp32 aux
    for (int aux_mode = 0; aux_mode < 3; ++aux_mode) {
      if (aux_mode > 0 && std::strcmp(c.name, "GELU_BIAS") == 0) continue;
      std::printf("%s (m=%d n=%d k=%d, aux %s):\n", c.name, m, n, k,
                  aux_mode == 0 ? "bf16" : aux_mode == 1 ? "type unset" : "fp32");
      hipMemcpy(dAux, hAux.data(), hAux.size() * 2, hipMemcpyHostToDevice);
      hipMemcpy(dBias, bias.data(), m * 4, hipMemcpyHostToDevice);
      hipMemset(dD, 0, (size_t)m * n * 2);
      hipblasLtMatmulDesc_t desc;
      CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
      hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
      CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
      CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
      CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &c.epi, sizeof(c.epi)));
      if (c.has_bias || c.bias_out) {
        const int32_t bt = HIP_R_32F;
        CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
        CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &dBias, sizeof(dBias)));
      }
      const int64_t ldaux = m;
      const int32_t at = aux_mode == 2 ? HIP_R_32F : HIP_R_16BF;
      CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &dAux, sizeof(dAux)));
      CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ldaux, sizeof(ldaux)));
      if (aux_mode != 1)
        CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at)));
      hipblasLtMatrixLayout_t la, lb, ld;
      CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, k, m, k));
      CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, k, n, k));
      CK(hipblasLtMatrixLayoutCreate(&ld, HIP_R_16BF, m, n, m));
      hipblasLtMatmulPreference_t pref;
      hipblasLtMatmulPreferenceCreate(&pref);
      uint64_t wsz = ws;
      hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz, sizeof(wsz));
      hipblasLtMatmulHeuristicResult_t res[16];
      int cnt = 0;
      const auto hs = hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, ld, ld, pref, 16, res, &cnt);
      std::printf("  heuristic status %d, %d algos\n", (int)hs, cnt);
      for (int a = 0; a < cnt && a < (aux_mode == 0 ? 3 : (aux_mode == 1 ? 1 : 0)); ++a) {
        hipMemcpy(dAux, hAux.data(), hAux.size() * 2, hipMemcpyHostToDevice);
        hipMemcpy(dBias, bias.data(), m * 4, hipMemcpyHostToDevice);
        const float one = 1.f, zero = 0.f;
        const auto st = hipblasLtMatmul(h, desc, &one, dA, la, dB, lb, &zero, dD, ld, dD, ld, &res[a].algo, dWs, ws, 0);
        hipDeviceSynchronize();
        std::vector<uint16_t> oD((size_t)m * n), oAux(hAux.size());
        std::vector<float> outB(m);
        hipMemcpy(oD.data(), dD, oD.size() * 2, hipMemcpyDeviceToHost);
        hipMemcpy(oAux.data(), dAux, oAux.size() * 2, hipMemcpyDeviceToHost);
        hipMemcpy(outB.data(), dBias, m * 4, hipMemcpyDeviceToHost);
        std::vector<float> D(oD.size()), AUX(oAux.size());
        for (size_t i = 0; i < D.size(); ++i) D[i] = bf2f(oD[i]);
        for (size_t i = 0; i < AUX.size(); ++i) AUX[i] = bf2f(oAux[i]);
        std::printf("  algo %d: matmul status %d\n", a, (int)st);
        std::vector<float> ref(D.size()), ref2(D.size()), ref3(D.size()), ref4(D.size());
        if (!c.aux_in) {
          for (int j = 0; j < n; ++j)
            for (int i = 0; i < m; ++i) {
              const size_t q = i + (size_t)j * m;
              const float pre = G[q] + (c.has_bias ? bias[i] : 0.f);
              ref[q] = gelu_tanh(pre);
              ref2[q] = pre;
            }
          std::printf("    D vs gelu_tanh(AB+b) %.3e | D vs AB+b %.3e | aux vs AB+b %.3e\n", rel(D, ref), rel(D, ref2),
                      rel(AUX, ref2));
        } else {
          for (int j = 0; j < n; ++j)
            for (int i = 0; i < m; ++i) {
              const size_t q = i + (size_t)j * m;
              const size_t qt = (size_t)(q % n) * m + q / n;  // aux read with swapped dims
              ref[q] = G[q] * dgelu_tanh(fAux[q]);
              ref2[q] = G[q] * dgelu_erf(fAux[q]);
              ref3[q] = G[q] * dgelu_tanh(fAux[qt % fAux.size()]);
              ref4[q] = G[q];
            }
          std::printf("    D vs AB*gelu'_tanh(aux) %.3e | *gelu'_erf(aux) %.3e | aux transposed %.3e | plain AB %.3e\n",
                      rel(D, ref), rel(D, ref2), rel(D, ref3), rel(D, ref4));
          if (c.bias_out) {
            std::vector<float> cs(m, 0.f), csd(m, 0.f);
            for (int j = 0; j < n; ++j)
              for (int i = 0; i < m; ++i) {
                cs[i] += ref[i + (size_t)j * m];
                csd[i] += D[i + (size_t)j * m];
              }
            std::printf("    bias-grad out vs rowsum(ref) %.3e | vs rowsum(D) %.3e\n", rel(outB, cs), rel(outB, csd));
          }
        }
      }
      hipblasLtMatmulPreferenceDestroy(pref);
      hipblasLtMatrixLayoutDestroy(la);
      hipblasLtMatrixLayoutDestroy(lb);
      hipblasLtMatrixLayoutDestroy(ld);
      hipblasLtMatmulDescDestroy(desc);
    }
  }
  hipblasLtDestroy(h);
  std::printf("PROBE_DONE\n");
  return 0;
}

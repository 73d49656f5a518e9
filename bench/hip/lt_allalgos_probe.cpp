// hipBLASLt exhaustive-solution probe for the ALBERT GEMM shapes (gfx950, ROCm 7.2).
//
// dedloc's plan cache (csrc/host/lt_gemm.cpp) autotunes over the top-64 candidates of
// hipblasLtMatmulAlgoGetHeuristic.  This probe times EVERY solution hipblaslt_ext::getAllAlgos
// knows for the same problem type (supported ones only) to see whether a faster kernel exists
// outside the heuristic's list.  Result (profiles/allalgos2_*.log, random operands): the forward
// GEMMs have direct-to-LDS 256x256 solutions 11-13% faster back to back than the top-64's best;
// the weight-gradient GEMMs none.  Inside the model step the gain shrinks to +0.4%
// (profiles/lt_exhaustive_tune_b512.log), which is why lt_gemm.cpp keeps the search opt-in.
//
// Row-major contract as in lt_gemm.cpp: D[M,N] = op(A)[M,K] . op(B)[K,N], handed to hipBLASLt as the
// column-major D^T = op(B)^T op(A)^T.
//   wgrad: A = dY [K=T, M] (transA), B = X [T, N], D fp32 [S, M, N] (token-split batch S)
//   fwd  : A = X [M=T, K], B = W [N, K] (transB), D bf16 [M, N]
//
//   hipcc --offload-arch=gfx950 -O2 bench/hip/lt_allalgos_probe.cpp -lhipblaslt -o bench/hip/probe_lt_allalgos
//   ./probe_lt_allalgos wgrad M N T S | fwd M N K | fwdb M N K  (fwdb: with the fp32 bias epilogue)
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

// pseudo-random bf16 in [-1, 1) (constant operands let the chip clock higher and flatter the
// timings by 10-30%: the first version of this probe filled 0x3c3c and overstated every kernel)
__global__ void fill_random(uint16_t* p, long n, uint32_t seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    const float f = (float)(h & 0xffff) / 32768.f - 1.f;
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    p[i] = (uint16_t)(u >> 16);
  }
}

#define CK(x)                                                                       \
  do {                                                                              \
    auto _s = (x);                                                                  \
    if (_s != 0) { std::printf("%s -> %d\n", #x, (int)_s); std::exit(1); }        \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 5) {
    std::printf("usage: %s wgrad M N T S | fwd M N K | fwdb M N K\n", argv[0]);
    return 1;
  }
  const std::string mode = argv[1];
  const bool wg = mode == "wgrad";
  const bool with_bias = mode == "fwdb";  // forward with the fp32-bias epilogue (what the model uses)
  const long M = std::atol(argv[2]), N = std::atol(argv[3]), KT = std::atol(argv[4]);
  const int S = wg && argc > 5 ? std::atoi(argv[5]) : 1;
  const long K = wg ? KT / S : KT;  // per-batch reduction length
  const int transA = wg ? 1 : 0, transB = wg ? 0 : 1;
  // our operands (row-major)
  const long a_elems = wg ? KT * M : M * K, b_elems = wg ? KT * N : N * K;
  const long lda = wg ? M : K, ldb = wg ? N : K;
  const size_t d_bytes = (size_t)S * M * N * (wg ? 4 : 2);
  void *A, *B, *D, *ws;
  const size_t wsz = 128ull << 20;
  CK(hipMalloc(&A, a_elems * 2));
  CK(hipMalloc(&B, b_elems * 2));
  CK(hipMalloc(&D, d_bytes));
  CK(hipMalloc(&ws, wsz));
  fill_random<<<4096, 256>>>((uint16_t*)A, a_elems, 1u);
  fill_random<<<4096, 256>>>((uint16_t*)B, b_elems, 2u);
  void* bias = nullptr;
  CK(hipMalloc(&bias, N * 4));
  CK(hipMemset(bias, 0, N * 4));
  hipblasLtHandle_t h;
  CK(hipblasLtCreate(&h));
  hipblasLtMatmulDesc_t desc;
  CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const hipblasOperation_t opA = transB ? HIPBLAS_OP_T : HIPBLAS_OP_N;  // hip "A" = our B
  const hipblasOperation_t opB = transA ? HIPBLAS_OP_T : HIPBLAS_OP_N;  // hip "B" = our A
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof(opA)));
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof(opB)));
  if (with_bias) {
    const hipblasLtEpilogue_t epi = HIPBLASLT_EPILOGUE_BIAS;
    const int32_t bt = HIP_R_32F;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
  }
  const hipDataType dt = wg ? HIP_R_32F : HIP_R_16BF;
  hipblasLtMatrixLayout_t la, lb, ld;
  const uint64_t a_rows = transB ? K : N, a_cols = transB ? N : K;
  const uint64_t b_rows = transA ? M : K, b_cols = transA ? K : M;
  CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, a_rows, a_cols, ldb));
  CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, b_rows, b_cols, lda));
  CK(hipblasLtMatrixLayoutCreate(&ld, dt, N, M, N));
  if (S > 1) {
    const int32_t bc = S;
    const int64_t sa = K * ldb, sb = K * lda, sd = M * N;
    CK(hipblasLtMatrixLayoutSetAttribute(la, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc)));
    CK(hipblasLtMatrixLayoutSetAttribute(la, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &sa, sizeof(sa)));
    CK(hipblasLtMatrixLayoutSetAttribute(lb, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc)));
    CK(hipblasLtMatrixLayoutSetAttribute(lb, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &sb, sizeof(sb)));
    CK(hipblasLtMatrixLayoutSetAttribute(ld, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc)));
    CK(hipblasLtMatrixLayoutSetAttribute(ld, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &sd, sizeof(sd)));
  }
  const float one = 1.f, beta = wg ? 1.f : 0.f;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double flop = 2.0 * M * N * K * S;
  auto time_algo = [&](hipblasLtMatmulAlgo_t& algo, int reps) -> double {
    if (hipblasLtMatmul(h, desc, &one, B, la, A, lb, &beta, D, ld, D, ld, &algo, ws, wsz, 0) != HIPBLAS_STATUS_SUCCESS)
      return -1;
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) hipblasLtMatmul(h, desc, &one, B, la, A, lb, &beta, D, ld, D, ld, &algo, ws, wsz, 0);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / reps * 1e3;  // us
  };

  // 1. the heuristic's top 64 (what lt_gemm.cpp autotunes over)
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  uint64_t w = wsz;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &w, sizeof(w));
  std::vector<hipblasLtMatmulHeuristicResult_t> heur(64);
  int nh = 0;
  hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, ld, ld, pref, 64, heur.data(), &nh);
  double best_h = 1e30;
  std::string best_h_name;
  for (int i = 0; i < nh; ++i) {
    const double us = time_algo(heur[i].algo, 3);
    if (us > 0 && us < best_h) {
      best_h = us;
      best_h_name = hipblaslt_ext::getKernelNameFromAlgo(h, heur[i].algo);
    }
  }
  std::printf("{\"mode\": \"%s\", \"M\": %ld, \"N\": %ld, \"K_total\": %ld, \"S\": %d, \"heuristic_candidates\": %d, "
              "\"heuristic_best_us\": %.1f, \"heuristic_best_tflops\": %.1f, \"heuristic_best\": \"%s\"}\n",
              mode.c_str(), M, N, KT, S, nh, best_h, flop / best_h * 1e-6, best_h_name.c_str());
  std::fflush(stdout);

  // 2. every solution of the problem type
  std::vector<hipblasLtMatmulHeuristicResult_t> all;
  CK(hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, opA, opB, HIP_R_16BF, HIP_R_16BF, dt, dt,
                                HIPBLAS_COMPUTE_32F, all));
  std::vector<std::pair<double, int>> timed;
  int supported = 0;
  for (size_t i = 0; i < all.size(); ++i) {
    size_t need = 0;
    if (hipblaslt_ext::matmulIsAlgoSupported(h, desc, &one, la, lb, &beta, ld, ld, all[i].algo, need) !=
            HIPBLAS_STATUS_SUCCESS ||
        need > wsz)
      continue;
    ++supported;
    const double us = time_algo(all[i].algo, 2);
    if (us > 0) timed.emplace_back(us, (int)i);
    if (supported % 100 == 0) {
      std::printf("  ... %d supported timed of %zu\n", supported, all.size());
      std::fflush(stdout);
    }
  }
  std::sort(timed.begin(), timed.end());
  // re-time the 8 fastest with more repetitions
  std::vector<std::pair<double, int>> top;
  for (size_t k = 0; k < timed.size() && k < 8; ++k)
    top.emplace_back(time_algo(all[timed[k].second].algo, 10), timed[k].second);
  std::sort(top.begin(), top.end());
  std::printf("{\"all_algos\": %zu, \"supported\": %d}\n", all.size(), supported);
  for (auto& t : top)
    std::printf("{\"us\": %.1f, \"tflops\": %.1f, \"index\": %d, \"kernel\": \"%s\"}\n", t.first, flop / t.first * 1e-6,
                hipblaslt_ext::getIndexFromAlgo(all[t.second].algo),
                hipblaslt_ext::getKernelNameFromAlgo(h, all[t.second].algo).c_str());
  std::printf("PROBE_DONE\n");
  return 0;
}

// hipBLASLt GEMM entry point (csrc/host/lt_gemm.cpp).  Row-major contract, see the .cpp header.
#pragma once
#include <hip/hip_runtime.h>

enum DlLtEpilogue { DL_LT_NONE = 0, DL_LT_BIAS = 1, DL_LT_GELU_AUX_BIAS = 2, DL_LT_DGELU_BGRAD = 3, DL_LT_GELU_BIAS = 4 };

struct DlLtArgs {
  int transA = 0, transB = 0;
  int M = 0, N = 0, K = 0;
  const void* A = nullptr;
  long lda = 0;
  const void* B = nullptr;
  long ldb = 0;
  void* D = nullptr;
  const void* C = nullptr;  // beta * C is added (same layout as D); nullptr -> C = D
  long ldd = 0;
  int d_f32 = 0;       // D (and C) fp32, else bf16
  int in_f32 = 0;      // A/B fp32, else bf16
  float beta = 0.f;
  int epilogue = DL_LT_NONE;
  const void* bias = nullptr;  // [N]; for DGELU_BGRAD this is the bias-gradient OUTPUT
  int bias_f32 = 1;
  void* aux = nullptr;         // [M, N] bf16 (ldaux): GELU pre-activation (written fwd, read bwd)
  long ldaux = 0;
  // strided batch (e.g. split-K over the token dimension: batch b reads A/B at +b*strideA/B and
  // writes its own partial D at +b*strideD); strides in elements
  int batch = 1;
  long strideA = 0, strideB = 0, strideD = 0;
};

// 0 on success; < 0 when hipBLASLt has no solution (callers fall back)
int dl_lt_matmul(const DlLtArgs& a, hipStream_t st);
int dl_lt_plan_count();

// Stand-alone timing harness for gemm8.hip (not part of the library): the NT GEMM on an ALBERT
// shape, outside torch.  The round-2/3 probe variants (no epilogue, no output stores, desynchronised
// first wave) were compiled from #ifdef hooks inside the shipped kernel; those hooks were removed
// (VERDICT r4): to re-run a probe, copy gemm8.hip next to this file, edit the copy, and include it
// instead.  Their results stay in profiles/README.md.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I dedloc_amd/csrc/include bench/hip/gemm8_probe.hip -o probe
#include "../../dedloc_amd/csrc/kernels/gemm8.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 131072, N = argc > 2 ? atoi(argv[2]) : 3072, K = argc > 3 ? atoi(argv[3]) : 1024;
  bf16_t *A, *B, *C;
  float* Cf;
  DL_HIP_CHECK(hipMalloc(&A, (size_t)M * K * 2));
  DL_HIP_CHECK(hipMalloc(&B, (size_t)N * K * 2));
  DL_HIP_CHECK(hipMalloc(&C, (size_t)M * N * 2));
  DL_HIP_CHECK(hipMalloc(&Cf, 4096 * 4));
  std::vector<uint16_t> h((size_t)M * K);
  uint32_t s = 12345;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = 0x3c00 | ((s >> 9) & 0x7f) | ((s >> 16) & 0x8000); }
  DL_HIP_CHECK(hipMemcpy(A, h.data(), (size_t)M * K * 2, hipMemcpyHostToDevice));
  DL_HIP_CHECK(hipMemcpy(B, h.data(), (size_t)N * K * 2, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int it = 0; it < 3; ++it)
    dl_gemm8(0, 0, 0, A, K, B, K, M, N, K, C, N, Cf, 0, 0, 0, nullptr, nullptr, 0, nullptr, 0, nullptr, 1, 0);
  hipEventRecord(e0, 0);
  const int iters = 20;
  for (int it = 0; it < iters; ++it)
    dl_gemm8(0, 0, 0, A, K, B, K, M, N, K, C, N, Cf, 0, 0, 0, nullptr, nullptr, 0, nullptr, 0, nullptr, 1, 0);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / iters;
  printf("{\"probe\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"us\": %.1f, \"tflops\": %.1f}\n", argc > 4 ? argv[4] : "",
         M, N, K, us, 2.0 * M * N * K / us / 1e6);
  return 0;
}

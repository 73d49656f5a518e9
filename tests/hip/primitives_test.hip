// Standalone gfx950 primitive checks (run on the GPU box): MFMA 32x32x16 bf16 operand/result
// layout, ds_read_b64_tr_b16 semantics through the generic->LDS pointer cast used by
// attention.hip, and the accumulator-as-operand chain.  Prints mismatch counts; exit code != 0 on
// any mismatch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef short s4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4_t lds_s4;

__global__ void mfma_layout(const float* A, const float* B, float* C) {
  // A [32][16], B [16][32] row-major fp32 (small ints); lane (r,h) loads A[r][8h+j], B[8h+j][r]
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)A[r * 16 + 8 * h + j];
    b[j] = (__bf16)B[(8 * h + j) * 32 + r];
  }
  floatx16 c;
  for (int i = 0; i < 16; ++i) c[i] = 0.f;
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int i = 0; i < 16; ++i) C[l * 16 + i] = c[i];
}

__device__ __forceinline__ s4_t tr_generic(const unsigned char* tile, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(tile + off));
}

__global__ void tr_read(short* out, int use_generic) {
  __shared__ __attribute__((aligned(16))) short lds[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) lds[i] = (short)i;  // value = row*64 + col
  __syncthreads();
  const int l = threadIdx.x, i = l & 15, g = l >> 4;
  const int row = 4 * g + (i >> 2), col = 16 * g + 4 * (i & 3);
  const int off = (row * 64 + col) * 2;
  s4_t v;
  if (use_generic) v = tr_generic(reinterpret_cast<const unsigned char*>(lds), off);
  else v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)((__attribute__((address_space(3))) char*)lds + off));
  for (int q = 0; q < 4; ++q) out[l * 4 + q] = v[q];
}

int main() {
  int bad = 0;
  // ---- MFMA layout
  std::vector<float> A(32 * 16), B(16 * 32), C(64 * 16);
  for (int i = 0; i < 32 * 16; ++i) A[i] = (float)((i * 7) % 5 - 2);
  for (int i = 0; i < 16 * 32; ++i) B[i] = (float)((i * 3) % 7 - 3);
  float *dA, *dB, *dC;
  hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dC, C.size() * 4);
  hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
  mfma_layout<<<1, 64>>>(dA, dB, dC);
  hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
  int mb = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 16; ++i) {
      const int row = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5), col = l & 31;
      float ref = 0;
      for (int k = 0; k < 16; ++k) ref += A[row * 16 + k] * B[k * 32 + col];
      if (ref != C[l * 16 + i]) ++mb;
    }
  printf("mfma 32x32x16 layout mismatches: %d\n", mb);
  bad += mb;
  // ---- tr read
  for (int gen = 0; gen < 2; ++gen) {
    short* dO;
    hipMalloc(&dO, 64 * 4 * 2);
    tr_read<<<1, 64>>>(dO, gen);
    std::vector<short> O(256);
    hipMemcpy(O.data(), dO, 512, hipMemcpyDeviceToHost);
    int mt = 0;
    for (int l = 0; l < 64; ++l) {
      const int i = l & 15, g = l >> 4;
      for (int q = 0; q < 4; ++q) {
        const int exp = (4 * g + q) * 64 + 16 * g + i;
        if (O[l * 4 + q] != exp) {
          if (mt < 4) printf("  lane %d elem %d got %d (row %d col %d) expected %d\n", l, q, O[l * 4 + q],
                             O[l * 4 + q] / 64, O[l * 4 + q] % 64, exp);
          ++mt;
        }
      }
    }
    printf("tr_read (%s pointer) mismatches: %d\n", gen ? "generic" : "lds", mt);
    bad += mt;
  }
  printf(bad ? "FAIL\n" : "OK\n");
  return bad ? 1 : 0;
}

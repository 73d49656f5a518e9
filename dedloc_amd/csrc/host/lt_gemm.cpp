// Library GEMMs with fused epilogues through hipBLASLt, called directly (no ATen detour), with a
// per-shape algorithm cache and first-call autotuning.
//
// Row-major contract used by the rest of dedloc (all matrices row-major):
//   D[M,N] = op(A)[M,K] · op(B)[K,N]  (+ beta·D) (+ bias[N]) -> epilogue
//   A is [M,K] (lda) or, with transA, [K,M];  B is [K,N] (ldb) or, with transB, [N,K].
// hipBLASLt is column-major, so we hand it the transposed problem D^T[N,M] = op(B)^T · op(A)^T:
// its matrix "A" is our B and its "B" is our A, with m = N, n = M.  Bias vectors then run along
// the column-major rows = our output features, exactly what Linear layers need, and the
// DGELU_BGRAD bias gradient is the sum over tokens.
//
// Epilogues: BIAS (fp32 bias read in the epilogue — no per-call bias cast kernel) and beta=1
// accumulation with a separate C (residual-branch sums, fp32 weight-gradient accumulation).
// GELU_AUX_BIAS / DGELU_BGRAD are wired but NOT used: on ROCm 7.2 / gfx950 neither has a solution
// (bench/hip/lt_epilogue_probe.cpp, profiles/hipblaslt_gelu_epilogue_probe.log).
//
// Plan choice, at the first call of a (layout, shape, epilogue) key:
//   1. the tuning database (DEDLOC_LT_DB, default the in-package lt_tuning_gfx950.txt written by
//      python on import): key -> hipBLASLt solution index, verified with matmulIsAlgoSupported;
//   2. otherwise autotune: time the heuristic's top-64 candidates; with DEDLOC_LT_EXHAUSTIVE=1, for
//      large bf16-output problems (forward / data-gradient GEMMs) also EVERY supported solution of
//      the problem type (hipblaslt_ext::getAllAlgos, ~230 runnable per plan, about 5 s each).  In
//      isolation the heuristic list misses direct-to-LDS 256x256 kernels that run the forward
//      GEMMs 11-13% faster back to back on random operands (bench/hip/lt_allalgos_probe.cpp,
//      profiles/allalgos2_*.log), but inside the model step the heuristic's stream-K picks hold up:
//      micro-step 936.5 (exhaustive) vs 932.6 (heuristic) samples/s on one box
//      (profiles/lt_exhaustive_tune_b512.log), so the search is opt-in; its results for the
//      micro-batch-512 shapes ship as lt_tuning_gfx950.txt (935.3 from the database on the same box,
//      and no tuning at start-up).  Newly tuned keys are appended to DEDLOC_LT_DB_OUT.
#include <algorithm>
#include <utility>
#include <vector>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <mutex>
#include <tuple>
#include <vector>

#include "dl_lt.h"

namespace {

struct Key {
  int ta, tb, M, N, K;
  long lda, ldb, ldd, ldaux;
  int d_f32, in_f32, beta_nz, epi, bias_f32, dev, batch;
  long sA, sB, sD;
  bool operator<(const Key& o) const {
    return std::tie(ta, tb, M, N, K, lda, ldb, ldd, ldaux, d_f32, in_f32, beta_nz, epi, bias_f32, dev, batch, sA, sB,
                    sD) < std::tie(o.ta, o.tb, o.M, o.N, o.K, o.lda, o.ldb, o.ldd, o.ldaux, o.d_f32, o.in_f32,
                                   o.beta_nz, o.epi, o.bias_f32, o.dev, o.batch, o.sA, o.sB, o.sD);
  }
};

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, ld = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
  bool ok = false;
};

struct DevState {
  hipblasLtHandle_t handle = nullptr;
  void* workspace = nullptr;
  size_t ws_size = 0;
  void* scratch = nullptr;  // autotuning output sink
  size_t scratch_size = 0;
};

std::mutex g_mu;
std::map<Key, Plan> g_plans;

// ---- tuning database: one "key index" line per plan (key = every Key field but the device)
std::string key_str(const Key& k) {
  std::ostringstream o;
  o << k.ta << ',' << k.tb << ',' << k.M << ',' << k.N << ',' << k.K << ',' << k.lda << ',' << k.ldb << ',' << k.ldd
    << ',' << k.ldaux << ',' << k.d_f32 << ',' << k.in_f32 << ',' << k.beta_nz << ',' << k.epi << ',' << k.bias_f32
    << ',' << k.batch << ',' << k.sA << ',' << k.sB << ',' << k.sD;
  return o.str();
}

std::map<std::string, int>& tuning_db() {
  static std::map<std::string, int> db;
  static bool loaded = false;
  if (!loaded) {
    loaded = true;
    if (const char* path = std::getenv("DEDLOC_LT_DB")) {
      std::ifstream f(path);
      std::string key;
      int idx;
      while (f >> key >> idx) db[key] = idx;
    }
  }
  return db;
}

void record_tuning(const std::string& key, int idx) {
  tuning_db()[key] = idx;
  if (const char* out = std::getenv("DEDLOC_LT_DB_OUT")) {
    std::ofstream f(out, std::ios::app);
    f << key << ' ' << idx << '\n';
  }
}
std::map<int, DevState> g_dev;

constexpr size_t kWorkspace = 128ull << 20;

hipblasLtEpilogue_t to_lt(int epi) {
  switch (epi) {
    case DL_LT_BIAS: return HIPBLASLT_EPILOGUE_BIAS;
    case DL_LT_GELU_AUX_BIAS: return HIPBLASLT_EPILOGUE_GELU_AUX_BIAS;
    case DL_LT_DGELU_BGRAD: return HIPBLASLT_EPILOGUE_DGELU_BGRAD;
    case DL_LT_GELU_BIAS: return HIPBLASLT_EPILOGUE_GELU_BIAS;
    default: return HIPBLASLT_EPILOGUE_DEFAULT;
  }
}

DevState* dev_state(int dev) {
  DevState& s = g_dev[dev];
  if (!s.handle) {
    if (hipblasLtCreate(&s.handle) != HIPBLAS_STATUS_SUCCESS) return nullptr;
    if (hipMalloc(&s.workspace, kWorkspace) != hipSuccess) return nullptr;
    s.ws_size = kWorkspace;
  }
  return &s;
}

bool set_ptrs(hipblasLtMatmulDesc_t desc, const DlLtArgs& a) {
  if (a.epilogue != DL_LT_NONE) {
    const void* bias = a.bias;
    if (hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)) !=
        HIPBLAS_STATUS_SUCCESS)
      return false;
  }
  if (a.epilogue == DL_LT_GELU_AUX_BIAS || a.epilogue == DL_LT_DGELU_BGRAD) {
    void* aux = a.aux;
    if (hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux)) !=
        HIPBLAS_STATUS_SUCCESS)
      return false;
  }
  return true;
}

bool build_plan(Plan& p, const DlLtArgs& a, DevState* s, hipStream_t st, const std::string& kstr) {
  const hipDataType in_t = a.in_f32 ? HIP_R_32F : HIP_R_16BF;
  const hipDataType d_t = a.d_f32 ? HIP_R_32F : HIP_R_16BF;
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return false;
  // hip "A" = our B, hip "B" = our A
  const hipblasOperation_t opA = a.transB ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  const hipblasOperation_t opB = a.transA ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof(opA));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof(opB));
  const hipblasLtEpilogue_t epi = to_lt(a.epilogue);
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
  if (a.epilogue != DL_LT_NONE) {
    const int32_t bt = a.bias_f32 ? HIP_R_32F : HIP_R_16BF;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
  }
  if (a.epilogue == DL_LT_GELU_AUX_BIAS || a.epilogue == DL_LT_DGELU_BGRAD) {
    const int64_t ldaux = a.ldaux;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ldaux, sizeof(ldaux));
    const int32_t at = HIP_R_16BF;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at));
  }
  // stored (pre-op) shapes, column-major
  const uint64_t a_rows = a.transB ? a.K : a.N, a_cols = a.transB ? a.N : a.K;
  const uint64_t b_rows = a.transA ? a.M : a.K, b_cols = a.transA ? a.K : a.M;
  if (hipblasLtMatrixLayoutCreate(&p.la, in_t, a_rows, a_cols, a.ldb) != HIPBLAS_STATUS_SUCCESS) return false;
  if (hipblasLtMatrixLayoutCreate(&p.lb, in_t, b_rows, b_cols, a.lda) != HIPBLAS_STATUS_SUCCESS) return false;
  if (hipblasLtMatrixLayoutCreate(&p.ld, d_t, a.N, a.M, a.ldd) != HIPBLAS_STATUS_SUCCESS) return false;
  if (a.batch > 1) {
    const int32_t bc = a.batch;
    const int64_t sa = a.strideB, sb = a.strideA, sd = a.strideD;  // hip "A" = our B, hip "B" = our A
    hipblasLtMatrixLayoutSetAttribute(p.la, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc));
    hipblasLtMatrixLayoutSetAttribute(p.la, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &sa, sizeof(sa));
    hipblasLtMatrixLayoutSetAttribute(p.lb, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc));
    hipblasLtMatrixLayoutSetAttribute(p.lb, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &sb, sizeof(sb));
    hipblasLtMatrixLayoutSetAttribute(p.ld, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc));
    hipblasLtMatrixLayoutSetAttribute(p.ld, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &sd, sizeof(sd));
  }
  if (!set_ptrs(p.desc, a)) return false;

  const float alpha_one = 1.f;
  const bool dbg = std::getenv("DEDLOC_LT_DEBUG") != nullptr;
  {  // 1. tuning database
    auto it = tuning_db().find(kstr);
    if (it != tuning_db().end()) {
      std::vector<int> idx{it->second};
      std::vector<hipblasLtMatmulHeuristicResult_t> r;
      size_t need = 0;
      if (hipblaslt_ext::getAlgosFromIndex(s->handle, idx, r) == HIPBLAS_STATUS_SUCCESS && !r.empty() &&
          hipblaslt_ext::matmulIsAlgoSupported(s->handle, p.desc, &alpha_one, p.la, p.lb, &a.beta, p.ld, p.ld,
                                               r[0].algo, need) == HIPBLAS_STATUS_SUCCESS &&
          need <= s->ws_size) {
        p.algo = r[0].algo;
        p.ws = need;
        p.ok = true;
        if (dbg) std::fprintf(stderr, "[lt] plan %s: tuning database solution %d\n", kstr.c_str(), it->second);
        return true;
      }
      if (dbg) std::fprintf(stderr, "[lt] plan %s: database solution %d not usable, retuning\n", kstr.c_str(), it->second);
    }
  }

  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  uint64_t wsz = s->ws_size;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz, sizeof(wsz));
  const char* tune_env = std::getenv("DEDLOC_LT_TUNE");
  // candidates timed per shape (once, at the first call): DEDLOC_LT_TUNE=0 takes the heuristic's
  // first choice, =N times the top N (default 64: the top 16 missed faster kernels on some shapes)
  const int want = !tune_env ? 64 : std::max(1, std::atoi(tune_env));
  std::vector<hipblasLtMatmulHeuristicResult_t> res(want);
  int n = 0;
  const hipblasStatus_t hs =
      hipblasLtMatmulAlgoGetHeuristic(s->handle, p.desc, p.la, p.lb, p.ld, p.ld, pref, want, res.data(), &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (std::getenv("DEDLOC_LT_DEBUG"))
    std::fprintf(stderr, "[lt] plan ta=%d tb=%d M=%d N=%d K=%d epi=%d d_f32=%d beta=%g: heuristic status %d, %d algos\n",
                 a.transA, a.transB, a.M, a.N, a.K, a.epilogue, a.d_f32, a.beta, (int)hs, n);
  if (hs != HIPBLAS_STATUS_SUCCESS || n <= 0) return false;

  // 2. autotune over candidate algos: the heuristic list, plus every supported solution of the
  // problem type for large bf16-output problems
  std::vector<hipblasLtMatmulAlgo_t> cand;
  std::vector<size_t> cand_ws;
  for (int i = 0; i < n; ++i)
    if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= s->ws_size) {
      cand.push_back(res[i].algo);
      cand_ws.push_back(res[i].workspaceSize);
    }
  if (cand.empty()) return false;
  const double flops = 2.0 * a.M * a.N * a.K * std::max(1, a.batch);
  const char* ex_env = std::getenv("DEDLOC_LT_EXHAUSTIVE");
  static const double min_flops = [] {  // DEDLOC_LT_EXHAUSTIVE_MIN_GFLOP: problem-size floor (default 200)
    const char* e = std::getenv("DEDLOC_LT_EXHAUSTIVE_MIN_GFLOP");
    return (e ? std::atof(e) : 200.0) * 1e9;
  }();
  const bool exhaustive = (ex_env && ex_env[0] == '1') && !a.d_f32 && !a.in_f32 && flops >= min_flops &&
                          a.epilogue != DL_LT_GELU_AUX_BIAS && a.epilogue != DL_LT_DGELU_BGRAD;
  int best = 0;
  if (cand.size() > 1 || exhaustive) {
    // time every candidate into a scratch output (inputs are read-only)
    const size_t d_bytes = (size_t)(a.batch > 1 ? a.strideD * a.batch : a.ldd * a.M) * (a.d_f32 ? 4 : 2);
    const size_t aux_bytes = (a.aux ? (size_t)a.ldaux * a.M * 2 : 0);
    const size_t bias_bytes = (size_t)a.N * 4;
    const size_t need = d_bytes + aux_bytes + bias_bytes + 256;
    if (s->scratch_size < need) {
      if (s->scratch) hipFree(s->scratch);
      s->scratch = nullptr;
      s->scratch_size = 0;
      if (hipMalloc(&s->scratch, need) == hipSuccess) s->scratch_size = need;
    }
    if (s->scratch) {
      char* base = static_cast<char*>(s->scratch);
      DlLtArgs t = a;
      t.D = base;
      if (a.epilogue == DL_LT_GELU_AUX_BIAS) t.aux = base + d_bytes;  // aux is an output there
      if (a.epilogue == DL_LT_DGELU_BGRAD) t.bias = base + d_bytes + aux_bytes;  // bias-grad output
      set_ptrs(p.desc, t);
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      const float one = 1.f;
      auto run = [&](hipblasLtMatmulAlgo_t& algo) {
        return hipblasLtMatmul(s->handle, p.desc, &one, a.B, p.la, a.A, p.lb, &a.beta, t.D, p.ld, t.D, p.ld, &algo,
                               s->workspace, s->ws_size, st);
      };
      auto time_ms = [&](hipblasLtMatmulAlgo_t& algo, int reps) {
        hipEventRecord(e0, st);
        for (int r = 0; r < reps; ++r) run(algo);
        hipEventRecord(e1, st);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        return ms / reps;
      };
      // round 1: every heuristic candidate, 3 runs
      std::vector<std::pair<float, int>> timed;
      for (size_t i = 0; i < cand.size(); ++i) {
        if (run(cand[i]) != HIPBLAS_STATUS_SUCCESS) continue;
        timed.emplace_back(time_ms(cand[i], 3), (int)i);
      }
      std::sort(timed.begin(), timed.end());
      std::vector<std::pair<float, int>> finalists(timed.begin(), timed.begin() + std::min<size_t>(4, timed.size()));
      if (exhaustive) {  // every supported solution once (after an untimed first launch)
        std::vector<hipblasLtMatmulHeuristicResult_t> all;
        const hipDataType io = HIP_R_16BF;
        const hipDataType dt = a.d_f32 ? HIP_R_32F : HIP_R_16BF;
        const hipblasOperation_t opA = a.transB ? HIPBLAS_OP_T : HIPBLAS_OP_N;
        const hipblasOperation_t opB = a.transA ? HIPBLAS_OP_T : HIPBLAS_OP_N;
        std::vector<std::pair<float, int>> ex;
        const size_t first = cand.size();
        if (hipblaslt_ext::getAllAlgos(s->handle, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, opA, opB, io, io, dt, dt,
                                       HIPBLAS_COMPUTE_32F, all) == HIPBLAS_STATUS_SUCCESS) {
          for (auto& r : all) {
            size_t w = 0;
            if (hipblaslt_ext::matmulIsAlgoSupported(s->handle, p.desc, &one, p.la, p.lb, &a.beta, p.ld, p.ld, r.algo,
                                                     w) != HIPBLAS_STATUS_SUCCESS ||
                w > s->ws_size)
              continue;
            if (run(r.algo) != HIPBLAS_STATUS_SUCCESS) continue;
            cand.push_back(r.algo);
            cand_ws.push_back(w);
            ex.emplace_back(time_ms(r.algo, 1), (int)(cand.size() - 1));
          }
        }
        std::sort(ex.begin(), ex.end());
        for (size_t k = 0; k < ex.size() && k < 4; ++k) finalists.push_back(ex[k]);
        std::fprintf(stderr, "[lt] exhaustive tune M=%d N=%d K=%d batch=%d: %zu heuristic + %zu supported solutions\n",
                     a.M, a.N, a.K, a.batch, first, cand.size() - first);
      }
      // round 2: the finalists again with 10 runs each, so a single noisy round-1 timing (clock
      // ramp, a neighbour's traffic) cannot pick the plan
      float best_ms = 1e30f;
      for (auto& f : finalists) {
        const float ms = time_ms(cand[f.second], 10);
        if (ms < best_ms) {
          best_ms = ms;
          best = f.second;
        }
      }
      if (exhaustive || dbg)
        std::fprintf(stderr, "[lt] plan M=%d N=%d K=%d: %.1f us (%s)\n", a.M, a.N, a.K, best_ms * 1e3,
                     best >= n ? "exhaustive" : "heuristic");
      hipEventDestroy(e0);
      hipEventDestroy(e1);
      set_ptrs(p.desc, a);
    }
  }
  p.algo = cand[best];
  p.ws = cand_ws[best];
  p.ok = true;
  if (exhaustive) record_tuning(kstr, hipblaslt_ext::getIndexFromAlgo(p.algo));
  return true;
}

}  // namespace

int dl_lt_matmul(const DlLtArgs& a, hipStream_t st) {
  int dev = 0;
  hipGetDevice(&dev);
  Key k{a.transA, a.transB, a.M, a.N, a.K, a.lda, a.ldb, a.ldd, a.ldaux, a.d_f32, a.in_f32, a.beta != 0.f,
        a.epilogue, a.bias_f32, dev, a.batch, a.strideA, a.strideB, a.strideD};
  std::lock_guard<std::mutex> lock(g_mu);
  DevState* s = dev_state(dev);
  if (!s) return -2;
  auto it = g_plans.find(k);
  if (it == g_plans.end()) {
    Plan p;
    if (!build_plan(p, a, s, st, key_str(k))) p.ok = false;
    it = g_plans.emplace(k, p).first;
  }
  Plan& p = it->second;
  if (!p.ok) return -1;
  if (!set_ptrs(p.desc, a)) return -3;
  const float one = 1.f;
  const float beta = a.beta;
  const void* C = a.C ? a.C : a.D;
  const hipblasStatus_t r = hipblasLtMatmul(s->handle, p.desc, &one, a.B, p.la, a.A, p.lb, &beta, C, p.ld, a.D,
                                            p.ld, &p.algo, s->workspace, s->ws_size, st);
  return r == HIPBLAS_STATUS_SUCCESS ? 0 : -4;
}

int dl_lt_plan_count() {
  std::lock_guard<std::mutex> lock(g_mu);
  return (int)g_plans.size();
}

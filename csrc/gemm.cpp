// Autotuned hipBLASLt GEMMs for the transformer's projections.
//
//   st_amd::gemm_(out, a, b, trans_a, trans_b, alpha, beta)
//     out[M,N] = alpha * op(a) @ op(b) + beta * out      (row-major views)
//     a, b bf16; out bf16 or fp32 (fp32 + beta=1 = the weight-gradient GEMM
//     accumulating straight into the fp32 main_grad arena).
//
// Why not torch.mm: PyTorch asks hipBLASLt for ONE heuristic solution per
// shape; on gfx950 the fp32-output weight-gradient GEMM lands on a 256x256x32
// macro-tile that runs ~1.0 PF/s while deeper-K solutions exist.  Here the
// first call of every (shape, layout, dtype, beta) key times the top
// heuristic candidates (ST_GEMM_TUNE_CANDIDATES, default 24) on scratch
// outputs and caches the fastest -- an in-process autotuner in the spirit of
// TunableOp but covering the mixed-precision epilogue too.  Candidates are run
// on SCRATCH C/D buffers so tuning never perturbs the accumulating output.
//
// hipBLASLt is column-major: a row-major [M,N] output is a column-major
// [N,M] matrix, so D^T = op(b)^T op(a)^T is issued with the operands swapped.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

#define ST_BLT_CHECK(expr)                                                              \
  do {                                                                                  \
    hipblasStatus_t _s = (expr);                                                        \
    TORCH_CHECK(_s == HIPBLAS_STATUS_SUCCESS, "hipBLASLt call failed (", (int)_s, "): " #expr); \
  } while (0)

struct Key {
  int64_t m, n, k, lda, ldb, ldc;
  int opa, opb, td, beta_nz, dev;
  bool operator==(const Key& o) const {
    return m == o.m && n == o.n && k == o.k && lda == o.lda && ldb == o.ldb && ldc == o.ldc &&
           opa == o.opa && opb == o.opb && td == o.td && beta_nz == o.beta_nz && dev == o.dev;
  }
};
struct KeyHash {
  size_t operator()(const Key& x) const {
    size_t h = 1469598103934665603ull;
    for (int64_t v : {x.m, x.n, x.k, x.lda, x.ldb, x.ldc, (int64_t)x.opa, (int64_t)x.opb, (int64_t)x.td,
                      (int64_t)x.beta_nz, (int64_t)x.dev})
      h = (h ^ (size_t)v) * 1099511628211ull;
    return h;
  }
};

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
  float best_ms = 0.f;
  int n_candidates = 0;
};

std::mutex g_mu;
std::unordered_map<Key, Plan, KeyHash> g_plans;
hipblasLtHandle_t g_handles[64] = {};
constexpr size_t kMaxWorkspace = 128ull << 20;

hipblasLtHandle_t handle_for(int dev) {
  if (!g_handles[dev]) ST_BLT_CHECK(hipblasLtCreate(&g_handles[dev]));
  return g_handles[dev];
}

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v ? std::atoi(v) : dflt;
}

// workspace from the caching allocator, kept per device
at::Tensor& workspace(const at::Device& d) {
  static at::Tensor ws[64];
  auto& t = ws[d.index()];
  if (!t.defined()) t = at::empty({(int64_t)kMaxWorkspace}, at::TensorOptions().dtype(at::kByte).device(d));
  return t;
}

Plan make_plan(const Key& key, hipDataType td, const at::Tensor& a, const at::Tensor& b, at::Tensor& out,
               float alpha, float beta, hipStream_t st) {
  Plan p;
  auto h = handle_for(key.dev);
  ST_BLT_CHECK(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t opa = (hipblasOperation_t)key.opa, opb = (hipblasOperation_t)key.opb;
  ST_BLT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)));
  ST_BLT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)));
  // column-major problem: D[m, n] = opA(A)[m, k] opB(B)[k, n]
  const int64_t a_rows = opa == HIPBLAS_OP_N ? key.m : key.k, a_cols = opa == HIPBLAS_OP_N ? key.k : key.m;
  const int64_t b_rows = opb == HIPBLAS_OP_N ? key.k : key.n, b_cols = opb == HIPBLAS_OP_N ? key.n : key.k;
  ST_BLT_CHECK(hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, a_rows, a_cols, key.lda));
  ST_BLT_CHECK(hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, b_rows, b_cols, key.ldb));
  ST_BLT_CHECK(hipblasLtMatrixLayoutCreate(&p.lc, td, key.m, key.n, key.ldc));

  hipblasLtMatmulPreference_t pref;
  ST_BLT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t wsz = kMaxWorkspace;
  ST_BLT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz,
                                                     sizeof(wsz)));
  const int want = std::max(1, env_int("ST_GEMM_TUNE_CANDIDATES", 24));
  std::vector<hipblasLtMatmulHeuristicResult_t> res(want);
  int got = 0;
  ST_BLT_CHECK(hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.la, p.lb, p.lc, p.lc, pref, want, res.data(), &got));
  hipblasLtMatmulPreferenceDestroy(pref);
  TORCH_CHECK(got > 0, "hipBLASLt: no solution for GEMM m=", key.m, " n=", key.n, " k=", key.k);
  p.algo = res[0].algo;
  p.ws = res[0].workspaceSize;
  if (env_int("ST_GEMM_TUNE_ALL", 0)) {  // exhaustive: every solution of this problem type
    std::vector<hipblasLtMatmulHeuristicResult_t> all;
    if (hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, opa, opb, HIP_R_16BF, HIP_R_16BF,
                                   td, td, HIPBLAS_COMPUTE_32F, all) == HIPBLAS_STATUS_SUCCESS) {
      res.clear();
      for (auto& r : all) {
        size_t ws = 0;
        if (hipblaslt_ext::matmulIsAlgoSupported(h, p.desc, &alpha, p.la, p.lb, &beta, p.lc, p.lc, r.algo, ws) ==
                HIPBLAS_STATUS_SUCCESS &&
            ws <= kMaxWorkspace) {
          r.workspaceSize = ws;
          r.state = HIPBLAS_STATUS_SUCCESS;
          res.push_back(r);
        }
      }
      got = (int)res.size();
    }
  }
  p.n_candidates = got;
  if (got == 1 || env_int("ST_GEMM_TUNE", 1) == 0) return p;

  // time candidates on scratch outputs (beta != 0 reads C: scratch C = D)
  auto scratch = at::empty_like(out);
  void* wsp = workspace(out.device()).data_ptr();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = std::max(1, env_int("ST_GEMM_TUNE_REPS", 3));
  float best = 1e30f;
  for (int i = 0; i < got; ++i) {
    if (res[i].state != HIPBLAS_STATUS_SUCCESS || res[i].workspaceSize > kMaxWorkspace) continue;
    auto run = [&]() {
      return hipblasLtMatmul(h, p.desc, &alpha, b.data_ptr(), p.la, a.data_ptr(), p.lb, &beta,
                             scratch.data_ptr(), p.lc, scratch.data_ptr(), p.lc, &res[i].algo, wsp,
                             res[i].workspaceSize, st);
    };
    if (run() != HIPBLAS_STATUS_SUCCESS) continue;  // warm-up (and support check)
    hipEventRecord(e0, st);
    for (int r = 0; r < reps; ++r) run();
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) {
      best = ms;
      p.algo = res[i].algo;
      p.ws = res[i].workspaceSize;
    }
  }
  p.best_ms = best / reps;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return p;
}

void check_operand(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 2, "gemm: ", name,
              " must be a 2-D bf16 GPU tensor");
  TORCH_CHECK(t.stride(1) == 1 && t.stride(0) >= t.size(1), "gemm: ", name, " rows must be contiguous");
}

// out[M,N] = alpha * op(a) @ op(b) + beta * out
void gemm_(at::Tensor out, const at::Tensor& a, const at::Tensor& b, bool trans_a, bool trans_b, double alpha,
           double beta) {
  check_operand(a, "a");
  check_operand(b, "b");
  TORCH_CHECK(out.is_cuda() && out.dim() == 2 && out.stride(1) == 1 && out.stride(0) >= out.size(1),
              "gemm: out must be a row-contiguous 2-D GPU tensor");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat, "gemm: out bf16 or fp32");
  TORCH_CHECK(a.device() == out.device() && b.device() == out.device(), "gemm: operands on different devices");
  const int64_t M = out.size(0), N = out.size(1);
  const int64_t K = trans_a ? a.size(0) : a.size(1);
  TORCH_CHECK((trans_a ? a.size(1) : a.size(0)) == M, "gemm: op(a) rows != out rows");
  TORCH_CHECK((trans_b ? b.size(0) : b.size(1)) == N, "gemm: op(b) cols != out cols");
  TORCH_CHECK((trans_b ? b.size(1) : b.size(0)) == K, "gemm: inner dimensions differ");
  if (M == 0 || N == 0) return;
  c10::hip::HIPGuardMasqueradingAsCUDA g(out.device());
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();
  if (K == 0) {
    if (beta == 0.0) out.zero_();
    else if (beta != 1.0) out.mul_(beta);
    return;
  }
  // column-major view: D^T[N,M] = op(b)^T [N,K] x op(a)^T [K,M]
  Key key;
  key.m = N;
  key.n = M;
  key.k = K;
  key.opa = trans_b ? HIPBLAS_OP_T : HIPBLAS_OP_N;  // b row-major [K,N] == col-major [N,K]
  key.opb = trans_a ? HIPBLAS_OP_T : HIPBLAS_OP_N;  // a row-major [M,K] == col-major [K,M]
  key.lda = b.stride(0);
  key.ldb = a.stride(0);
  key.ldc = out.stride(0);
  key.td = out.scalar_type() == at::kFloat ? 1 : 0;
  key.beta_nz = beta != 0.0;
  key.dev = out.device().index();
  const hipDataType td = key.td ? HIP_R_32F : HIP_R_16BF;
  const float fa = (float)alpha, fb = (float)beta;
  Plan* plan;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_plans.find(key);
    if (it == g_plans.end()) it = g_plans.emplace(key, make_plan(key, td, a, b, out, fa, fb, st)).first;
    plan = &it->second;
  }
  void* wsp = plan->ws ? workspace(out.device()).data_ptr() : nullptr;
  ST_BLT_CHECK(hipblasLtMatmul(handle_for(key.dev), plan->desc, &fa, b.data_ptr(), plan->la, a.data_ptr(),
                               plan->lb, &fb, out.data_ptr(), plan->lc, out.data_ptr(), plan->lc, &plan->algo,
                               wsp, plan->ws, st));
}

at::Tensor gemm(const at::Tensor& a, const at::Tensor& b, bool trans_a, bool trans_b) {
  const int64_t M = trans_a ? a.size(1) : a.size(0);
  const int64_t N = trans_b ? b.size(0) : b.size(1);
  auto out = at::empty({M, N}, a.options());
  gemm_(out, a, b, trans_a, trans_b, 1.0, 0.0);
  return out;
}

// (m, n, k, out_is_fp32, beta_nz, best_ms, candidates) of every tuned problem
std::vector<double> gemm_tuning_report() {
  std::lock_guard<std::mutex> lk(g_mu);
  std::vector<double> r;
  for (auto& kv : g_plans) {
    r.insert(r.end(), {(double)kv.first.n, (double)kv.first.m, (double)kv.first.k, (double)kv.first.td,
                       (double)kv.first.beta_nz, (double)kv.second.best_ms, (double)kv.second.n_candidates});
  }
  return r;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(st_amd, m) {
  m.def("gemm_(Tensor(a!) out, Tensor a, Tensor b, bool trans_a, bool trans_b, float alpha, float beta) -> ()");
  m.def("gemm(Tensor a, Tensor b, bool trans_a, bool trans_b) -> Tensor");
  m.def("gemm_tuning_report() -> float[]", &gemm_tuning_report);
}

TORCH_LIBRARY_IMPL(st_amd, CUDA, m) {
  m.impl("gemm_", &gemm_);
  m.impl("gemm", &gemm);
}

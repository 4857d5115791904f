// TORCH_LIBRARY registration of every scaletorch_amd HIP kernel as a
// `torch.ops.st_amd.*` custom op (CUDA dispatch key == HIP on ROCm).
//
// The kernels themselves live in csrc/*.hip behind plain `extern "C"`
// launchers (no torch headers in device code, so they compile in seconds);
// this file only validates shapes/dtypes, allocates outputs through the
// PyTorch caching allocator and launches on the current HIP stream.  Shape
// checks here are the host-side guard required before any hand-written kernel
// touches memory: a kernel is never launched on a shape its grid does not
// cover.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

extern "C" {
int st_rmsnorm_fwd(const void* x, const void* res, const void* w, void* y, void* sum_out,
                   float* rstd, int rows, int h, float eps, hipStream_t st);
int st_rmsnorm_bwd(const void* dy, const void* s, const void* w, const float* rstd,
                   const void* dres, void* ds, float* partial, float* dw_out, int rows, int h,
                   hipStream_t st);
int st_rmsnorm_bwd_nwaves(int rows);
int st_rope_inplace(void* x, const float* cos_t, const float* sin_t, const int64_t* pos, int B,
                    int S, int NH, int D, int64_t sB, int64_t sS, int64_t sH, int pos_offset,
                    int backward, int64_t max_pos, hipStream_t st);
int st_swiglu_fwd(const void* gu, void* out, int64_t N, int64_t I, const int* nvalid, hipStream_t st);
int st_swiglu_bwd(const void* dout, const void* gu, void* dgu, int64_t N, int64_t I, const int* nvalid,
                  hipStream_t st);
int st_adamw_step(float* master, void* m, void* v, int states_bf16, const void* g, int g_is_bf16,
                  void* p, const float* clip, int64_t n, float lr, float b1, float b2, float eps,
                  float wd, float bc1, float bc2_sqrt, uint32_t sr_step, int64_t sr_base, hipStream_t st);
int st_adamw_wt_step(float* master, void* m, void* v, int states_bf16, const void* g, int g_is_bf16,
                     void* p, void* wt, int R, int C, const float* clip, float lr, float b1, float b2,
                     float eps, float wd, float bc1, float bc2_sqrt, uint32_t sr_step, int64_t sr_base, hipStream_t st);
int st_sumsq_partials();
int st_sumsq(const void* g, int g_is_bf16, int64_t n, float* partial, float* out, hipStream_t st);
int st_xent_fwd(const void* logits, int64_t ld, const int64_t* tgt, int64_t N, int V,
                int64_t vocab_start, float* lse, float* tlogit, hipStream_t st);
int st_xent_bwd(const void* logits, int64_t ld, const int64_t* tgt, int64_t N, int V,
                int64_t vocab_start, const float* lse, const float* dloss, void* dlogits,
                int64_t ldd, hipStream_t st);
int st_flash_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int Sq,
                 int Sk, int H, int Hkv, int D, int64_t sqb, int64_t sqs, int64_t sqh,
                 int64_t skb, int64_t sks, int64_t skh, int64_t svb, int64_t svs, int64_t svh,
                 int64_t sob, int64_t sos, int64_t soh, float scale, int causal, int64_t q_offset,
                 int64_t k_offset, hipStream_t st);
int st_flash_bwd_preprocess(const void* o, const void* dout, const float* lse, float* delta, float* nlse2,
                            int B, int S, int H,
                            int D, int64_t sob, int64_t sos, int64_t soh, int64_t sdb, int64_t sds,
                            int64_t sdh, hipStream_t st);
int st_flash_bwd(const void* q, const void* k, const void* v, const void* dout, const float* lse,
                 const float* delta, const float* nlse2, void* dq, void* dk, void* dv, int B, int Sq, int Sk,
                 int H, int Hkv, int D, int64_t sqb, int64_t sqs, int64_t sqh, int64_t skb,
                 int64_t sks, int64_t skh, int64_t svb, int64_t svs, int64_t svh, int64_t sdb,
                 int64_t sds, int64_t sdh, int64_t sdqb, int64_t sdqs, int64_t sdqh, int64_t sdkb,
                 int64_t sdks, int64_t sdkh, float scale, int causal, int64_t q_offset,
                 int64_t k_offset, float* part, void* dsw, int phases, hipStream_t st);
int64_t st_flash_bwd_part_elems(int B, int Sq, int Sk, int H, int Hkv, int D, int causal);
int64_t st_flash_bwd_ds_elems(int B, int Sq, int Sk, int H, int D, int causal, int64_t q_offset,
                              int64_t k_offset);
int st_wgrad_gemm(const void* A, int64_t lda, const void* B, int64_t ldb, float* C, int64_t ldc, int M,
                  int N, int T, int beta, int variant, float* ws, hipStream_t st);
int64_t st_wgrad_ws_elems(int M, int N, int T, int variant);
int st_wgrad_grouped(const void* A, int64_t lda, const void* B, int64_t ldb, float* C, int64_t ldc, int64_t strideC,
                     int M, int N, int G, const int* offs, int T_total, int beta, hipStream_t st);
int64_t st_grouped_gemm_slots(int T, int G);
int st_gemm4w(const void* X, int64_t ldx, const void* W, int64_t ldw, int64_t strideW, void* Y, int64_t ldy,
              const int* offs, const int* tile_end, int T, int G, int N, int K, hipStream_t st);
int st_gemm4w_swiglu(const void* X, int64_t ldx, const void* W, int64_t ldw, void* GU, int64_t ldgu, void* H,
                     int64_t ldh, int T, int I, int K, hipStream_t st);
int st_gemm4w_swiglu_grouped(const void* X, int64_t ldx, const void* W, int64_t ldw, int64_t strideW, void* GU,
                             int64_t ldgu, void* H, int64_t ldh, const int* offs, const int* tile_end, int T, int G,
                             int I, int K, hipStream_t st);
int st_grouped_gemm_bm();
int st_grouped_gemm(const void* X, int64_t ldx, const void* W, int64_t ldw, int64_t strideW, void* Y, int64_t ldy,
                    const int* offs, const int* tile_end, int T, int G, int N, int K, int wn, hipStream_t st);
int st_grouped_gemm_ex(const void* X, int64_t ldx, const void* W, int64_t ldw, int64_t strideW, void* Y,
                       int64_t ldy, const int* offs, const int* tile_end, int T, int G, int N, int K, int wn,
                       int epi, void* Y2, int64_t ld2, hipStream_t st);
int st_xgmi_header_bytes();
int st_xgmi_max_ranks();
int64_t st_xgmi_create(int rank, int world, int64_t cap, int64_t epoch_base);
int st_xgmi_handle(int64_t id, void* out64);
int st_xgmi_open(int64_t id, int r, const void* handle64);
int st_xgmi_set_peer(int64_t id, int r, int64_t peer_id);
int st_xgmi_all_reduce(int64_t id, const void* in, void* out, int64_t n, int dtype, int mode, int blocks,
                       hipStream_t st);
int st_xgmi_pair(int64_t id, const void* in, void* out, int64_t n, int dtype, int mode, int partner, int blocks,
                 hipStream_t st);
int st_xgmi_collective_sim(const int64_t* ids, const void* const* ins, void* const* outs, const int* partners,
                           int world, int64_t n, int dtype, int mode, int blocks, hipStream_t st);
int st_xgmi_all_reduce_sim(const int64_t* ids, const void* const* ins, void* const* outs, int world, int64_t n,
                           int dtype, int mode, int blocks, hipStream_t st);
int st_xgmi_error(int64_t id);
int st_xgmi_ep_exchange(int64_t id, const void* in, void* out, const int* M, int E, int El, int64_t row_elems,
                        int64_t in_rows, int64_t out_rows, int64_t area_rows_needed, int dtype, int dir, int blocks,
                        hipStream_t st);
int st_xgmi_ep_exchange_sim(const int64_t* ids, const void* const* ins, void* const* outs, const int* M, int world,
                            int E, int El, int64_t row_elems, int64_t in_rows, int64_t out_rows,
                            int64_t area_rows_needed, int dtype, int dir, int blocks, hipStream_t st);
int st_xgmi_set_timeout(int64_t id, double seconds);
int st_xgmi_world(int64_t id);
int st_xgmi_destroy(int64_t id);
int st_qknorm_rope_bwd_blocks();
int st_qknorm_rope_fwd(void* qkv, void* xsave, float* rstd, const void* wq, const void* wk, const float* cos_t,
                       const float* sin_t, const int64_t* pos, int64_t N, int S, int H, int Hkv, int D, float eps,
                       int64_t max_pos, hipStream_t st);
int st_qknorm_rope_bwd(void* dqkv, const void* xsave, const float* rstd, const void* wq, const void* wk,
                       const float* cos_t, const float* sin_t, const int64_t* pos, int64_t N, int S, int H, int Hkv,
                       int D, int64_t max_pos, float* partial, float* dw_out, hipStream_t st);
int st_transpose_bf16(const void* src, void* dst, int R, int C, int64_t lds_src, int64_t lds_dst, hipStream_t st);
int st_embedding_bwd(const int64_t* sorted_ids, const int64_t* order, const void* dy, int64_t ldd, float* grad,
                     int64_t ldg, float* partial, int T, int H, int64_t V, hipStream_t st);
int64_t st_embedding_bwd_partial_floats(int T, int H);
int st_lse_merge(float* out, float* lse, const void* bout, const float* blse, int B, int S, int H,
                 int D, int64_t sbb, int64_t sbs, int64_t sbh, hipStream_t st);
}

namespace {

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define ST_CHECK_RC(rc, name) \
  TORCH_CHECK((rc) == 0, "st_amd::" name " launch failed with code ", (rc))

void check_bf16_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16, got ", t.scalar_type());
}

// Every auxiliary tensor a kernel dereferences must live on the same GPU as
// the primary operand: a host pointer handed to a kernel is an illegal-address
// fault on the device, so it is rejected here instead.
void check_same_gpu(const at::Tensor& t, const at::Tensor& ref, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.device() == ref.device(), name, " must be on ", ref.device(), ", got ",
              t.device());
}

// ---------------------------------------------------------------- RMSNorm
std::vector<at::Tensor> rmsnorm_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& res,
                                    const at::Tensor& w, double eps) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "weight");
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous(), "rmsnorm: x and weight must be contiguous");
  const int64_t h = x.size(-1);
  TORCH_CHECK(w.numel() == h, "rmsnorm: weight size ", w.numel(), " != hidden ", h);
  TORCH_CHECK(h % 8 == 0 && h <= 8192, "rmsnorm: hidden must be a multiple of 8 and <= 8192");
  const int64_t rows = x.numel() / h;
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto y = at::empty_like(x);
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  at::Tensor s;
  const void* rp = nullptr;
  if (res.has_value() && res->defined()) {
    check_bf16_cuda(*res, "residual");
    TORCH_CHECK(res->is_contiguous() && res->sizes() == x.sizes(), "rmsnorm: residual shape");
    s = at::empty_like(x);
    rp = res->data_ptr();
  } else {
    s = at::empty({0}, x.options());
  }
  int rc = st_rmsnorm_fwd(x.data_ptr(), rp, w.data_ptr(), y.data_ptr(),
                          rp ? s.data_ptr() : nullptr, rstd.data_ptr<float>(), (int)rows, (int)h,
                          (float)eps, cur_stream());
  ST_CHECK_RC(rc, "rmsnorm_fwd");
  return {y, rstd, s};
}

at::Tensor rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& s, const at::Tensor& w,
                       const at::Tensor& rstd, const c10::optional<at::Tensor>& dres,
                       at::Tensor dw_accum) {
  check_bf16_cuda(dy, "dy");
  check_bf16_cuda(s, "s");
  check_bf16_cuda(w, "weight");
  TORCH_CHECK(dy.is_contiguous() && s.is_contiguous() && dy.sizes() == s.sizes(), "rmsnorm_bwd: shapes");
  const int64_t h = s.size(-1);
  const int64_t rows = s.numel() / h;
  TORCH_CHECK(rstd.numel() == rows && rstd.scalar_type() == at::kFloat, "rmsnorm_bwd: rstd");
  TORCH_CHECK(dw_accum.numel() == h && dw_accum.scalar_type() == at::kFloat &&
                  dw_accum.is_contiguous(), "rmsnorm_bwd: dw_accum must be fp32 [h]");
  check_same_gpu(dy, s, "dy");
  check_same_gpu(w, s, "weight");
  check_same_gpu(rstd, s, "rstd");
  check_same_gpu(dw_accum, s, "dw_accum");
  c10::hip::HIPGuardMasqueradingAsCUDA g(s.device());
  const void* dp = nullptr;
  if (dres.has_value() && dres->defined()) {
    check_bf16_cuda(*dres, "dres");
    TORCH_CHECK(dres->is_contiguous() && dres->sizes() == s.sizes(), "rmsnorm_bwd: dres shape");
    dp = dres->data_ptr();
  }
  auto ds = at::empty_like(s);
  const int nw = st_rmsnorm_bwd_nwaves((int)rows);
  auto partial = at::empty({(int64_t)nw * h}, s.options().dtype(at::kFloat));
  int rc = st_rmsnorm_bwd(dy.data_ptr(), s.data_ptr(), w.data_ptr(), rstd.data_ptr<float>(), dp,
                          ds.data_ptr(), partial.data_ptr<float>(), dw_accum.data_ptr<float>(),
                          (int)rows, (int)h, cur_stream());
  ST_CHECK_RC(rc, "rmsnorm_bwd");
  return ds;
}

// ---------------------------------------------------------------- RoPE
void rope_(at::Tensor x, const at::Tensor& cos_t, const at::Tensor& sin_t,
           const c10::optional<at::Tensor>& pos, int64_t pos_offset, bool backward) {
  check_bf16_cuda(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.stride(3) == 1, "rope: x must be [B,S,NH,D] with contiguous D");
  const int64_t B = x.size(0), S = x.size(1), NH = x.size(2), D = x.size(3);
  TORCH_CHECK(D % 16 == 0, "rope: head_dim must be a multiple of 16");
  TORCH_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat &&
                  cos_t.is_contiguous() && sin_t.is_contiguous() && cos_t.size(-1) == D / 2,
              "rope: tables must be fp32 contiguous [max_pos, D/2]");
  const int64_t maxpos = cos_t.size(0);
  check_same_gpu(cos_t, x, "cos table");
  check_same_gpu(sin_t, x, "sin table");
  TORCH_CHECK(sin_t.sizes() == cos_t.sizes(), "rope: cos/sin tables differ in shape");
  const int64_t* pp = nullptr;
  if (pos.has_value() && pos->defined()) {
    TORCH_CHECK(pos->scalar_type() == at::kLong && pos->is_contiguous() && pos->numel() == B * S,
                "rope: position_ids must be int64 [B,S]");
    check_same_gpu(*pos, x, "position_ids");
    pp = pos->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(S + pos_offset <= maxpos && pos_offset >= 0, "rope: positions exceed table");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  int rc = st_rope_inplace(x.data_ptr(), cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), pp,
                           (int)B, (int)S, (int)NH, (int)D, x.stride(0), x.stride(1), x.stride(2),
                           (int)pos_offset, backward ? 1 : 0, maxpos, cur_stream());
  ST_CHECK_RC(rc, "rope_");
}

// ---------------------------------------------------------------- SwiGLU
// nvalid (optional int32 device scalar view, e.g. offs[-1:]): rows at or past it are skipped
static const int* nvalid_ptr(const c10::optional<at::Tensor>& nv, const at::Tensor& ref) {
  if (!nv.has_value() || !nv->defined()) return nullptr;
  TORCH_CHECK(nv->scalar_type() == at::kInt && nv->numel() >= 1 && nv->is_cuda() && nv->device() == ref.device(),
              "swiglu: nvalid must be an int32 tensor on the same GPU");
  return nv->data_ptr<int>();
}

at::Tensor swiglu_fwd(const at::Tensor& gu, const c10::optional<at::Tensor>& nvalid) {
  check_bf16_cuda(gu, "gate_up");
  TORCH_CHECK(gu.is_contiguous() && gu.size(-1) % 16 == 0, "swiglu: [.., 2I] contiguous, I%8==0");
  const int64_t I = gu.size(-1) / 2, N = gu.numel() / gu.size(-1);
  auto sizes = gu.sizes().vec();
  sizes.back() = I;
  c10::hip::HIPGuardMasqueradingAsCUDA g(gu.device());
  auto out = at::empty(sizes, gu.options());
  int rc = st_swiglu_fwd(gu.data_ptr(), out.data_ptr(), N, I, nvalid_ptr(nvalid, gu), cur_stream());
  ST_CHECK_RC(rc, "swiglu_fwd");
  return out;
}

at::Tensor swiglu_bwd(const at::Tensor& dout, const at::Tensor& gu, const c10::optional<at::Tensor>& nvalid) {
  check_bf16_cuda(dout, "dout");
  check_bf16_cuda(gu, "gate_up");
  TORCH_CHECK(gu.is_contiguous() && dout.is_contiguous(), "swiglu_bwd: contiguous inputs");
  const int64_t I = gu.size(-1) / 2, N = gu.numel() / gu.size(-1);
  TORCH_CHECK(dout.numel() == N * I, "swiglu_bwd: dout shape");
  c10::hip::HIPGuardMasqueradingAsCUDA g(gu.device());
  auto dgu = at::empty_like(gu);
  int rc = st_swiglu_bwd(dout.data_ptr(), gu.data_ptr(), dgu.data_ptr(), N, I, nvalid_ptr(nvalid, gu),
                         cur_stream());
  ST_CHECK_RC(rc, "swiglu_bwd");
  return dgu;
}

// ---------------------------------------------------------------- AdamW / norms
void adamw_step_(at::Tensor master, at::Tensor exp_avg, at::Tensor exp_avg_sq,
                 const at::Tensor& grad, const c10::optional<at::Tensor>& param,
                 const c10::optional<at::Tensor>& clip_coef, double lr, double beta1, double beta2,
                 double eps, double weight_decay, int64_t step, int64_t sr_base) {
  TORCH_CHECK(master.is_cuda() && master.scalar_type() == at::kFloat && master.is_contiguous(),
              "adamw: master must be contiguous fp32 on GPU");
  const int64_t n = master.numel();
  TORCH_CHECK(exp_avg.numel() == n && exp_avg_sq.numel() == n && grad.numel() == n,
              "adamw: arena sizes differ");
  const bool sbf = exp_avg.scalar_type() == at::kBFloat16;
  TORCH_CHECK((exp_avg.scalar_type() == at::kFloat || sbf) && exp_avg_sq.scalar_type() == exp_avg.scalar_type() &&
                  exp_avg.is_contiguous() && exp_avg_sq.is_contiguous() && grad.is_contiguous(),
              "adamw: states must be contiguous fp32 or bf16 (both the same)");
  TORCH_CHECK(grad.scalar_type() == at::kFloat || grad.scalar_type() == at::kBFloat16,
              "adamw: grad must be fp32 or bf16");
  TORCH_CHECK(n % 4 == 0, "adamw: arena length must be a multiple of 4");
  check_same_gpu(exp_avg, master, "exp_avg");
  check_same_gpu(exp_avg_sq, master, "exp_avg_sq");
  check_same_gpu(grad, master, "grad");
  void* pp = nullptr;
  if (param.has_value() && param->defined()) {
    check_bf16_cuda(*param, "param");
    check_same_gpu(*param, master, "param");
    TORCH_CHECK(param->numel() == n && param->is_contiguous(), "adamw: param arena");
    pp = param->data_ptr();
  }
  const float* cp = nullptr;
  if (clip_coef.has_value() && clip_coef->defined()) {
    TORCH_CHECK(clip_coef->scalar_type() == at::kFloat && clip_coef->numel() == 1, "adamw: clip");
    check_same_gpu(*clip_coef, master, "clip_coef");
    cp = clip_coef->data_ptr<float>();
  }
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  c10::hip::HIPGuardMasqueradingAsCUDA g(master.device());
  int rc = st_adamw_step(master.data_ptr<float>(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(),
                         sbf ? 1 : 0, grad.data_ptr(),
                         grad.scalar_type() == at::kBFloat16 ? 1 : 0, pp, cp, n, (float)lr,
                         (float)beta1, (float)beta2, (float)eps, (float)weight_decay, (float)bc1,
                         (float)std::sqrt(bc2), (uint32_t)step, sr_base, cur_stream());
  ST_CHECK_RC(rc, "adamw_step_");
}

// AdamW over one 2-D weight's arena run that also writes the updated bf16 weight
// transposed into `wt` [C, R] (param is the [R, C] weight view of the arena)
void adamw_wt_step_(at::Tensor master, at::Tensor exp_avg, at::Tensor exp_avg_sq, const at::Tensor& grad,
                    at::Tensor param, at::Tensor wt, const c10::optional<at::Tensor>& clip_coef, double lr,
                    double beta1, double beta2, double eps, double weight_decay, int64_t step, int64_t sr_base) {
  TORCH_CHECK(param.dim() == 2 && param.is_contiguous(), "adamw_wt: param must be a contiguous 2-D weight");
  check_bf16_cuda(param, "param");
  check_bf16_cuda(wt, "wt");
  const int64_t R = param.size(0), C = param.size(1), n = R * C;
  TORCH_CHECK(wt.dim() == 2 && wt.size(0) == C && wt.size(1) == R && wt.is_contiguous(), "adamw_wt: wt must be [C, R]");
  TORCH_CHECK(R % 64 == 0 && C % 64 == 0 && R <= INT32_MAX && C <= INT32_MAX, "adamw_wt: R, C multiples of 64");
  TORCH_CHECK(master.is_cuda() && master.scalar_type() == at::kFloat && master.is_contiguous() && master.numel() == n,
              "adamw_wt: master must be contiguous fp32 of the weight's size");
  const bool sbf = exp_avg.scalar_type() == at::kBFloat16;
  TORCH_CHECK((exp_avg.scalar_type() == at::kFloat || sbf) && exp_avg_sq.scalar_type() == exp_avg.scalar_type() &&
                  exp_avg.is_contiguous() && exp_avg_sq.is_contiguous() && exp_avg.numel() == n &&
                  exp_avg_sq.numel() == n,
              "adamw_wt: states must be contiguous fp32 or bf16 of the weight's size");
  TORCH_CHECK((grad.scalar_type() == at::kFloat || grad.scalar_type() == at::kBFloat16) && grad.is_contiguous() &&
                  grad.numel() == n,
              "adamw_wt: grad must be contiguous fp32 or bf16 of the weight's size");
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&exp_avg, &exp_avg_sq, &grad, &param, &wt})
    check_same_gpu(*t, master, "adamw_wt operand");
  const float* cp = nullptr;
  if (clip_coef.has_value() && clip_coef->defined()) {
    TORCH_CHECK(clip_coef->scalar_type() == at::kFloat && clip_coef->numel() == 1, "adamw_wt: clip");
    check_same_gpu(*clip_coef, master, "clip_coef");
    cp = clip_coef->data_ptr<float>();
  }
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  c10::hip::HIPGuardMasqueradingAsCUDA g(master.device());
  int rc = st_adamw_wt_step(master.data_ptr<float>(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(), sbf ? 1 : 0,
                            grad.data_ptr(), grad.scalar_type() == at::kBFloat16 ? 1 : 0, param.data_ptr(),
                            wt.data_ptr(), (int)R, (int)C, cp, (float)lr, (float)beta1, (float)beta2, (float)eps,
                            (float)weight_decay, (float)bc1, (float)std::sqrt(bc2), (uint32_t)step, sr_base, cur_stream());
  ST_CHECK_RC(rc, "adamw_wt_step_");
}

// grad[V, H] fp32 += rows of dy[T, H] bf16 grouped by token id; sorted_ids / order from a
// STABLE sort of the ids (deterministic: fixed summation order, no atomics)
void embedding_bwd_(at::Tensor grad, const at::Tensor& dy, const at::Tensor& sorted_ids, const at::Tensor& order) {
  check_bf16_cuda(dy, "dy");
  check_same_gpu(grad, dy, "grad");
  check_same_gpu(sorted_ids, dy, "sorted_ids");
  check_same_gpu(order, dy, "order");
  TORCH_CHECK(grad.scalar_type() == at::kFloat && grad.dim() == 2 && grad.stride(1) == 1, "embedding_bwd_: grad fp32 [V, H]");
  TORCH_CHECK(dy.dim() == 2 && dy.stride(1) == 1 && dy.size(1) == grad.size(1), "embedding_bwd_: dy [T, H]");
  TORCH_CHECK(sorted_ids.scalar_type() == at::kLong && order.scalar_type() == at::kLong && sorted_ids.is_contiguous() &&
                  order.is_contiguous() && sorted_ids.numel() == dy.size(0) && order.numel() == dy.size(0),
              "embedding_bwd_: int64 sorted_ids / order of length T");
  TORCH_CHECK(dy.size(1) % 4 == 0 && dy.stride(0) % 4 == 0 && grad.stride(0) % 4 == 0, "embedding_bwd_: H % 4");
  TORCH_CHECK(dy.size(0) < (1LL << 31) && dy.size(1) < (1LL << 31), "embedding_bwd_: dims");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(dy.device());
  // per-block partial sums of long runs (split across workgroups, reduced in block order)
  at::Tensor partial = at::empty({st_embedding_bwd_partial_floats((int)dy.size(0), (int)dy.size(1))},
                                 dy.options().dtype(at::kFloat));
  int rc = st_embedding_bwd(sorted_ids.data_ptr<int64_t>(), order.data_ptr<int64_t>(), dy.data_ptr(), dy.stride(0),
                            grad.data_ptr<float>(), grad.stride(0), partial.data_ptr<float>(), (int)dy.size(0),
                            (int)dy.size(1), grad.size(0), cur_stream());
  ST_CHECK_RC(rc, "embedding_bwd_");
}

void transpose_(const at::Tensor& src, at::Tensor dst) {
  check_bf16_cuda(src, "src");
  check_bf16_cuda(dst, "dst");
  check_same_gpu(dst, src, "dst");
  TORCH_CHECK(src.dim() == 2 && dst.dim() == 2, "transpose_: 2-D tensors");
  const int64_t R = src.size(0), C = src.size(1);
  TORCH_CHECK(dst.size(0) == C && dst.size(1) == R, "transpose_: dst must be [C, R]");
  TORCH_CHECK(R % 64 == 0 && C % 64 == 0, "transpose_: both dims must be multiples of 64");
  TORCH_CHECK(src.stride(1) == 1 && dst.stride(1) == 1 && src.stride(0) % 8 == 0 && dst.stride(0) % 8 == 0 &&
                  src.stride(0) >= C && dst.stride(0) >= R,
              "transpose_: row-major with 16-B aligned rows");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(src.data_ptr()) % 16) == 0 &&
                  (reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16) == 0, "transpose_: 16-B aligned");
  TORCH_CHECK(R < (1LL << 31) && C < (1LL << 31), "transpose_: dims");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(src.device());
  int rc = st_transpose_bf16(src.data_ptr(), dst.data_ptr(), (int)R, (int)C, src.stride(0), dst.stride(0),
                             cur_stream());
  ST_CHECK_RC(rc, "transpose_");
}

void sumsq_(const at::Tensor& g, at::Tensor out) {
  TORCH_CHECK(g.is_cuda() && g.is_contiguous() && g.numel() % 4 == 0, "sumsq: contiguous, n%4==0");
  TORCH_CHECK(g.scalar_type() == at::kFloat || g.scalar_type() == at::kBFloat16, "sumsq: dtype");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() >= 1, "sumsq: out fp32");
  check_same_gpu(out, g, "out");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(g.device());
  auto partial = at::empty({st_sumsq_partials()}, g.options().dtype(at::kFloat));
  int rc = st_sumsq(g.data_ptr(), g.scalar_type() == at::kBFloat16 ? 1 : 0, g.numel(),
                    partial.data_ptr<float>(), out.data_ptr<float>(), cur_stream());
  ST_CHECK_RC(rc, "sumsq_");
}

// ---------------------------------------------------------------- weight-gradient GEMM
// out[M,N] fp32 (+)= dy[T,M]^T @ x[T,N]; returns false when the shape is not one the
// kernel tiles (caller falls back to hipBLASLt).
bool wgrad_gemm_(at::Tensor out, const at::Tensor& dy, const at::Tensor& x, int64_t beta, int64_t variant) {
  check_bf16_cuda(dy, "dy");
  check_bf16_cuda(x, "x");
  check_same_gpu(x, dy, "x");
  check_same_gpu(out, dy, "out");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && out.dim() == 2, "wgrad_gemm: 2-D operands");
  TORCH_CHECK(out.scalar_type() == at::kFloat, "wgrad_gemm: out must be fp32");
  TORCH_CHECK(dy.size(0) == x.size(0) && out.size(0) == dy.size(1) && out.size(1) == x.size(1),
              "wgrad_gemm: shapes ", dy.sizes(), " x ", x.sizes(), " -> ", out.sizes());
  if (dy.stride(1) != 1 || x.stride(1) != 1 || out.stride(1) != 1) return false;
  const int64_t T = dy.size(0), M = dy.size(1), N = x.size(1);
  if (T > INT32_MAX || M > INT32_MAX || N > INT32_MAX) return false;
  c10::hip::HIPGuardMasqueradingAsCUDA g(out.device());
  // tail-split partials (csrc/wgrad_gemm.hip): stream-ordered caching-allocator scratch
  const int64_t wse = st_wgrad_ws_elems((int)M, (int)N, (int)T, (int)variant);
  at::Tensor ws;
  if (wse > 0) ws = at::empty({wse}, out.options());
  int rc = st_wgrad_gemm(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), out.data_ptr<float>(),
                         out.stride(0), (int)M, (int)N, (int)T, beta ? 1 : 0, (int)variant,
                         wse > 0 ? ws.data_ptr<float>() : nullptr, cur_stream());
  if (rc == -2) return false;
  ST_CHECK_RC(rc, "wgrad_gemm_");
  return true;
}

// out[g] fp32 [G, M, N] (+)= dy[rows of g]^T @ x[rows of g], rows of g = [offs[g-1], offs[g])
// (int32 inclusive prefix sums on the device).  One launch for every expert; false when
// the kernel does not tile the shape.
bool wgrad_grouped_(at::Tensor out, const at::Tensor& dy, const at::Tensor& x, const at::Tensor& offs, int64_t beta) {
  check_bf16_cuda(dy, "dy");
  check_bf16_cuda(x, "x");
  check_same_gpu(x, dy, "x");
  check_same_gpu(out, dy, "out");
  check_same_gpu(offs, dy, "offs");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && out.dim() == 3, "wgrad_grouped: dy [T,M], x [T,N], out [G,M,N]");
  TORCH_CHECK(out.scalar_type() == at::kFloat, "wgrad_grouped: out must be fp32");
  TORCH_CHECK(offs.scalar_type() == at::kInt && offs.dim() == 1 && offs.is_contiguous() && offs.size(0) == out.size(0),
              "wgrad_grouped: offs int32 [G]");
  TORCH_CHECK(dy.size(0) == x.size(0) && out.size(1) == dy.size(1) && out.size(2) == x.size(1),
              "wgrad_grouped: shapes ", dy.sizes(), " x ", x.sizes(), " -> ", out.sizes());
  if (dy.stride(1) != 1 || x.stride(1) != 1 || out.stride(2) != 1) return false;
  const int64_t T = dy.size(0), M = dy.size(1), N = x.size(1), G = out.size(0);
  if (T > INT32_MAX || M > INT32_MAX || N > INT32_MAX || G > INT32_MAX) return false;
  c10::hip::HIPGuardMasqueradingAsCUDA g(out.device());
  int rc = st_wgrad_grouped(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), out.data_ptr<float>(),
                            out.stride(1), out.stride(0), (int)M, (int)N, (int)G, offs.data_ptr<int>(), (int)T,
                            beta ? 1 : 0, cur_stream());
  if (rc == -2) return false;
  ST_CHECK_RC(rc, "wgrad_grouped_");
  return true;
}

// Grouped expert GEMM (csrc/grouped_gemm.hip): y[T, N] = x[T, K] @ (wn ? w[g] : w[g]^T) over the
// row ranges [offs[g-1], offs[g]); w is [G, N, K] (wn = false) or [G, K, N] (wn = true).  Rows
// of y past offs[G-1] are left unwritten.  Returns an undefined tensor when the kernel does
// not tile the shape (caller falls back).
at::Tensor grouped_gemm(const at::Tensor& x, const at::Tensor& w, const at::Tensor& offs, bool wn) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "w");
  check_same_gpu(w, x, "w");
  check_same_gpu(offs, x, "offs");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 3, "grouped_gemm: x [T, K], w [G, ., .]");
  TORCH_CHECK(offs.scalar_type() == at::kInt && offs.dim() == 1 && offs.is_contiguous() && offs.size(0) == w.size(0),
              "grouped_gemm: offs int32 [G]");
  const int64_t T = x.size(0), K = x.size(1), G = w.size(0);
  const int64_t N = wn ? w.size(2) : w.size(1);
  TORCH_CHECK((wn ? w.size(1) : w.size(2)) == K, "grouped_gemm: inner dims ", x.sizes(), " x ", w.sizes());
  if (x.stride(1) != 1 || w.stride(2) != 1 || T == 0 || T > INT32_MAX || N > INT32_MAX || K > INT32_MAX)
    return at::Tensor();
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  const int bm = st_grouped_gemm_bm();
  // per-group M-tile counts -> inclusive prefix (device; the host never reads the offsets)
  at::Tensor counts = at::diff(offs, 1, 0, at::zeros({1}, offs.options()));
  at::Tensor tile_end = at::cumsum(at::floor_divide(counts + (bm - 1), bm), 0, at::kInt);
  at::Tensor y = at::empty({T, N}, x.options());
  int rc = st_grouped_gemm(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(1), w.stride(0), y.data_ptr(),
                           y.stride(0), offs.data_ptr<int>(), tile_end.data_ptr<int>(), (int)T, (int)G, (int)N,
                           (int)K, wn ? 1 : 0, cur_stream());
  if (rc == -2) return at::Tensor();
  ST_CHECK_RC(rc, "grouped_gemm");
  return y;
}

// One-wave-per-SIMD TN GEMM (csrc/gemm4w.hip): y[T, N] = x[T, K] @ w[g]^T over the row ranges
// [offs[g-1], offs[g]); w [G, N, K] (K contiguous).  Undefined tensor when the kernel does not
// tile the shape.
at::Tensor gemm4w(const at::Tensor& x, const at::Tensor& w, const at::Tensor& offs) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "w");
  check_same_gpu(w, x, "w");
  check_same_gpu(offs, x, "offs");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 3 && w.size(2) == x.size(1), "gemm4w: x [T, K], w [G, N, K]");
  TORCH_CHECK(offs.scalar_type() == at::kInt && offs.dim() == 1 && offs.is_contiguous() && offs.size(0) == w.size(0),
              "gemm4w: offs int32 [G]");
  const int64_t T = x.size(0), K = x.size(1), G = w.size(0), N = w.size(1);
  if (x.stride(1) != 1 || w.stride(2) != 1 || T == 0 || T > INT32_MAX || N > INT32_MAX || K > INT32_MAX)
    return at::Tensor();
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  at::Tensor counts = at::diff(offs, 1, 0, at::zeros({1}, offs.options()));
  at::Tensor tile_end = at::cumsum(at::floor_divide(counts + 255, 256), 0, at::kInt);
  at::Tensor y = at::empty({T, N}, x.options());
  int rc = st_gemm4w(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(1), w.stride(0), y.data_ptr(), y.stride(0),
                     offs.data_ptr<int>(), tile_end.data_ptr<int>(), (int)T, (int)G, (int)N, (int)K, cur_stream());
  if (rc == -2) return at::Tensor();
  ST_CHECK_RC(rc, "gemm4w");
  return y;
}

// Dense gate|up GEMM with the SwiGLU epilogue (csrc/gemm4w.hip, whole-tile-fragment LDS-DMA
// kernel): x [T, K] (any row stride), w [2I, K] = gate rows then up rows; returns
// {gu [T, 2I], h [T, I] = silu(gate) * up}, or {} when the kernel does not take the shape.
std::vector<at::Tensor> gemm_swiglu(const at::Tensor& x, const at::Tensor& w) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "w");
  check_same_gpu(w, x, "w");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && w.size(1) == x.size(1) && w.size(0) % 2 == 0,
              "gemm_swiglu: x [T, K], w [2I, K]");
  const int64_t T = x.size(0), K = x.size(1), I = w.size(0) / 2;
  if (x.stride(1) != 1 || w.stride(1) != 1 || T == 0 || T > INT32_MAX || I > INT32_MAX / 2 || K > INT32_MAX) return {};
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  at::Tensor gu = at::empty({T, 2 * I}, x.options());
  at::Tensor h = at::empty({T, I}, x.options());
  int rc = st_gemm4w_swiglu(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), gu.data_ptr(), gu.stride(0),
                            h.data_ptr(), h.stride(0), (int)T, (int)I, (int)K, cur_stream());
  if (rc == -2) return {};
  ST_CHECK_RC(rc, "gemm_swiglu");
  return {gu, h};
}

// Grouped gate|up GEMM + SwiGLU epilogue on the one-wave-per-SIMD kernel (csrc/gemm4w.hip):
// x [T, K], w [G, 2I, K], offs int32 [G] (inclusive); returns {gu [T, 2I], h [T, I]} (rows past
// offs[G-1] unwritten), or {} when the kernel does not take the shape.
std::vector<at::Tensor> gemm4w_swiglu_grouped(const at::Tensor& x, const at::Tensor& w, const at::Tensor& offs) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "w");
  check_same_gpu(w, x, "w");
  check_same_gpu(offs, x, "offs");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 3 && w.size(2) == x.size(1) && w.size(1) % 2 == 0,
              "gemm4w_swiglu_grouped: x [T, K], w [G, 2I, K]");
  TORCH_CHECK(offs.scalar_type() == at::kInt && offs.dim() == 1 && offs.is_contiguous() && offs.size(0) == w.size(0),
              "gemm4w_swiglu_grouped: offs int32 [G]");
  const int64_t T = x.size(0), K = x.size(1), G = w.size(0), I = w.size(1) / 2;
  if (x.stride(1) != 1 || w.stride(2) != 1 || T == 0 || T > INT32_MAX || I > INT32_MAX / 2 || K > INT32_MAX) return {};
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  at::Tensor counts = at::diff(offs, 1, 0, at::zeros({1}, offs.options()));
  at::Tensor tile_end = at::cumsum(at::floor_divide(counts + 255, 256), 0, at::kInt);
  at::Tensor gu = at::empty({T, 2 * I}, x.options());
  at::Tensor h = at::empty({T, I}, x.options());
  int rc = st_gemm4w_swiglu_grouped(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(1), w.stride(0), gu.data_ptr(),
                                    gu.stride(0), h.data_ptr(), h.stride(0), offs.data_ptr<int>(),
                                    tile_end.data_ptr<int>(), (int)T, (int)G, (int)I, (int)K, cur_stream());
  if (rc == -2) return {};
  ST_CHECK_RC(rc, "gemm4w_swiglu_grouped");
  return {gu, h};
}

// Grouped gate|up GEMM with the SwiGLU epilogue: w [G, 2I, K]; returns {gu [T, 2I], a [T, I]}
// (rows past offs[G-1] unwritten), or {} when the kernel does not take the shape.
std::vector<at::Tensor> grouped_gemm_swiglu(const at::Tensor& x, const at::Tensor& w, const at::Tensor& offs) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "w");
  check_same_gpu(w, x, "w");
  check_same_gpu(offs, x, "offs");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 3 && w.size(2) == x.size(1) && w.size(1) % 2 == 0,
              "grouped_gemm_swiglu: x [T, K], w [G, 2I, K]");
  TORCH_CHECK(offs.scalar_type() == at::kInt && offs.dim() == 1 && offs.is_contiguous() && offs.size(0) == w.size(0),
              "grouped_gemm_swiglu: offs int32 [G]");
  const int64_t T = x.size(0), K = x.size(1), G = w.size(0), N = w.size(1), I = N / 2;
  if (x.stride(1) != 1 || !w.is_contiguous() || T == 0 || T > INT32_MAX) return {};
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  const int bm = st_grouped_gemm_bm();
  at::Tensor counts = at::diff(offs, 1, 0, at::zeros({1}, offs.options()));
  at::Tensor tile_end = at::cumsum(at::floor_divide(counts + (bm - 1), bm), 0, at::kInt);
  at::Tensor gu = at::empty({T, N}, x.options());
  at::Tensor a = at::empty({T, I}, x.options());
  int rc = st_grouped_gemm_ex(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(1), w.stride(0), gu.data_ptr(), N,
                              offs.data_ptr<int>(), tile_end.data_ptr<int>(), (int)T, (int)G, (int)N, (int)K, 0, 1,
                              a.data_ptr(), I, cur_stream());
  if (rc == -2) return {};
  ST_CHECK_RC(rc, "grouped_gemm_swiglu");
  return {gu, a};
}

// Down-projection data gradient with the SwiGLU backward epilogue: w [G, K=h, I]
// (dy @ w[g]), gu [T, 2I] saved by the forward; returns dgu [T, 2I] (undefined when the
// kernel does not take the shape).
at::Tensor grouped_gemm_dswiglu(const at::Tensor& dy, const at::Tensor& w, const at::Tensor& offs,
                                const at::Tensor& gu) {
  check_bf16_cuda(dy, "dy");
  check_bf16_cuda(w, "w");
  check_bf16_cuda(gu, "gu");
  check_same_gpu(w, dy, "w");
  check_same_gpu(gu, dy, "gu");
  check_same_gpu(offs, dy, "offs");
  TORCH_CHECK(dy.dim() == 2 && w.dim() == 3 && w.size(1) == dy.size(1), "grouped_gemm_dswiglu: dy [T, K], w [G, K, I]");
  const int64_t T = dy.size(0), K = dy.size(1), G = w.size(0), I = w.size(2);
  TORCH_CHECK(gu.dim() == 2 && gu.size(0) == T && gu.size(1) == 2 * I && gu.is_contiguous(),
              "grouped_gemm_dswiglu: gu [T, 2I] contiguous");
  TORCH_CHECK(offs.scalar_type() == at::kInt && offs.dim() == 1 && offs.is_contiguous() && offs.size(0) == G,
              "grouped_gemm_dswiglu: offs int32 [G]");
  if (dy.stride(1) != 1 || !w.is_contiguous() || T == 0 || T > INT32_MAX) return at::Tensor();
  c10::hip::HIPGuardMasqueradingAsCUDA g(dy.device());
  const int bm = st_grouped_gemm_bm();
  at::Tensor counts = at::diff(offs, 1, 0, at::zeros({1}, offs.options()));
  at::Tensor tile_end = at::cumsum(at::floor_divide(counts + (bm - 1), bm), 0, at::kInt);
  at::Tensor dgu = at::empty({T, 2 * I}, dy.options());
  int rc = st_grouped_gemm_ex(dy.data_ptr(), dy.stride(0), w.data_ptr(), w.stride(1), w.stride(0), dgu.data_ptr(),
                              2 * I, offs.data_ptr<int>(), tile_end.data_ptr<int>(), (int)T, (int)G, (int)I, (int)K,
                              1, 2, gu.data_ptr(), 2 * I, cur_stream());
  if (rc == -2) return at::Tensor();
  ST_CHECK_RC(rc, "grouped_gemm_dswiglu");
  return dgu;
}

// ---------------------------------------------------------------- xGMI all-reduce
// Stateful helpers around csrc/xgmi_allreduce.hip (catch-all kernels: most take no tensor).
int64_t xgmi_create(int64_t rank, int64_t world, int64_t cap, int64_t epoch_base) {
  int64_t id = st_xgmi_create((int)rank, (int)world, cap, epoch_base);
  TORCH_CHECK(id >= 0, "xgmi_create failed (", id, ")");
  return id;
}
at::Tensor xgmi_handle(int64_t id) {
  auto t = at::zeros({64}, at::TensorOptions().dtype(at::kByte));
  int rc = st_xgmi_handle(id, t.data_ptr());
  TORCH_CHECK(rc == 0, "hipIpcGetMemHandle failed (", rc, ")");
  return t;
}
void xgmi_open(int64_t id, int64_t r, const at::Tensor& h) {
  TORCH_CHECK(!h.is_cuda() && h.numel() == 64 && h.scalar_type() == at::kByte, "xgmi_open: uint8[64] CPU handle");
  auto hc = h.contiguous();
  int rc = st_xgmi_open(id, (int)r, hc.data_ptr());
  TORCH_CHECK(rc == 0, "hipIpcOpenMemHandle for peer ", r, " failed (", rc, ")");
}
void xgmi_set_peer(int64_t id, int64_t r, int64_t peer) {
  TORCH_CHECK(st_xgmi_set_peer(id, (int)r, peer) == 0, "xgmi_set_peer");
}
// elements n the kernels are told about: the tensor (all-reduce), the per-rank
// contribution (all-gather: out = world x in) or the output (reduce-scatter: in = world x out)
static int64_t xgmi_count(int64_t mode, int64_t world, const at::Tensor& inp, const at::Tensor& out) {
  if (mode == 2) {
    TORCH_CHECK(out.numel() == world * inp.numel(), "xgmi all_gather: out must hold world x input elements");
    return inp.numel();
  }
  if (mode == 3) {
    TORCH_CHECK(inp.numel() == world * out.numel(), "xgmi reduce_scatter: input must hold world x out elements");
    return out.numel();
  }
  if (mode == 4) {
    TORCH_CHECK(inp.numel() == out.numel() && inp.numel() % world == 0, "xgmi all_to_all: world equal chunks");
    return inp.numel() / world;
  }
  if (mode == 5) {
    TORCH_CHECK(out.numel() == 2 * inp.numel(), "xgmi pair all_gather: out must hold 2 x input elements");
    return inp.numel();
  }
  if (mode == 6) {
    TORCH_CHECK(inp.numel() == 2 * out.numel(), "xgmi pair reduce_scatter: input must hold 2 x out elements");
    return out.numel();
  }
  TORCH_CHECK(mode == 0 || mode == 1, "xgmi: mode 0..6");
  TORCH_CHECK(inp.numel() == out.numel(), "xgmi all_reduce: same size");
  return inp.numel();
}

void xgmi_all_reduce(int64_t id, const at::Tensor& inp, at::Tensor out, int64_t mode, int64_t blocks) {
  TORCH_CHECK(inp.is_cuda() && out.is_cuda() && inp.device() == out.device(), "xgmi: GPU tensors");
  TORCH_CHECK(inp.is_contiguous() && out.is_contiguous() && inp.scalar_type() == out.scalar_type(),
              "xgmi: contiguous, same dtype");
  TORCH_CHECK(inp.scalar_type() == at::kBFloat16 || inp.scalar_type() == at::kFloat, "xgmi: bf16 or fp32");
  const int world = st_xgmi_world(id);
  TORCH_CHECK(world > 0, "xgmi: unknown communicator");
  const int64_t n = xgmi_count(mode, world, inp, out);
  TORCH_CHECK(mode < 2 || inp.data_ptr() != out.data_ptr(), "xgmi all_gather/reduce_scatter: out-of-place only");
  c10::hip::HIPGuardMasqueradingAsCUDA g(inp.device());
  int rc = st_xgmi_all_reduce(id, inp.data_ptr(), out.data_ptr(), n, inp.scalar_type() == at::kBFloat16 ? 0 : 1,
                              (int)mode, (int)blocks, cur_stream());
  TORCH_CHECK(rc == 0, "xgmi collective failed (", rc, "): size must be a multiple of 8 and fit the buffer");
}
// pair collective (mode 5 all-gather / 6 reduce-scatter) with `partner` over multiple paths
void xgmi_pair(int64_t id, const at::Tensor& inp, at::Tensor out, int64_t mode, int64_t partner, int64_t blocks) {
  TORCH_CHECK(mode == 5 || mode == 6, "xgmi_pair: mode 5 or 6");
  TORCH_CHECK(inp.is_cuda() && out.is_cuda() && inp.device() == out.device(), "xgmi: GPU tensors");
  TORCH_CHECK(inp.is_contiguous() && out.is_contiguous() && inp.scalar_type() == out.scalar_type(),
              "xgmi: contiguous, same dtype");
  TORCH_CHECK(inp.scalar_type() == at::kBFloat16 || inp.scalar_type() == at::kFloat, "xgmi: bf16 or fp32");
  TORCH_CHECK(inp.data_ptr() != out.data_ptr(), "xgmi pair: out-of-place only");
  const int world = st_xgmi_world(id);
  TORCH_CHECK(world > 0, "xgmi: unknown communicator");
  const int64_t n = xgmi_count(mode, world, inp, out);
  c10::hip::HIPGuardMasqueradingAsCUDA g(inp.device());
  int rc = st_xgmi_pair(id, inp.data_ptr(), out.data_ptr(), n, inp.scalar_type() == at::kBFloat16 ? 0 : 1, (int)mode,
                        (int)partner, (int)blocks, cur_stream());
  TORCH_CHECK(rc == 0, "xgmi pair collective failed (", rc, ")");
}
void xgmi_set_timeout(int64_t id, double seconds) {
  TORCH_CHECK(st_xgmi_set_timeout(id, seconds) == 0, "xgmi_set_timeout: bad id or value");
}
void xgmi_all_reduce_sim(std::vector<int64_t> ids, std::vector<at::Tensor> ins, std::vector<at::Tensor> outs,
                         int64_t mode, int64_t blocks, c10::OptionalArrayRef<int64_t> partners) {
  const size_t w = ids.size();
  TORCH_CHECK(w >= 1 && ins.size() == w && outs.size() == w, "xgmi_all_reduce_sim: one in/out per rank");
  std::vector<const void*> ip(w);
  std::vector<void*> op(w);
  const int64_t n = xgmi_count(mode, (int64_t)w, ins[0], outs[0]);
  for (size_t r = 0; r < w; ++r) {
    TORCH_CHECK(ins[r].is_cuda() && outs[r].is_cuda() && ins[r].is_contiguous() && outs[r].is_contiguous() &&
                    ins[r].numel() == ins[0].numel() && outs[r].numel() == outs[0].numel() &&
                    ins[r].scalar_type() == ins[0].scalar_type() && outs[r].scalar_type() == ins[0].scalar_type() &&
                    ins[r].device() == ins[0].device() && outs[r].device() == ins[0].device(),
                "xgmi_all_reduce_sim: matching contiguous GPU tensors");
    ip[r] = ins[r].data_ptr();
    op[r] = outs[r].data_ptr();
  }
  TORCH_CHECK(ins[0].scalar_type() == at::kBFloat16 || ins[0].scalar_type() == at::kFloat, "xgmi: bf16 or fp32");
  c10::hip::HIPGuardMasqueradingAsCUDA g(ins[0].device());
  std::vector<int> pr;
  if (partners.has_value()) {
    TORCH_CHECK(partners->size() == w, "xgmi_all_reduce_sim: one partner per rank");
    for (int64_t x : *partners) pr.push_back((int)x);
  }
  int rc = st_xgmi_collective_sim(ids.data(), ip.data(), op.data(), pr.empty() ? nullptr : pr.data(), (int)w, n,
                                  ins[0].scalar_type() == at::kBFloat16 ? 0 : 1, (int)mode, (int)blocks,
                                  cur_stream());
  TORCH_CHECK(rc == 0, "xgmi_all_reduce_sim failed (", rc, ")");
}
// Expert-parallel exchange with device counts M [world, E] int32 (csrc/xgmi_allreduce.hip):
// dir 0 dispatch (in: this rank's rows sorted by global expert -> out: its experts' rows,
// expert-major, out.size(0) = the host bound R_max), dir 1 combine (the reverse).
static void check_ep_args(const at::Tensor& inp, const at::Tensor& out, const at::Tensor& M, int64_t world) {
  TORCH_CHECK(inp.is_cuda() && out.is_cuda() && inp.device() == out.device(), "xgmi_ep_exchange: GPU tensors");
  TORCH_CHECK(inp.dim() == 2 && out.dim() == 2 && inp.size(1) == out.size(1) && inp.is_contiguous() &&
                  out.is_contiguous() && inp.scalar_type() == out.scalar_type(),
              "xgmi_ep_exchange: contiguous [rows, h] in / out of one dtype");
  TORCH_CHECK(inp.scalar_type() == at::kBFloat16 || inp.scalar_type() == at::kFloat, "xgmi: bf16 or fp32");
  TORCH_CHECK(inp.size(1) % 8 == 0, "xgmi_ep_exchange: row width must be a multiple of 8");
  TORCH_CHECK(M.is_cuda() && M.device() == inp.device() && M.scalar_type() == at::kInt && M.dim() == 2 &&
                  M.size(0) == world && M.is_contiguous(),
              "xgmi_ep_exchange: M int32 [world, E] on the same GPU");
  TORCH_CHECK(inp.data_ptr() != out.data_ptr(), "xgmi_ep_exchange: out-of-place only");
}
void xgmi_ep_exchange(int64_t id, const at::Tensor& inp, at::Tensor out, const at::Tensor& M, int64_t El,
                      int64_t dir, int64_t area_rows, int64_t blocks) {
  const int world = st_xgmi_world(id);
  TORCH_CHECK(world > 0, "xgmi: unknown communicator");
  check_ep_args(inp, out, M, world);
  c10::hip::HIPGuardMasqueradingAsCUDA g(inp.device());
  int rc = st_xgmi_ep_exchange(id, inp.data_ptr(), out.data_ptr(), M.data_ptr<int>(), (int)M.size(1), (int)El,
                               inp.size(1), inp.size(0), out.size(0), area_rows,
                               inp.scalar_type() == at::kBFloat16 ? 0 : 1, (int)dir, (int)blocks, cur_stream());
  TORCH_CHECK(rc == 0, "xgmi_ep_exchange failed (", rc, "): E = El x world <= 256, rows must fit the buffer");
}
void xgmi_ep_exchange_sim(std::vector<int64_t> ids, std::vector<at::Tensor> ins, std::vector<at::Tensor> outs,
                          const at::Tensor& M, int64_t El, int64_t dir, int64_t area_rows, int64_t blocks) {
  const size_t w = ids.size();
  TORCH_CHECK(w >= 1 && ins.size() == w && outs.size() == w, "xgmi_ep_exchange_sim: one in/out per rank");
  std::vector<const void*> ip(w);
  std::vector<void*> op(w);
  for (size_t r = 0; r < w; ++r) {
    check_ep_args(ins[r], outs[r], M, (int64_t)w);
    TORCH_CHECK(ins[r].sizes() == ins[0].sizes() && outs[r].sizes() == outs[0].sizes() &&
                    ins[r].scalar_type() == ins[0].scalar_type() && ins[r].device() == ins[0].device(),
                "xgmi_ep_exchange_sim: matching tensors on every rank");
    ip[r] = ins[r].data_ptr();
    op[r] = outs[r].data_ptr();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(ins[0].device());
  int rc = st_xgmi_ep_exchange_sim(ids.data(), ip.data(), op.data(), M.data_ptr<int>(), (int)w, (int)M.size(1),
                                   (int)El, ins[0].size(1), ins[0].size(0), outs[0].size(0), area_rows,
                                   ins[0].scalar_type() == at::kBFloat16 ? 0 : 1, (int)dir, (int)blocks,
                                   cur_stream());
  TORCH_CHECK(rc == 0, "xgmi_ep_exchange_sim failed (", rc, ")");
}
int64_t xgmi_error(int64_t id) { return st_xgmi_error(id); }
void xgmi_destroy(int64_t id) { st_xgmi_destroy(id); }

// ---------------------------------------------------------------- fused QK-norm + RoPE
// qkv [B, S, H + 2 Hkv, D] contiguous bf16, modified in place (q, k heads).
static void check_qknorm_args(const at::Tensor& qkv, const at::Tensor& wq, const at::Tensor& wk,
                              const at::Tensor& cos, const at::Tensor& sin, const c10::optional<at::Tensor>& pos,
                              int64_t H, int64_t Hkv) {
  check_bf16_cuda(qkv, "qkv");
  check_bf16_cuda(wq, "q_norm.weight");
  check_bf16_cuda(wk, "k_norm.weight");
  TORCH_CHECK(qkv.dim() == 4 && qkv.is_contiguous() && qkv.size(2) == H + 2 * Hkv, "qknorm_rope: qkv [B,S,H+2Hkv,D]");
  const int64_t D = qkv.size(3);
  TORCH_CHECK(D == 64 || D == 128, "qknorm_rope: head_dim 64 or 128");
  TORCH_CHECK(wq.numel() == D && wk.numel() == D && wq.is_contiguous() && wk.is_contiguous(), "qknorm_rope: weights [D]");
  TORCH_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat && cos.is_contiguous() &&
                  sin.is_contiguous() && cos.dim() == 2 && cos.size(1) == D / 2 && sin.sizes() == cos.sizes(),
              "qknorm_rope: fp32 cos/sin [max_pos, D/2]");
  check_same_gpu(wq, qkv, "q_norm.weight");
  check_same_gpu(wk, qkv, "k_norm.weight");
  check_same_gpu(cos, qkv, "cos");
  check_same_gpu(sin, qkv, "sin");
  if (pos.has_value() && pos->defined()) {
    TORCH_CHECK(pos->scalar_type() == at::kLong && pos->is_contiguous() &&
                    pos->numel() == qkv.size(0) * qkv.size(1), "qknorm_rope: position ids int64 [B,S]");
    check_same_gpu(*pos, qkv, "position_ids");
  }
}

std::vector<at::Tensor> qknorm_rope_fwd_(at::Tensor qkv, const at::Tensor& wq, const at::Tensor& wk,
                                         const at::Tensor& cos, const at::Tensor& sin,
                                         const c10::optional<at::Tensor>& pos, int64_t H, int64_t Hkv, double eps) {
  check_qknorm_args(qkv, wq, wk, cos, sin, pos, H, Hkv);
  const int64_t B = qkv.size(0), S = qkv.size(1), D = qkv.size(3);
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  auto xsave = at::empty({B * S, H + Hkv, D}, qkv.options());
  auto rstd = at::empty({B * S, H + Hkv}, qkv.options().dtype(at::kFloat));
  const int64_t* pp = (pos.has_value() && pos->defined()) ? pos->data_ptr<int64_t>() : nullptr;
  int rc = st_qknorm_rope_fwd(qkv.data_ptr(), xsave.data_ptr(), rstd.data_ptr<float>(), wq.data_ptr(), wk.data_ptr(),
                              cos.data_ptr<float>(), sin.data_ptr<float>(), pp, B * S, (int)S, (int)H, (int)Hkv,
                              (int)D, (float)eps, cos.size(0), cur_stream());
  ST_CHECK_RC(rc, "qknorm_rope_fwd_");
  return {xsave, rstd};
}

// returns dw [2, D] fp32 (q-norm, k-norm weight gradients); dqkv modified in place
at::Tensor qknorm_rope_bwd_(at::Tensor dqkv, const at::Tensor& xsave, const at::Tensor& rstd, const at::Tensor& wq,
                            const at::Tensor& wk, const at::Tensor& cos, const at::Tensor& sin,
                            const c10::optional<at::Tensor>& pos, int64_t H, int64_t Hkv) {
  check_qknorm_args(dqkv, wq, wk, cos, sin, pos, H, Hkv);
  const int64_t B = dqkv.size(0), S = dqkv.size(1), D = dqkv.size(3);
  check_bf16_cuda(xsave, "xsave");
  check_same_gpu(xsave, dqkv, "xsave");
  check_same_gpu(rstd, dqkv, "rstd");
  TORCH_CHECK(xsave.is_contiguous() && xsave.numel() == B * S * (H + Hkv) * D, "qknorm_rope_bwd: xsave shape");
  TORCH_CHECK(rstd.is_contiguous() && rstd.scalar_type() == at::kFloat && rstd.numel() == B * S * (H + Hkv),
              "qknorm_rope_bwd: rstd shape");
  c10::hip::HIPGuardMasqueradingAsCUDA g(dqkv.device());
  auto dw = at::zeros({2, D}, dqkv.options().dtype(at::kFloat));
  auto partial = at::empty({(int64_t)st_qknorm_rope_bwd_blocks() * 2 * D}, dqkv.options().dtype(at::kFloat));
  const int64_t* pp = (pos.has_value() && pos->defined()) ? pos->data_ptr<int64_t>() : nullptr;
  int rc = st_qknorm_rope_bwd(dqkv.data_ptr(), xsave.data_ptr(), rstd.data_ptr<float>(), wq.data_ptr(), wk.data_ptr(),
                              cos.data_ptr<float>(), sin.data_ptr<float>(), pp, B * S, (int)S, (int)H, (int)Hkv,
                              (int)D, cos.size(0), partial.data_ptr<float>(), dw.data_ptr<float>(), cur_stream());
  ST_CHECK_RC(rc, "qknorm_rope_bwd_");
  return dw;
}

// ---------------------------------------------------------------- cross-entropy
std::vector<at::Tensor> xent_fwd(const at::Tensor& logits, const at::Tensor& tgt,
                                 int64_t vocab_start) {
  check_bf16_cuda(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "xent: logits [N, V] row-major");
  TORCH_CHECK(tgt.scalar_type() == at::kLong && tgt.is_contiguous() && tgt.numel() == logits.size(0),
              "xent: targets int64 [N]");
  check_same_gpu(tgt, logits, "target");
  const int64_t N = logits.size(0), V = logits.size(1);
  TORCH_CHECK(V % 8 == 0 && logits.stride(0) % 8 == 0, "xent: V and row stride must be %8");
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  auto lse = at::empty({N}, logits.options().dtype(at::kFloat));
  auto tl = at::empty({N}, logits.options().dtype(at::kFloat));
  int rc = st_xent_fwd(logits.data_ptr(), logits.stride(0), tgt.data_ptr<int64_t>(), N, (int)V,
                       vocab_start, lse.data_ptr<float>(), tl.data_ptr<float>(), cur_stream());
  ST_CHECK_RC(rc, "xent_fwd");
  return {lse, tl};
}

void xent_bwd_(const at::Tensor& logits, const at::Tensor& tgt, int64_t vocab_start,
               const at::Tensor& lse, const at::Tensor& dloss, at::Tensor dlogits) {
  check_bf16_cuda(logits, "logits");
  check_bf16_cuda(dlogits, "dlogits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1 && dlogits.sizes() == logits.sizes() &&
                  dlogits.stride(1) == 1, "xent_bwd: shapes");
  const int64_t N = logits.size(0), V = logits.size(1);
  TORCH_CHECK(lse.numel() == N && dloss.numel() == N && tgt.numel() == N, "xent_bwd: row vectors");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && dloss.scalar_type() == at::kFloat &&
                  lse.is_contiguous() && dloss.is_contiguous(), "xent_bwd: fp32 lse/dloss");
  TORCH_CHECK(tgt.scalar_type() == at::kLong && tgt.is_contiguous(), "xent_bwd: targets int64");
  check_same_gpu(tgt, logits, "target");
  check_same_gpu(lse, logits, "lse");
  check_same_gpu(dloss, logits, "dloss");
  check_same_gpu(dlogits, logits, "dlogits");
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  int rc = st_xent_bwd(logits.data_ptr(), logits.stride(0), tgt.data_ptr<int64_t>(), N, (int)V,
                       vocab_start, lse.data_ptr<float>(), dloss.data_ptr<float>(),
                       dlogits.data_ptr(), dlogits.stride(0), cur_stream());
  ST_CHECK_RC(rc, "xent_bwd_");
}

// ---------------------------------------------------------------- flash attention
// q [B, Sq, H, D], k/v [B, Sk, Hkv, D] (strided views, D contiguous), out
// [B, Sq, H, D] contiguous, lse [B, H, Sq] fp32.  q_offset/k_offset are the
// global positions of row 0 of q / k (context-parallel blocks); causal masks
// key j > query i in global coordinates.
void check_qkv(const at::Tensor& t, const char* n, int64_t D) {
  check_bf16_cuda(t, n);
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1 && t.size(3) == D, n, ": expected [B,S,H,D] with contiguous D");
  TORCH_CHECK(t.stride(2) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(0) % 8 == 0,
              n, ": strides must be multiples of 8 elements");
}

std::vector<at::Tensor> flash_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                  double scale, bool causal, int64_t q_offset, int64_t k_offset) {
  const int64_t D = q.size(3);
  TORCH_CHECK(D == 64 || D == 128, "flash_fwd: head_dim must be 64 or 128");
  check_qkv(q, "q", D);
  check_qkv(k, "k", D);
  check_qkv(v, "v", D);
  const int64_t B = q.size(0), Sq = q.size(1), H = q.size(2), Sk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(k.size(0) == B && v.size(0) == B && v.size(1) == Sk && v.size(2) == Hkv, "flash_fwd: k/v shapes");
  TORCH_CHECK(H % Hkv == 0, "flash_fwd: H must be a multiple of Hkv");
  check_same_gpu(k, q, "k");
  check_same_gpu(v, q, "v");
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  auto o = at::empty({B, Sq, H, D}, q.options());
  auto lse = at::empty({B, H, Sq}, q.options().dtype(at::kFloat));
  int rc = st_flash_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(),
                        (int)B, (int)Sq, (int)Sk, (int)H, (int)Hkv, (int)D, q.stride(0), q.stride(1),
                        q.stride(2), k.stride(0), k.stride(1), k.stride(2), v.stride(0), v.stride(1),
                        v.stride(2), o.stride(0), o.stride(1), o.stride(2), (float)scale,
                        causal ? 1 : 0, q_offset, k_offset, cur_stream());
  ST_CHECK_RC(rc, "flash_fwd");
  return {o, lse};
}

// Returns (dq, dk, dv) bf16: dq [B,Sq,H,D], dk/dv [B,Sk,Hkv,D].  Optional
// preallocated outputs (any (b,s,h) strides with contiguous D, e.g. slices of
// one fused dQKV buffer) are written in place and returned.
// GQA is native: dk/dv are accumulated over the H/Hkv query heads of each kv
// head, never expanded.
std::vector<at::Tensor> flash_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k,
                                  const at::Tensor& v, const at::Tensor& o, const at::Tensor& lse,
                                  double scale, bool causal, int64_t q_offset, int64_t k_offset,
                                  const c10::optional<at::Tensor>& dq_out,
                                  const c10::optional<at::Tensor>& dk_out,
                                  const c10::optional<at::Tensor>& dv_out, int64_t ds_mode) {
  const int64_t D = q.size(3);
  TORCH_CHECK(D == 64 || D == 128, "flash_bwd: head_dim must be 64 or 128");
  check_qkv(q, "q", D);
  check_qkv(k, "k", D);
  check_qkv(v, "v", D);
  check_qkv(o, "o", D);
  check_qkv(dout, "dout", D);
  const int64_t B = q.size(0), Sq = q.size(1), H = q.size(2), Sk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(o.sizes() == q.sizes() && dout.sizes() == q.sizes(), "flash_bwd: o/dout shapes");
  TORCH_CHECK(k.sizes() == v.sizes() && k.size(0) == B, "flash_bwd: k/v shapes");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == B * H * Sq,
              "flash_bwd: lse [B,H,Sq] fp32");
  TORCH_CHECK(H % Hkv == 0, "flash_bwd: H must be a multiple of Hkv");
  for (auto* t : {&k, &v, &o, &dout, &lse}) check_same_gpu(*t, q, "flash_bwd operand");
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  auto delta = at::empty({B, H, Sq}, q.options().dtype(at::kFloat));
  auto nlse2 = at::empty({B, H, Sq}, q.options().dtype(at::kFloat));
  int rc = st_flash_bwd_preprocess(o.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(),
                                   nlse2.data_ptr<float>(), (int)B, (int)Sq, (int)H, (int)D, o.stride(0), o.stride(1), o.stride(2),
                                   dout.stride(0), dout.stride(1), dout.stride(2), cur_stream());
  ST_CHECK_RC(rc, "flash_bwd_preprocess");
  auto pick = [&](const c10::optional<at::Tensor>& t, at::IntArrayRef shape, const char* n) {
    if (t.has_value() && t->defined()) {
      check_qkv(*t, n, D);
      check_same_gpu(*t, q, n);
      TORCH_CHECK(t->sizes() == shape, n, ": wrong shape");
      return *t;
    }
    return at::empty(shape, q.options());
  };
  auto dq = pick(dq_out, q.sizes(), "dq_out");
  auto dk = pick(dk_out, k.sizes(), "dk_out");
  auto dv = pick(dv_out, v.sizes(), "dv_out");
  TORCH_CHECK(dk.strides() == dv.strides(), "flash_bwd: dk_out/dv_out must share strides");
  // fp32 partials of the dK/dV query-range split (short grids only; csrc/flash_attn.hip)
  const int64_t pe = st_flash_bwd_part_elems((int)B, (int)Sq, (int)Sk, (int)H, (int)Hkv, (int)D, causal ? 1 : 0);
  at::Tensor part;
  if (pe > 0) part = at::empty({pe}, q.options().dtype(at::kFloat));
  // dS workspace of the dS-materialising backward (transient: freed on return); ds_mode 0
  // forces the one-shot (recompute dQ) backward, -1 lets st_flash_bwd_ds_elems decide
  const int64_t dse = ds_mode == 0 ? 0
                                   : st_flash_bwd_ds_elems((int)B, (int)Sq, (int)Sk, (int)H, (int)D, causal ? 1 : 0,
                                                           q_offset, k_offset);
  at::Tensor dsw;
  if (dse > 0) dsw = at::empty({dse}, q.options());
  rc = st_flash_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(),
                    delta.data_ptr<float>(), nlse2.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                    (int)B, (int)Sq, (int)Sk, (int)H, (int)Hkv, (int)D, q.stride(0), q.stride(1),
                    q.stride(2), k.stride(0), k.stride(1), k.stride(2), v.stride(0), v.stride(1),
                    v.stride(2), dout.stride(0), dout.stride(1), dout.stride(2), dq.stride(0),
                    dq.stride(1), dq.stride(2), dk.stride(0), dk.stride(1), dk.stride(2),
                    (float)scale, causal ? 1 : 0, q_offset, k_offset,
                    pe > 0 ? part.data_ptr<float>() : nullptr, dse > 0 ? dsw.data_ptr() : nullptr, 3,
                    cur_stream());
  ST_CHECK_RC(rc, "flash_bwd");
  return {dq, dk, dv};
}

// First phase of the dS-materialising backward on its own: delta, then dK / dV with the
// dS^T tiles stored into the returned workspace.  Returns {dk, dv, ws}; ws is EMPTY (and
// nothing ran) when the dS path does not apply -- the caller then runs flash_bwd.
std::vector<at::Tensor> flash_bwd_kv(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k,
                                     const at::Tensor& v, const at::Tensor& o, const at::Tensor& lse, double scale,
                                     bool causal, int64_t q_offset, int64_t k_offset,
                                     const c10::optional<at::Tensor>& dk_out,
                                     const c10::optional<at::Tensor>& dv_out) {
  const int64_t D = q.size(3);
  TORCH_CHECK(D == 64 || D == 128, "flash_bwd_kv: head_dim must be 64 or 128");
  for (auto* t : {&q, &k, &v, &o, &dout}) check_qkv(*t, "flash_bwd_kv operand", D);
  const int64_t B = q.size(0), Sq = q.size(1), H = q.size(2), Sk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(o.sizes() == q.sizes() && dout.sizes() == q.sizes() && k.sizes() == v.sizes() && k.size(0) == B,
              "flash_bwd_kv: shapes");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == B * H * Sq,
              "flash_bwd_kv: lse [B,H,Sq] fp32");
  TORCH_CHECK(H % Hkv == 0, "flash_bwd_kv: H must be a multiple of Hkv");
  for (auto* t : {&k, &v, &o, &dout, &lse}) check_same_gpu(*t, q, "flash_bwd_kv operand");
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  const int64_t dse = st_flash_bwd_ds_elems((int)B, (int)Sq, (int)Sk, (int)H, (int)D, causal ? 1 : 0, q_offset,
                                            k_offset);
  auto pick = [&](const c10::optional<at::Tensor>& t, at::IntArrayRef shape, const char* n) {
    if (t.has_value() && t->defined()) {
      check_qkv(*t, n, D);
      check_same_gpu(*t, q, n);
      TORCH_CHECK(t->sizes() == shape, n, ": wrong shape");
      return *t;
    }
    return at::empty(shape, q.options());
  };
  auto dk = pick(dk_out, k.sizes(), "dk_out");
  auto dv = pick(dv_out, v.sizes(), "dv_out");
  if (dse <= 0) return {dk, dv, at::empty({0}, q.options())};
  TORCH_CHECK(dk.strides() == dv.strides(), "flash_bwd_kv: dk_out/dv_out must share strides");
  auto delta = at::empty({B, H, Sq}, q.options().dtype(at::kFloat));
  auto nlse2 = at::empty({B, H, Sq}, q.options().dtype(at::kFloat));
  int rc = st_flash_bwd_preprocess(o.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(),
                                   nlse2.data_ptr<float>(), (int)B, (int)Sq, (int)H,
                                   (int)D, o.stride(0), o.stride(1), o.stride(2), dout.stride(0), dout.stride(1),
                                   dout.stride(2), cur_stream());
  ST_CHECK_RC(rc, "flash_bwd_kv preprocess");
  const int64_t pe = st_flash_bwd_part_elems((int)B, (int)Sq, (int)Sk, (int)H, (int)Hkv, (int)D, causal ? 1 : 0);
  at::Tensor part;
  if (pe > 0) part = at::empty({pe}, q.options().dtype(at::kFloat));
  auto ws = at::empty({dse}, q.options());
  rc = st_flash_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(),
                    delta.data_ptr<float>(), nlse2.data_ptr<float>(), nullptr, dk.data_ptr(), dv.data_ptr(), (int)B,
                    (int)Sq, (int)Sk, (int)H,
                    (int)Hkv, (int)D, q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2),
                    v.stride(0), v.stride(1), v.stride(2), dout.stride(0), dout.stride(1), dout.stride(2), 0, 0, 0,
                    dk.stride(0), dk.stride(1), dk.stride(2), (float)scale, causal ? 1 : 0, q_offset, k_offset,
                    pe > 0 ? part.data_ptr<float>() : nullptr, ws.data_ptr(), 1, cur_stream());
  ST_CHECK_RC(rc, "flash_bwd_kv");
  return {dk, dv, ws};
}

// Second phase: dQ = dS K from flash_bwd_kv's workspace (on the caller's current stream).
at::Tensor flash_bwd_q_ds(const at::Tensor& q, const at::Tensor& k, const at::Tensor& ws, double scale, bool causal,
                          int64_t q_offset, int64_t k_offset, const c10::optional<at::Tensor>& dq_out) {
  const int64_t D = q.size(3);
  check_qkv(q, "q", D);
  check_qkv(k, "k", D);
  check_same_gpu(k, q, "k");
  check_same_gpu(ws, q, "ws");
  const int64_t B = q.size(0), Sq = q.size(1), H = q.size(2), Sk = k.size(1), Hkv = k.size(2);
  const int64_t dse = st_flash_bwd_ds_elems((int)B, (int)Sq, (int)Sk, (int)H, (int)D, causal ? 1 : 0, q_offset,
                                            k_offset);
  TORCH_CHECK(dse > 0 && ws.numel() == dse && ws.scalar_type() == at::kBFloat16,
              "flash_bwd_q_ds: workspace does not match this problem");
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  at::Tensor dq;
  if (dq_out.has_value() && dq_out->defined()) {
    dq = *dq_out;
    check_qkv(dq, "dq_out", D);
    check_same_gpu(dq, q, "dq_out");
    TORCH_CHECK(dq.sizes() == q.sizes(), "dq_out: wrong shape");
  } else {
    dq = at::empty(q.sizes(), q.options());
  }
  int rc = st_flash_bwd(q.data_ptr(), k.data_ptr(), k.data_ptr(), q.data_ptr(), nullptr, nullptr, nullptr, dq.data_ptr(),
                        nullptr, nullptr, (int)B, (int)Sq, (int)Sk, (int)H, (int)Hkv, (int)D, q.stride(0), q.stride(1),
                        q.stride(2), k.stride(0), k.stride(1), k.stride(2), k.stride(0), k.stride(1), k.stride(2),
                        q.stride(0), q.stride(1), q.stride(2), dq.stride(0), dq.stride(1), dq.stride(2), 0, 0, 0,
                        (float)scale, causal ? 1 : 0, q_offset, k_offset, nullptr, ws.data_ptr(), 2, cur_stream());
  ST_CHECK_RC(rc, "flash_bwd_q_ds");
  return dq;
}

// In-place online-softmax merge of a partial attention block into a running
// (out fp32 [B,S,H,D], lse fp32 [B,H,S]) pair -- the ring-attention combine.
void lse_merge_(at::Tensor out, at::Tensor lse, const at::Tensor& bout, const at::Tensor& blse) {
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.dim() == 4, "lse_merge: out");
  check_qkv(bout, "block_out", out.size(3));
  TORCH_CHECK(bout.sizes() == out.sizes(), "lse_merge: block_out shape");
  const int64_t B = out.size(0), S = out.size(1), H = out.size(2), D = out.size(3);
  TORCH_CHECK(lse.scalar_type() == at::kFloat && blse.scalar_type() == at::kFloat &&
                  lse.is_contiguous() && blse.is_contiguous() && lse.numel() == B * H * S &&
                  blse.numel() == B * H * S, "lse_merge: lse [B,H,S] fp32");
  TORCH_CHECK(D % 8 == 0, "lse_merge: D % 8");
  TORCH_CHECK(out.is_cuda(), "lse_merge: out must be a GPU tensor");
  check_same_gpu(lse, out, "lse");
  check_same_gpu(bout, out, "block_out");
  check_same_gpu(blse, out, "block_lse");
  c10::hip::HIPGuardMasqueradingAsCUDA g(out.device());
  int rc = st_lse_merge(out.data_ptr<float>(), lse.data_ptr<float>(), bout.data_ptr(),
                        blse.data_ptr<float>(), (int)B, (int)S, (int)H, (int)D, bout.stride(0),
                        bout.stride(1), bout.stride(2), cur_stream());
  ST_CHECK_RC(rc, "lse_merge_");
}

}  // namespace

TORCH_LIBRARY(st_amd, m) {
  m.def("rmsnorm_fwd(Tensor x, Tensor? residual, Tensor weight, float eps) -> Tensor[]");
  m.def("rmsnorm_bwd(Tensor dy, Tensor s, Tensor weight, Tensor rstd, Tensor? dres, Tensor(a!) dw_accum) -> Tensor");
  m.def("rope_(Tensor(a!) x, Tensor cos, Tensor sin, Tensor? pos, int pos_offset, bool backward) -> ()");
  m.def("swiglu_fwd(Tensor gate_up, Tensor? nvalid=None) -> Tensor");
  m.def("swiglu_bwd(Tensor dout, Tensor gate_up, Tensor? nvalid=None) -> Tensor");
  m.def("adamw_step_(Tensor(a!) master, Tensor(b!) exp_avg, Tensor(c!) exp_avg_sq, Tensor grad, Tensor(d!)? param, Tensor? clip_coef, float lr, float beta1, float beta2, float eps, float weight_decay, int step, int sr_base=0) -> ()");
  m.def("adamw_wt_step_(Tensor(a!) master, Tensor(b!) exp_avg, Tensor(c!) exp_avg_sq, Tensor grad, Tensor(d!) param, Tensor(e!) wt, Tensor? clip_coef, float lr, float beta1, float beta2, float eps, float weight_decay, int step, int sr_base=0) -> ()");
  m.def("sumsq_(Tensor g, Tensor(a!) out) -> ()");
  m.def("transpose_(Tensor src, Tensor(a!) dst) -> ()");
  m.def("embedding_bwd_(Tensor(a!) grad, Tensor dy, Tensor sorted_ids, Tensor order) -> ()");
  m.def("xent_fwd(Tensor logits, Tensor target, int vocab_start) -> Tensor[]");
  m.def("xent_bwd_(Tensor logits, Tensor target, int vocab_start, Tensor lse, Tensor dloss, Tensor(a!) dlogits) -> ()");
  m.def("flash_fwd(Tensor q, Tensor k, Tensor v, float scale, bool causal, int q_offset, int k_offset) -> Tensor[]");
  m.def("flash_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, float scale, bool causal, int q_offset, int k_offset, Tensor(a!)? dq_out=None, Tensor(b!)? dk_out=None, Tensor(c!)? dv_out=None, int ds_mode=-1) -> Tensor[]");
  m.def("flash_bwd_kv(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, float scale, bool causal, int q_offset, int k_offset, Tensor(a!)? dk_out=None, Tensor(b!)? dv_out=None) -> Tensor[]");
  m.def("flash_bwd_q_ds(Tensor q, Tensor k, Tensor ws, float scale, bool causal, int q_offset, int k_offset, Tensor(a!)? dq_out=None) -> Tensor");
  m.def("wgrad_gemm_(Tensor(a!) out, Tensor dy, Tensor x, int beta, int variant=0) -> bool");
  m.def("wgrad_grouped_(Tensor(a!) out, Tensor dy, Tensor x, Tensor offs, int beta) -> bool");
  m.def("grouped_gemm(Tensor x, Tensor w, Tensor offs, bool wn) -> Tensor");
  m.def("grouped_gemm_swiglu(Tensor x, Tensor w, Tensor offs) -> Tensor[]");
  m.def("gemm_swiglu(Tensor x, Tensor w) -> Tensor[]");
  m.def("gemm4w_swiglu_grouped(Tensor x, Tensor w, Tensor offs) -> Tensor[]");
  m.def("gemm4w(Tensor x, Tensor w, Tensor offs) -> Tensor");
  m.def("grouped_gemm_dswiglu(Tensor dy, Tensor w, Tensor offs, Tensor gu) -> Tensor");
  m.def("xgmi_create(int rank, int world, int cap, int epoch_base) -> int", &xgmi_create);
  m.def("xgmi_handle(int id) -> Tensor", &xgmi_handle);
  m.def("xgmi_open(int id, int r, Tensor handle) -> ()", &xgmi_open);
  m.def("xgmi_set_peer(int id, int r, int peer) -> ()", &xgmi_set_peer);
  m.def("xgmi_all_reduce(int id, Tensor inp, Tensor(a!) out, int mode, int blocks) -> ()", &xgmi_all_reduce);
  m.def("xgmi_all_reduce_sim(int[] ids, Tensor[] ins, Tensor(a!)[] outs, int mode, int blocks, int[]? partners=None) -> ()",
        &xgmi_all_reduce_sim);
  m.def("xgmi_pair(int id, Tensor inp, Tensor(a!) out, int mode, int partner, int blocks) -> ()", &xgmi_pair);
  m.def("xgmi_error(int id) -> int", &xgmi_error);
  m.def("xgmi_ep_exchange(int id, Tensor inp, Tensor(a!) out, Tensor M, int El, int dir, int area_rows, int blocks) -> ()",
        &xgmi_ep_exchange);
  m.def("xgmi_ep_exchange_sim(int[] ids, Tensor[] ins, Tensor(a!)[] outs, Tensor M, int El, int dir, int area_rows, int blocks) -> ()",
        &xgmi_ep_exchange_sim);
  m.def("xgmi_set_timeout(int id, float seconds) -> ()", &xgmi_set_timeout);
  m.def("xgmi_destroy(int id) -> ()", &xgmi_destroy);
  m.def("qknorm_rope_fwd_(Tensor(a!) qkv, Tensor wq, Tensor wk, Tensor cos, Tensor sin, Tensor? pos, int H, int Hkv, float eps) -> Tensor[]");
  m.def("qknorm_rope_bwd_(Tensor(a!) dqkv, Tensor xsave, Tensor rstd, Tensor wq, Tensor wk, Tensor cos, Tensor sin, Tensor? pos, int H, int Hkv) -> Tensor");
  m.def("lse_merge_(Tensor(a!) out, Tensor(b!) lse, Tensor block_out, Tensor block_lse) -> ()");
}

TORCH_LIBRARY_IMPL(st_amd, CUDA, m) {
  m.impl("rmsnorm_fwd", &rmsnorm_fwd);
  m.impl("rmsnorm_bwd", &rmsnorm_bwd);
  m.impl("rope_", &rope_);
  m.impl("swiglu_fwd", &swiglu_fwd);
  m.impl("swiglu_bwd", &swiglu_bwd);
  m.impl("adamw_step_", &adamw_step_);
  m.impl("adamw_wt_step_", &adamw_wt_step_);
  m.impl("sumsq_", &sumsq_);
  m.impl("transpose_", &transpose_);
  m.impl("embedding_bwd_", &embedding_bwd_);
  m.impl("xent_fwd", &xent_fwd);
  m.impl("xent_bwd_", &xent_bwd_);
  m.impl("flash_fwd", &flash_fwd);
  m.impl("flash_bwd", &flash_bwd);
  m.impl("flash_bwd_kv", &flash_bwd_kv);
  m.impl("flash_bwd_q_ds", &flash_bwd_q_ds);
  m.impl("lse_merge_", &lse_merge_);
  m.impl("wgrad_gemm_", &wgrad_gemm_);
  m.impl("wgrad_grouped_", &wgrad_grouped_);
  m.impl("grouped_gemm", &grouped_gemm);
  m.impl("grouped_gemm_swiglu", &grouped_gemm_swiglu);
  m.impl("gemm_swiglu", &gemm_swiglu);
  m.impl("gemm4w_swiglu_grouped", &gemm4w_swiglu_grouped);
  m.impl("gemm4w", &gemm4w);
  m.impl("grouped_gemm_dswiglu", &grouped_gemm_dswiglu);
  m.impl("qknorm_rope_fwd_", &qknorm_rope_fwd_);
  m.impl("qknorm_rope_bwd_", &qknorm_rope_bwd_);
}

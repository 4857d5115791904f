// torch.ops.st_amd.moe_* registrations for csrc/moe.hip (host-side shape
// checks + output allocation; kernels launched on the current HIP stream).
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

extern "C" {
int st_moe_topk_softmax(const float* logits, int T, int E, int k, int renorm, float* probs, float* topw, int* topi,
                        hipStream_t st);
int st_moe_permute_workspace_ints(int64_t n, int E);
int st_moe_permute(const int* ids, int64_t n, int E, int* workspace, int* pos, int* sorted_entry, int* counts,
                   int* offsets, hipStream_t st);
int st_moe_gather_rows(const void* x, const int* sorted_entry, int64_t rows, int h, int k, void* xs, hipStream_t st);
int st_moe_combine(const void* y, const float* w, const int* pos, int64_t T, int h, int k, void* out, hipStream_t st);
int st_moe_combine_bwd(const void* dout, const void* y, const float* w, const int* pos, const int* sorted_entry,
                       int64_t T, int h, int k, void* dy, float* dw, hipStream_t st);
}

namespace {

inline hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define MOE_RC(rc, name) TORCH_CHECK((rc) == 0, "st_amd::" name " launch failed with code ", (rc))

void need(const at::Tensor& t, at::ScalarType dt, int dim, const char* name, const at::Tensor* ref = nullptr) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == dt && t.dim() == dim && t.is_contiguous(), "moe: ", name,
              " must be a contiguous ", dim, "-D ", dt, " GPU tensor");
  if (ref) TORCH_CHECK(t.device() == ref->device(), "moe: ", name, " on a different device");
}

// logits fp32 [T, E] -> probs fp32 [T, E], topw fp32 [T, k], topi int32 [T, k]
std::vector<at::Tensor> moe_topk_softmax(const at::Tensor& logits, int64_t k, bool renorm) {
  need(logits, at::kFloat, 2, "logits");
  const int64_t T = logits.size(0), E = logits.size(1);
  TORCH_CHECK(k >= 1 && k <= 8 && k <= E && E <= 512, "moe_topk_softmax: need 1 <= k <= min(8, E), E <= 512");
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  auto probs = at::empty_like(logits);
  auto topw = at::empty({T, k}, logits.options());
  auto topi = at::empty({T, k}, logits.options().dtype(at::kInt));
  MOE_RC(st_moe_topk_softmax(logits.data_ptr<float>(), (int)T, (int)E, (int)k, renorm ? 1 : 0,
                             probs.data_ptr<float>(), topw.data_ptr<float>(), topi.data_ptr<int>(), stream()),
         "moe_topk_softmax");
  return {probs, topw, topi};
}

// ids int32 [n] in [0, E) -> pos [n], sorted_entry [n], counts [E], offsets [E+1]  (stable by entry)
std::vector<at::Tensor> moe_permute(const at::Tensor& ids, int64_t E) {
  need(ids, at::kInt, 1, "ids");
  const int64_t n = ids.size(0);
  TORCH_CHECK(E >= 1 && E <= 4096, "moe_permute: 1 <= E <= 4096");
  c10::hip::HIPGuardMasqueradingAsCUDA g(ids.device());
  auto opt = ids.options();
  auto ws = at::empty({std::max<int64_t>(1, st_moe_permute_workspace_ints(n, (int)E))}, opt);
  auto pos = at::empty({n}, opt), sorted = at::empty({n}, opt);
  auto counts = at::empty({E}, opt), offsets = at::empty({E + 1}, opt);
  MOE_RC(st_moe_permute(ids.data_ptr<int>(), n, (int)E, ws.data_ptr<int>(), pos.data_ptr<int>(),
                        sorted.data_ptr<int>(), counts.data_ptr<int>(), offsets.data_ptr<int>(), stream()),
         "moe_permute");
  return {pos, sorted, counts, offsets};
}

// x bf16 [T, h], sorted_entry int32 [T*k] -> xs bf16 [T*k, h] (row p = x[sorted_entry[p] / k])
at::Tensor moe_gather_rows(const at::Tensor& x, const at::Tensor& sorted_entry, int64_t k) {
  need(x, at::kBFloat16, 2, "x");
  need(sorted_entry, at::kInt, 1, "sorted_entry", &x);
  TORCH_CHECK(sorted_entry.size(0) == x.size(0) * k, "moe_gather_rows: sorted_entry must have T*k entries");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto xs = at::empty({sorted_entry.size(0), x.size(1)}, x.options());
  MOE_RC(st_moe_gather_rows(x.data_ptr(), sorted_entry.data_ptr<int>(), xs.size(0), (int)x.size(1), (int)k,
                            xs.data_ptr(), stream()),
         "moe_gather_rows");
  return xs;
}

// y bf16 [T*k, h] sorted rows, w fp32 [T, k] (None: weight 1), pos int32 [T*k] -> out bf16 [T, h]
at::Tensor moe_combine(const at::Tensor& y, const c10::optional<at::Tensor>& w, const at::Tensor& pos, int64_t k) {
  need(y, at::kBFloat16, 2, "y");
  need(pos, at::kInt, 1, "pos", &y);
  TORCH_CHECK(pos.size(0) == y.size(0) && y.size(0) % k == 0, "moe_combine: pos/y sizes");
  const int64_t T = y.size(0) / k;
  const float* wp = nullptr;
  if (w.has_value() && w->defined()) {
    need(*w, at::kFloat, 2, "w", &y);
    TORCH_CHECK(w->size(0) == T && w->size(1) == k, "moe_combine: w must be [T, k]");
    wp = w->data_ptr<float>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(y.device());
  auto out = at::empty({T, y.size(1)}, y.options());
  MOE_RC(st_moe_combine(y.data_ptr(), wp, pos.data_ptr<int>(), T, (int)y.size(1), (int)k, out.data_ptr(), stream()),
         "moe_combine");
  return out;
}

// -> dy bf16 [T*k, h] (sorted rows), dw fp32 [T, k] (empty when not needed)
std::vector<at::Tensor> moe_combine_bwd(const at::Tensor& dout, const at::Tensor& y, const at::Tensor& w,
                                        const at::Tensor& pos, const at::Tensor& sorted_entry, int64_t k,
                                        bool need_dw) {
  need(dout, at::kBFloat16, 2, "dout");
  need(y, at::kBFloat16, 2, "y", &dout);
  need(w, at::kFloat, 2, "w", &dout);
  need(pos, at::kInt, 1, "pos", &dout);
  need(sorted_entry, at::kInt, 1, "sorted_entry", &dout);
  const int64_t T = dout.size(0);
  TORCH_CHECK(y.size(0) == T * k && pos.size(0) == T * k && sorted_entry.size(0) == T * k && w.size(0) == T &&
                  w.size(1) == k && y.size(1) == dout.size(1),
              "moe_combine_bwd: shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA g(dout.device());
  auto dy = at::empty_like(y);
  at::Tensor dw = need_dw ? at::empty({T, k}, w.options()) : at::empty({0}, w.options());
  MOE_RC(st_moe_combine_bwd(dout.data_ptr(), y.data_ptr(), w.data_ptr<float>(), pos.data_ptr<int>(),
                            sorted_entry.data_ptr<int>(), T, (int)dout.size(1), (int)k, dy.data_ptr(),
                            need_dw ? dw.data_ptr<float>() : nullptr, stream()),
         "moe_combine_bwd");
  return {dy, dw};
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(st_amd, m) {
  m.def("moe_topk_softmax(Tensor logits, int k, bool renorm) -> Tensor[]");
  m.def("moe_permute(Tensor ids, int num_experts) -> Tensor[]");
  m.def("moe_gather_rows(Tensor x, Tensor sorted_entry, int k) -> Tensor");
  m.def("moe_combine(Tensor y, Tensor? w, Tensor pos, int k) -> Tensor");
  m.def("moe_combine_bwd(Tensor dout, Tensor y, Tensor w, Tensor pos, Tensor sorted_entry, int k, bool need_dw) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(st_amd, CUDA, m) {
  m.impl("moe_topk_softmax", &moe_topk_softmax);
  m.impl("moe_permute", &moe_permute);
  m.impl("moe_gather_rows", &moe_gather_rows);
  m.impl("moe_combine", &moe_combine);
  m.impl("moe_combine_bwd", &moe_combine_bwd);
}

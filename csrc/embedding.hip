// Deterministic embedding backward: grad[id] += sum of dY rows of every token
// that looked up `id`, summed in token order, without atomics.
//
// Reference: autograd's F.embedding backward (scaletorch/models/llama.py:382-420,
// embedding_dense_backward: atomics) -- fp32 atomics make the sum order, and so
// the result bits, differ run to run.  Here the token ids are sorted stably on
// device (torch.sort(stable=True): equal ids keep token order), and ONE workgroup
// per run of equal ids (the workgroup at the run's first position; the others
// exit) adds the run's rows in that order and updates the fp32 gradient row with
// a plain read-add-write: no two workgroups touch the same row.  One pass over
// dY (T x H bf16) plus one read-write of the touched gradient rows.
#include "common.h"

using namespace st;

namespace {

__global__ __launch_bounds__(256) void embedding_bwd_kernel(const int64_t* __restrict__ sorted_ids,
                                                            const int64_t* __restrict__ order,
                                                            const bf16_t* __restrict__ dy, int64_t ldd,
                                                            float* __restrict__ grad, int64_t ldg, int T, int H,
                                                            int64_t V) {
  const int i = blockIdx.x;
  const int64_t id = sorted_ids[i];
  if (i > 0 && sorted_ids[i - 1] == id) return;  // not the first position of its run
  if (id < 0 || id >= V) return;
  int j = i + 1;
  while (j < T && sorted_ids[j] == id) ++j;
  float* g = grad + id * ldg;
  for (int c = threadIdx.x * 4; c < H; c += blockDim.x * 4) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (int k = i; k < j; ++k) {
      const uint2 v = *reinterpret_cast<const uint2*>(dy + order[k] * ldd + c);
      a0 += __uint_as_float(v.x << 16);
      a1 += __uint_as_float(v.x & 0xffff0000u);
      a2 += __uint_as_float(v.y << 16);
      a3 += __uint_as_float(v.y & 0xffff0000u);
    }
    float4 o = *reinterpret_cast<const float4*>(g + c);
    o.x += a0;
    o.y += a1;
    o.z += a2;
    o.w += a3;
    *reinterpret_cast<float4*>(g + c) = o;
  }
}

}  // namespace

extern "C" int st_embedding_bwd(const int64_t* sorted_ids, const int64_t* order, const void* dy, int64_t ldd,
                                float* grad, int64_t ldg, int T, int H, int64_t V, hipStream_t st) {
  if (T <= 0) return 0;
  if (H % 4 || ldd % 4 || ldg % 4) return -2;
  embedding_bwd_kernel<<<(unsigned)T, 256, 0, st>>>(sorted_ids, order, (const bf16_t*)dy, ldd, grad, ldg, T, H, V);
  return (int)hipGetLastError();
}

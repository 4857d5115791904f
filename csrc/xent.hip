// Vocab-parallel softmax cross-entropy on bf16 logits.
//
// Reference: F.cross_entropy(logits.view(-1, V), targets) after an all-gather
// of the vocab-sharded logits (scaletorch/trainer/train_step.py:89-103,
// scaletorch/parallel/tensor_parallel/tensor_parallel.py:142/247).  Here each
// rank keeps its [N, V/tp] shard:
//   fwd: per row, local log-sum-exp and the target logit if the target id is
//        in this rank's [vocab_start, vocab_start + V_local) slice;
//        (the caller combines lse across TP ranks: only [N] floats move, never
//        the [N, V] logits);
//   bwd: dlogits = (exp(x - lse_global) - onehot) * dloss, written IN PLACE
//        over the logits when asked (no second [N, V] buffer).
// One 256-thread block per row, 16-byte loads, online (max, sum) per lane.
#include "common.h"

using namespace st;

namespace {

ST_DEVICE void merge_ms(float& m, float& s, float m2, float s2) {
  const float mx = fmaxf(m, m2);
  if (mx == -INFINITY) { m = mx; s = 0.f; return; }
  s = s * __expf(m - mx) + s2 * __expf(m2 - mx);
  m = mx;
}

__global__ __launch_bounds__(256) void xent_fwd_kernel(const bf16_t* __restrict__ logits, int64_t ld,
                                                        const int64_t* __restrict__ tgt, int V,
                                                        int64_t vocab_start, float* __restrict__ lse,
                                                        float* __restrict__ tlogit) {
  __shared__ float sm[4], ss[4];
  const int64_t row = blockIdx.x;
  const bf16_t* x = logits + row * ld;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
    float f[8];
    unpack8(ld8(x + c), f);
    float bm = f[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) bm = fmaxf(bm, f[i]);
    const float mx = fmaxf(m, bm);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += __expf(f[i] - mx);
    s = s * __expf(m - mx) + acc;
    m = mx;
  }
  // wave reduce of (m, s)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    merge_ms(m, s, m2, s2);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sm[wid] = m; ss[wid] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], Ssum = ss[0];
    for (int k = 1; k < 4; ++k) merge_ms(M, Ssum, sm[k], ss[k]);
    lse[row] = M + __logf(Ssum);
    const int64_t t = tgt[row] - vocab_start;
    tlogit[row] = (t >= 0 && t < V) ? bf2f(x[t]) : 0.f;
  }
}

__global__ __launch_bounds__(256) void xent_bwd_kernel(const bf16_t* __restrict__ logits, int64_t ld,
                                                        const int64_t* __restrict__ tgt, int V,
                                                        int64_t vocab_start, const float* __restrict__ lse,
                                                        const float* __restrict__ dloss,
                                                        bf16_t* __restrict__ dlogits, int64_t ldd) {
  const int64_t row = blockIdx.x;
  const bf16_t* x = logits + row * ld;
  bf16_t* dx = dlogits + row * ldd;
  const float L = lse[row], d = dloss[row];
  const int64_t t = tgt[row] - vocab_start;
  for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
    float f[8], o[8];
    unpack8(ld8(x + c), f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float p = __expf(f[i] - L);
      o[i] = (p - ((int64_t)(c + i) == t ? 1.f : 0.f)) * d;
    }
    st8(dx + c, pack8(o));
  }
}

}  // namespace

extern "C" {

int st_xent_fwd(const void* logits, int64_t ld, const int64_t* tgt, int64_t N, int V,
                int64_t vocab_start, float* lse, float* tlogit, hipStream_t st) {
  if (V % 8 != 0 || ld % 8 != 0) return -2;
  if (N == 0) return 0;
  xent_fwd_kernel<<<dim3((unsigned)N), 256, 0, st>>>((const bf16_t*)logits, ld, tgt, V, vocab_start,
                                                    lse, tlogit);
  return (int)hipGetLastError();
}

int st_xent_bwd(const void* logits, int64_t ld, const int64_t* tgt, int64_t N, int V,
                int64_t vocab_start, const float* lse, const float* dloss, void* dlogits,
                int64_t ldd, hipStream_t st) {
  if (V % 8 != 0 || ld % 8 != 0 || ldd % 8 != 0) return -2;
  if (N == 0) return 0;
  xent_bwd_kernel<<<dim3((unsigned)N), 256, 0, st>>>((const bf16_t*)logits, ld, tgt, V, vocab_start,
                                                    lse, dloss, (bf16_t*)dlogits, ldd);
  return (int)hipGetLastError();
}

}  // extern "C"

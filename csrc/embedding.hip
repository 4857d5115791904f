// Deterministic embedding backward: grad[id] += sum of dY rows of every token
// that looked up `id`, summed in a fixed order, without atomics.
//
// Reference: autograd's F.embedding backward (scaletorch/models/llama.py:382-420,
// embedding_dense_backward: atomics) -- fp32 atomics make the sum order, and so
// the result bits, differ run to run.  Here the token ids are sorted stably on
// device (torch.sort(stable=True): equal ids keep token order).  A "run" is a
// range of equal sorted ids; each workgroup finds its run by binary search in the
// sorted ids (2 x log2 T scalar loads, no host work, no extra passes).
//
//  * short run (<= kSeg rows): the workgroup at the run's first position adds the
//    run's rows in order and updates the fp32 gradient row (read-add-write: no two
//    workgroups touch the same row);
//  * long run (a pad / EOS id, or many tokens of one id): cut at ABSOLUTE kSeg
//    blocks of the sorted positions, so one long run is summed by ~len/kSeg
//    workgroups in parallel instead of one CU reading it serially.  The piece of a
//    run inside block b goes to partial[b][sub]; a block meets at most two long
//    runs (a long run that starts inside a block outlasts it), so sub = 0 for the
//    piece covering the block start and 1 for a run that starts inside the block.
//    A second kernel sums a long run's pieces in block order into the gradient row.
// Both passes use fixed summation orders: bitwise reproducible.  Ids < 0 (masked
// tokens, e.g. out-of-shard ids under TP) sort first and are skipped.
#include "common.h"

using namespace st;

namespace {

constexpr int kSeg = 64;  // sorted positions per block; longer runs are split

// first index in [0, T) with s[idx] >= id (lower) / > id (upper)
ST_DEVICE int lower_bound(const int64_t* s, int T, int64_t id) {
  int lo = 0, hi = T;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (s[mid] < id) lo = mid + 1; else hi = mid;
  }
  return lo;
}

ST_DEVICE int upper_bound(const int64_t* s, int T, int64_t id) {
  int lo = 0, hi = T;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (s[mid] <= id) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// sum dY rows order[k], k in [a, b), columns [c, c+4) -> fp32 x4
ST_DEVICE float4 sum_rows(const int64_t* __restrict__ order, const bf16_t* __restrict__ dy, int64_t ldd, int a,
                          int b, int c) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  for (int k = a; k < b; ++k) {
    const uint2 v = *reinterpret_cast<const uint2*>(dy + order[k] * ldd + c);
    a0 += __uint_as_float(v.x << 16);
    a1 += __uint_as_float(v.x & 0xffff0000u);
    a2 += __uint_as_float(v.y << 16);
    a3 += __uint_as_float(v.y & 0xffff0000u);
  }
  return make_float4(a0, a1, a2, a3);
}

__global__ __launch_bounds__(256) void embedding_bwd_kernel(const int64_t* __restrict__ sorted_ids,
                                                            const int64_t* __restrict__ order,
                                                            const bf16_t* __restrict__ dy, int64_t ldd,
                                                            float* __restrict__ grad, int64_t ldg,
                                                            float* __restrict__ partial, int T, int H,
                                                            int64_t V) {
  const int i = blockIdx.x;
  const int64_t id = sorted_ids[i];
  if (id < 0 || id >= V) return;
  const bool run_head = (i == 0 || sorted_ids[i - 1] != id);
  const bool block_head = (i % kSeg) == 0;
  if (!run_head && !block_head) return;  // neither a run start nor a block start
  const int rs = run_head ? i : lower_bound(sorted_ids, i, id);
  const int re = upper_bound(sorted_ids + i, T - i, id) + i;
  if (re - rs <= kSeg) {
    if (!run_head) return;
    float* g = grad + id * ldg;
    for (int c = threadIdx.x * 4; c < H; c += blockDim.x * 4) {
      const float4 s = sum_rows(order, dy, ldd, rs, re, c);
      float4 o = *reinterpret_cast<const float4*>(g + c);
      o.x += s.x;
      o.y += s.y;
      o.z += s.z;
      o.w += s.w;
      *reinterpret_cast<float4*>(g + c) = o;
    }
    return;
  }
  // long run: this workgroup owns the run's piece inside block b = i / kSeg
  const int b = i / kSeg;
  const int end = min(re, (b + 1) * kSeg);
  const int sub = (rs > b * kSeg) ? 1 : 0;
  float* p = partial + ((int64_t)b * 2 + sub) * H;
  for (int c = threadIdx.x * 4; c < H; c += blockDim.x * 4)
    *reinterpret_cast<float4*>(p + c) = sum_rows(order, dy, ldd, i, end, c);
}

// second pass: the head of every long run adds its pieces, in block order
__global__ __launch_bounds__(256) void embedding_bwd_reduce_kernel(const int64_t* __restrict__ sorted_ids,
                                                                   float* __restrict__ grad, int64_t ldg,
                                                                   const float* __restrict__ partial, int T, int H,
                                                                   int64_t V) {
  const int i = blockIdx.x;
  const int64_t id = sorted_ids[i];
  if (id < 0 || id >= V) return;
  if (i > 0 && sorted_ids[i - 1] == id) return;
  const int re = upper_bound(sorted_ids + i, T - i, id) + i;
  if (re - i <= kSeg) return;
  const int b0 = i / kSeg, b1 = (re - 1) / kSeg;
  float* g = grad + id * ldg;
  for (int c = threadIdx.x * 4; c < H; c += blockDim.x * 4) {
    float4 o = *reinterpret_cast<const float4*>(g + c);
    for (int b = b0; b <= b1; ++b) {
      const int sub = (b == b0 && i > b * kSeg) ? 1 : 0;
      const float4 s = *reinterpret_cast<const float4*>(partial + ((int64_t)b * 2 + sub) * H + c);
      o.x += s.x;
      o.y += s.y;
      o.z += s.z;
      o.w += s.w;
    }
    *reinterpret_cast<float4*>(g + c) = o;
  }
}

}  // namespace

// partial: scratch of st_embedding_bwd_partial_floats(T, H) floats
extern "C" int64_t st_embedding_bwd_partial_floats(int T, int H) {
  return (int64_t)((T + kSeg - 1) / kSeg) * 2 * H;
}

extern "C" int st_embedding_bwd(const int64_t* sorted_ids, const int64_t* order, const void* dy, int64_t ldd,
                                float* grad, int64_t ldg, float* partial, int T, int H, int64_t V, hipStream_t st) {
  if (T <= 0) return 0;
  if (H % 4 || ldd % 4 || ldg % 4) return -2;
  embedding_bwd_kernel<<<(unsigned)T, 256, 0, st>>>(sorted_ids, order, (const bf16_t*)dy, ldd, grad, ldg, partial,
                                                    T, H, V);
  embedding_bwd_reduce_kernel<<<(unsigned)T, 256, 0, st>>>(sorted_ids, grad, ldg, partial, T, H, V);
  return (int)hipGetLastError();
}

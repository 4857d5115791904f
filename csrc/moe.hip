// Mixture-of-Experts routing kernels for gfx950: fused softmax + top-k router,
// deterministic (stable) token permutation by expert, expert-row gather and
// the weighted combine -- forward and backward, no atomics on the data path.
//
// Reference behaviour: MoERouter / MoEExperts dispatch in
// scaletorch/models/model_qwen3_moe.py:30-171 (softmax -> topk -> renorm,
// per-expert `nonzero` gathers with host syncs, index_add combine).
//
// Layout conventions: T tokens, k slots per token, E experts.  An "entry" is
// (token t, slot s) at index i = t*k + s.  The permutation sorts entries by
// expert, ties in entry order (stable), so results are bitwise reproducible:
//   pos[i]         : row of entry i in the expert-sorted buffer
//   sorted_entry[p]: entry at sorted row p (inverse of pos)
//   counts[e], offsets[e] (exclusive prefix of counts)
#include "common.h"

using namespace st;

namespace {

// ---------------------------------------------------------------- router
// One wave per token: softmax over E logits (fp32), top-k by k rounds of a
// wave-wide argmax (ties -> lower expert id, like torch.topk on equal values
// in practice), optional renormalisation of the selected probabilities.
template <int EPL>  // experts per lane (E <= 64 * EPL)
__global__ __launch_bounds__(256) void topk_softmax_kernel(const float* __restrict__ logits, int T, int E, int k,
                                                           int renorm, float* __restrict__ probs,
                                                           float* __restrict__ topw, int* __restrict__ topi) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const float* row = logits + (int64_t)t * E;
  float v[EPL];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    const int e = lane + 64 * j;
    v[j] = e < E ? row[e] : -INFINITY;
    mx = fmaxf(mx, v[j]);
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    const int e = lane + 64 * j;
    v[j] = e < E ? __expf(v[j] - mx) : 0.f;
    sum += v[j];
  }
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    const int e = lane + 64 * j;
    v[j] *= inv;
    if (e < E) probs[(int64_t)t * E + e] = v[j];
  }
  float selsum = 0.f;
  float selw[8];
  int seli[8];
  for (int s = 0; s < k; ++s) {
    float best = -1.f;
    int bi = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      const int e = lane + 64 * j;
      if (e < E && (v[j] > best || (v[j] == best && e < bi))) {
        best = v[j];
        bi = e;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) {
        best = ob;
        bi = oi;
      }
    }
    selw[s] = best;
    seli[s] = bi;
    selsum += best;
    // knock the winner out
#pragma unroll
    for (int j = 0; j < EPL; ++j)
      if (lane + 64 * j == bi) v[j] = -2.f;
  }
  if (lane < k) {
    float w = 0.f;
    int id = 0;
    for (int s = 0; s < k; ++s)
      if (s == lane) {
        w = selw[s];
        id = seli[s];
      }
    topw[(int64_t)t * k + lane] = renorm ? w / selsum : w;
    topi[(int64_t)t * k + lane] = id;
  }
}

// ---------------------------------------------------------------- permutation
constexpr int kBlockEntries = 1024;

// A: per-block expert histogram
__global__ __launch_bounds__(256) void hist_kernel(const int* __restrict__ ids, int64_t n, int E,
                                                   int* __restrict__ block_counts) {
  extern __shared__ int h[];
  for (int e = threadIdx.x; e < E; e += 256) h[e] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kBlockEntries;
  for (int i = threadIdx.x; i < kBlockEntries; i += 256) {
    const int64_t g = base + i;
    if (g < n) atomicAdd(&h[ids[g]], 1);  // LDS counter: order-independent
  }
  __syncthreads();
  for (int e = threadIdx.x; e < E; e += 256) block_counts[(int64_t)blockIdx.x * E + e] = h[e];
}

// B: one workgroup: expert totals, exclusive offsets, per-(block, expert) bases
__global__ __launch_bounds__(256) void scan_kernel(const int* __restrict__ block_counts, int nblocks, int E,
                                                   int* __restrict__ block_base, int* __restrict__ counts,
                                                   int* __restrict__ offsets) {
  extern __shared__ int tot[];
  for (int e = threadIdx.x; e < E; e += 256) {
    int run = 0;
    for (int b = 0; b < nblocks; ++b) {
      block_base[(int64_t)b * E + e] = run;
      run += block_counts[(int64_t)b * E + e];
    }
    tot[e] = run;
    counts[e] = run;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int e = 0; e < E; ++e) {
      offsets[e] = run;
      run += tot[e];
    }
    offsets[E] = run;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < E; e += 256) {
    const int off = offsets[e];
    for (int b = 0; b < nblocks; ++b) block_base[(int64_t)b * E + e] += off;
  }
}

// C: one wave per block walks its entries in order; rank among equal experts
// inside each 64-entry group via shuffles -> stable positions.
__global__ __launch_bounds__(64) void rank_kernel(const int* __restrict__ ids, int64_t n, int E,
                                                  const int* __restrict__ block_base, int* __restrict__ pos,
                                                  int* __restrict__ sorted_entry) {
  extern __shared__ int cur[];
  const int lane = threadIdx.x;
  for (int e = lane; e < E; e += 64) cur[e] = block_base[(int64_t)blockIdx.x * E + e];
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kBlockEntries;
  for (int g = 0; g < kBlockEntries; g += 64) {
    const int64_t i = base + g + lane;
    const bool valid = i < n;
    const int e = valid ? ids[i] : -1;
    int before = 0, total = 0;
    for (int j = 0; j < 64; ++j) {
      const int ej = __shfl(e, j, 64);
      before += (j < lane && ej == e) ? 1 : 0;
      total += (ej == e) ? 1 : 0;
    }
    int p = 0;
    if (valid) p = cur[e] + before;
    __syncthreads();  // every lane read cur[] before it moves
    if (valid && before + 1 == total) cur[e] += total;  // last lane of each expert group
    __syncthreads();
    if (valid) {
      pos[i] = p;
      sorted_entry[p] = (int)i;
    }
  }
}

// D: sorted rows <- token rows (16-B vectors)
__global__ __launch_bounds__(256) void gather_rows_kernel(const bf16_t* __restrict__ x, const int* __restrict__ sorted_entry,
                                                          int64_t rows, int h8, int k, bf16_t* __restrict__ xs) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= rows * h8) return;
  const int64_t p = t / h8;
  const int c = (int)(t % h8);
  const int64_t tok = sorted_entry[p] / k;
  st8(xs + p * (int64_t)h8 * 8 + c * 8, ld8(x + tok * (int64_t)h8 * 8 + c * 8));
}

// out[t] = sum_s w[t,s] * y[pos[t*k+s]]   (w == nullptr: plain sum, the permute backward)
__global__ __launch_bounds__(256) void combine_kernel(const bf16_t* __restrict__ y, const float* __restrict__ w,
                                                      const int* __restrict__ pos, int64_t T, int h8, int k,
                                                      bf16_t* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= T * h8) return;
  const int64_t tok = t / h8;
  const int c = (int)(t % h8);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < k; ++s) {
    const int64_t e = tok * k + s;
    const float ws = w ? w[e] : 1.f;
    float v[8];
    unpack8(ld8(y + (int64_t)pos[e] * h8 * 8 + c * 8), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += ws * v[j];
  }
  st8(out + tok * (int64_t)h8 * 8 + c * 8, pack8(acc));
}

// combine backward, sorted side: dy[p] = w[e] * dout[e / k]   (e = sorted_entry[p])
__global__ __launch_bounds__(256) void combine_bwd_rows_kernel(const bf16_t* __restrict__ dout,
                                                               const float* __restrict__ w,
                                                               const int* __restrict__ sorted_entry, int64_t rows,
                                                               int h8, int k, bf16_t* __restrict__ dy) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= rows * h8) return;
  const int64_t p = t / h8;
  const int c = (int)(t % h8);
  const int e = sorted_entry[p];
  const float ws = w[e];
  float v[8];
  unpack8(ld8(dout + (int64_t)(e / k) * h8 * 8 + c * 8), v);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] *= ws;
  st8(dy + p * (int64_t)h8 * 8 + c * 8, pack8(v));
}

// combine backward, weights: dw[e] = <dout[e / k], y[pos[e]]>   (one wave per entry)
__global__ __launch_bounds__(256) void combine_bwd_w_kernel(const bf16_t* __restrict__ dout,
                                                            const bf16_t* __restrict__ y, const int* __restrict__ pos,
                                                            int64_t n, int h8, int k, float* __restrict__ dw) {
  const int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (e >= n) return;
  const bf16_t* a = dout + (e / k) * (int64_t)h8 * 8;
  const bf16_t* b = y + (int64_t)pos[e] * h8 * 8;
  float acc = 0.f;
  for (int c = lane; c < h8; c += 64) {
    float va[8], vb[8];
    unpack8(ld8(a + c * 8), va);
    unpack8(ld8(b + c * 8), vb);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += va[j] * vb[j];
  }
  acc = wave_sum(acc);
  if (lane == 0) dw[e] = acc;
}

inline unsigned blocks_for(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

}  // namespace

extern "C" {

int st_moe_topk_softmax(const float* logits, int T, int E, int k, int renorm, float* probs, float* topw, int* topi,
                        hipStream_t st) {
  if (k < 1 || k > 8 || k > E || E > 512) return -2;
  if (T == 0) return 0;
  const unsigned g = blocks_for(T, 4);
  if (E <= 64) topk_softmax_kernel<1><<<g, 256, 0, st>>>(logits, T, E, k, renorm, probs, topw, topi);
  else if (E <= 128) topk_softmax_kernel<2><<<g, 256, 0, st>>>(logits, T, E, k, renorm, probs, topw, topi);
  else if (E <= 256) topk_softmax_kernel<4><<<g, 256, 0, st>>>(logits, T, E, k, renorm, probs, topw, topi);
  else topk_softmax_kernel<8><<<g, 256, 0, st>>>(logits, T, E, k, renorm, probs, topw, topi);
  return (int)hipGetLastError();
}

int st_moe_permute_workspace_ints(int64_t n, int E) {
  const int64_t nb = (n + kBlockEntries - 1) / kBlockEntries;
  return (int)(2 * nb * E);
}

// ids [n] (expert of every entry) -> pos [n], sorted_entry [n], counts [E], offsets [E+1]
int st_moe_permute(const int* ids, int64_t n, int E, int* workspace, int* pos, int* sorted_entry, int* counts,
                   int* offsets, hipStream_t st) {
  if (E < 1 || E > 4096) return -2;
  if (n == 0) {
    hipMemsetAsync(counts, 0, E * sizeof(int), st);
    hipMemsetAsync(offsets, 0, (E + 1) * sizeof(int), st);
    return (int)hipGetLastError();
  }
  const int nb = (int)((n + kBlockEntries - 1) / kBlockEntries);
  int* block_counts = workspace;
  int* block_base = workspace + (int64_t)nb * E;
  hist_kernel<<<nb, 256, E * sizeof(int), st>>>(ids, n, E, block_counts);
  scan_kernel<<<1, 256, E * sizeof(int), st>>>(block_counts, nb, E, block_base, counts, offsets);
  rank_kernel<<<nb, 64, E * sizeof(int), st>>>(ids, n, E, block_base, pos, sorted_entry);
  return (int)hipGetLastError();
}

int st_moe_gather_rows(const void* x, const int* sorted_entry, int64_t rows, int h, int k, void* xs, hipStream_t st) {
  if (h % 8) return -2;
  if (rows == 0) return 0;
  const int h8 = h / 8;
  gather_rows_kernel<<<blocks_for(rows * h8, 256), 256, 0, st>>>((const bf16_t*)x, sorted_entry, rows, h8, k,
                                                                  (bf16_t*)xs);
  return (int)hipGetLastError();
}

int st_moe_combine(const void* y, const float* w, const int* pos, int64_t T, int h, int k, void* out, hipStream_t st) {
  if (h % 8) return -2;
  if (T == 0) return 0;
  const int h8 = h / 8;
  combine_kernel<<<blocks_for(T * h8, 256), 256, 0, st>>>((const bf16_t*)y, w, pos, T, h8, k, (bf16_t*)out);
  return (int)hipGetLastError();
}

int st_moe_combine_bwd(const void* dout, const void* y, const float* w, const int* pos, const int* sorted_entry,
                       int64_t T, int h, int k, void* dy, float* dw, hipStream_t st) {
  if (h % 8) return -2;
  if (T == 0) return 0;
  const int h8 = h / 8;
  const int64_t n = T * k;
  combine_bwd_rows_kernel<<<blocks_for(n * h8, 256), 256, 0, st>>>((const bf16_t*)dout, w, sorted_entry, n, h8, k,
                                                                    (bf16_t*)dy);
  if (dw)
    combine_bwd_w_kernel<<<blocks_for(n, 4), 256, 0, st>>>((const bf16_t*)dout, (const bf16_t*)y, pos, n, h8, k, dw);
  return (int)hipGetLastError();
}

}  // extern "C"

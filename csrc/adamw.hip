// Fused AdamW over FLAT parameter arenas + global-norm reduction.
//
// Reference: torch.optim.AdamW(fused=True) on bf16 params with bf16 states
// (scaletorch/trainer/model_builder.py:119-134) and a local clip_grad_norm_
// (scaletorch/trainer/train_step.py:122-136).  Here:
//   * every trainable tensor of one dtype lives in ONE contiguous arena, so the
//     whole optimizer step is ONE bandwidth-bound launch (no multi-tensor
//     chunk lists, no per-parameter launches);
//   * fp32 master weights + fp32 exp_avg/exp_avg_sq; the bf16 model copy is
//     written in the same pass;
//   * the clip coefficient is read from DEVICE memory (computed from the
//     all-reduced global norm), so clipping needs no host synchronisation;
//   * grads may be fp32 (main_grad arena) or bf16.
#include "common.h"

#include <cstdlib>

using namespace st;

namespace {

template <typename G>
ST_DEVICE float4 load_g4(const G* g, int64_t i);
template <>
ST_DEVICE float4 load_g4<float>(const float* g, int64_t i) {
  return ld4f(g + i);
}
template <>
ST_DEVICE float4 load_g4<bf16_t>(const bf16_t* g, int64_t i) {
  uint2 v = *reinterpret_cast<const uint2*>(g + i);
  return make_float4(__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u),
                     __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u));
}

template <typename G>
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ master, float* __restrict__ m,
                                                     float* __restrict__ v, const G* __restrict__ g,
                                                     bf16_t* __restrict__ p, const float* __restrict__ clip,
                                                     int64_t n4, float lr, float b1, float b2, float eps,
                                                     float wd, float bc1, float bc2_sqrt) {
  const float cs = clip ? *clip : 1.f;
  const float step = lr / bc1, decay = 1.f - lr * wd;
  // Two 16-B chunks per thread per iteration, all loads issued before any math
  // (10 independent HBM streams in flight per thread); every byte is touched
  // exactly once, so loads/stores are non-temporal (no L2 pollution).
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n4; t += 2 * stride) {
    int64_t ii[2] = {t * 4, (t + stride) * 4};
    const int nv = (t + stride < n4) ? 2 : 1;
    f32x4 w[2], mm[2], vv[2];
    float4 gg[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u < nv) {
        w[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(master + ii[u]));
        mm[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(m + ii[u]));
        vv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(v + ii[u]));
        gg[u] = load_g4<G>(g, ii[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u >= nv) continue;
      const float ga[4] = {gg[u].x, gg[u].y, gg[u].z, gg[u].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float gk = ga[k] * cs;
        mm[u][k] = b1 * mm[u][k] + (1.f - b1) * gk;
        vv[u][k] = b2 * vv[u][k] + (1.f - b2) * gk * gk;
        const float denom = sqrtf(vv[u][k]) / bc2_sqrt + eps;
        w[u][k] = w[u][k] * decay - step * mm[u][k] / denom;
      }
      __builtin_nontemporal_store(w[u], reinterpret_cast<f32x4*>(master + ii[u]));
      __builtin_nontemporal_store(mm[u], reinterpret_cast<f32x4*>(m + ii[u]));
      __builtin_nontemporal_store(vv[u], reinterpret_cast<f32x4*>(v + ii[u]));
      if (p) {
        uint2 o;
        o.x = pack_bf16x2(w[u][0], w[u][1]);
        o.y = pack_bf16x2(w[u][2], w[u][3]);
        *reinterpret_cast<uint2*>(p + ii[u]) = o;
      }
    }
  }
}

// Stage 1 of the squared L2 norm: per-block partial sums (deterministic).
template <typename G>
__global__ __launch_bounds__(256) void sumsq_kernel(const G* __restrict__ g, int64_t n4,
                                                     float* __restrict__ partial) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n4;
       t += (int64_t)gridDim.x * blockDim.x) {
    float4 v = load_g4<G>(g, t * 4);
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

// Stage 2: one block sums the partials and ADDS into out[0] (so several
// arenas can accumulate into one global sum of squares).
__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ partial, int n,
                                                            float* __restrict__ out) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) acc += partial[i];
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) out[0] += acc;
}

constexpr int kNormBlocks = 1024;

inline unsigned grid_for(int64_t n4) {
  int64_t b = (n4 + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (unsigned)b;
}

}  // namespace

extern "C" {

// ST_ADAMW_BLOCKS caps the grid (grid-stride loop): a small grid leaves most CUs
// to the GEMMs of the forward pass the side-stream update overlaps (optim.py).
static unsigned adamw_grid(int64_t n4) {
  const char* e = std::getenv("ST_ADAMW_BLOCKS");  // read per launch: same-process A/B (tools/ab_step.py)
  const long cap = e ? std::atol(e) : 0L;
  unsigned g = grid_for(n4);
  if (cap > 0 && g > (unsigned)cap) g = (unsigned)cap;
  return g;
}

int st_adamw_step(float* master, float* m, float* v, const void* g, int g_is_bf16, void* p,
                  const float* clip, int64_t n, float lr, float b1, float b2, float eps, float wd,
                  float bc1, float bc2_sqrt, hipStream_t st) {
  if (n % 4 != 0) return -2;
  const int64_t n4 = n / 4;
  if (n4 == 0) return 0;
  if (g_is_bf16)
    adamw_kernel<bf16_t><<<adamw_grid(n4), 256, 0, st>>>(master, m, v, (const bf16_t*)g, (bf16_t*)p,
                                                       clip, n4, lr, b1, b2, eps, wd, bc1, bc2_sqrt);
  else
    adamw_kernel<float><<<adamw_grid(n4), 256, 0, st>>>(master, m, v, (const float*)g, (bf16_t*)p,
                                                      clip, n4, lr, b1, b2, eps, wd, bc1, bc2_sqrt);
  return (int)hipGetLastError();
}

int st_sumsq_partials() { return kNormBlocks; }

// out[0] += sum(g^2).  `partial` must hold kNormBlocks floats.
int st_sumsq(const void* g, int g_is_bf16, int64_t n, float* partial, float* out, hipStream_t st) {
  if (n % 4 != 0) return -2;
  const int64_t n4 = n / 4;
  unsigned blocks = grid_for(n4);
  if (blocks > kNormBlocks) blocks = kNormBlocks;
  if (g_is_bf16)
    sumsq_kernel<bf16_t><<<blocks, 256, 0, st>>>((const bf16_t*)g, n4, partial);
  else
    sumsq_kernel<float><<<blocks, 256, 0, st>>>((const float*)g, n4, partial);
  sum_partials_kernel<<<1, 256, 0, st>>>(partial, (int)blocks, out);
  return (int)hipGetLastError();
}

}  // extern "C"

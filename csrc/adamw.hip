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
//   * grads may be fp32 (main_grad arena) or bf16;
//   * bf16 moments are stored with STOCHASTIC rounding: a hashed 16-bit offset per
//     (element, step, moment: the two halves of one 32-bit hash) is added to the fp32
//     bits before truncation, so the stored
//     moment is unbiased.  Round-to-nearest froze exp_avg_sq at beta2 = 0.999, where the
//     per-step change (0.1 %) is below bf16's half-ulp.  The hash is
//     mirrored bit-for-bit by scaletorch_amd/optim.py ``sr_offsets``.
#include "common.h"

#include <cstdlib>
#include <type_traits>

using namespace st;

namespace {

// Every byte these passes touch is touched once per step (gradients read by the norm and the
// update, parameters and W^T written for a forward that reads them long after), and the passes
// run on a side stream beside the forward / backward GEMMs: all their accesses carry the
// non-temporal hint, so the stream does not evict the GEMMs' re-read tiles from L2.
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
template <typename G>
ST_DEVICE float4 load_g4(const G* g, int64_t i);
template <>
ST_DEVICE float4 load_g4<float>(const float* g, int64_t i) {
  const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g + i));
  return make_float4(v[0], v[1], v[2], v[3]);
}
template <>
ST_DEVICE float4 load_g4<bf16_t>(const bf16_t* g, int64_t i) {
  const u32x2_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x2_t*>(g + i));
  return make_float4(__uint_as_float(v[0] << 16), __uint_as_float(v[0] & 0xffff0000u),
                     __uint_as_float(v[1] << 16), __uint_as_float(v[1] & 0xffff0000u));
}
ST_DEVICE void store_p4(bf16_t* p, uint32_t lo, uint32_t hi) {  // 4 bf16 parameters
  const u32x2_t v = {lo, hi};
  __builtin_nontemporal_store(v, reinterpret_cast<u32x2_t*>(p));
}
ST_DEVICE void store_wt8(bf16_t* p, const BF8& o) {  // 8 bf16 of W^T
  const u32x4_t v = {o.w[0], o.w[1], o.w[2], o.w[3]};
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4_t*>(p));
}

// Optimizer moments: fp32 (default) or bf16 (ST optimizer_state_dtype="bf16": the
// reference's own state precision, torch AdamW on bf16 params; the fp32 master
// weights stay).  bf16 moments cut the pass from 30 to 22 B/param.
template <typename S>
ST_DEVICE f32x4 load_s4(const S* s, int64_t i);
template <>
ST_DEVICE f32x4 load_s4<float>(const float* s, int64_t i) {
  return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(s + i));
}
template <>
ST_DEVICE f32x4 load_s4<bf16_t>(const bf16_t* s, int64_t i) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(s + i));
  f32x4 r;
  r[0] = __uint_as_float(v[0] << 16);
  r[1] = __uint_as_float(v[0] & 0xffff0000u);
  r[2] = __uint_as_float(v[1] << 16);
  r[3] = __uint_as_float(v[1] & 0xffff0000u);
  return r;
}
// 32-bit integer mixer (lowbias32): cheap, full avalanche; optim.py mirrors it in int64.
ST_DEVICE uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// key of one step; the element index is its ARENA index (launch base + local), so a ZeRO-1
// shard rounds exactly as the replicated arena does
ST_DEVICE uint32_t sr_key(uint32_t step) { return mix32(step * 0x9e3779b9u); }
// 16 random bits for exp_avg (low half) and 16 for exp_avg_sq (high half) of element idx:
// ONE mix per element (the high-word mix is shared by the 4 elements of a chunk)
ST_DEVICE uint32_t sr_hash(uint32_t lo, uint32_t hi_mix) { return mix32(lo ^ hi_mix); }
// stochastic fp32 -> bf16: add 16 random low bits, truncate; NaN / Inf keep the plain cast
ST_DEVICE uint32_t sr_bf16(float x, uint32_t r16) {
  const uint32_t u = __float_as_uint(x);
  if ((u & 0x7f800000u) == 0x7f800000u) return f2bf(x);
  return (u + r16) >> 16;
}

template <typename S>
ST_DEVICE void store_s4(S* s, int64_t i, f32x4 v, const uint32_t (&r)[4]);
template <>
ST_DEVICE void store_s4<float>(float* s, int64_t i, f32x4 v, const uint32_t (&)[4]) {
  __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(s + i));
}
template <>
ST_DEVICE void store_s4<bf16_t>(bf16_t* s, int64_t i, f32x4 v, const uint32_t (&r)[4]) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  u32x2 o;
  o[0] = sr_bf16(v[0], r[0]) | (sr_bf16(v[1], r[1]) << 16);
  o[1] = sr_bf16(v[2], r[2]) | (sr_bf16(v[3], r[3]) << 16);
  __builtin_nontemporal_store(o, reinterpret_cast<u32x2*>(s + i));
}
// random words of the 4 elements at arena index gi (a multiple of 4: one high word)
template <typename S>
ST_DEVICE void sr_words(int64_t gi, uint32_t key, uint32_t (&rm)[4], uint32_t (&rv)[4]) {
  if constexpr (std::is_same<S, bf16_t>::value) {
    const uint32_t hm = mix32((uint32_t)((uint64_t)gi >> 32) ^ key);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t h = sr_hash((uint32_t)gi + k, hm);
      rm[k] = h & 0xffffu;
      rv[k] = h >> 16;
    }
  }
}

// One element of the AdamW update, shared by the flat and the W^T-writing kernels so
// both compile to the same instruction sequence (explicit fmas, no contraction left to
// the scheduler): the fused pass is bitwise equal to the flat one.
ST_DEVICE void adam_elem(float& w, float& m, float& v, float g, float b1, float b2, float eps, float step,
                         float decay, float bc2_sqrt) {
#pragma clang fp contract(off)
  m = __builtin_fmaf(b1, m, (1.f - b1) * g);
  v = __builtin_fmaf(b2, v, ((1.f - b2) * g) * g);
  const float denom = sqrtf(v) / bc2_sqrt + eps;
  w = __builtin_fmaf(w, decay, -(step * (m / denom)));
}

template <typename G, typename S>
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ master, S* __restrict__ m,
                                                     S* __restrict__ v, const G* __restrict__ g,
                                                     bf16_t* __restrict__ p, const float* __restrict__ clip,
                                                     int64_t n4, float lr, float b1, float b2, float eps,
                                                     float wd, float bc1, float bc2_sqrt, uint32_t sr_step,
                                                     int64_t sr_base) {
  const float cs = clip ? *clip : 1.f;
  const float step = lr / bc1, decay = 1.f - lr * wd;
  const uint32_t key = sr_key(sr_step);
  // Two 4-element chunks per thread per iteration, all loads issued before any math
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
        mm[u] = load_s4<S>(m, ii[u]);
        vv[u] = load_s4<S>(v, ii[u]);
        gg[u] = load_g4<G>(g, ii[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u >= nv) continue;
      const float ga[4] = {gg[u].x, gg[u].y, gg[u].z, gg[u].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float wk = w[u][k], mk = mm[u][k], vk = vv[u][k];
        adam_elem(wk, mk, vk, ga[k] * cs, b1, b2, eps, step, decay, bc2_sqrt);
        w[u][k] = wk;
        mm[u][k] = mk;
        vv[u][k] = vk;
      }
      __builtin_nontemporal_store(w[u], reinterpret_cast<f32x4*>(master + ii[u]));
      uint32_t rm[4] = {}, rv[4] = {};
      sr_words<S>(ii[u] + sr_base, key, rm, rv);
      store_s4<S>(m, ii[u], mm[u], rm);
      store_s4<S>(v, ii[u], vv[u], rv);
      if (p) store_p4(p + ii[u], pack_bf16x2(w[u][0], w[u][1]), pack_bf16x2(w[u][2], w[u][3]));
    }
  }
}

// AdamW over ONE 2-D weight [R, C] (a contiguous run of the arena) that ALSO writes
// the updated bf16 weight transposed, W^T [C, R], for the data-gradient GEMM's TN
// layout (ops/grad.py): the side-stream transpose the next forward would launch per
// weight re-reads W (2 B/elt) in a separate pass -- here the update already holds the
// new values in registers, so W^T costs only its 2 B/elt of writes and no launch.
// Tile 64 x 64 per 256-thread workgroup: 16 lanes x 4 fp32 cover one 256-B row of
// master / m / v / g (4 passes of 16 rows, all loads issued before any math); the
// bf16 results go row-major to p and into a padded LDS tile, which is read back by
// columns so each lane stores 16 B of W^T (8 lanes = one 128-B W^T row segment).
constexpr int kWT = 64, kWLd = kWT + 2;

template <typename G, typename S>
__global__ __launch_bounds__(256) void adamw_wt_kernel(float* __restrict__ master, S* __restrict__ m,
                                                        S* __restrict__ v, const G* __restrict__ g,
                                                        bf16_t* __restrict__ p, bf16_t* __restrict__ wt,
                                                        const float* __restrict__ clip, int R, int C, float lr,
                                                        float b1, float b2, float eps, float wd, float bc1,
                                                        float bc2_sqrt, uint32_t sr_step, int64_t sr_base) {
  __shared__ bf16_t tile[kWT * kWLd];
  const float cs = clip ? *clip : 1.f;
  const float step = lr / bc1, decay = 1.f - lr * wd;
  // same keys and element indices as the flat kernel over this weight: bitwise-equal moments
  const uint32_t key = sr_key(sr_step);
  const int tiles_c = C / kWT;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int r0 = (b / tiles_c) * kWT, c0 = (b % tiles_c) * kWT;
  const int t = threadIdx.x;
  const int lc = (t & 15) * 4, lr0 = t >> 4;  // 4 columns of one row; rows lr0 + 16 * pass
  f32x4 w[4], mm[4], vv[4];
  float4 gg[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t i = (int64_t)(r0 + lr0 + 16 * u) * C + c0 + lc;
    w[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(master + i));
    mm[u] = load_s4<S>(m, i);
    vv[u] = load_s4<S>(v, i);
    gg[u] = load_g4<G>(g, i);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t i = (int64_t)(r0 + lr0 + 16 * u) * C + c0 + lc;
    const float ga[4] = {gg[u].x, gg[u].y, gg[u].z, gg[u].w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float wk = w[u][k], mk = mm[u][k], vk = vv[u][k];
      adam_elem(wk, mk, vk, ga[k] * cs, b1, b2, eps, step, decay, bc2_sqrt);
      w[u][k] = wk;
      mm[u][k] = mk;
      vv[u][k] = vk;
    }
    __builtin_nontemporal_store(w[u], reinterpret_cast<f32x4*>(master + i));
    uint32_t rm[4] = {}, rv[4] = {};
    sr_words<S>(i + sr_base, key, rm, rv);
    store_s4<S>(m, i, mm[u], rm);
    store_s4<S>(v, i, vv[u], rv);
    const uint32_t lo = pack_bf16x2(w[u][0], w[u][1]), hi = pack_bf16x2(w[u][2], w[u][3]);
    store_p4(p + i, lo, hi);
    // padded LDS row (132 B): 4-B aligned only
    uint32_t* d = reinterpret_cast<uint32_t*>(tile + (lr0 + 16 * u) * kWLd + lc);
    d[0] = lo;
    d[1] = hi;
  }
  __syncthreads();
  const int chunk = t & 7, row = t >> 3;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int oc = row + 32 * q;  // W^T row = W column
    BF8 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t a = tile[(chunk * 8 + 2 * j) * kWLd + oc];
      const uint32_t c = tile[(chunk * 8 + 2 * j + 1) * kWLd + oc];
      o.w[j] = a | (c << 16);
    }
    store_wt8(wt + (int64_t)(c0 + oc) * R + r0 + chunk * 8, o);
  }
}

template <typename S>
int launch_adamw_wt(float* master, S* m, S* v, const void* g, int g_is_bf16, void* p, void* wt,
                    const float* clip, int R, int C, float lr, float b1, float b2, float eps, float wd,
                    float bc1, float bc2_sqrt, uint32_t sr_step, int64_t sr_base, hipStream_t st) {
  if (R % kWT || C % kWT || R <= 0 || C <= 0) return -2;
  const int64_t blocks = (int64_t)(R / kWT) * (C / kWT);
  if (blocks > 0x7fffffff) return -3;
  if (g_is_bf16)
    adamw_wt_kernel<bf16_t, S><<<(unsigned)blocks, 256, 0, st>>>(master, m, v, (const bf16_t*)g, (bf16_t*)p,
                                                                 (bf16_t*)wt, clip, R, C, lr, b1, b2, eps, wd,
                                                                 bc1, bc2_sqrt, sr_step, sr_base);
  else
    adamw_wt_kernel<float, S><<<(unsigned)blocks, 256, 0, st>>>(master, m, v, (const float*)g, (bf16_t*)p,
                                                                (bf16_t*)wt, clip, R, C, lr, b1, b2, eps, wd,
                                                                bc1, bc2_sqrt, sr_step, sr_base);
  return 0;
}

// Stage 1 of the squared L2 norm: per-block partial sums (deterministic).
template <typename G>
__global__ __launch_bounds__(256) void sumsq_kernel(const G* __restrict__ g, int64_t n4,
                                                     float* __restrict__ partial) {
  __shared__ float red[4];
  // four independent 16-byte loads in flight per lane: with one (a load -> wait -> FMA chain)
  // the 1,024-block grid kept ~16 KiB per CU in flight and read at 2.15 TB/s
  // (profiles/r05/step_kernels_mbs6_v2.csv)
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  for (; t + 3 * stride < n4; t += 4 * stride) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = load_g4<G>(g, (t + u * stride) * 4);
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += v[u].x * v[u].x + v[u].y * v[u].y + v[u].z * v[u].z + v[u].w * v[u].w;
  }
  for (; t < n4; t += stride) {
    const float4 v = load_g4<G>(g, t * 4);
    a[0] += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  float acc = (a[0] + a[1]) + (a[2] + a[3]);
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

// ST_ADAMW_BLOCKS caps the grid (grid-stride loop): a small grid leaves most CUs
// to the GEMMs of the forward pass the side-stream update overlaps (optim.py).
unsigned adamw_grid(int64_t n4) {
  const char* e = std::getenv("ST_ADAMW_BLOCKS");  // read per launch: same-process A/B (tools/ab_step.py)
  const long cap = e ? std::atol(e) : 0L;
  unsigned g = grid_for(n4);
  if (cap > 0 && g > (unsigned)cap) g = (unsigned)cap;
  return g;
}

template <typename S>
void launch_adamw(float* master, S* m, S* v, const void* g, int g_is_bf16, void* p,
                         const float* clip, int64_t n4, float lr, float b1, float b2, float eps,
                         float wd, float bc1, float bc2_sqrt, uint32_t sr_step, int64_t sr_base, hipStream_t st) {
  if (g_is_bf16)
    adamw_kernel<bf16_t, S><<<adamw_grid(n4), 256, 0, st>>>(master, m, v, (const bf16_t*)g, (bf16_t*)p,
                                                          clip, n4, lr, b1, b2, eps, wd, bc1, bc2_sqrt, sr_step, sr_base);
  else
    adamw_kernel<float, S><<<adamw_grid(n4), 256, 0, st>>>(master, m, v, (const float*)g, (bf16_t*)p,
                                                         clip, n4, lr, b1, b2, eps, wd, bc1, bc2_sqrt, sr_step, sr_base);
}

}  // namespace

extern "C" {

// states_bf16: exp_avg / exp_avg_sq are bf16 arrays (else fp32)
int st_adamw_step(float* master, void* m, void* v, int states_bf16, const void* g, int g_is_bf16,
                  void* p, const float* clip, int64_t n, float lr, float b1, float b2, float eps,
                  float wd, float bc1, float bc2_sqrt, uint32_t sr_step, int64_t sr_base, hipStream_t st) {
  if (n % 4 != 0) return -2;
  const int64_t n4 = n / 4;
  if (n4 == 0) return 0;
  if (states_bf16)
    launch_adamw<bf16_t>(master, (bf16_t*)m, (bf16_t*)v, g, g_is_bf16, p, clip, n4, lr, b1, b2, eps, wd,
                         bc1, bc2_sqrt, sr_step, sr_base, st);
  else
    launch_adamw<float>(master, (float*)m, (float*)v, g, g_is_bf16, p, clip, n4, lr, b1, b2, eps, wd, bc1,
                        bc2_sqrt, sr_step, sr_base, st);
  return (int)hipGetLastError();
}

// AdamW over one [R, C] weight run + its bf16 transpose W^T [C, R] (see adamw_wt_kernel)
int st_adamw_wt_step(float* master, void* m, void* v, int states_bf16, const void* g, int g_is_bf16,
                     void* p, void* wt, int R, int C, const float* clip, float lr, float b1, float b2,
                     float eps, float wd, float bc1, float bc2_sqrt, uint32_t sr_step, int64_t sr_base, hipStream_t st) {
  const int rc = states_bf16
                     ? launch_adamw_wt<bf16_t>(master, (bf16_t*)m, (bf16_t*)v, g, g_is_bf16, p, wt, clip, R, C,
                                               lr, b1, b2, eps, wd, bc1, bc2_sqrt, sr_step, sr_base, st)
                     : launch_adamw_wt<float>(master, (float*)m, (float*)v, g, g_is_bf16, p, wt, clip, R, C, lr,
                                              b1, b2, eps, wd, bc1, bc2_sqrt, sr_step, sr_base, st);
  if (rc) return rc;
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

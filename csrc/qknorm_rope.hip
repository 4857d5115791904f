// Fused per-head QK-RMSNorm + RoPE for Qwen3-style attention, in place on the
// fused QKV GEMM output [N = B*S rows, H + 2*Hkv heads, D].
//
// Reference: Qwen3Attention (scaletorch/models/model_qwen3.py:179-180, :209-210:
// q_norm / k_norm per head BEFORE rotary) followed by apply_rotary_pos_emb
// (scaletorch/models/attention_utils.py:170-192).  Unfused that is, per layer:
// two .contiguous() copies of q and k, two RMSNorm launches, a torch.cat back into
// the QKV buffer and an in-place RoPE pass -- six HBM round trips of q and k and,
// backward, the mirror image plus weight-gradient column sums.  Here:
//   forward : one pass -- each row (token, head) of q and k is read once, its
//             pre-norm copy saved for backward, normalised (fp32 statistics),
//             scaled by the q- or k-norm weight, rotated and written back in place;
//   backward: one pass on the attention backward's dQ / dK (in place) -- inverse
//             rotation, RMSNorm backward, and per-block partial sums of the two
//             weight gradients (no atomics; a second tiny kernel adds the partials
//             in block order, so results are bitwise deterministic).
// Lane mapping: a row of D bf16 is D/16 lanes x (8 elements of the first half +
// the 8 rotation partners of the second half), so RoPE needs no cross-lane
// traffic and the sum of squares is a D/16-lane butterfly.
#include "common.h"

using namespace st;

namespace {

template <int D>
struct RowMap {
  static constexpr int L = D / 16;  // lanes per row (8 for D = 128, 4 for D = 64)
};

ST_DEVICE void ld8f(const float* p, float (&f)[8]) {
  float4 a = ld4f(p), b = ld4f(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

template <int D>
ST_DEVICE float row_sum(float v) {
#pragma unroll
  for (int o = 1; o < RowMap<D>::L; o <<= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// rows are (token n, head h) for h in [0, NQK = H + Hkv); 256 threads per block
template <int D>
__global__ __launch_bounds__(256) void qknorm_rope_fwd_kernel(
    bf16_t* __restrict__ qkv, bf16_t* __restrict__ xsave, float* __restrict__ rstd_out,
    const bf16_t* __restrict__ wq, const bf16_t* __restrict__ wk, const float* __restrict__ cos_t,
    const float* __restrict__ sin_t, const int64_t* __restrict__ pos, int64_t N, int S, int H, int NQK, int NHT,
    float eps, int64_t max_pos) {
  constexpr int L = RowMap<D>::L, HALF = D / 2;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int j = (int)(t % L);
  const int64_t row = t / L;  // n * NQK + h
  const bool live = row < N * NQK;
  const int64_t n = live ? row / NQK : 0;
  const int h = live ? (int)(row % NQK) : 0;
  float x1[8], x2[8];
  bf16_t* base = qkv + (n * NHT + h) * D + 8 * j;
  BF8 raw1{}, raw2{};
  if (live) {
    raw1 = ld8(base);
    raw2 = ld8(base + HALF);
  }
  unpack8(raw1, x1);
  unpack8(raw2, x2);
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) ss += x1[i] * x1[i] + x2[i] * x2[i];
  ss = row_sum<D>(ss);  // every lane of the row group takes part (no early return)
  if (!live) return;
  const float r = rsqrtf(ss / D + eps);
  // pre-norm copy for backward (rows of the saved buffer are [n, h] with NQK heads)
  bf16_t* sv = xsave + row * D + 8 * j;
  st8(sv, raw1);
  st8(sv + HALF, raw2);
  if (j == 0) rstd_out[row] = r;
  const bf16_t* w = h < H ? wq : wk;
  float w1[8], w2[8];
  unpack8(ld8(w + 8 * j), w1);
  unpack8(ld8(w + HALF + 8 * j), w2);
  int64_t p = pos ? pos[n] : (int64_t)(n % S);
  p = p < 0 ? 0 : (p >= max_pos ? max_pos - 1 : p);
  float c[8], sn[8];
  ld8f(cos_t + p * HALF + 8 * j, c);
  ld8f(sin_t + p * HALF + 8 * j, sn);
  float o1[8], o2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float y1 = x1[i] * r * w1[i], y2 = x2[i] * r * w2[i];
    o1[i] = y1 * c[i] - y2 * sn[i];
    o2[i] = y2 * c[i] + y1 * sn[i];
  }
  st8(base, pack8(o1));
  st8(base + HALF, pack8(o2));
}

// Backward, in place on dqkv's q / k heads.  Per block: grid-stride over rows;
// each lane keeps its 16 columns' weight-gradient partial for q and for k, the
// block reduces them over its row groups in LDS and writes partial[block][2][D].
template <int D>
__global__ __launch_bounds__(256) void qknorm_rope_bwd_kernel(
    bf16_t* __restrict__ dqkv, const bf16_t* __restrict__ xsave, const float* __restrict__ rstd,
    const bf16_t* __restrict__ wq, const bf16_t* __restrict__ wk, const float* __restrict__ cos_t,
    const float* __restrict__ sin_t, const int64_t* __restrict__ pos, int64_t N, int S, int H, int NQK, int NHT,
    int64_t max_pos, float* __restrict__ partial) {
  constexpr int L = RowMap<D>::L, HALF = D / 2, GROUPS = 256 / L;
  __shared__ float red[GROUPS][2 * D];
  const int j = threadIdx.x % L, grp = threadIdx.x / L;
  float aq1[8], aq2[8], ak1[8], ak2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) aq1[i] = aq2[i] = ak1[i] = ak2[i] = 0.f;
  float wq1[8], wq2[8], wk1[8], wk2[8];
  unpack8(ld8(wq + 8 * j), wq1);
  unpack8(ld8(wq + HALF + 8 * j), wq2);
  unpack8(ld8(wk + 8 * j), wk1);
  unpack8(ld8(wk + HALF + 8 * j), wk2);
  const int64_t rows = N * NQK;
  const int64_t rows_per_iter = (int64_t)gridDim.x * GROUPS;
  for (int64_t row0 = (int64_t)blockIdx.x * GROUPS; row0 < rows; row0 += rows_per_iter) {
    const int64_t row = row0 + grp;
    const bool live = row < rows;
    const int64_t n = live ? row / NQK : 0;
    const int h = live ? (int)(row % NQK) : 0;
    const bool isq = h < H;
    float g1[8], g2[8], x1[8], x2[8];
    bf16_t* base = dqkv + (n * NHT + h) * D + 8 * j;
    float r = 0.f;
    if (live) {
      unpack8(ld8(base), g1);
      unpack8(ld8(base + HALF), g2);
      unpack8(ld8(xsave + row * D + 8 * j), x1);
      unpack8(ld8(xsave + row * D + HALF + 8 * j), x2);
      r = rstd[row];
      int64_t p = pos ? pos[n] : (int64_t)(n % S);
      p = p < 0 ? 0 : (p >= max_pos ? max_pos - 1 : p);
      float c[8], sn[8];
      ld8f(cos_t + p * HALF + 8 * j, c);
      ld8f(sin_t + p * HALF + 8 * j, sn);
#pragma unroll
      for (int i = 0; i < 8; ++i) {  // inverse rotation: R(theta)^T
        const float a = g1[i] * c[i] + g2[i] * sn[i];
        const float b = g2[i] * c[i] - g1[i] * sn[i];
        g1[i] = a;
        g2[i] = b;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) g1[i] = g2[i] = x1[i] = x2[i] = 0.f;
    }
    float w1[8], w2[8];  // per-element select: stays in registers
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      w1[i] = isq ? wq1[i] : wk1[i];
      w2[i] = isq ? wq2[i] : wk2[i];
    }
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) dot += g1[i] * w1[i] * x1[i] + g2[i] * w2[i] * x2[i];
    dot = row_sum<D>(dot);
    if (live) {
      const float k3 = r * r * r * dot / D;
      float d1[8], d2[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        d1[i] = r * g1[i] * w1[i] - x1[i] * k3;
        d2[i] = r * g2[i] * w2[i] - x2[i] * k3;
        const float e1 = g1[i] * x1[i] * r, e2 = g2[i] * x2[i] * r;
        if (isq) {
          aq1[i] += e1;
          aq2[i] += e2;
        } else {
          ak1[i] += e1;
          ak2[i] += e2;
        }
      }
      st8(base, pack8(d1));
      st8(base + HALF, pack8(d2));
    }
  }
  // block reduction of the weight-gradient partials (fixed order: deterministic)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    red[grp][8 * j + i] = aq1[i];
    red[grp][HALF + 8 * j + i] = aq2[i];
    red[grp][D + 8 * j + i] = ak1[i];
    red[grp][D + HALF + 8 * j + i] = ak2[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * D; c += 256) {
    float s = 0.f;
    for (int g = 0; g < GROUPS; ++g) s += red[g][c];
    partial[(int64_t)blockIdx.x * 2 * D + c] = s;
  }
}

// out[c] += sum_p partial[p][c] for c < C (C % 4 == 0), in a fixed order: a block owns
// 64 columns (16 lanes x float4) and splits the P partial rows over 16 row groups whose
// sums fold through LDS in group order (one serial 512-row walk per column took 118 us
// per call: 7 % of a Qwen3-0.6B step).
__global__ __launch_bounds__(256) void partial_colsum_kernel(const float* __restrict__ partial, int P, int C,
                                                             float* __restrict__ out) {
  __shared__ float4 red[16][16];
  const int q = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + q * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < C) {
    for (int p = g; p < P; p += 16) {
      const float4 v = *reinterpret_cast<const float4*>(partial + (int64_t)p * C + c);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  red[g][q] = acc;
  __syncthreads();
  if (g == 0 && c < C) {
    float4 t = red[0][q];
#pragma unroll
    for (int k = 1; k < 16; ++k) {
      t.x += red[k][q].x; t.y += red[k][q].y; t.z += red[k][q].z; t.w += red[k][q].w;
    }
    out[c + 0] += t.x;
    out[c + 1] += t.y;
    out[c + 2] += t.z;
    out[c + 3] += t.w;
  }
}

constexpr int kBwdBlocks = 512;

}  // namespace

extern "C" {

int st_qknorm_rope_bwd_blocks() { return kBwdBlocks; }

int st_qknorm_rope_fwd(void* qkv, void* xsave, float* rstd, const void* wq, const void* wk, const float* cos_t,
                       const float* sin_t, const int64_t* pos, int64_t N, int S, int H, int Hkv, int D, float eps,
                       int64_t max_pos, hipStream_t st) {
  if (D != 64 && D != 128) return -2;
  const int NQK = H + Hkv, NHT = H + 2 * Hkv;
  const int64_t lanes = N * NQK * (D / 16);
  if (lanes == 0) return 0;
  const unsigned blocks = (unsigned)((lanes + 255) / 256);
  if (D == 128)
    qknorm_rope_fwd_kernel<128><<<blocks, 256, 0, st>>>((bf16_t*)qkv, (bf16_t*)xsave, rstd, (const bf16_t*)wq,
                                                        (const bf16_t*)wk, cos_t, sin_t, pos, N, S, H, NQK, NHT,
                                                        eps, max_pos);
  else
    qknorm_rope_fwd_kernel<64><<<blocks, 256, 0, st>>>((bf16_t*)qkv, (bf16_t*)xsave, rstd, (const bf16_t*)wq,
                                                       (const bf16_t*)wk, cos_t, sin_t, pos, N, S, H, NQK, NHT,
                                                       eps, max_pos);
  return (int)hipGetLastError();
}

// dw_out: fp32 [2, D] (q-norm then k-norm weight gradient), ACCUMULATED into.
// partial: fp32 scratch of kBwdBlocks * 2 * D.
int st_qknorm_rope_bwd(void* dqkv, const void* xsave, const float* rstd, const void* wq, const void* wk,
                       const float* cos_t, const float* sin_t, const int64_t* pos, int64_t N, int S, int H, int Hkv,
                       int D, int64_t max_pos, float* partial, float* dw_out, hipStream_t st) {
  if (D != 64 && D != 128) return -2;
  const int NQK = H + Hkv, NHT = H + 2 * Hkv;
  const int64_t rows = N * NQK;
  const int groups = 256 / (D / 16);
  int64_t need = (rows + groups - 1) / groups;
  const int blocks = (int)(need < kBwdBlocks ? (need < 1 ? 1 : need) : kBwdBlocks);
  if (D == 128)
    qknorm_rope_bwd_kernel<128><<<blocks, 256, 0, st>>>((bf16_t*)dqkv, (const bf16_t*)xsave, rstd,
                                                        (const bf16_t*)wq, (const bf16_t*)wk, cos_t, sin_t, pos, N,
                                                        S, H, NQK, NHT, max_pos, partial);
  else
    qknorm_rope_bwd_kernel<64><<<blocks, 256, 0, st>>>((bf16_t*)dqkv, (const bf16_t*)xsave, rstd,
                                                       (const bf16_t*)wq, (const bf16_t*)wk, cos_t, sin_t, pos, N,
                                                       S, H, NQK, NHT, max_pos, partial);
  partial_colsum_kernel<<<(2 * D + 63) / 64, 256, 0, st>>>(partial, blocks, 2 * D, dw_out);
  return (int)hipGetLastError();
}

}  // extern "C"

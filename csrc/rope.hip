// Rotary position embedding (rotate-half convention, as HF Llama/Qwen3 and
// scaletorch/models/attention_utils.py:170-192), applied IN PLACE on strided
// q/k head views -- typically the q and k sections of the fused QKV GEMM output
// [B, S, H + 2*Hkv, D], so no transpose/copy of q or k is ever materialised.
//
// * explicit global positions (position_ids) make CP / zig-zag chunks correct,
//   fixing the reference's "slice [:S] of a cp-partitioned table" bug
//   (scaletorch/parallel/context_parallel/context_parallel.py:427-473);
// * the cos/sin tables are precomputed fp32 [max_pos, D/2] (no on-device trig,
//   cdna_hip_programming.md App. B 'Element-wise');
// * each lane rotates 8 (x_i, x_{i+D/2}) pairs with two 16-byte loads/stores;
// * backward is the same kernel with sin negated (R(theta)^T = R(-theta)).
#include "common.h"

using namespace st;

namespace {

__global__ __launch_bounds__(256) void rope_kernel(bf16_t* __restrict__ x, const float* __restrict__ cos_t,
                                                    const float* __restrict__ sin_t,
                                                    const int64_t* __restrict__ pos, int B, int S, int NH,
                                                    int D, int64_t sB, int64_t sS, int64_t sH,
                                                    int pos_offset, float sin_sign, int64_t total,
                                                    int64_t max_pos) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int half = D >> 1;
  const int per_head = half >> 3;  // lanes per head (8 pairs each)
  const int j = (int)(t % per_head);
  int64_t r = t / per_head;
  const int h = (int)(r % NH);
  r /= NH;
  const int s = (int)(r % S);
  const int b = (int)(r / S);
  int64_t p = pos ? pos[(int64_t)b * S + s] : (int64_t)(s + pos_offset);
  // position ids are data: clamp into the table instead of reading out of bounds
  p = p < 0 ? 0 : (p >= max_pos ? max_pos - 1 : p);
  bf16_t* base = x + b * sB + s * sS + h * sH + j * 8;
  float x1[8], x2[8], c[8], sn[8];
  unpack8(ld8(base), x1);
  unpack8(ld8(base + half), x2);
  const float* cp = cos_t + p * half + j * 8;
  const float* sp = sin_t + p * half + j * 8;
  float4 c0 = ld4f(cp), c1 = ld4f(cp + 4), s0 = ld4f(sp), s1 = ld4f(sp + 4);
  c[0] = c0.x; c[1] = c0.y; c[2] = c0.z; c[3] = c0.w; c[4] = c1.x; c[5] = c1.y; c[6] = c1.z; c[7] = c1.w;
  sn[0] = s0.x; sn[1] = s0.y; sn[2] = s0.z; sn[3] = s0.w; sn[4] = s1.x; sn[5] = s1.y; sn[6] = s1.z; sn[7] = s1.w;
  float o1[8], o2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float si = sn[i] * sin_sign;
    o1[i] = x1[i] * c[i] - x2[i] * si;
    o2[i] = x2[i] * c[i] + x1[i] * si;
  }
  st8(base, pack8(o1));
  st8(base + half, pack8(o2));
}

}  // namespace

extern "C" int st_rope_inplace(void* x, const float* cos_t, const float* sin_t, const int64_t* pos,
                               int B, int S, int NH, int D, int64_t sB, int64_t sS, int64_t sH,
                               int pos_offset, int backward, int64_t max_pos, hipStream_t st) {
  if (D % 16 != 0) return -2;
  const int64_t total = (int64_t)B * S * NH * (D / 16);
  if (total == 0) return 0;
  const int64_t blocks = (total + 255) / 256;
  rope_kernel<<<dim3((unsigned)blocks), dim3(256), 0, st>>>((bf16_t*)x, cos_t, sin_t, pos, B, S, NH, D,
                                                             sB, sS, sH, pos_offset,
                                                             backward ? -1.f : 1.f, total, max_pos);
  return (int)hipGetLastError();
}

// SwiGLU on the output of ONE fused gate|up GEMM: gu = x @ [W_gate; W_up]^T is
// [N, 2I] with the gate in columns [0, I) and up in [I, 2I) of every row.
//   fwd: out = silu(g) * u                          [N, I]
//   bwd: dg = dout * u * silu'(g), du = dout * silu(g)  -> [N, 2I]
// Reference: down(silu(gate(x)) * up(x)), scaletorch/models/llama.py:236-249
// (two separate GEMMs + three elementwise kernels there; here one GEMM + one
// bandwidth-bound kernel with 16-byte accesses).
#include "common.h"

using namespace st;

namespace {

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ gu,
                                                          bf16_t* __restrict__ out, int64_t I8,
                                                          int64_t total) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = t / I8, c = t - row * I8;
    const bf16_t* gp = gu + row * (I8 * 16) + c * 8;
    float g[8], u[8], o[8];
    unpack8(ld8(gp), g);
    unpack8(ld8(gp + I8 * 8), u);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = silu(g[i]) * u[i];
    st8(out + row * (I8 * 8) + c * 8, pack8(o));
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ dout,
                                                          const bf16_t* __restrict__ gu,
                                                          bf16_t* __restrict__ dgu, int64_t I8,
                                                          int64_t total) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = t / I8, c = t - row * I8;
    const int64_t off = row * (I8 * 16) + c * 8;
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(ld8(gu + off), g);
    unpack8(ld8(gu + off + I8 * 8), u);
    unpack8(ld8(dout + row * (I8 * 8) + c * 8), d);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float sg = 1.f / (1.f + __expf(-g[i]));
      const float sl = g[i] * sg;
      du[i] = d[i] * sl;
      dg[i] = d[i] * u[i] * (sg + sl * (1.f - sg));
    }
    st8(dgu + off, pack8(dg));
    st8(dgu + off + I8 * 8, pack8(du));
  }
}

inline unsigned grid_for(int64_t total) {
  int64_t b = (total + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (unsigned)b;
}

}  // namespace

extern "C" int st_swiglu_fwd(const void* gu, void* out, int64_t N, int64_t I, hipStream_t st) {
  if (I % 8 != 0) return -2;
  const int64_t total = N * (I / 8);
  if (total == 0) return 0;
  swiglu_fwd_kernel<<<grid_for(total), 256, 0, st>>>((const bf16_t*)gu, (bf16_t*)out, I / 8, total);
  return (int)hipGetLastError();
}

extern "C" int st_swiglu_bwd(const void* dout, const void* gu, void* dgu, int64_t N, int64_t I,
                             hipStream_t st) {
  if (I % 8 != 0) return -2;
  const int64_t total = N * (I / 8);
  if (total == 0) return 0;
  swiglu_bwd_kernel<<<grid_for(total), 256, 0, st>>>((const bf16_t*)dout, (const bf16_t*)gu,
                                                     (bf16_t*)dgu, I / 8, total);
  return (int)hipGetLastError();
}

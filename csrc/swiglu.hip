// SwiGLU on the output of ONE fused gate|up GEMM: gu = x @ [W_gate; W_up]^T is
// [N, 2I] with the gate in columns [0, I) and up in [I, 2I) of every row.
//   fwd: out = silu(g) * u                          [N, I]
//   bwd: dg = dout * u * silu'(g), du = dout * silu(g)  -> [N, 2I]
// Reference: down(silu(gate(x)) * up(x)), scaletorch/models/llama.py:236-249
// (two separate GEMMs + three elementwise kernels there; here one GEMM + one
// bandwidth-bound kernel with 16-byte accesses).
#include <cstdlib>

#include "common.h"

using namespace st;

namespace {

// 2-D mapping: blockIdx.y walks rows (no 64-bit division per element), each lane
// owns U 16-byte column vectors 256 apart so U loads per operand are in flight
// before the first use (the grid-stride one-vector loop held only one).
template <int U>
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ gu,
                                                          bf16_t* __restrict__ out, int64_t I8,
                                                          int64_t N, const int* __restrict__ nvalid) {
  if (nvalid) N = min(N, (int64_t)max(0, *nvalid));  // rows past the device count: not touched
  const int64_t c0 = (int64_t)blockIdx.x * (256 * U) + threadIdx.x;
  for (int64_t row = blockIdx.y; row < N; row += gridDim.y) {
    const bf16_t* gp = gu + row * (I8 * 16);
    BF8 rg[U], ru[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t c = c0 + u * 256;
      if (c < I8) {
        rg[u] = ld8(gp + c * 8);
        ru[u] = ld8(gp + I8 * 8 + c * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t c = c0 + u * 256;
      if (c < I8) {
        float g[8], v[8], o[8];
        unpack8(rg[u], g);
        unpack8(ru[u], v);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = silu(g[i]) * v[i];
        st8(out + row * (I8 * 8) + c * 8, pack8(o));
      }
    }
  }
}

template <int U>
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ dout,
                                                          const bf16_t* __restrict__ gu,
                                                          bf16_t* __restrict__ dgu, int64_t I8,
                                                          int64_t N, const int* __restrict__ nvalid) {
  if (nvalid) N = min(N, (int64_t)max(0, *nvalid));
  const int64_t c0 = (int64_t)blockIdx.x * (256 * U) + threadIdx.x;
  for (int64_t row = blockIdx.y; row < N; row += gridDim.y) {
    const int64_t base = row * (I8 * 16);
    BF8 rg[U], ru[U], rd[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t c = c0 + u * 256;
      if (c < I8) {
        rg[u] = ld8(gu + base + c * 8);
        ru[u] = ld8(gu + base + I8 * 8 + c * 8);
        rd[u] = ld8(dout + row * (I8 * 8) + c * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t c = c0 + u * 256;
      if (c < I8) {
        float g[8], v[8], d[8], dg[8], du[8];
        unpack8(rg[u], g);
        unpack8(ru[u], v);
        unpack8(rd[u], d);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float sg = 1.f / (1.f + __expf(-g[i]));
          const float sl = g[i] * sg;
          du[i] = d[i] * sl;
          dg[i] = d[i] * v[i] * (sg + sl * (1.f - sg));
        }
        st8(dgu + base + c * 8, pack8(dg));
        st8(dgu + base + I8 * 8 + c * 8, pack8(du));
      }
    }
  }
}

inline dim3 grid_for(int64_t I8, int64_t N, int U) {
  const int64_t gx = (I8 + 256 * U - 1) / (256 * U);
  // ST_SWIGLU_ROWS caps the row dimension of the grid (blocks then walk several rows)
  static const int64_t cap = [] {
    const char* e = std::getenv("ST_SWIGLU_ROWS");
    const long v = e ? std::atol(e) : 0;
    return (int64_t)(v > 0 && v < 65535 ? v : 65535);
  }();
  const int64_t gy = N < cap ? N : cap;
  return dim3((unsigned)gx, (unsigned)gy);
}

// Column vectors per lane: 1 (Llama-3-8B I = 14336 -> I8 = 1792 = 7 full blocks of 256 per
// row; 2 vectors per lane left the 4th block of a row half-empty).  Isolated at 6 x 4096 rows
// (scripts/gpu_swiglu_ab.sh): fwd 5.19-5.32 -> 5.61 TB/s, bwd 5.20-5.25 -> 5.74 TB/s.
// ST_SWIGLU_U = 1 / 2 / 4 / 7 for A/B.
inline int pick_u(int64_t I8) {
  static const int forced = [] {
    const char* e = std::getenv("ST_SWIGLU_U");
    return e ? std::atoi(e) : 0;
  }();
  if (forced == 1 || forced == 2 || forced == 4 || forced == 7) return forced;
  return 1;
}

#define ST_SWIGLU_DISPATCH(KERNEL, ...)                                              \
  switch (pick_u(I8)) {                                                               \
    case 1: KERNEL<1><<<grid_for(I8, N, 1), 256, 0, st>>>(__VA_ARGS__); break;         \
    case 4: KERNEL<4><<<grid_for(I8, N, 4), 256, 0, st>>>(__VA_ARGS__); break;         \
    case 7: KERNEL<7><<<grid_for(I8, N, 7), 256, 0, st>>>(__VA_ARGS__); break;         \
    default: KERNEL<2><<<grid_for(I8, N, 2), 256, 0, st>>>(__VA_ARGS__); break;        \
  }

}  // namespace

// nvalid (may be null): device int32 row count -- rows at or past it are skipped (the
// R_max-row expert buffers of the dropless EP dispatch, models/moe.py)
extern "C" int st_swiglu_fwd(const void* gu, void* out, int64_t N, int64_t I, const int* nvalid, hipStream_t st) {
  if (I % 8 != 0) return -2;
  const int64_t I8 = I / 8;
  if (N == 0 || I8 == 0) return 0;
  ST_SWIGLU_DISPATCH(swiglu_fwd_kernel, (const bf16_t*)gu, (bf16_t*)out, I8, N, nvalid)
  return (int)hipGetLastError();
}

extern "C" int st_swiglu_bwd(const void* dout, const void* gu, void* dgu, int64_t N, int64_t I,
                             const int* nvalid, hipStream_t st) {
  if (I % 8 != 0) return -2;
  const int64_t I8 = I / 8;
  if (N == 0 || I8 == 0) return 0;
  ST_SWIGLU_DISPATCH(swiglu_bwd_kernel, (const bf16_t*)dout, (const bf16_t*)gu, (bf16_t*)dgu, I8, N, nvalid)
  return (int)hipGetLastError();
}

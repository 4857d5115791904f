// Shared device helpers for the scaletorch_amd CDNA4 (gfx950) kernels.
//
// Conventions used by every kernel in csrc/:
//  * wave64: a wavefront is 64 lanes; all cross-lane reductions below are
//    64-wide (never the 32-wide warp idiom).
//  * bf16 is carried as raw 16-bit patterns (uint16_t) in memory and widened to
//    fp32 in registers; narrowing uses the hardware round-to-nearest-even
//    conversion (clang lowers the __bf16 cast to v_cvt_pk_bf16_f32 at -O3,
//    which keeps NaN a NaN).
//  * memory-bound kernels move 16 bytes per lane per access (8 x bf16) so a
//    wave touches one contiguous 1 KiB segment per instruction.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define ST_DEVICE __device__ __forceinline__

namespace st {

constexpr int kWave = 64;

typedef uint16_t bf16_t;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));   // 8 bf16 = 4 VGPRs (MFMA A/B fragment)
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

ST_DEVICE float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

ST_DEVICE bf16_t f2bf(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(bf16_t, b);
}

// Pack two floats into one dword of two bf16 (lo in bits 0..15).
ST_DEVICE uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// 16-byte vector of 8 bf16 <-> 8 floats.
struct alignas(16) BF8 {
  uint32_t w[4];
};

ST_DEVICE void unpack8(const BF8& v, float (&f)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v.w[i] << 16);
    f[2 * i + 1] = __uint_as_float(v.w[i] & 0xffff0000u);
  }
}

ST_DEVICE BF8 pack8(const float (&f)[8]) {
  BF8 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v.w[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
  return v;
}

ST_DEVICE BF8 ld8(const bf16_t* p) { return *reinterpret_cast<const BF8*>(p); }
ST_DEVICE void st8(bf16_t* p, const BF8& v) { *reinterpret_cast<BF8*>(p) = v; }

ST_DEVICE float4 ld4f(const float* p) { return *reinterpret_cast<const float4*>(p); }
ST_DEVICE void st4f(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// Full-wave (64-lane) butterfly reductions.
ST_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
ST_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Block-wide sum for blockDim.x = NT threads (multiple of 64); `red` must hold
// NT/64 floats of LDS. Every thread returns the total.
template <int NT>
ST_DEVICE float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

ST_DEVICE float silu(float x) { return x / (1.f + __expf(-x)); }

// Bijective XCD-aware remap of a 1-D block id: blocks that the dispatcher
// deals round-robin to the same XCD (b % 8 equal) get a contiguous range of
// logical ids, so neighbouring tiles share an L2 (speed only, never
// correctness).
ST_DEVICE int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

}  // namespace st

#define ST_HIP_CHECK(expr)                                                   \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess) return (int)_e;                                    \
  } while (0)

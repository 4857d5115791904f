// bf16 2-D transpose [R, C] -> [C, R] through LDS (gfx950).
//
// Used to keep a K-contiguous copy W^T of every linear weight for the data-
// gradient GEMM: dX = dY W is an "NN" GEMM on the row-major weight, which
// hipBLASLt runs ~10 % slower on MI355X than the "TN" form dX = dY (W^T)^T that
// the forward pass uses (profiles/r02: 1.38 vs 1.58 PF/s).  One transpose per
// weight per step, issued on a side stream during the forward pass, buys the
// faster layout for every backward data-gradient GEMM.
//
// Tile: 64 x 64 bf16 per 256-thread workgroup.  Loads are 16 B per lane
// (8 lanes cover one 128-B tile row), the tile goes to LDS with a 2-element
// row pad (row stride 33 dwords: the 8 rows one wave reads per output chunk
// fall on distinct banks), and each lane gathers the 8 values of one 16-B
// output vector, so stores are 16 B per lane and 128 B per 8 lanes.
#include "common.h"

using namespace st;

namespace {

constexpr int kT = 64;       // tile edge
constexpr int kPad = 2;      // bf16 elements of row padding
constexpr int kLd = kT + kPad;

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst,
                                                             int R, int C, int64_t lds_src, int64_t lds_dst) {
  __shared__ bf16_t tile[kT * kLd];
  const int tiles_c = C / kT;
  const int nwg = gridDim.x;
  const int b = xcd_remap(blockIdx.x, nwg);
  const int r0 = (b / tiles_c) * kT, c0 = (b % tiles_c) * kT;
  const int t = threadIdx.x;
  const int chunk = t & 7, row = t >> 3;  // 8 lanes x 16 B = one 128-B tile row, 32 rows per pass
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = row + 32 * p;
    BF8 v = ld8(src + (int64_t)(r0 + r) * lds_src + c0 + chunk * 8);
    bf16_t* d = tile + r * kLd + chunk * 8;
    // row stride is not 16-B aligned (padded): 4 x 4-B stores
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<uint32_t*>(d + 2 * i) = v.w[i];
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int oc = row + 32 * p;  // output row = input column
    BF8 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t lo = tile[(chunk * 8 + 2 * i) * kLd + oc];
      const uint32_t hi = tile[(chunk * 8 + 2 * i + 1) * kLd + oc];
      o.w[i] = lo | (hi << 16);
    }
    st8(dst + (int64_t)(c0 + oc) * lds_dst + r0 + chunk * 8, o);
  }
}

}  // namespace

extern "C" int st_transpose_bf16(const void* src, void* dst, int R, int C, int64_t lds_src, int64_t lds_dst,
                                 hipStream_t st) {
  if (R % kT || C % kT || R <= 0 || C <= 0) return -2;
  const int64_t blocks = (int64_t)(R / kT) * (C / kT);
  if (blocks > 0x7fffffff) return -3;
  transpose_bf16_kernel<<<(unsigned)blocks, 256, 0, st>>>((const bf16_t*)src, (bf16_t*)dst, R, C, lds_src, lds_dst);
  return (int)hipGetLastError();
}

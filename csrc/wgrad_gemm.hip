// Weight-gradient GEMM for gfx950: C[M,N] (fp32) = beta * C + sum_t A[t,m] * B[t,n]
//
// The product every linear layer's backward needs for dW = dY^T X: both bf16
// operands are TOKEN-major ([T, M] and [T, N], the feature dimension
// contiguous), i.e. the reduction index is the strided one for BOTH.  hipBLASLt
// serves this layout (its "NT" form) with shallow-K macro tiles at ~0.9-1.1 PF/s
// on gfx950 while the same sizes with K-contiguous operands run at 1.25-1.4 PF/s
// (profiles/gemm_microbench.json); the fp32 output accumulates straight into the
// main_grad arena (beta = 1), or overwrites it on the step's first write
// (beta = 0, ops/grad.py).  Reference call site: the wgrad of
// LinearWithAsyncAllReduce (scaletorch/parallel/tensor_parallel/tp_comms.py:288-311)
// and autograd's F.linear backward.
//
// Design (CDNA4-first):
//   * 256x256 output tile, 8 waves (2 along M x 4 along N, 128x64 per wave),
//     v_mfma_f32_32x32x16_bf16, 8 accumulators (128 acc registers) per lane.
//   * the K loop walks T in 64-token tiles; each tile of A and B is staged
//     global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds) EXACTLY as stored
//     (rows = tokens, 256-byte rows of 128 features, XOR-swizzled on the source
//     address), and BOTH MFMA operands are read with ds_read_b64_tr_b16, which
//     delivers the token (reduction) index down a lane's fragment: no transpose
//     pass, no staging registers, no ds_write.  The same permuted k order is
//     used for A and B, so the pairing inside the MFMA is consistent.
//   * two LDS stages (2 x 64 KiB): the next tile's DMA is issued at the top of
//     a step and retired by the end-of-step barrier.
//   * XCD-aware tile order: the dispatcher deals workgroups round-robin to the
//     8 XCDs; the bijective remap gives each XCD a contiguous range of tiles,
//     grouped 4 M-blocks x N so the ~32 tiles an XCD runs at once share their
//     A and B token slices in its L2.
#include <cstdlib>
#include <type_traits>

#include "common.h"

using namespace st;

namespace {

typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
typedef __bf16 bfx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_t;

constexpr int BM = 256, BN = 256, BK = 32, NT = 512;
constexpr int RB = 256;               // bytes per LDS image row: 128 bf16 features
constexpr int IMG = BK * RB;          // one [32 tokens][128 features] image: 8 KiB
constexpr int STAGE = 4 * IMG;        // A0 A1 B0 B1: 32 KiB
constexpr int NBUF = 4;               // ring of 4 stages = 128 KiB, 3 in flight
constexpr int NDMA = STAGE / (NT * 16);  // LDS-DMA instructions per lane per stage (4)
constexpr int GROUP_M = 4;

// 256-B rows, 16-B chunks: both the transposed reads and the DMA fill are
// bank-conflict free with this XOR (cdna_hip_programming.md T10 image (b)).
ST_DEVICE int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
ST_DEVICE int lds_off(int row, int ch) { return row * RB + 16 * (ch ^ swz(row)); }

ST_DEVICE bfx8 lds_tr(const lds_t* p0, const lds_t* p1) {
  bfx4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bfx4 __attribute__((address_space(3)))*)p0);
  bfx4 b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bfx4 __attribute__((address_space(3)))*)p1);
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// Buffer resource words (base, stride 0, num_records, raw-buffer flags), wave-uniform.
typedef int i32x4 __attribute__((ext_vector_type(4)));
ST_DEVICE i32x4 make_rsrc(const bf16_t* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  i32x4 r;
  r[0] = (int)__builtin_amdgcn_readfirstlane((uint32_t)a);
  r[1] = (int)(__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) & 0xffffu);
  r[2] = (int)__builtin_amdgcn_readfirstlane(bytes);
  r[3] = 0x00020000;
  return r;
}

// LDS-DMA issued from inline asm: hipcc does not see it as an LDS write, so it
// does not drain it (vmcnt(0)) before the tile's transposed reads the way it
// does for the builtin form -- the wait is placed by hand (end of step), which
// is what lets the next tile's DMA overlap this tile's MFMAs.  M0 = the wave's
// LDS destination base; lane l lands at base + 16 l.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved: nothing else in this kernel uses it
ST_DEVICE void lds_dma16(const i32x4& rs, uint32_t lds_base, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(lds_base), "v"(voff), "s"(rs)
               : "memory", "m0");
}
#pragma clang diagnostic pop

template <int PROBE, int MF>
__global__ __launch_bounds__(NT, 2) void wgrad_gemm_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                           const bf16_t* __restrict__ B, int64_t ldb,
                                                           float* __restrict__ C, int64_t ldc, int M, int N,
                                                           int T, int beta) {
  __shared__ __attribute__((aligned(16))) char smem_raw[NBUF * STAGE];
  lds_t* smem = (lds_t*)smem_raw;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nbm = M / BM, nbn = N / BN, nwg = nbm * nbn;

  // ---- tile of this workgroup: XCD remap, then GROUP_M x nbn grouping
  const int logical = xcd_remap((int)blockIdx.x, nwg);
  const int per_group = GROUP_M * nbn;
  const int first_bm = (logical / per_group) * GROUP_M;
  const int gsz = min(nbm - first_bm, GROUP_M);
  const int in_group = logical % per_group;
  const int bm = first_bm + in_group % gsz, bn = in_group / gsz;
  const int m0 = bm * BM, n0 = bn * BN;

  // ---- DMA plan: wave w fills rows [16 (w&1), +16) of image (w>>1) of a stage
  const int img = wid >> 1, part = wid & 1;
  const bf16_t* src = img < 2 ? A + m0 + 128 * img : B + n0 + 128 * (img - 2);
  const int64_t ld = img < 2 ? lda : ldb;
  const uint32_t stride_b = (uint32_t)(ld * 2);
  const i32x4 rs = make_rsrc(src, (uint32_t)(((int64_t)(T - 1) * ld + 128) * 2));
  uint32_t voff[NDMA];
#pragma unroll
  for (int i = 0; i < NDMA; ++i) {
    const int a = part * (IMG / 2) + i * 1024 + lane * 16;
    const int row = a / RB, pos = (a % RB) / 16;
    voff[i] = (uint32_t)row * stride_b + (uint32_t)((pos ^ swz(row)) * 16);
  }
  const uint32_t dma_base = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)smem + (uint32_t)(img * IMG + part * (IMG / 2)));
  auto dma = [&](int buf, int kt) {
    const uint32_t o = (uint32_t)(kt * BK) * stride_b;
#pragma unroll
    for (int i = 0; i < NDMA; ++i) lds_dma16(rs, dma_base + buf * STAGE + i * 1024, voff[i] + o);
  };

  // ---- fragment read plan (lane-constant offsets): element j of lane (r, h) of a
  // transposed read at k-step s is image[16s + 8(j>>2) + 4h + (j&3)][32 dt + r]
  const int h = lane >> 5, g = (lane >> 4) & 1, q = (lane >> 2) & 3, pp = lane & 3;
  const int wm = wid >> 2, wn = wid & 3;
  const int a_img = wm * IMG, b_img = (2 + (wn >> 1)) * IMG, b_dt0 = (wn & 1) * 2;
  int atr[4][2], btr[2][2];  // never indexed by a runtime value (registers, not scratch)
  // 16x16x32 plan: lane group G = lane>>4 reads token rows 8G..8G+7 (natural k
  // order) of 16 feature columns 16 f .. 16 f + 15
  const int G = lane >> 4;
  int atr16[8][2], btr16[4][2];
  if constexpr (MF == 32) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        atr[dt][hf] = lds_off(4 * h + q + 8 * hf, 4 * dt + 2 * g + (pp >> 1)) + 8 * (pp & 1);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        btr[j][hf] = lds_off(4 * h + q + 8 * hf, 4 * (b_dt0 + j) + 2 * g + (pp >> 1)) + 8 * (pp & 1);
    }
  } else {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
      for (int f = 0; f < 8; ++f) atr16[f][hf] = lds_off(8 * G + 4 * hf + q, 2 * f + (pp >> 1)) + 8 * (pp & 1);
#pragma unroll
      for (int f = 0; f < 4; ++f)
        btr16[f][hf] = lds_off(8 * G + 4 * hf + q, 2 * (4 * (wn & 1) + f) + (pp >> 1)) + 8 * (pp & 1);
    }
  }

  f32x16 acc[4][2];
  f32x4 acc16[8][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc16[i][j][r] = 0.f;

  // ---- K loop: a ring of NBUF stages, NBUF-1 tiles in flight.  Top of step kt:
  // wait (counted vmcnt) until this wave's DMA of tile kt landed, barrier (every
  // wave's DMA landed + every wave finished reading tile kt-1), refill the stage
  // tile kt-1 used with tile kt+NBUF-1, then 2 k-steps of MFMAs on tile kt.
  const int KT = T / BK;
#pragma unroll
  for (int p = 0; p < NBUF - 1; ++p)
    if (p < KT) dma(p, p);

  auto step = [&](auto bufc, int kt) {
    constexpr int BUF = decltype(bufc)::value;
    if (kt + 2 < KT) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NDMA) : "memory");
    else if (kt + 1 < KT) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NBUF - 1 < KT && PROBE != 1) dma((BUF + NBUF - 1) % NBUF, kt + NBUF - 1);
    const lds_t* st = smem + BUF * STAGE;
    if constexpr (MF == 16) {
      const lds_t* ab = st + a_img;
      const lds_t* bb = st + b_img;
      bfx8 af[8], bf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = lds_tr(bb + btr16[j][0], bb + btr16[j][1]);
#pragma unroll
      for (int i = 0; i < 8; ++i) af[i] = lds_tr(ab + atr16[i][0], ab + atr16[i][1]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc16[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc16[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      asm volatile("" ::: "memory");
      return;
    }
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const lds_t* ab = st + a_img + 16 * s * RB;
      const lds_t* bb = st + b_img + 16 * s * RB;
      bfx8 af[4], bf[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = lds_tr(ab + atr[i][0], ab + atr[i][1]);
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = lds_tr(bb + btr[j][0], bb + btr[j][1]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("" ::: "memory");
  };
  for (int kt = 0; kt < KT; kt += NBUF) {
    step(std::integral_constant<int, 0>(), kt);
    if (kt + 1 < KT) step(std::integral_constant<int, 1>(), kt + 1);
    if (kt + 2 < KT) step(std::integral_constant<int, 2>(), kt + 2);
    if (kt + 3 < KT) step(std::integral_constant<int, 3>(), kt + 3);
  }

  const int mb = m0 + wm * 128, nb = n0 + wn * 64, c = lane & 31;
  if constexpr (MF == 16) {  // C/D: row = 4 (lane>>4) + reg (M), column = lane&15 (N)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = mb + 16 * i + 4 * G + r;
          float* p = C + (int64_t)m * ldc + nb + 16 * j + (lane & 15);
          *p = beta ? *p + acc16[i][j][r] : acc16[i][j][r];
        }
    return;
  }
  // ---- epilogue: C/D row = (reg&3) + 8(reg>>2) + 4h (M), column = lane&31 (N)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mb + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        float* p = C + (int64_t)m * ldc + nb + 32 * j + c;
        *p = beta ? *p + acc[i][j][r] : acc[i][j][r];
      }
}

}  // namespace

extern "C" {

// 0 on success; -2: shape not supported by this kernel (caller falls back).
int st_wgrad_gemm(const void* A, int64_t lda, const void* B, int64_t ldb, float* C, int64_t ldc, int M,
                  int N, int T, int beta, hipStream_t st) {
  if (M <= 0 || N <= 0 || T <= 0) return -2;
  if (M % BM || N % BN || T % BK) return -2;
  if (lda % 8 || ldb % 8 || lda < M || ldb < N || ldc < N) return -2;
  if (((uintptr_t)A | (uintptr_t)B) % 16 || (uintptr_t)C % 4) return -2;
  // 32-bit buffer offsets: the last row of each operand must be addressable
  if (((int64_t)(T - 1) * lda + M) * 2 >= (int64_t)1 << 32) return -2;
  if (((int64_t)(T - 1) * ldb + N) * 2 >= (int64_t)1 << 32) return -2;
  const int nwg = (M / BM) * (N / BN);
  // ST_WGRAD_PROBE=1: timing probe only (no K-loop DMA: compute ceiling) -- wrong results
  const char* pe = std::getenv("ST_WGRAD_PROBE");
  const int probe = pe ? std::atoi(pe) : 0;
  // ST_WGRAD_MFMA=32: v_mfma_f32_32x32x16_bf16 variant (default 16x16x32: ~+5-8 % on random data)
  const char* me = std::getenv("ST_WGRAD_MFMA");
  const int mf = me ? std::atoi(me) : 16;
  const bf16_t *a = (const bf16_t*)A, *b = (const bf16_t*)B;
  const int bt = beta ? 1 : 0;
  if (mf == 16) {
    if (probe == 1) wgrad_gemm_kernel<1, 16><<<nwg, NT, 0, st>>>(a, lda, b, ldb, C, ldc, M, N, T, bt);
    else wgrad_gemm_kernel<0, 16><<<nwg, NT, 0, st>>>(a, lda, b, ldb, C, ldc, M, N, T, bt);
  } else {
    if (probe == 1) wgrad_gemm_kernel<1, 32><<<nwg, NT, 0, st>>>(a, lda, b, ldb, C, ldc, M, N, T, bt);
    else wgrad_gemm_kernel<0, 32><<<nwg, NT, 0, st>>>(a, lda, b, ldb, C, ldc, M, N, T, bt);
  }
  return (int)hipGetLastError();
}

}  // extern "C"

// Grouped (MoE expert) GEMM for gfx950 with a DEVICE offset table:
//   for every group g:  Y[rows of g] = X[rows of g] @ op(W[g])
//   rows of g = [offs[g-1], offs[g])  (int32 inclusive prefix sums, never read by the host)
//
// Two weight layouts, one kernel template:
//   * WT (forward):      W[g] is [N][K] (K contiguous)  -> Y = X W^T   (x @ w.t() per expert)
//   * WN (data grad):    W[g] is [K][N] (N contiguous)  -> Y = X W     (dy @ w per expert)
// X / Y are token-major [T][K] / [T][N] with row strides.  Reference: the grouped-matmul
// autograd of scaletorch/models/npu_patch.py:94-127 (npu_grouped_matmul); on ROCm,
// torch._grouped_mm runs one small hipBLASLt GEMM per group after reading the offsets on
// the host (profiles/r03/moe_qwen3_30b_a3b_proxy_breakdown.txt: ~1,500 launches and 56 ms
// of idle per step at 128 experts) -- this is ONE launch per product.
//
// Design (CDNA4-first; the synchronisation skeleton is the 4-stage ring of
// csrc/wgrad_gemm.hip):
//   * 256 x BN output tile (BN = 256 or 128), 8 waves, 16x16x32 bf16 MFMA, K in 64-wide
//     tiles, double-buffered (128 KiB of LDS at BN = 256): tile kt+1's LDS-DMA (inline asm,
//     so hipcc does not drain it) is issued right after the barrier that retires tile kt
//     and runs under tile kt's MFMAs.
//   * grid = (ceil(T/256) + G) M-tile slots x N-tiles (an upper bound of sum_g ceil(n_g/256));
//     a workgroup maps its slot to (group, M-tile) by a binary search of the per-group
//     tile-count prefix (device, computed by the caller); surplus slots exit at once.
//   * rows past a group's end: the buffer descriptor's range ends at the group's last
//     row, so they load as zeros and are not stored.
//   * LDS images, both filled by DMA pieces of 8 rows x 128 B (full lines from HBM) and
//     conflict-free for their reads by construction:
//       row image (X, and W in WT layout): [row][8 chunks of 8 k], chunk c of row r at
//         c ^ ((r >> 1) & 7) -- the A/B fragment of a 32-k sub-step is ONE ds_read_b128;
//       column image (W in WN layout): [64-col block][k][4 x 32-B column slots], slot at
//         slot ^ csw(k), read by ds_read_b64_tr_b16 (k down the lane's fragment).
#include <cstdlib>
#include <type_traits>

#include "common.h"

// timing probes only (variant builds, wrong results): 1 = no wait for the DMA, 2 = no DMA
#ifndef ST_GMM_PROBE
#define ST_GMM_PROBE 0
#endif

using namespace st;

namespace {

typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
typedef __bf16 bfx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_t;
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 256, BK = 64, NT = 512;

ST_DEVICE i32x4 make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  i32x4 r;
  r[0] = (int)__builtin_amdgcn_readfirstlane((uint32_t)a);
  r[1] = (int)(__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) & 0xffffu);
  r[2] = (int)__builtin_amdgcn_readfirstlane(bytes);
  r[3] = 0x00020000;
  return r;
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved: nothing else in this kernel uses it
ST_DEVICE void lds_dma16(const i32x4& rs, uint32_t lds_base, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(lds_base), "v"(voff), "s"(rs)
               : "memory", "m0");
}
#pragma clang diagnostic pop

ST_DEVICE bfx8 lds_b128(const lds_t* p) { return *(const bfx8 __attribute__((address_space(3)))*)p; }
ST_DEVICE bfx4 lds_tr(const lds_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bfx4 __attribute__((address_space(3)))*)p);
}
ST_DEVICE bfx8 cat8(bfx4 a, bfx4 b) { return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7); }

// row image: [row][8 x 16-B chunks of k], chunk c of row r stored at c ^ rsw(r): the 16
// rows x 2 chunks a ds_read_b128 lane group touches land in 16 distinct 16-B slots
ST_DEVICE int rsw(int r) { return (r >> 1) & 7; }
// column image: [64-col block][k][4 x 32-B column slots], slot stored at slot ^ csw(k): the
// 8 k-rows of a transposed-read half land in 8 distinct 32-B slots
ST_DEVICE int csw(int k) { return ((k >> 1) & 1) | (((k >> 3) & 1) << 1); }

template <int BN, bool WN>
struct Geo {
  static constexpr int WM = BN == 256 ? 2 : 4, WNV = 8 / WM;  // wave grid
  static constexpr int TM = BM / WM, TN = BN / WNV;           // per-wave tile
  static constexpr int FM = TM / 16, FN = TN / 16;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int A_PIECES = A_BYTES / 1024, PIECES = STAGE / 1024;
  static constexpr int NDMA = PIECES / 8;
  static_assert(PIECES % 8 == 0, "stage must split evenly over 8 waves");
  static_assert(NDMA % 2 == 0, "SPREAD issues half of a wave's pieces per 32-k sub-step");
};

// first g with tile_end[g] > s (tile_end = inclusive prefix of per-group M-tile counts)
ST_DEVICE int find_group(const int* __restrict__ tile_end, int G, int s) {
  int lo = 0, hi = G;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (tile_end[mid] <= s) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// EPI (epilogue): 0 = Y = X op(W);
//   1 = SwiGLU forward (WT, BN = 256): W[g] = [gate rows 0..I | up rows I..2I]; N-tile t
//       computes gate columns [128 t, 128 t + 128) AND the matching up columns (the B
//       image's rows are drawn from both halves: wave w's 64 columns = 32 gate + the 32
//       up columns of the same features, so gate and up of one feature meet in ONE
//       lane's registers); writes gu (Y, [rows, 2I]) for the backward and
//       a = silu(gate) * up (Y2, [rows, I]) straight from the fp32 accumulators;
//   2 = SwiGLU backward (WN): the tile is da = dY W_down[g] ([rows, I]); the epilogue
//       reads gate / up from gu (Y2, [rows, 2I]) and writes dgu = [d gate | d up] (Y,
//       [rows, 2I]) -- the separate swiglu_bwd pass and the da round-trip disappear.
template <int BN, bool WN, bool SPREAD = false, int EPI = 0>
__global__ __launch_bounds__(NT, 1) void grouped_gemm_kernel(const bf16_t* __restrict__ X, int64_t ldx,
                                                             const bf16_t* __restrict__ W, int64_t ldw,
                                                             int64_t strideW, bf16_t* __restrict__ Y, int64_t ldy,
                                                             const int* __restrict__ offs,
                                                             const int* __restrict__ tile_end, int G, int N,
                                                             int K, int order, bf16_t* __restrict__ Y2,
                                                             int64_t ld2, int I) {
  static_assert(EPI != 1 || (BN == 256 && !WN), "SwiGLU forward epilogue: WT layout, 256-wide tiles");
  static_assert(EPI != 2 || WN, "SwiGLU backward epilogue: WN layout");
  using Gm = Geo<BN, WN>;
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * Gm::STAGE];
  lds_t* smem = (lds_t*)smem_raw;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nbn = N / BN;

  // ---- work item: (M-tile slot, N-tile); slot -> (group, M-tile of the group).
  // order 1: XCD-aware remap, then super-rows of 8 slots walked N-tile-major, so the ~32
  // workgroups an XCD holds at once share 8 X tiles and 4 weight tiles in its L2;
  // order 0: slot-major (each X tile swept across all N-tiles before the next)
  int slot, nt;
  if (order == 1) {
    const int nslots = (int)gridDim.x / nbn;
    const int idx = xcd_remap((int)blockIdx.x, (int)gridDim.x);
    const int per = 8 * nbn, grp = idx / per, in = idx % per;
    const int gsz = min(8, nslots - grp * 8);
    slot = grp * 8 + in % gsz;
    nt = in / gsz;
  } else {
    slot = (int)blockIdx.x / nbn;
    nt = (int)blockIdx.x % nbn;
  }
  const int total_slots = tile_end[G - 1];
  if (slot >= total_slots) return;  // uniform over the workgroup: no barrier reached yet
  const int g = find_group(tile_end, G, slot);
  const int first_slot = g ? tile_end[g - 1] : 0;
  const int row0 = (g ? offs[g - 1] : 0) + (slot - first_slot) * BM;
  const int rows = min(BM, offs[g] - row0);  // >= 1 by construction
  const int n0 = nt * BN;

  // ---- operands: X rows [row0, row0 + rows) -- the descriptor ends at the last valid
  // row, so DMA of rows past it (next group / past T) reads zeros
  const bf16_t* xb = X + (int64_t)row0 * ldx;
  const i32x4 rsX = make_rsrc(xb, (uint32_t)(((int64_t)(rows - 1) * ldx + K) * 2));
  const bf16_t* wb = W + (int64_t)g * strideW + (EPI == 1 ? 0 : (WN ? (int64_t)n0 : (int64_t)n0 * ldw));
  const i32x4 rsW = make_rsrc(wb, (uint32_t)(EPI == 1 ? ((int64_t)(N - 1) * ldw + K) * 2
                                            : WN ? ((int64_t)(K - 1) * ldw + BN) * 2
                                                 : ((int64_t)(BN - 1) * ldw + K) * 2));
  const uint32_t sX = (uint32_t)(ldx * 2), sW = (uint32_t)(ldw * 2);

  // ---- DMA plan: every 1-KiB piece is 8 rows x 128 B (8 rows of 64 k, or 8 k-rows of 64
  // columns); wave w fills pieces [w NDMA, (w+1) NDMA) of a stage, lane L the 16 B at L*16
  uint32_t voff[Gm::NDMA];
  bool isA[Gm::NDMA];
#pragma unroll
  for (int i = 0; i < Gm::NDMA; ++i) {
    const int p = wid * Gm::NDMA + i;  // wave-uniform
    isA[i] = p < Gm::A_PIECES;
    const int q = isA[i] ? p : p - Gm::A_PIECES;
    const int pr = q * 8 + (lane >> 3), pc = lane & 7;  // row of the image, physical 16-B chunk
    if (isA[i] || !WN) {
      int src = pr;  // EPI 1: image row pr -> gate / up row of the weight (see the EPI note)
      if (EPI == 1 && !isA[i]) {
        const int wb64 = pr >> 6, w = pr & 63;
        src = (w < 32 ? 0 : I) + 128 * nt + 32 * wb64 + (w & 31);
      }
      voff[i] = (uint32_t)src * (isA[i] ? sX : sW) + (uint32_t)((pc ^ rsw(pr)) * 16);
    } else {  // column image: block cb = q / 8, k-row kr, logical 32-B slot
      const int cb = q >> 3, kr = (q & 7) * 8 + (lane >> 3);
      const int logical = (((pc >> 1) ^ csw(kr)) << 1) | (pc & 1);
      voff[i] = (uint32_t)kr * sW + (uint32_t)((cb * 64 + logical * 8) * 2);
    }
  }
  const uint32_t dma_base =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem + (uint32_t)(wid * Gm::NDMA * 1024));
  auto dma_piece = [&](int buf, int kt, int i) {
    const uint32_t kx = (uint32_t)(kt * BK * 2);             // row images: k along the row
    const uint32_t kw = WN ? (uint32_t)(kt * BK) * sW : kx;  // column image: k = row
    lds_dma16(isA[i] ? rsX : rsW, dma_base + buf * Gm::STAGE + i * 1024, voff[i] + (isA[i] ? kx : kw));
  };
  auto dma = [&](int buf, int kt) {
#pragma unroll
    for (int i = 0; i < Gm::NDMA; ++i) dma_piece(buf, kt, i);
  };

  // ---- fragment read plan (16x16x32, natural k order: lane group gq holds k 8gq..8gq+7
  // of a 32-k sub-step = 16-B chunk 4s + gq)
  const int gq = lane >> 4, rr = lane & 15;
  const int wm = wid / Gm::WNV, wn = wid % Gm::WNV;
  const int am = wm * Gm::TM, bnn = wn * Gm::TN;
  int aoff[Gm::FM][2], boff[Gm::FN][2];
#pragma unroll
  for (int f = 0; f < Gm::FM; ++f) {
    const int r = am + 16 * f + rr;
#pragma unroll
    for (int st = 0; st < 2; ++st) aoff[f][st] = r * 128 + 16 * ((4 * st + gq) ^ rsw(r));
  }
#pragma unroll
  for (int f = 0; f < Gm::FN; ++f) {
    const int nn = bnn + 16 * f;
    if (WN) {  // lane 4q+p of group gq: k-row 8gq+q (+4 for the 2nd read, +32 per sub-step)
      const int q = (lane >> 2) & 3, p = lane & 3;
      const int kr = 8 * gq + q, sl = (nn & 63) >> 4;
      boff[f][0] = Gm::A_BYTES + (nn >> 6) * 8192 + kr * 128 + 32 * (sl ^ csw(kr)) + 8 * p;
      boff[f][1] = boff[f][0] + 4 * 128;  // k-rows 8gq+4..8gq+7: same swizzle (csw ignores k bit 2)
    } else {
      const int r = nn + rr;
#pragma unroll
      for (int st = 0; st < 2; ++st) boff[f][st] = Gm::A_BYTES + r * 128 + 16 * ((4 * st + gq) ^ rsw(r));
    }
  }

  f32x4 acc[Gm::FM][Gm::FN];
#pragma unroll
  for (int i = 0; i < Gm::FM; ++i)
#pragma unroll
    for (int j = 0; j < Gm::FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;

  // ---- K loop: double-buffered 64-k tiles; tile kt+1's DMA is issued right after the
  // barrier that retires tile kt, and runs under tile kt's MFMAs
  const int KT = K / BK;
  dma(0, 0);
  auto tile = [&](auto bufc, int kt) {
    constexpr int BUF = decltype(bufc)::value;
#if ST_GMM_PROBE == 0
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bool more = kt + 1 < KT;
#if ST_GMM_PROBE != 2
    if (!SPREAD && more) dma(BUF ^ 1, kt + 1);
#endif
    const lds_t* stg = smem + BUF * Gm::STAGE;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      bfx8 af[Gm::FM], bf[Gm::FN];
#pragma unroll
      for (int j = 0; j < Gm::FN; ++j) {
        if (WN) bf[j] = cat8(lds_tr(stg + boff[j][0] + st * 32 * 128), lds_tr(stg + boff[j][1] + st * 32 * 128));
        else bf[j] = lds_b128(stg + boff[j][st]);
      }
#pragma unroll
      for (int i = 0; i < Gm::FM; ++i) af[i] = lds_b128(stg + aoff[i][st]);
      __builtin_amdgcn_s_setprio(1);
      // SPREAD: the next tile's DMA pieces go out one at a time between this sub-step's MFMAs
      // (NP per sub-step, evenly spaced) instead of in one burst after the barrier
      constexpr int NM = Gm::FM * Gm::FN, NP = Gm::NDMA / 2;
#pragma unroll
      for (int i = 0; i < Gm::FM; ++i)
#pragma unroll
        for (int j = 0; j < Gm::FN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
          if constexpr (SPREAD) {
#pragma unroll
            for (int q = 0; q < NP; ++q)
              if (i * Gm::FN + j == (q * NM) / NP + NM / (2 * NP) && ST_GMM_PROBE != 2) {
                __builtin_amdgcn_sched_barrier(0);
                if (more) dma_piece(BUF ^ 1, kt + 1, st * NP + q);
                __builtin_amdgcn_sched_barrier(0);
              }
          }
        }
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("" ::: "memory");
  };
  for (int kt = 0; kt < KT; kt += 2) {
    tile(std::integral_constant<int, 0>(), kt);
    if (kt + 1 < KT) tile(std::integral_constant<int, 1>(), kt + 1);
  }

  // ---- epilogue: 16x16 C/D row = 4 (lane>>4) + reg (M), column = lane & 15 (N); rows past
  // the group's end are not stored
  if constexpr (EPI == 1) {
    static_assert(Gm::FN == 4, "32 gate + 32 up columns per wave");
    const int cb = 128 * nt + 32 * wn + (lane & 15);  // gate feature of fragment 0
    bf16_t* gub = Y + (int64_t)row0 * ldy;
    bf16_t* ab = Y2 + (int64_t)row0 * ld2;
#pragma unroll
    for (int i = 0; i < Gm::FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = am + 16 * i + 4 * gq + r;
        if (m < rows) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const float gv = acc[i][j][r], uv = acc[i][j + 2][r];
            const int c = cb + 16 * j;
            gub[(int64_t)m * ldy + c] = f2bf(gv);
            gub[(int64_t)m * ldy + I + c] = f2bf(uv);
            ab[(int64_t)m * ld2 + c] = f2bf(silu(gv) * uv);
          }
        }
      }
  } else if constexpr (EPI == 2) {
    const int cb = n0 + bnn + (lane & 15);
    const bf16_t* gub = Y2 + (int64_t)row0 * ld2;
    bf16_t* db = Y + (int64_t)row0 * ldy;
#pragma unroll
    for (int i = 0; i < Gm::FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = am + 16 * i + 4 * gq + r;
        if (m < rows) {
#pragma unroll
          for (int j = 0; j < Gm::FN; ++j) {
            const int c = cb + 16 * j;
            const float gv = bf2f(gub[(int64_t)m * ld2 + c]), uv = bf2f(gub[(int64_t)m * ld2 + I + c]);
            const float d = acc[i][j][r];
            const float sg = 1.f / (1.f + __expf(-gv)), sl = gv * sg;
            db[(int64_t)m * ldy + c] = f2bf(d * uv * (sg + sl * (1.f - sg)));
            db[(int64_t)m * ldy + I + c] = f2bf(d * sl);
          }
        }
      }
  } else {
    bf16_t* yb = Y + (int64_t)row0 * ldy + n0 + bnn + (lane & 15);
#pragma unroll
    for (int i = 0; i < Gm::FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = am + 16 * i + 4 * gq + r;
        if (m < rows) {
#pragma unroll
          for (int j = 0; j < Gm::FN; ++j) yb[(int64_t)m * ldy + 16 * j] = f2bf(acc[i][j][r]);
        }
      }
  }
}

// ============================================================ 8-phase variant (BN = 256)
// The synchronisation skeleton of csrc/wgrad_gemm.hip's wgrad8_kernel (the 256² 8-phase
// template of cdna_hip_programming.md) on this file's operand images: 256 x 256 tile,
// BK = 64, 8 waves as 2 (M) x 4 (N); wave (wr, wc) owns the four 64 x 32 quadrants (mq, nq)
// at rows mq*128 + wr*64, columns nq*128 + wc*32.  Quadrant (mq, nq) reads only the X
// half-image mq ([128 rows][64 k] row image) and the W half-image nq (row image in the WT
// layout, [2 x 64-col blocks][64 k] column image in WN), 16 KiB each, so a K-tile is
// consumed half-image by half-image in four phases -- (0,0) (0,1) (1,1) (1,0), reads p0 X0+W0,
// p1 W1, p2 X1, p3 none (W0 / W1 fragments stay in registers) -- while the next tiles'
// half-images stream into a ring of 8 slots behind them (LEAD 4, counted vmcnt, raw
// barriers; waves 4-7 one barrier behind waves 0-3, so on every SIMD one wave reads while
// its partner runs MFMAs).  The 2-phase kernel above waits vmcnt(0) at every K-tile.
// EPI 1 (SwiGLU forward): W half-image 0 = gate rows, 1 = up rows of the tile's 128
// features, so a lane holds gate (acc[.][j]) and up (acc[.][2 + j]) of the same feature.
namespace g8 {
constexpr int IMGB = 16384;  // one half-image: 128 rows x 64 k (or 64 k-rows x 128 cols) bf16
constexpr int SLOTS = 8, LEAD = 4;
}  // namespace g8

template <bool WN, int EPI>
__global__ __launch_bounds__(NT, 1) void grouped8_kernel(const bf16_t* __restrict__ X, int64_t ldx,
                                                         const bf16_t* __restrict__ W, int64_t ldw, int64_t strideW,
                                                         bf16_t* __restrict__ Y, int64_t ldy,
                                                         const int* __restrict__ offs,
                                                         const int* __restrict__ tile_end, int G, int N, int K,
                                                         bf16_t* __restrict__ Y2, int64_t ld2, int I) {
  using namespace g8;
  static_assert(EPI != 1 || !WN, "SwiGLU forward epilogue: WT layout");
  static_assert(EPI != 2 || WN, "SwiGLU backward epilogue: WN layout");
  __shared__ __attribute__((aligned(16))) char smem_raw[SLOTS * IMGB];
  lds_t* smem = (lds_t*)smem_raw;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wid >> 2, wr = grp, wc = wid & 3;
  // EPI 1: N = 2I columns of gu, one N-tile per 128 features (gate + up)
  const int nbn = EPI == 1 ? I / 128 : N / 256;
  const int slot = (int)blockIdx.x / nbn, nt = (int)blockIdx.x % nbn;
  const int total_slots = tile_end[G - 1];
  if (slot >= total_slots) return;  // uniform over the workgroup: no barrier reached yet
  const int g = find_group(tile_end, G, slot);
  const int first_slot = g ? tile_end[g - 1] : 0;
  const int row0 = (g ? offs[g - 1] : 0) + (slot - first_slot) * BM;
  const int rows = min(BM, offs[g] - row0);  // >= 1 by construction
  const int n0 = nt * 256;

  // ---- descriptors: X rows past the group's end and W rows / columns past the tile read as 0
  const bf16_t* xb = X + (int64_t)row0 * ldx;
  const i32x4 rsX = make_rsrc(xb, (uint32_t)(((int64_t)(rows - 1) * ldx + K) * 2));
  const bf16_t* wb = W + (int64_t)g * strideW;
  const i32x4 rsW = make_rsrc(wb, (uint32_t)(WN ? ((int64_t)(K - 1) * ldw + N) * 2 : ((int64_t)(N - 1) * ldw + K) * 2));
  const uint32_t sX = (uint32_t)(ldx * 2), sW = (uint32_t)(ldw * 2);

  // ---- DMA: half-image h (issue order X = 0: X0, 1: W0, 2: W1, 3: X1) of K-tile kt; wave w
  // fills pieces 2w, 2w + 1 (1 KiB each: 8 rows x 128 B, or 8 k-rows x 128 B of a 64-col
  // block); lane L lands at 16 L of its piece
  uint32_t vX[2], vWr[2][2], vWc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = 2 * wid + i, pr = q * 8 + (lane >> 3), pc = lane & 7;
    const uint32_t ch = (uint32_t)((pc ^ rsw(pr)) * 16);
    vX[i] = (uint32_t)pr * sX + ch;
    // WT row image of W half nq: tile columns nq*128 + pr -> weight row
#pragma unroll
    for (int nq = 0; nq < 2; ++nq) {
      const int src = EPI == 1 ? (nq ? I : 0) + 128 * nt + pr : n0 + nq * 128 + pr;
      vWr[nq][i] = (uint32_t)src * sW + ch;
    }
    // WN column image: block cb = q / 8, k-row kr, logical 32-B slot
    const int cb = q >> 3, kr = (q & 7) * 8 + (lane >> 3);
    const int logical = (((pc >> 1) ^ csw(kr)) << 1) | (pc & 1);
    vWc[i] = (uint32_t)kr * sW + (uint32_t)((cb * 64 + logical * 8) * 2);
  }
  const uint32_t ldsw = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem + (uint32_t)(wid * 2048));
  auto ring_dma = [&](auto xc, int slot_i, int kt, int piece) {
    constexpr int Xh = decltype(xc)::value;
    constexpr bool isX = (Xh == 0 || Xh == 3);
    constexpr int half = (Xh == 2 || Xh == 3) ? 1 : 0;
    uint32_t v;
    if constexpr (isX) {
      v = vX[piece] + (uint32_t)(half * 128) * sX + (uint32_t)(kt * BK * 2);
    } else if constexpr (WN) {
      v = vWc[piece] + (uint32_t)(kt * BK) * sW + (uint32_t)((n0 + half * 128) * 2);
    } else {
      v = vWr[half][piece] + (uint32_t)(kt * BK * 2);
    }
    lds_dma16(isX ? rsX : rsW, ldsw + (uint32_t)(slot_i * IMGB + piece * 1024), v);
  };

  // ---- fragment reads (16x16x32; lane group gq = lane >> 4 holds k 8gq .. 8gq+7 of a
  // 32-k sub-step ks): A rows wr*64 + 16 i of a X half-image, B columns wc*32 + 16 j of a W one
  const int gq = lane >> 4, rr = lane & 15;
  int aoff[4][2], boff[2][2][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = wr * 64 + 16 * i + rr;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) aoff[i][ks] = r * 128 + 16 * ((4 * ks + gq) ^ rsw(r));
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int nn = wc * 32 + 16 * j;  // column within the half-image
    if (WN) {
      const int q = (lane >> 2) & 3, p = lane & 3;
      const int kr = 8 * gq + q, sl = (nn & 63) >> 4;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        boff[j][ks][0] = (nn >> 6) * 8192 + (kr + 32 * ks) * 128 + 32 * (sl ^ csw(kr)) + 8 * p;
        boff[j][ks][1] = boff[j][ks][0] + 4 * 128;
      }
    } else {
      const int r = nn + rr;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) boff[j][ks][0] = boff[j][ks][1] = r * 128 + 16 * ((4 * ks + gq) ^ rsw(r));
    }
  }
  auto read_b = [&](const lds_t* img, int j, int ks) -> bfx8 {
    if constexpr (WN) return cat8(lds_tr(img + boff[j][ks][0]), lds_tr(img + boff[j][ks][1]));
    else return lds_b128(img + boff[j][ks][0]);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;
  bfx8 af[4][2] = {}, b0[2][2] = {}, b1[2][2] = {};

  auto bar = [] {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;

  const int KT = K / BK;
  const int NH = 4 * KT;  // half-images of the whole K loop
  // prologue: half-images 0 .. LEAD-1 (K-tile 0); 0 (X0) and 1 (W0) retired for phase 0
#pragma unroll
  for (int pc = 0; pc < 2; ++pc) ring_dma(I0(), 0, 0, pc);
#pragma unroll
  for (int pc = 0; pc < 2; ++pc) ring_dma(I1(), 1, 0, pc);
#pragma unroll
  for (int pc = 0; pc < 2; ++pc) ring_dma(I2(), 2, 0, pc);
#pragma unroll
  for (int pc = 0; pc < 2; ++pc) ring_dma(I3(), 3, 0, pc);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (LEAD - 2)) : "memory");
  bar();
  if (grp == 1) bar();  // the stagger: waves 4-7 run one barrier behind

  auto phase = [&](auto pc, int kt) {
    constexpr int P = decltype(pc)::value;
    constexpr int MQ = (P == 0 || P == 1) ? 0 : 1, NQ = (P == 0 || P == 3) ? 0 : 1;
    const int n0h = 4 * kt;
    // slots read this phase: X0 = n0h, W0 = n0h + 1, W1 = n0h + 2, X1 = n0h + 3
    const lds_t* ai = smem + ((n0h + (MQ ? 3 : 0)) % SLOTS) * IMGB;
    if constexpr (P == 0 || P == 2) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) af[i][ks] = lds_b128(ai + aoff[i][ks]);
    }
    if constexpr (P == 0 || P == 1) {
      const lds_t* bi = smem + ((n0h + 1 + NQ) % SLOTS) * IMGB;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bfx8 v = read_b(bi, j, ks);
          if constexpr (NQ == 0) b0[j][ks] = v;
          else b1[j][ks] = v;
        }
    }
    // retire what the NEXT phase reads (p3 -> X0/W0 of kt+1, p0 -> W1, p1 -> X1, p2 -> none)
    const int issue = n0h + P + LEAD;  // this phase's DMA (issued under its MFMAs)
    if (issue <= NH) {
      if constexpr (P == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (LEAD - 2)) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (LEAD - 3)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();
    if constexpr (P == 0 || P == 2) {
#pragma unroll
      for (int i = 2; i < 4; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) af[i][ks] = lds_b128(ai + aoff[i][ks]);
    }
    const int islot = issue % SLOTS, ikt = kt + (P + LEAD) / 4;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const bfx8 bv = NQ == 0 ? b0[j][ks] : b1[j][ks];
          acc[MQ * 4 + i][NQ * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bv, acc[MQ * 4 + i][NQ * 2 + j], 0, 0, 0);
        }
      // the next half-image, one 1-KiB piece after the 4th and the 8th MFMA
      if ((i == 0 || i == 1) && issue < NH) {
        __builtin_amdgcn_sched_barrier(0);
        ring_dma(std::integral_constant<int, (P + LEAD) % 4>(), islot, ikt, i);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    bar();
  };
  for (int kt = 0; kt < KT; ++kt) {
    phase(I0(), kt);
    phase(I1(), kt);
    phase(I2(), kt);
    phase(I3(), kt);
  }
  if (grp == 0) bar();  // same barrier count in both groups

  // ---- epilogue: acc[i][j] = rows (i >> 2)*128 + wr*64 + 16 (i & 3) + 4 gq + r, columns
  // (j >> 1)*128 + wc*32 + 16 (j & 1) + (lane & 15) of the tile; rows past the group unstored
  const int cl = lane & 15;
  if constexpr (EPI == 1) {
    bf16_t* gub = Y + (int64_t)row0 * ldy;
    bf16_t* ab = Y2 + (int64_t)row0 * ld2;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = (i >> 2) * 128 + wr * 64 + 16 * (i & 3) + 4 * gq + r;
        if (m < rows) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const float gv = acc[i][j][r], uv = acc[i][j + 2][r];
            const int c = 128 * nt + wc * 32 + 16 * j + cl;
            gub[(int64_t)m * ldy + c] = f2bf(gv);
            gub[(int64_t)m * ldy + I + c] = f2bf(uv);
            ab[(int64_t)m * ld2 + c] = f2bf(silu(gv) * uv);
          }
        }
      }
  } else if constexpr (EPI == 2) {
    const bf16_t* gub = Y2 + (int64_t)row0 * ld2;
    bf16_t* db = Y + (int64_t)row0 * ldy;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = (i >> 2) * 128 + wr * 64 + 16 * (i & 3) + 4 * gq + r;
        if (m < rows) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int c = n0 + (j >> 1) * 128 + wc * 32 + 16 * (j & 1) + cl;
            const float gv = bf2f(gub[(int64_t)m * ld2 + c]), uv = bf2f(gub[(int64_t)m * ld2 + I + c]);
            const float d = acc[i][j][r];
            const float sg = 1.f / (1.f + __expf(-gv)), sl = gv * sg;
            db[(int64_t)m * ldy + c] = f2bf(d * uv * (sg + sl * (1.f - sg)));
            db[(int64_t)m * ldy + I + c] = f2bf(d * sl);
          }
        }
      }
  } else {
    bf16_t* yb = Y + (int64_t)row0 * ldy + n0 + wc * 32 + cl;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = (i >> 2) * 128 + wr * 64 + 16 * (i & 3) + 4 * gq + r;
        if (m < rows) {
#pragma unroll
          for (int j = 0; j < 4; ++j) yb[(int64_t)m * ldy + (j >> 1) * 128 + 16 * (j & 1)] = f2bf(acc[i][j][r]);
        }
      }
  }
}

}  // namespace

extern "C" {

// M-tile slots to launch for T rows in G groups (upper bound of sum_g ceil(n_g / 256)).
int64_t st_grouped_gemm_slots(int T, int G) { return (int64_t)(T + BM - 1) / BM + G; }
int st_grouped_gemm_bm() { return BM; }

// Y[T, N] (bf16, rows of each group) = X[T, K] @ (wn ? W[g] : W[g]^T); W[g] is [K][N] when
// wn, else [N][K].  offs / tile_end: int32 [G] device (tile_end = inclusive prefix of
// ceil(n_g / 256)).  epi 1: SwiGLU forward (wn = 0, N = 2I, I % 128 == 0): Y = gu [T, 2I],
// Y2 = a [T, I]; epi 2: SwiGLU backward (wn = 1, N = I): Y = dgu [T, 2I], Y2 = gu [T, 2I]
// (read).  0 on success, -2 unsupported shape.
int st_grouped_gemm_ex(const void* X, int64_t ldx, const void* W, int64_t ldw, int64_t strideW, void* Y,
                       int64_t ldy, const int* offs, const int* tile_end, int T, int G, int N, int K, int wn,
                       int epi, void* Y2, int64_t ld2, hipStream_t st) {
  if (T <= 0 || G <= 0 || N <= 0 || K <= 0) return -2;
  if (K % BK || N % 128) return -2;  // K: whole 64-k tiles
  if (ldx % 8 || ldw % 8 || ldy % 8 || ldx < K || (wn ? ldw < N : ldw < K)) return -2;
  if (((uintptr_t)X | (uintptr_t)W | (uintptr_t)Y) % 16) return -2;
  if (((int64_t)(T + BM) * ldx) * 2 >= (int64_t)1 << 32) return -2;  // 32-bit buffer offsets
  if ((wn ? (int64_t)K * ldw : (int64_t)N * ldw) * 2 >= (int64_t)1 << 32) return -2;
  int I = 0;
  if (epi == 0) {
    if (ldy < N) return -2;
  } else if (epi == 1) {
    I = N / 2;
    if (wn || N % 256 || I % 128 || !Y2 || ldy < N || ld2 < I || ld2 % 8) return -2;
  } else if (epi == 2) {
    I = N;
    if (!wn || !Y2 || ldy < 2 * I || ld2 < 2 * I || ld2 % 8) return -2;
  } else {
    return -2;
  }
  const int bn = (N % 256 == 0) ? 256 : 128;
  const int64_t grid = st_grouped_gemm_slots(T, G) * (N / bn);
  if (grid >= (1LL << 31)) return -2;
  const bf16_t *x = (const bf16_t*)X, *w = (const bf16_t*)W;
  bf16_t* y = (bf16_t*)Y;
  bf16_t* y2 = (bf16_t*)Y2;
  // 1: XCD-grouped tile order -- measured 2-19 % SLOWER than slot-major on every MoE and
  // dense shape (profiles/r03/grouped_gemm_order_ab.log): slot-major stays the default
  const char* oe = std::getenv("ST_GMM_ORDER");
  const int order = oe ? std::atoi(oe) : 0;
  // ST_GMM_DMA_SPREAD=1: next-tile DMA pieces interleaved with the MFMAs (A/B)
  const char* se = std::getenv("ST_GMM_DMA_SPREAD");
  const bool spread = se && std::atoi(se) == 1 && epi == 0;
#define ARGS x, ldx, w, ldw, strideW, y, ldy, offs, tile_end, G, N, K, order, y2, ld2, I
#define LAUNCH(BNV, WNV)                                                                         \
  do {                                                                                           \
    if (spread)                                                                                  \
      grouped_gemm_kernel<BNV, WNV, true, 0><<<(unsigned)grid, NT, 0, st>>>(ARGS);               \
    else                                                                                         \
      grouped_gemm_kernel<BNV, WNV, false, 0><<<(unsigned)grid, NT, 0, st>>>(ARGS);              \
  } while (0)
  // 8-phase kernel for 256-wide tiles (ST_GMM_8PHASE=0: the 2-phase kernel, A/B)
  const char* p8e = std::getenv("ST_GMM_8PHASE");
  const bool p8 = bn == 256 && !spread && !(p8e && std::atoi(p8e) == 0);
#define ARGS8 x, ldx, w, ldw, strideW, y, ldy, offs, tile_end, G, N, K, y2, ld2, I
  if (p8) {
    if (epi == 1) grouped8_kernel<false, 1><<<(unsigned)grid, NT, 0, st>>>(ARGS8);
    else if (epi == 2) grouped8_kernel<true, 2><<<(unsigned)grid, NT, 0, st>>>(ARGS8);
    else if (wn) grouped8_kernel<true, 0><<<(unsigned)grid, NT, 0, st>>>(ARGS8);
    else grouped8_kernel<false, 0><<<(unsigned)grid, NT, 0, st>>>(ARGS8);
  } else if (epi == 1) {
    grouped_gemm_kernel<256, false, false, 1><<<(unsigned)grid, NT, 0, st>>>(ARGS);
  } else if (epi == 2) {
    if (bn == 256) grouped_gemm_kernel<256, true, false, 2><<<(unsigned)grid, NT, 0, st>>>(ARGS);
    else grouped_gemm_kernel<128, true, false, 2><<<(unsigned)grid, NT, 0, st>>>(ARGS);
  } else if (bn == 256) {
    if (wn) LAUNCH(256, true); else LAUNCH(256, false);
  } else {
    if (wn) LAUNCH(128, true); else LAUNCH(128, false);
  }
#undef LAUNCH
#undef ARGS
#undef ARGS8
  return (int)hipGetLastError();
}

int st_grouped_gemm(const void* X, int64_t ldx, const void* W, int64_t ldw, int64_t strideW, void* Y, int64_t ldy,
                    const int* offs, const int* tile_end, int T, int G, int N, int K, int wn, hipStream_t st) {
  return st_grouped_gemm_ex(X, ldx, W, ldw, strideW, Y, ldy, offs, tile_end, T, G, N, K, wn, 0, nullptr, 0, st);
}

}  // extern "C"

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
//   * 256x256 output tile, 8 waves (2 along M x 4 along N, 128x64 per wave), or
//     256x128 (4 x 2 waves, 64x64 per wave) when the 256-wide grid would leave a
//     partial last wave of workgroups on the 256 CUs; v_mfma_f32_16x16x32_bf16
//     (on random operands it holds a higher clock than 32x32x16: +5-8 % here).
//   * the K loop walks T in 64-token tiles; each tile of A and B is staged
//     global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds) EXACTLY as stored
//     (rows = tokens, 256-byte rows of 128 features, XOR-swizzled on the source
//     address), and BOTH MFMA operands are read with ds_read_b64_tr_b16, which
//     delivers the token (reduction) index down a lane's fragment: no transpose
//     pass, no staging registers, no ds_write.  The same permuted k order is
//     used for A and B, so the pairing inside the MFMA is consistent.
//   * K loop over 32-token tiles through a ring of 4 LDS stages with 3 tiles in
//     flight: the DMA is issued from inline asm (so hipcc does not drain it
//     before the transposed reads) and retired by a counted vmcnt + s_barrier.
//   * tried and dropped (profiles/r02/wgrad_v3_pipelined_ab.log): a schedule that
//     reads the next step's fragments into a second register set under the
//     current step's MFMAs (one barrier per step after the MFMAs) ran 4-15 %
//     SLOWER at T = 16384 -- the exposed cost here is not LDS read latency.
//   * XCD-aware tile order: the dispatcher deals workgroups round-robin to the
//     8 XCDs; the bijective remap gives each XCD a contiguous range of tiles,
//     grouped 4 M-blocks x N so the ~32 tiles an XCD runs at once share their
//     A and B token slices in its L2.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"

using namespace st;

namespace {

typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
typedef __bf16 bfx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_t;

constexpr int BM = 256, BK = 32, NT = 512;
constexpr int RB = 256;               // bytes per LDS image row: 128 bf16 features
constexpr int IMG = BK * RB;          // one [32 tokens][128 features] image: 8 KiB
constexpr int NBUF = 4;               // ring of 4 stages, 3 tiles in flight
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
// does for the builtin form -- the wait is placed by hand, which is what lets
// the next tiles' DMA overlap this tile's MFMAs.  M0 = the wave's LDS
// destination base; lane l lands at base + 16 l.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved: nothing else in this kernel uses it
ST_DEVICE void lds_dma16(const i32x4& rs, uint32_t lds_base, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(lds_base), "v"(voff), "s"(rs)
               : "memory", "m0");
}
#pragma clang diagnostic pop

// ---- tail split (split-K over the token range for the last, partial wave of tiles)
// A grid of nt tiles on 256 CUs (one workgroup per CU) runs ceil(nt/256) rounds; when
// nt % 256 != 0 the last round leaves CUs idle (down 4096x14336: 896 tiles = 3.5 rounds,
// qkv 6144x4096: 1.5, TP-sharded projections: < 1).  The first nfull = 256 * floor(nt/256)
// tiles run whole; each of the remaining `tail` tiles is cut into `split` token ranges,
// so the last round is split x shorter.  Range 0 of a tail tile accumulates into C with
// beta like a whole tile; ranges 1.. write fp32 partials to a workspace that
// wgrad_tail_reduce adds to C in range order afterwards (same stream): deterministic,
// no atomics, no inter-workgroup flags.
struct SplitPlan {
  float* ws;
  int nfull, tail, split;
};
struct WItem {
  int m0, n0;    // tile origin in the full output
  int k0, T;     // token range [k0, k0 + T)
  int beta;
  float* C;      // where the tile goes: C itself, or its workspace slot
  int64_t ldc;
  int cm0, cn0;  // origin of the tile inside *C (m0/n0, or 0/0 in the workspace)
};

// tile index -> (bm, bn): GROUP_M M-blocks x all N-blocks per group, so the ~32 tiles one
// XCD runs at once share their A and B token slices in its L2
ST_DEVICE void group_tile(int idx, int nbm, int nbn, int& bm, int& bn) {
  const int per_group = GROUP_M * nbn;
  const int first_bm = (idx / per_group) * GROUP_M;
  const int gsz = min(nbm - first_bm, GROUP_M);
  const int in_group = idx % per_group;
  bm = first_bm + in_group % gsz;
  bn = in_group / gsz;
}

// workgroup b -> work item.  Blocks are dealt round-robin to the 8 XCDs (b % 8 shares an
// XCD), so XCD x's j-th block takes the j-th item of a contiguous per-XCD range: first of
// the whole tiles, then of the (range-major) tail units, keeping one XCD's concurrent
// units on the same token range and neighbouring tiles.
template <int TBM, int TBN>
ST_DEVICE WItem work_item(int b, int nbm, int nbn, int T, int beta, float* C, int64_t ldc, const SplitPlan& sp) {
  WItem w{0, 0, 0, T, beta, C, ldc, 0, 0};
  int idx;
  bool direct = true;
  if (sp.split <= 1) {
    idx = xcd_remap(b, nbm * nbn);
  } else if (b < sp.nfull) {
    idx = (b & 7) * (sp.nfull >> 3) + (b >> 3);
  } else {
    const int u = b - sp.nfull, per = (sp.tail * sp.split) >> 3;
    const int ux = (u & 7) * per + (u >> 3);
    const int s = ux / sp.tail, tl = ux % sp.tail;
    idx = sp.nfull + tl;
    w.T = T / sp.split;
    w.k0 = s * w.T;
    if (s > 0) {
      direct = false;
      w.C = sp.ws + ((int64_t)(s - 1) * sp.tail + tl) * (TBM * TBN);
      w.ldc = TBN;
      w.beta = 0;
    }
  }
  int bm, bn;
  group_tile(idx, nbm, nbn, bm, bn);
  w.m0 = bm * TBM;
  w.n0 = bn * TBN;
  if (direct) {
    w.cm0 = w.m0;
    w.cn0 = w.n0;
  }
  return w;
}

template <int BN>
__global__ __launch_bounds__(256) void wgrad_tail_reduce(float* __restrict__ C, int64_t ldc,
                                                         const float* __restrict__ ws, int nbm, int nbn,
                                                         SplitPlan sp) {
  const int tl = blockIdx.y;
  int bm, bn;
  group_tile(sp.nfull + tl, nbm, nbn, bm, bn);
  const int e = (blockIdx.x * 256 + threadIdx.x) * 4;  // element of the BM x BN tile
  const int r = e / BN, c = e % BN;
  f32x4* pc = (f32x4*)(C + (int64_t)(bm * BM + r) * ldc + bn * BN + c);
  f32x4 acc = *pc;
  for (int s = 1; s < sp.split; ++s) acc += *(const f32x4*)(ws + ((int64_t)(s - 1) * sp.tail + tl) * (BM * BN) + e);
  *pc = acc;
}

template <int BN>
struct Geo {
  static constexpr int WM = BN == 256 ? 2 : 4, WN = 8 / WM;  // wave grid
  static constexpr int TM = BM / WM, TN = BN / WN;           // per-wave tile
  static constexpr int FM = TM / 16, FN = TN / 16;           // 16x16 fragments per wave
  static constexpr int NIMG = (BM + BN) / 128;               // 128-feature images per stage
  static constexpr int STAGE = NIMG * IMG;
  static constexpr int PIECES = STAGE / 1024;                // 1 KiB DMA pieces per stage
  static constexpr int NDMA = PIECES / 8;                    // per wave (and per lane)
  static_assert(PIECES % 8 == 0, "stage must split evenly over 8 waves");
};

// Grouped launch (MoE experts): G independent products C_g = beta C_g + A_g^T B_g whose
// token ranges are [offs[g-1], offs[g]) of the same A / B (offs = inclusive prefix sum of
// the per-expert row counts, on the device: the host never reads them).  Every group
// has the same M x N, so the grid is G x tiles, expert-major: the ~256 workgroups in
// flight at any time belong to ONE expert (as in a per-expert launch), and the XCD remap
// runs inside each expert's tiles.  (Remapping over the whole grid put a different
// expert on every XCD: 8 experts' operands competing for the Infinity Cache, 26 % slower
// on the Mixtral proxy, profiles/r03/moe_grouped_wgrad.md.)
struct GroupPlan {
  const int* offs;  // [G] inclusive offsets (int32), device
  int G;
  int64_t strideC;  // elements between consecutive C_g
};

template <int BN>
ST_DEVICE WItem group_item(int b, int nbm, int nbn, int beta, float* C, int64_t ldc, const GroupPlan& gp) {
  const int tiles = nbm * nbn;
  const int g = b / tiles, t = xcd_remap(b % tiles, tiles);
  const int k0 = g ? gp.offs[g - 1] : 0;
  WItem w{0, 0, k0, gp.offs[g] - k0, beta, C + (int64_t)g * gp.strideC, ldc, 0, 0};
  int bm, bn;
  group_tile(t, nbm, nbn, bm, bn);
  w.m0 = w.cm0 = bm * BM;
  w.n0 = w.cn0 = bn * BN;
  return w;
}

template <int PROBE, int BN, bool GROUPED = false>
__global__ __launch_bounds__(NT, 2) void wgrad_gemm_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                           const bf16_t* __restrict__ B, int64_t ldb,
                                                           float* __restrict__ C, int64_t ldc, int M, int N,
                                                           int T, int beta, SplitPlan sp, GroupPlan gp) {
  using Gm = Geo<BN>;
  __shared__ __attribute__((aligned(16))) char smem_raw[NBUF * Gm::STAGE];
  lds_t* smem = (lds_t*)smem_raw;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int nbm = M / BM, nbn = N / BN;

  // ---- work item of this workgroup: tile (XCD-aware, GROUP_M x nbn grouping), token range
  const WItem w = GROUPED ? group_item<BN>((int)blockIdx.x, nbm, nbn, beta, C, ldc, gp)
                          : work_item<BM, BN>((int)blockIdx.x, nbm, nbn, T, beta, C, ldc, sp);
  if (GROUPED && w.T <= 0 && w.beta) return;  // expert received no tokens: C_g unchanged
  const int m0 = w.m0, n0 = w.n0;
  A += (int64_t)w.k0 * lda;
  B += (int64_t)w.k0 * ldb;
  T = w.T;

  // ---- DMA plan: a stage is NIMG images [32 tokens][128 features] (A images
  // first); wave w fills the 1 KiB pieces [w NDMA, (w+1) NDMA) of it.  Image
  // boundaries are 8 KiB, so a piece never straddles two images.
  const i32x4 rsA = make_rsrc(A + m0, (uint32_t)(T > 0 ? ((int64_t)(T - 1) * lda + BM) * 2 : 0));
  const i32x4 rsB = make_rsrc(B + n0, (uint32_t)(T > 0 ? ((int64_t)(T - 1) * ldb + BN) * 2 : 0));
  const uint32_t sA = (uint32_t)(lda * 2), sB = (uint32_t)(ldb * 2);
  uint32_t voff[Gm::NDMA];
  bool isA[Gm::NDMA];
#pragma unroll
  for (int i = 0; i < Gm::NDMA; ++i) {
    const int piece = (wid * Gm::NDMA + i) * 1024;  // wave-uniform
    const int a = piece + lane * 16;
    const int im = piece / IMG, row = (a % IMG) / RB, pos = (a % RB) / 16;
    isA[i] = im < BM / 128;
    const int col_b = 256 * (isA[i] ? im : im - BM / 128);
    voff[i] = (uint32_t)row * (isA[i] ? sA : sB) + (uint32_t)(col_b + 16 * (pos ^ swz(row)));
  }
  const uint32_t dma_base =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem + (uint32_t)(wid * Gm::NDMA * 1024));
  auto dma = [&](int buf, int kt) {
    const uint32_t oA = (uint32_t)(kt * BK) * sA, oB = (uint32_t)(kt * BK) * sB;
#pragma unroll
    for (int i = 0; i < Gm::NDMA; ++i)
      lds_dma16(isA[i] ? rsA : rsB, dma_base + buf * Gm::STAGE + i * 1024, voff[i] + (isA[i] ? oA : oB));
  };

  // ---- fragment read plan (16x16x32): lane group G = lane>>4 reads token rows
  // 8G..8G+7 (natural k order) of 16 feature columns; lane 4q+p of the group
  // addresses row q, columns 4p..4p+3 (T10).
  const int G = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int wm = wid / Gm::WN, wn = wid % Gm::WN;
  const int am = wm * Gm::TM, bnn = wn * Gm::TN;  // wave's first row / column inside the tile
  int atr[Gm::FM][2], btr[Gm::FN][2];             // never indexed by a runtime value
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
    for (int f = 0; f < Gm::FM; ++f) {
      const int col = am + 16 * f;  // feature column inside the A half-images
      atr[f][hf] = (col / 128) * IMG + lds_off(8 * G + 4 * hf + q, ((col % 128) / 8) + (pp >> 1)) + 8 * (pp & 1);
    }
#pragma unroll
    for (int f = 0; f < Gm::FN; ++f) {
      const int col = bnn + 16 * f;
      btr[f][hf] = (BM / 128 + col / 128) * IMG + lds_off(8 * G + 4 * hf + q, ((col % 128) / 8) + (pp >> 1)) +
                   8 * (pp & 1);
    }
  }

  f32x4 acc[Gm::FM][Gm::FN];
#pragma unroll
  for (int i = 0; i < Gm::FM; ++i)
#pragma unroll
    for (int j = 0; j < Gm::FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;

  // ---- K loop: a ring of NBUF stages, NBUF-1 tiles in flight.  Top of step kt:
  // wait (counted vmcnt) until this wave's DMA of tile kt landed, barrier (every
  // wave's DMA landed + every wave finished reading tile kt-1), refill the stage
  // tile kt-1 used with tile kt+NBUF-1, then the tile's MFMAs.
  const int KT = (T + BK - 1) / BK;  // a ragged last tile reads rows >= T as zeros (buffer range)
#pragma unroll
  for (int p = 0; p < NBUF - 1; ++p)
    if (p < KT) dma(p, p);

  auto step = [&](auto bufc, int kt) {
    constexpr int BUF = decltype(bufc)::value;
    if (kt + 2 < KT) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * Gm::NDMA) : "memory");
    else if (kt + 1 < KT) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Gm::NDMA) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NBUF - 1 < KT && PROBE != 1) dma((BUF + NBUF - 1) % NBUF, kt + NBUF - 1);
    const lds_t* st = smem + BUF * Gm::STAGE;
    bfx8 af[Gm::FM], bf[Gm::FN];
#pragma unroll
    for (int j = 0; j < Gm::FN; ++j) bf[j] = lds_tr(st + btr[j][0], st + btr[j][1]);
#pragma unroll
    for (int i = 0; i < Gm::FM; ++i) af[i] = lds_tr(st + atr[i][0], st + atr[i][1]);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < Gm::FM; ++i)
#pragma unroll
      for (int j = 0; j < Gm::FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("" ::: "memory");
  };
  for (int kt = 0; kt < KT; kt += NBUF) {
    step(std::integral_constant<int, 0>(), kt);
    if (kt + 1 < KT) step(std::integral_constant<int, 1>(), kt + 1);
    if (kt + 2 < KT) step(std::integral_constant<int, 2>(), kt + 2);
    if (kt + 3 < KT) step(std::integral_constant<int, 3>(), kt + 3);
  }

  // ---- epilogue: 16x16 C/D row = 4 (lane>>4) + reg (M), column = lane&15 (N)
#pragma unroll
  for (int i = 0; i < Gm::FM; ++i)
#pragma unroll
    for (int j = 0; j < Gm::FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = w.cm0 + am + 16 * i + 4 * G + r;
        float* p = w.C + (int64_t)m * w.ldc + w.cn0 + bnn + 16 * j + (lane & 15);
        *p = w.beta ? *p + acc[i][j][r] : acc[i][j][r];
      }
}

// ============================================================ 8-phase variant
// 256x256 tile, BK = 64 tokens, 8 waves as 2 (M) x 4 (N), wave (wr, wc) owning
// the four 64x32 quadrants (mq, nq) at rows mq*128 + wr*64, columns nq*128 + wc*32:
// quadrant (mq, nq) reads ONLY the A half-image mq and the B half-image nq
// ([64 tokens][128 features], 16 KiB each), so a K-tile is consumed half-image by
// half-image and the next tile's half-images stream in behind it.  Four phases
// per K-tile, quadrants (0,0) (0,1) (1,1) (1,0):
//   reads (p0: A0+B0, p1: B1, p2: A1, p3: none -- B0/B1 stay in registers)
//   + counted vmcnt retiring what the NEXT phase reads     | barrier |
//   16 MFMAs (quadrant x 64 tokens), with one half-image of tile t+1 issued
//   by LDS-DMA between them (p0 A0, p1 B0, p2 B1, p3 A1)  | barrier |
// (DMA issued from the reading section instead measured 3-7 % slower: the
// read section, not the MFMA section, was the longer one.)
// Waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave issues
// its LDS reads and DMA while its partner runs MFMAs (cdna_hip_programming.md
// "The 256² 8-phase template"; counted waits + raw barriers only: a DMA stays
// in flight across every barrier).  Every read of a half-image is ordered after
// the issuing waves' vmcnt AND one extra barrier (the stagger), since the wait
// for phase p+1's data sits before phase p's first barrier.
namespace p8 {
constexpr int BK = 64;
constexpr int IMGB = BK * RB;    // [64 tokens][128 features]: 16 KiB

}  // namespace p8

// Half-images live in a ring of SLOTS 16-KiB slots: half-image n = 4 kt + X (X in issue
// order: 0 = A0, 1 = B0, 2 = B1, 3 = A1) in slot n % SLOTS; phase P of tile kt issues
// half-image 4 kt + P + LEAD, LEAD = SLOTS - 4, into the slot last read at phase <= P of
// tile kt - 1.  SLOTS = 8 (LEAD 4) is the two-K-tile double buffer; written as a ring it
// runs 1-2 % faster than the buffer-indexed form it replaced (profiles/r03/wgrad_ring.md).
// Deeper leads (9 / 10 slots, the whole 160 KiB) measured 13-15 % SLOWER: the slot index
// is no longer a power of two, and its per-read address adds cost 19 % with the DMA off.
// Probes on the same box (gate_up / down at T = 24,576): no K-loop DMA 1.60 PF/s; DMA from
// an L2-hot source 1.33; DMA never waited for 1.23; as shipped 1.24 -- the DMA's cost is
// its traffic through the CU and the L2 misses, not its latency, so a deeper ring cannot
// buy it back.
template <int X>
ST_DEVICE void ring_dma(const i32x4& rsA, const i32x4& rsB, uint32_t ldsw, const uint32_t (&vA)[2],
                        const uint32_t (&vB)[2], uint32_t sA, uint32_t sB, int slot, int kt, int piece) {
  constexpr bool isA = (X == 0 || X == 3);
  constexpr uint32_t col = (X == 2 || X == 3) ? 256u : 0u;  // byte offset of feature 128
  const uint32_t koff = (uint32_t)(kt * p8::BK) * (isA ? sA : sB) + col;
  const uint32_t v = piece ? (isA ? vA[1] : vB[1]) : (isA ? vA[0] : vB[0]);
  lds_dma16(isA ? rsA : rsB, ldsw + (uint32_t)(slot * p8::IMGB + piece * 1024), v + koff);
}

// PROBE (timing probes, wrong results): 1 = no K-loop DMA, 2 = no K-loop LDS reads,
// 3 = DMA never waited for in the loop, 4 = every DMA from K-tile 0 (L2-hot)
template <int PROBE, int SLOTS = 8>
__global__ __launch_bounds__(NT, 1) void wgrad8_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                           const bf16_t* __restrict__ B, int64_t ldb,
                                                           float* __restrict__ C, int64_t ldc, int M, int N,
                                                           int T, int beta, SplitPlan sp) {
  using namespace p8;
  constexpr int LEAD = SLOTS - 4;
  static_assert(LEAD >= 4 && LEAD <= 6, "lead of 4..6 half-images");
  __shared__ __attribute__((aligned(16))) char smem_raw[SLOTS * IMGB];
  lds_t* smem = (lds_t*)smem_raw;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wid >> 2, wr = grp, wc = wid & 3;
  const int nbm = M / BM, nbn = N / 256;
  const WItem w = work_item<BM, 256>((int)blockIdx.x, nbm, nbn, T, beta, C, ldc, sp);
  const int m0 = w.m0, n0 = w.n0;
  A += (int64_t)w.k0 * lda;
  B += (int64_t)w.k0 * ldb;
  T = w.T;

  const i32x4 rsA = make_rsrc(A + m0, (uint32_t)(((int64_t)(T - 1) * lda + BM) * 2));
  const i32x4 rsB = make_rsrc(B + n0, (uint32_t)(((int64_t)(T - 1) * ldb + 256) * 2));
  const uint32_t sA = (uint32_t)(lda * 2), sB = (uint32_t)(ldb * 2);
  uint32_t vA[2], vB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 4 * (2 * wid + i) + (lane >> 4), pos = lane & 15;
    const uint32_t c = (uint32_t)(16 * (pos ^ swz(row)));
    vA[i] = (uint32_t)row * sA + c;
    vB[i] = (uint32_t)row * sB + c;
  }
  const uint32_t ldsw = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem + (uint32_t)(wid * 2048));
  const int G = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  int aoff[4][2], boff[2][2];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      aoff[i][hf] = lds_off(8 * G + 4 * hf + q, ((wr * 64 + 16 * i) / 8) + (pp >> 1)) + 8 * (pp & 1);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      boff[j][hf] = lds_off(8 * G + 4 * hf + q, ((wc * 32 + 16 * j) / 8) + (pp >> 1)) + 8 * (pp & 1);
  }

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

  const int KT = (T + p8::BK - 1) / p8::BK;  // ragged last tile: rows >= T read as zeros
  const int NH = 4 * KT;             // half-images of the whole K loop
  // prologue: half-images 0 .. LEAD-1; 0 (A0) and 1 (B0) retired for phase 0
#pragma unroll
  for (int pc = 0; pc < 2; ++pc) ring_dma<0>(rsA, rsB, ldsw, vA, vB, sA, sB, 0, 0, pc);
#pragma unroll
  for (int pc = 0; pc < 2; ++pc) ring_dma<1>(rsA, rsB, ldsw, vA, vB, sA, sB, 1, 0, pc);
#pragma unroll
  for (int pc = 0; pc < 2; ++pc) ring_dma<2>(rsA, rsB, ldsw, vA, vB, sA, sB, 2, 0, pc);
#pragma unroll
  for (int pc = 0; pc < 2; ++pc) ring_dma<3>(rsA, rsB, ldsw, vA, vB, sA, sB, 3, 0, pc);
  if (LEAD > 4 && NH > 4) {
#pragma unroll
    for (int pc = 0; pc < 2; ++pc) ring_dma<0>(rsA, rsB, ldsw, vA, vB, sA, sB, 4, 1, pc);
  }
  if (LEAD > 5 && NH > 5) {
#pragma unroll
    for (int pc = 0; pc < 2; ++pc) ring_dma<1>(rsA, rsB, ldsw, vA, vB, sA, sB, 5, 1, pc);
  }
  if (NH >= LEAD) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (LEAD - 2)) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();
  if (grp == 1) bar();  // the stagger: waves 4-7 run one barrier behind

  auto phase = [&](auto pc, int kt) {
    constexpr int P = decltype(pc)::value;
    constexpr int MQ = (P == 0 || P == 1) ? 0 : 1, NQ = (P == 0 || P == 3) ? 0 : 1;
    const int n0h = 4 * kt;
    // half-image slots read this phase: A0 = n0h, B0 = n0h + 1, B1 = n0h + 2, A1 = n0h + 3
    const lds_t* ai = smem + ((n0h + (MQ ? 3 : 0)) % SLOTS) * IMGB;
    if constexpr (PROBE != 2 && (P == 0 || P == 2)) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) af[i][ks] = lds_tr(ai + aoff[i][0] + ks * 32 * RB, ai + aoff[i][1] + ks * 32 * RB);
    }
    if constexpr (PROBE != 2 && (P == 0 || P == 1)) {
      const lds_t* bi = smem + ((n0h + 1 + NQ) % SLOTS) * IMGB;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bfx8 v = lds_tr(bi + boff[j][0] + ks * 32 * RB, bi + boff[j][1] + ks * 32 * RB);
          if constexpr (NQ == 0) b0[j][ks] = v;
          else b1[j][ks] = v;
        }
    }
    // retire what the NEXT phase reads (p3 -> A0/B0 of kt+1, p0 -> B1, p1 -> A1, p2 -> none):
    // the last LEAD-3 (LEAD-2 at p2) half-images issued may stay in flight, unless the
    // issue stream was cut short at the end of the loop
    const int issue = n0h + P + LEAD;  // this phase's DMA (issued under its MFMAs)
    if (PROBE == 3) {
      // probe: DMA issued, never waited for inside the loop (wrong results)
    } else if (issue <= NH) {
      if constexpr (P == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (LEAD - 2)) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (LEAD - 3)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();
    if constexpr (PROBE != 2 && (P == 0 || P == 2)) {
#pragma unroll
      for (int i = 2; i < 4; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) af[i][ks] = lds_tr(ai + aoff[i][0] + ks * 32 * RB, ai + aoff[i][1] + ks * 32 * RB);
    }
    const int islot = issue % SLOTS, ikt = PROBE == 4 ? 0 : kt + (P + LEAD) / 4;  // probe 4: L2-hot source
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const bfx8 bv = NQ == 0 ? b0[j][ks] : b1[j][ks];
          acc[MQ * 4 + i][NQ * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bv,
                                                                                 acc[MQ * 4 + i][NQ * 2 + j], 0, 0, 0);
        }
      // the next half-image, one 1-KiB piece after the 4th and the 8th MFMA (spread over
      // the section instead, after the 8th and 16th: same time)
      if ((i == 0 || i == 1) && issue < NH && PROBE != 1) {
        __builtin_amdgcn_sched_barrier(0);
        ring_dma<(P + LEAD) % 4>(rsA, rsB, ldsw, vA, vB, sA, sB, islot, ikt, i);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    bar();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  for (int kt = 0; kt < KT; ++kt) {
    phase(I0(), kt);
    phase(I1(), kt);
    phase(I2(), kt);
    phase(I3(), kt);
  }
  if (grp == 0) bar();  // same barrier count in both groups
  if (PROBE == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = w.cm0 + (i >> 2) * 128 + wr * 64 + 16 * (i & 3) + 4 * G + r;
        float* p = w.C + (int64_t)m * w.ldc + w.cn0 + (j >> 1) * 128 + wc * 32 + 16 * (j & 1) + (lane & 15);
        *p = w.beta ? *p + acc[i][j][r] : acc[i][j][r];
      }
}


// ---- launch plan: kernel variant, tile width, tail split
struct Launch {
  int variant;  // 1 = 4-stage ring, 2 = 8-phase
  int bn;       // tile width (256 or 128; the 8-phase kernel is 256 only)
  int split;    // token ranges per tail tile (1 = none)
  int nfull, tail;
};

// Rounds of whole-tile time the grid takes on `cus` CUs with the tail cut `s` ways.
double rounds(int64_t nt, int s, int cus) {
  const int64_t nfull = (nt / cus) * cus, tail = nt - nfull;
  if (s <= 1 || tail == 0) return (double)((nt + cus - 1) / cus);
  return (double)(nfull / cus) + (double)((tail * s + cus - 1) / cus) / s;
}

// Split of the last partial round (1 = leave it).  Measured on MI355X
// (tools/bench_wgrad_split.py, T = 24576): cutting a last round that is at most half
// full in two wins (qkv 384 tiles +18 %, down 896 +3-12 %, TP-2 out 128 tiles +54 %),
// but a 3/4-full one cut in four loses 4-8 % (TP-2 qkv / down: the chip runs
// power-limited, so a partly idle round is not lost time in proportion, while the
// shorter units pay their prologue, epilogue and partial traffic four times).  Every
// range must be a whole number of K-tiles and the units must deal evenly over the 8 XCDs.
int pick_split(int64_t nt, int T, int bk, int cus, bool off) {
  const char* e = std::getenv("ST_WGRAD_SPLIT");  // 0: off (A/B); N > 1: force N ways
  const int forced = e ? std::atoi(e) : -1;
  const int64_t tail = nt % cus;
  if (off || forced == 0 || tail == 0) return 1;
  auto ok = [&](int s) { return T % (s * bk) == 0 && (tail * s) % 8 == 0 && (nt / cus) * cus % 8 == 0; };
  if (forced > 1) return ok(forced) ? forced : 1;
  if (tail * 2 > cus) return 1;
  for (int s = (int)std::min<int64_t>(8, cus / tail); s >= 2; --s)
    if (ok(s)) return s;
  return 1;
}

// -2: shape not supported (caller falls back)
int plan(int M, int N, int T, int variant, Launch& L) {
  if (M <= 0 || N <= 0 || T <= 0) return -2;
  if (M % BM || N % 128) return -2;  // any T: rows past T land in LDS as zeros (MoE experts)
  const int cus = 256;
  const bool nosplit = (variant & 16) != 0;  // +16: tail split off (ops/grad.py times both)
  variant &= 15;
  if (variant == 0) {
    const char* ve = std::getenv("ST_WGRAD_P8");
    variant = (ve && std::atoi(ve) == 1) ? 2 : 1;
  }
  L.variant = variant;
  if (variant == 2) {
    if (N % 256) return -2;
    L.bn = 256;
  } else {
    const char* be = std::getenv("ST_WGRAD_BN");  // force 128 / 256 (A/B)
    int bn = be ? std::atoi(be) : 0;
    if (bn != 128 && bn != 256) {
      // a 256x128 tile streams ~10 % less MFMA work per LDS byte: take it only where the
      // 256-wide grid, tail split included, would leave CUs idle for a real share of the time
      const int64_t t128 = (int64_t)(M / BM) * (N / 128);
      auto eff = [&](int64_t t, int bk) { return (double)t / cus / rounds(t, pick_split(t, T, bk, cus, nosplit), cus); };
      bn = (N % 256 == 0 && eff(t128 / 2, BK) * 1.08 >= eff(t128, BK)) ? 256 : 128;
    }
    if (bn == 256 && N % 256) return -2;
    L.bn = bn;
  }
  const int64_t nt = (int64_t)(M / BM) * (N / L.bn);
  L.split = pick_split(nt, T, variant == 2 ? p8::BK : BK, cus, nosplit);
  L.nfull = (int)((nt / cus) * cus);
  L.tail = (int)(nt - L.nfull);
  return 0;
}

}  // namespace

extern "C" {

int st_wgrad4(const void* A, int64_t lda, const void* B, int64_t ldb, float* C, int64_t ldc, int M, int N, int T,
              int beta, float* ws, hipStream_t st);
int64_t st_wgrad4_ws_elems(int M, int N, int T);
int st_wgrad4_grouped(const void* A, int64_t lda, const void* B, int64_t ldb, float* C, int64_t ldc,
                      int64_t strideC, int M, int N, int G, const int* offs, int T_total, int beta, hipStream_t st);

// fp32 workspace elements the tail split of this launch needs (0: none).
int64_t st_wgrad_ws_elems(int M, int N, int T, int variant) {
  if ((variant & 15) == 6) return (variant & 16) ? 0 : st_wgrad4_ws_elems(M, N, T);  // csrc/wgrad4.hip
  Launch L;
  if (plan(M, N, T, variant, L) || L.split <= 1) return 0;
  return (int64_t)(L.split - 1) * L.tail * BM * L.bn;
}

// 0 on success; -2: shape not supported by this kernel (caller falls back).
// variant: 0 = default (the 4-stage kernel, or the 8-phase one when ST_WGRAD_P8=1),
// 1 = the 4-stage kernel, 2 = the 8-phase kernel, 6 = csrc/wgrad4.hip (ops/grad.py times them per shape);
// + 16 = without the tail split.  ws: st_wgrad_ws_elems(...) fp32 elements (may be null when that is 0).
int st_wgrad_gemm(const void* A, int64_t lda, const void* B, int64_t ldb, float* C, int64_t ldc, int M,
                  int N, int T, int beta, int variant, float* ws, hipStream_t st) {
  if ((variant & 15) == 6)  // csrc/wgrad4.hip (+16: tail split off, no workspace)
    return st_wgrad4(A, lda, B, ldb, C, ldc, M, N, T, beta, (variant & 16) ? nullptr : ws, st);
  Launch L;
  if (plan(M, N, T, variant, L)) return -2;
  if (lda % 8 || ldb % 8 || lda < M || ldb < N || ldc < N) return -2;
  if (((uintptr_t)A | (uintptr_t)B) % 16 || (uintptr_t)C % 4) return -2;
  // 32-bit buffer offsets: every row a K-tile addresses -- up to T + 63 for a ragged last
  // tile -- must stay below 2^32 bytes, or its offset would wrap into range instead of
  // reading the descriptor's zero fill
  if (((int64_t)(T + 63) * lda + M) * 2 >= (int64_t)1 << 32) return -2;
  if (((int64_t)(T + 63) * ldb + N) * 2 >= (int64_t)1 << 32) return -2;
  if (L.split > 1 && (ws == nullptr || ldc % 4 || (uintptr_t)C % 16)) L.split = 1;  // the reduce reads C by 16 B
  const SplitPlan sp{ws, L.nfull, L.tail, L.split};
  const int nbm = M / BM, nbn = N / L.bn;
  const int grid = L.split > 1 ? L.nfull + L.tail * L.split : nbm * nbn;
  const bf16_t *a = (const bf16_t*)A, *b = (const bf16_t*)B;
  const int bt = beta ? 1 : 0;
#ifdef ST_PROBES
  // diagnostic library only (wrong results): 1 = no K-loop DMA, 2 = no LDS reads, 3 / 4 (8-phase)
  const char* pe = std::getenv("ST_WGRAD_PROBE");
  const int probe = pe ? std::atoi(pe) : 0;
  if (probe && L.variant == 2) {
    if (probe == 1) wgrad8_kernel<1><<<grid, NT, 0, st>>>(a, lda, b, ldb, C, ldc, M, N, T, bt, sp);
    else if (probe == 2) wgrad8_kernel<2><<<grid, NT, 0, st>>>(a, lda, b, ldb, C, ldc, M, N, T, bt, sp);
    else if (probe == 3) wgrad8_kernel<3><<<grid, NT, 0, st>>>(a, lda, b, ldb, C, ldc, M, N, T, bt, sp);
    else wgrad8_kernel<4><<<grid, NT, 0, st>>>(a, lda, b, ldb, C, ldc, M, N, T, bt, sp);
    return (int)hipGetLastError();
  }
  if (probe == 1) {
    if (L.bn == 256) wgrad_gemm_kernel<1, 256><<<grid, NT, 0, st>>>(a, lda, b, ldb, C, ldc, M, N, T, bt, sp, GroupPlan{});
    else wgrad_gemm_kernel<1, 128><<<grid, NT, 0, st>>>(a, lda, b, ldb, C, ldc, M, N, T, bt, sp, GroupPlan{});
    return (int)hipGetLastError();
  }
#endif
  if (L.variant == 2) wgrad8_kernel<0><<<grid, NT, 0, st>>>(a, lda, b, ldb, C, ldc, M, N, T, bt, sp);
  else if (L.bn == 256) wgrad_gemm_kernel<0, 256><<<grid, NT, 0, st>>>(a, lda, b, ldb, C, ldc, M, N, T, bt, sp, GroupPlan{});
  else wgrad_gemm_kernel<0, 128><<<grid, NT, 0, st>>>(a, lda, b, ldb, C, ldc, M, N, T, bt, sp, GroupPlan{});
  ST_HIP_CHECK(hipGetLastError());
  if (L.split > 1) {
    const dim3 rg(BM * L.bn / 1024, L.tail);
    if (L.bn == 256) wgrad_tail_reduce<256><<<rg, 256, 0, st>>>(C, ldc, ws, nbm, nbn, sp);
    else wgrad_tail_reduce<128><<<rg, 256, 0, st>>>(C, ldc, ws, nbm, nbn, sp);
  }
  return (int)hipGetLastError();
}

// Grouped weight gradient over G experts (MoE backward): C[g] (fp32, [G, M, N] with
// leading stride strideC) = beta * C[g] + A[rows of g]^T B[rows of g], rows of expert g =
// [offs[g-1], offs[g]) (int32 device prefix sums).  ONE launch for all experts, no host
// read of the counts; the 4-stage kernel handles any row count (ragged last K-tile zero
// filled).  T_total = rows of A / B (bounds every expert's range).  -2: unsupported shape.
int st_wgrad_grouped(const void* A, int64_t lda, const void* B, int64_t ldb, float* C, int64_t ldc,
                     int64_t strideC, int M, int N, int G, const int* offs, int T_total, int beta, hipStream_t st) {
  if (M <= 0 || N <= 0 || G <= 0) return -2;
  // csrc/wgrad4.hip's one-wave-per-SIMD kernel for experts of at least a chip's worth of 256 x 256
  // tiles (Mixtral: 1,792 per expert, proxy 136.3 -> 127.3 ms).  Small experts stay here: at
  // Qwen3-30B-A3B's 24-48 tiles per expert wgrad4 is faster alone but the proxy step 0.7 % slower
  // (its 128 KiB-LDS workgroups crowd out the concurrent streams; profiles/r05/wgrad4/).
  // ST_WGRAD_GROUPED4=1 / 0 forces it on / off.
  const char* g4 = std::getenv("ST_WGRAD_GROUPED4");
  const bool use4 = g4 ? std::atoi(g4) != 0 : (int64_t)(M / 256) * (N / 256) >= 256;
  if (use4) {
    const int rc = st_wgrad4_grouped(A, lda, B, ldb, C, ldc, strideC, M, N, G, offs, T_total, beta, st);
    if (rc != -2) return rc;
  }
  if (M % BM || N % 128 || lda % 8 || ldb % 8 || lda < M || ldb < N || ldc < N) return -2;
  if (((uintptr_t)A | (uintptr_t)B) % 16 || (uintptr_t)C % 4) return -2;
  if (((int64_t)(T_total + 63) * lda + M) * 2 >= (int64_t)1 << 32) return -2;
  if (((int64_t)(T_total + 63) * ldb + N) * 2 >= (int64_t)1 << 32) return -2;
  const int bn = (N % 256 == 0) ? 256 : 128;
  const int64_t grid = (int64_t)G * (M / BM) * (N / bn);
  if (grid >= (1LL << 31)) return -2;
  const GroupPlan gp{offs, G, strideC};
  const SplitPlan sp{nullptr, 0, 0, 1};
  const bf16_t *a = (const bf16_t*)A, *b = (const bf16_t*)B;
  const int bt = beta ? 1 : 0;
  if (bn == 256)
    wgrad_gemm_kernel<0, 256, true><<<(unsigned)grid, NT, 0, st>>>(a, lda, b, ldb, C, ldc, M, N, T_total, bt, sp, gp);
  else
    wgrad_gemm_kernel<0, 128, true><<<(unsigned)grid, NT, 0, st>>>(a, lda, b, ldb, C, ldc, M, N, T_total, bt, sp, gp);
  return (int)hipGetLastError();
}

}  // extern "C"

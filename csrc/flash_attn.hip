// Flash attention forward / backward for gfx950 (CDNA4), bf16 in / fp32 accumulate,
// head_dim 64 or 128, causal or full, GQA-native, with global position
// offsets for context-parallel (ring / zig-zag) blocks.
//
// Reference behaviour: F.scaled_dot_product_attention(q, k, v, is_causal) on
// K/V pre-expanded to H heads (scaletorch/models/attention_utils.py:130-152,
// scaletorch/models/llama.py:175-191) and the S^2-materialising ring block
// attention (scaletorch/parallel/context_parallel/context_parallel.py:266-364).
//
// Design (MI355X-first, not a CUDA tiling):
//   * MFMA v_mfma_f32_32x32x16_bf16; a wave owns 32 query rows (fwd, dQ) or 32
//     keys (dK/dV); 4 waves (256 threads) per workgroup.
//   * "swapped" products so every softmax statistic is LANE-LOCAL:
//       fwd   S^T = K Q^T   (query on the lane)  ->  O^T += V^T P^T
//       dQ    S^T, dP^T     (query on the lane)  ->  dQ^T += K^T dS^T
//       dK/dV S, dP         (key on the lane)    ->  dV^T += dO^T P, dK^T += Q^T dS
//     An accumulator whose ROW index is summed next is fed straight back as the
//     B operand (registers 8s..8s+7 -> k-step s, cdna_hip_programming.md §3);
//     the other operand is read with ds_read_b64_tr_b16 from a row-major LDS
//     image (T10), so no product needs an explicit transpose.
//   * one LDS image per tile, XOR-swizzled so both the 16-byte row reads and the
//     transposed reads are bank-conflict free (T2/T10).  Every LDS read in the
//     loops is `ds_read* vaddr offset:<imm>` on a lane-constant VGPR computed
//     once (LdsAddr); the double-buffer index is a template constant (the loop
//     is unrolled by two), so the loops carry no LDS address arithmetic.
//   * global -> LDS by LDS-DMA (`buffer_load_dwordx4 ... lds`, DmaStager): the
//     next tile is requested at the top of a step into the other buffer and
//     retired by the end-of-step barrier; buffer descriptors (T8/T20) give
//     32-bit offsets and zero-fill rows past the end of a sequence -- no
//     staging registers, no ds_write, no branches.
//   * with one wave per SIMD (backward kernels) fragment reads are issued a
//     k-step ahead and pinned above the MFMAs that precede their use
//     (sched_barrier); hipcc otherwise serialises read -> wait -> MFMA.
//   * online softmax in base 2 with raw v_exp_f32; the O rescale is deferred
//     until the running max grows by 2^8 (T13) and decided wave-uniformly.
//   * only the diagonal / tail blocks evaluate the causal mask.
//   * backward = preprocess (-delta = -rowsum(dO*O) and -lse*log2e per query row);
//     dK/dV kernel (per 128-key tile of one kv head, iterating every query head of
//     its GQA group x query blocks, so dK/dV are summed in registers).  Default
//     (ST_FLASH_BWD_DS=1): the dK/dV kernel also stores the dS it holds as bf16
//     dS^T tiles (raw MFMA fragment layout, compact causal workspace) and
//     dQ = dS K is a streaming kernel sharing each K tile over 4 query heads --
//     5 MFMA products instead of 7.  Otherwise a dQ kernel (per 128-query tile)
//     recomputes S and dP.  No atomics, no partial buffers, bitwise deterministic.
//   * dK/dV softmax per element: exp2(fma(S, c2, nlse2)) and one multiply (the dP
//     chain is seeded with -delta); the causal mask is a scalar branch applied
//     after the softmax, only on diagonal blocks.
//   * causal: workgroups are numbered heaviest-first so the dispatcher's
//     greedy fill is a longest-job-first schedule.
#include <cstdlib>
#include <type_traits>

#include "common.h"

using namespace st;

namespace {

typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
typedef __bf16 bfx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_t;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kRescaleThr = 8.f;  // log2 units: P entries stay <= 2^8 between rescales

// ---- LDS tile geometry: rows of D bf16, 16-byte chunks, XOR swizzle ----
template <int D>
ST_DEVICE int swz(int row) {
  if constexpr (D == 128) return ((row & 3) << 2) | ((row >> 2) & 3);
  else return (row >> 1) & 7;
}
template <int D>
ST_DEVICE int lds_off(int row, int ch) {
  return row * (2 * D) + 16 * (ch ^ swz<D>(row));
}

ST_DEVICE bfx8 lds_row(const lds_t* p) {
  return *reinterpret_cast<const bfx8 __attribute__((address_space(3)))*>(p);
}
ST_DEVICE bfx8 lds_tr(const lds_t* p0, const lds_t* p1) {
  bfx4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bfx4 __attribute__((address_space(3)))*)p0);
  bfx4 b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bfx4 __attribute__((address_space(3)))*)p1);
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// Lane-constant LDS offsets into one tile image.
//  rowf(tile, t, kk): 8 contiguous bf16 of tile row 32t + (lane&31), chunk
//    2kk + (lane>>5)  -- an MFMA A/B fragment in natural k order.
//  trf(tile, rbase, s, dt): element j of lane (r = lane&31, h = lane>>5) is
//    tile[rbase + 16s + 8(j>>2) + 4h + (j&3)][32dt + r] -- the operand whose k
//    index runs over tile ROWS, permuted to match an accumulator fed back as
//    the other operand (k-step s).
// Swizzle rows only depend on row & 15 (D=128) / bits 1..3 (D=64), so the
// 32-row sub-tile and 16-row k-step offsets are compile-time immediates.
template <int D>
struct LdsAddr {
  static constexpr int NKK = D / 16, NDT = D / 32, RB = 2 * D;
  int row[NKK];
  int tr[NDT][2];
  ST_DEVICE void init(int lane) {
    const int r = lane & 31, h = lane >> 5, g = (lane >> 4) & 1, q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) row[kk] = lds_off<D>(r, 2 * kk + h);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
        tr[dt][hf] = lds_off<D>(4 * h + q + 8 * hf, 4 * dt + 2 * g + (pp >> 1)) + 8 * (pp & 1);
  }
  ST_DEVICE bfx8 rowf(const lds_t* tile, int t, int kk) const {
    return lds_row(tile + t * 32 * RB + row[kk]);
  }
  ST_DEVICE bfx8 trf(const lds_t* tile, int rbase, int s, int dt) const {
    const lds_t* b = tile + (rbase + 16 * s) * RB;
    return lds_tr(b + tr[dt][0], b + tr[dt][1]);
  }
};

ST_DEVICE f32x16 mfma(bfx8 a, bfx8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Long-lived accumulators (dQ, dK, dV) live in the AGPR file for the whole
// loop: this file is built with -mllvm -amdgpu-mfma-vgpr-form so the
// compiler's own MFMAs (S, dP: read by VALU right away) stay in VGPRs, and
// these asm MFMAs pin the accumulate chains to AGPRs -- no per-iteration
// v_accvgpr copies.  `s_nop 1` covers the VALU-write -> MFMA-read hazard of
// the freshly converted B operand (cdna_hip_programming.md §5.7 item 2);
// MFMA -> MFMA on the same C needs none.
ST_DEVICE void mfma_acc(f32x16& c, bfx8 a, bfx8 b) {
  asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
// Ends the AGPR chains before compiler code reads them (8-pass XDL result ->
// any reader: >= 12 wait states).
template <int N>
ST_DEVICE void agpr_fence(f32x16 (&c)[N]) {
  if constexpr (N == 4)
    asm volatile("s_nop 15\n\ts_nop 3" : "+a"(c[0]), "+a"(c[1]), "+a"(c[2]), "+a"(c[3]));
  else
    asm volatile("s_nop 15\n\ts_nop 3" : "+a"(c[0]), "+a"(c[1]));
}

ST_DEVICE f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

typedef __bf16 bfx2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

ST_DEVICE bfx2 cvt2(float a, float b) {  // one v_cvt_pk_bf16_f32 (RNE)
  f32x2 v = {a, b};
  return __builtin_convertvector(v, bfx2);
}

// registers 8s..8s+7 of an accumulator -> bf16 fragment for k-step s
ST_DEVICE bfx8 acc_frag(const f32x16& a, int s) {
  const int o = 8 * s;
  const bfx2 p0 = cvt2(a[o], a[o + 1]), p1 = cvt2(a[o + 2], a[o + 3]);
  const bfx2 p2 = cvt2(a[o + 4], a[o + 5]), p3 = cvt2(a[o + 6], a[o + 7]);
  return __builtin_shufflevector(__builtin_shufflevector(p0, p1, 0, 1, 2, 3),
                                 __builtin_shufflevector(p2, p3, 0, 1, 2, 3), 0, 1, 2, 3, 4, 5, 6, 7);
}

// accumulator register -> row inside the 32x32 C tile, minus the 4h lane part
ST_DEVICE constexpr int acc_row0(int reg) { return (reg & 3) + 8 * (reg >> 2); }

ST_DEVICE float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Buffer descriptor over rows [0, rows) of a [rows, D] view with a row stride
// (elements); built from wave-uniform values only (T20) so no waterfall loops.
ST_DEVICE rsrc_t make_rsrc(const bf16_t* base, int rows, int64_t row_stride, int D) {
  const uint32_t bytes = rows > 0 ? (uint32_t)(((int64_t)(rows - 1) * row_stride + D) * 2) : 0u;
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

ST_DEVICE bfx8 bload_frag(rsrc_t rs, uint32_t off) {
  return __builtin_bit_cast(bfx8, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}

// Direct global -> LDS staging (buffer_load_dwordx4 ... lds): each wave
// instruction writes 1 KiB of LDS lane-linearly, so the XOR swizzle is applied
// on the SOURCE side -- lane l of a wave fetches the global chunk that belongs
// at LDS byte (base + 16 l) of the swizzled image.  No staging registers, no
// ds_write; rows past the descriptor's range land as zeros.
// Issued from inline asm (M0 = the wave's LDS base): hipcc cannot prove that
// the builtin form's LDS write misses the tile being read, so it drained every
// DMA with `s_waitcnt vmcnt(0)` before the step's first ds_read -- the next
// tile's load was never overlapped with this step's MFMAs.  Hidden from hipcc,
// the DMA is retired by hand at the end of the step (dma_barrier).
ST_DEVICE void lds_dma16(rsrc_t rs, lds_t* dst, uint32_t voff) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved: nothing else in these kernels uses it
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(m0), "v"(voff), "s"(rs)
               : "memory", "m0");
#pragma clang diagnostic pop
}

// The same 16-byte DMA with the non-temporal hint: for data read exactly once (the dS
// workspace in the dQ pass), so it streams past L2 instead of evicting re-read tiles.
ST_DEVICE void lds_dma16_nt(rsrc_t rs, lds_t* dst, uint32_t voff) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds"
               :
               : "s"(m0), "v"(voff), "s"(rs)
               : "memory", "m0");
#pragma clang diagnostic pop
}

// 4 bytes per lane (64 floats per wave-instruction): the per-query softmax
// statistics (lse, delta) of a 64-query block go through the same DMA path, so
// the loop carries no ordinary global load (hipcc would drain every DMA with
// vmcnt(0) to wait for it).
ST_DEVICE void lds_dma4(rsrc_t rs, lds_t* dst, uint32_t voff) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dword %1, %2, 0 offen lds"
               :
               : "s"(m0), "v"(voff), "s"(rs)
               : "memory", "m0");
#pragma clang diagnostic pop
}

ST_DEVICE rsrc_t make_rsrc_f32(const float* base, int n) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane((uint32_t)(n > 0 ? n * 4 : 0)),
                                           0x00020000);
}

// End of a pipeline step: this wave's LDS-DMA has landed (hipcc does not count
// the asm DMA, so the wait is explicit), then the workgroup barrier publishes
// every wave's tile and retires this step's LDS reads.
ST_DEVICE void dma_barrier() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

template <int D, int ROWS, int NWAVES = 4>  // the tile is split over the workgroup's NWAVES waves
struct DmaStager {
  static constexpr int RB = 2 * D, BYTES = ROWS * RB, PER_WAVE = BYTES / NWAVES, NI = PER_WAVE / 1024;
  static_assert(NI >= 1 && PER_WAVE % 1024 == 0, "tile must be whole KiB per wave");
  uint32_t voff[NI];
  uint32_t stride_bytes;
  int wave_base;
  ST_DEVICE void init(int wid, int lane, int64_t row_stride) {
    stride_bytes = (uint32_t)(row_stride * 2);
    wave_base = wid * PER_WAVE;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int a = wave_base + i * 1024 + lane * 16;
      const int row = a / RB, pos = (a % RB) / 16;
      voff[i] = (uint32_t)row * stride_bytes + (uint32_t)((pos ^ swz<D>(row)) * 16);
    }
  }
  ST_DEVICE void load(rsrc_t rs, lds_t* tile, int row0) const {
    const uint32_t o = (uint32_t)row0 * stride_bytes;
#pragma unroll
    for (int i = 0; i < NI; ++i) lds_dma16(rs, tile + wave_base + i * 1024, voff[i] + o);
  }
};

struct AttnParams {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  int B, Sq, Sk, H, Hkv;
  int64_t sqb, sqs, sqh, skb, sks, skh, svb, svs, svh;
  float scale;
  int causal;
  int64_t q_offset, k_offset;
  int64_t sxb, sxs, sxh;  // output strides (dQ for the dQ kernel, dK/dV for the dK/dV kernel)
};

template <int BUF>
using Buf = std::integral_constant<int, BUF>;

// Key-block range of a query tile [q0, q0+BM): blocks [0, nkb) are visible,
// blocks >= kb_mask need the per-element mask (diagonal, or the Sk tail when
// `tail_mask`).
template <int BM, int BN>
ST_DEVICE void key_blocks(const AttnParams& p, int q0, bool tail_mask, int& nkb, int& kb_mask) {
  nkb = (p.Sk + BN - 1) / BN;
  kb_mask = tail_mask ? p.Sk / BN : nkb;
  if (p.causal) {
    const int64_t last = p.q_offset + q0 + BM - 1 - p.k_offset;  // last key any row of the tile sees
    const int64_t lim = last < 0 ? 0 : last / BN + 1;
    if (lim < nkb) nkb = (int)lim;
    const int64_t full = p.q_offset + q0 - p.k_offset + 1;  // keys [0, full) visible to every row
    const int64_t fb = full <= 0 ? 0 : full / BN;
    if (fb < kb_mask) kb_mask = (int)fb;
  }
}

// Per-lane key limit inside key block kb for query row qg (global): key
// 32t + acc_row0(i) + 4h is visible iff it is <= the returned value.
ST_DEVICE int key_limit(const AttnParams& p, int kb, int BN, int64_t qg, int h, bool tail) {
  int64_t lim = tail ? (int64_t)p.Sk - 1 - (int64_t)kb * BN : (int64_t)BN;
  if (p.causal) {
    const int64_t c = qg - p.k_offset - (int64_t)kb * BN;
    if (c < lim) lim = c;
  }
  if (lim < -1) lim = -1;
  return (int)lim - 4 * h;
}

// ---- dS workspace of the dS-materialising backward (ST_FLASH_BWD_DS) ----
// The dK/dV kernel already holds dS = P (dP - delta) for every (query, key) it
// visits; instead of the dQ kernel recomputing S, dP and the softmax for the
// same pairs (3 of its MFMA products and all of its exp work), dK/dV stores dS
// once (bf16) and dQ becomes one product per tile, dQ^T += K^T dS^T.  With 288 GB
// of HBM the transient causal workspace (B*H*Sq*Sk bytes: 3.2 GB for Llama-3-8B
// at 6 x 4096) is affordable.
//
// Layout: per (b, q-head), the 64-key x 128-query tiles (kb, qt) that the dQ
// kernel visits, query tile major, key block minor, compact under the causal mask:
// tile (qt, kb) sits at prefix(qt) + kb, prefix(n) = sum_{t<n} nkb(t).  A tile is
// a dS^T tile [64 keys][128 queries] (16 KiB) in the dK/dV kernel's STORE order: one
// 1 KiB block per (key half wp, 64-query half qh, 32-query half u, 16-query group s),
// holding each lane's raw bf16 MFMA fragment -- lane (key r, half h) has the queries
// 16s + 4h + 0..3 (bytes 0-7) and 16s + 8 + 4h + 0..3 (bytes 8-15) -- at
// 16 (32 h + (r ^ (8 s + 4 h))).  So every dK/dV store instruction writes 1 KiB
// contiguous with no lane shuffles, and the dQ kernel DMAs the tile linearly into LDS
// where the XOR keeps its transposed reads (4 keys x 16 queries per 16-lane group)
// bank-conflict free.
//
// nkb(t) of query tile t (128 rows) is key_blocks<128, 64>'s nkb:
//   causal: clamp(2t + e, 0, NKB), e = floor((q_offset + 127 - k_offset) / 64) + 1
//   full:   NKB = ceil(Sk / 64)
__host__ __device__ inline int64_t ds_floordiv64(int64_t x) { return x >= 0 ? x / 64 : -((-x + 63) / 64); }
__host__ __device__ inline int ds_nkb(int causal, int Sk, int64_t q_offset, int64_t k_offset, int t) {
  const int NKB = (Sk + 63) / 64;
  if (!causal) return NKB;
  const int64_t v = 2 * (int64_t)t + ds_floordiv64(q_offset + 127 - k_offset) + 1;
  return v < 0 ? 0 : (v > NKB ? NKB : (int)v);
}
__host__ __device__ inline int64_t ds_prefix(int causal, int Sk, int64_t q_offset, int64_t k_offset, int n) {
  const int64_t NKB = (Sk + 63) / 64;
  if (n <= 0) return 0;
  if (!causal) return (int64_t)n * NKB;
  const int64_t e = ds_floordiv64(q_offset + 127 - k_offset) + 1;
  // first t with 2t + e >= 1 (t0) and with 2t + e >= NKB (t1); t1 >= t0 since NKB >= 1
  auto ceil_half = [](int64_t x) { return x >= 0 ? (x + 1) / 2 : -((-x) / 2); };
  int64_t t0 = ceil_half(1 - e), t1 = ceil_half(NKB - e);
  t0 = t0 < 0 ? 0 : (t0 > n ? n : t0);
  t1 = t1 < t0 ? t0 : (t1 > n ? n : t1);
  return (t1 - t0) * (t0 + t1 - 1) + e * (t1 - t0) + (n - t1) * NKB;
}
constexpr int kDsTile = 64 * 128;  // bf16 elements of one dS^T tile (16 KiB)
// byte offset of lane (key k in 0..63, half h)'s 16-byte fragment of block (qh, u, s)
ST_DEVICE int ds_off(int k, int qh, int u, int s, int h) {
  return 8192 * (k >> 5) + 4096 * qh + 2048 * u + 1024 * s + 512 * h + 16 * ((k & 31) ^ (8 * s + 4 * h));
}

// ============================================================== forward
// XCD: XCD-aware workgroup order (ST_FLASH_XCD=0 -> off, A/B).  HP: query heads per
// workgroup -- HP = 2 puts two heads of one GQA group in an 8-wave workgroup (waves
// 4s .. 4s+3 = head s), so every K / V tile is DMA'd into LDS once for both.
template <int D, bool XCD = true, int HP = 1>
__global__ __launch_bounds__(256 * HP, 2 / HP) void flash_fwd_kernel(AttnParams p, bf16_t* __restrict__ o,
                                                                     int64_t sob, int64_t sos, int64_t soh,
                                                                     float* __restrict__ lse) {
  constexpr int BM = 128, BN = 64, NKK = D / 16, NDT = D / 32;
  constexpr int TB = BN * D * 2;
  __shared__ __attribute__((aligned(16))) char smem_raw[4 * TB];  // K0 K1 V0 V1
  lds_t* smem = (lds_t*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, r = lane & 31, h = lane >> 5;
  const int wq = wid & 3;  // this wave's 32-query slice of the tile
  const int nqt = (p.Sq + BM - 1) / BM, id = blockIdx.x;
  int rank, b, hq;
  const int G = p.H / p.Hkv, BHk = p.B * p.Hkv, NG = G / HP;  // NG head groups per kv head
  if (XCD && BHk % 8 == 0) {
    // XCD-aware order (T1): the dispatcher deals workgroups round-robin to the 8 XCDs, so
    // XCD x = id % 8 takes every (batch, kv head) pair with index = x mod 8, all G query
    // heads of each: the K / V tiles its workgroups stream are shared by G concurrent
    // workgroups in that XCD's L2 instead of one per XCD.  Heaviest query tiles first.
    const int j = id >> 3, per_rank = (BHk >> 3) * NG, rem = j % per_rank;
    rank = j / per_rank;
    const int bhk = (id & 7) + 8 * (rem / NG);
    b = bhk / p.Hkv;
    hq = (bhk % p.Hkv) * G + (rem % NG) * HP;
  } else {
    const int BHG = p.B * p.H / HP;
    rank = id / BHG;
    b = (id % BHG) / (p.H / HP);
    hq = (id % (p.H / HP)) * HP;
  }
  hq += wid >> 2;
  const int qt = p.causal ? nqt - 1 - rank : rank;
  const int hk = hq / G;
  const int q0 = qt * BM, my_q = q0 + wq * 32 + r;

  const rsrc_t rq = make_rsrc(p.q + (int64_t)b * p.sqb + (int64_t)hq * p.sqh, p.Sq, p.sqs, D);
  const rsrc_t rk = make_rsrc(p.k + (int64_t)b * p.skb + (int64_t)hk * p.skh, p.Sk, p.sks, D);
  const rsrc_t rv = make_rsrc(p.v + (int64_t)b * p.svb + (int64_t)hk * p.svh, p.Sk, p.svs, D);

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[my_q][16kk + 8h .. +8]
  bfx8 qf[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk)
    qf[kk] = bload_frag(rq, (uint32_t)my_q * (uint32_t)(p.sqs * 2) + (2 * kk + h) * 16);

  // register fragments resident before the DMA pipeline starts: hipcc's own
  // vmcnt bookkeeping for these loads otherwise lands inside the loop, where
  // (the asm DMAs being invisible to it) a small vmcnt would wait for them
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  int nkb, kb_mask;
  key_blocks<BM, BN>(p, q0, true, nkb, kb_mask);

  LdsAddr<D> la;
  la.init(lane);
  DmaStager<D, BN, 4 * HP> sk, sv;
  sk.init(wid, lane, p.sks);
  sv.init(wid, lane, p.svs);

  f32x16 oacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) oacc[dt] = zero16();
  float m = -INFINITY, l = 0.f;
  const float c2 = p.scale * kLog2e;
  const int64_t qg = p.q_offset + my_q;

  if (nkb > 0) {
    sk.load(rk, smem, 0);
    sv.load(rv, smem + 2 * TB, 0);
  }
  dma_barrier();

  auto step = [&](auto bufc, int kb) {
    constexpr int BUF = decltype(bufc)::value;
    const bool more = kb + 1 < nkb;
    if (more) {
      sk.load(rk, smem + (BUF ^ 1) * TB, (kb + 1) * BN);
      sv.load(rv, smem + (2 + (BUF ^ 1)) * TB, (kb + 1) * BN);
    }
    const lds_t* kt = smem + BUF * TB;
    const lds_t* vt = smem + (2 + BUF) * TB;
    f32x16 s0 = zero16(), s1 = zero16();
    // K row fragments one k-step ahead, pinned above the MFMAs that precede
    // their use (hipcc otherwise emits read -> wait -> MFMA for every k-step)
    bfx8 fk[NKK][2];
    fk[0][0] = la.rowf(kt, 0, 0);
    fk[0][1] = la.rowf(kt, 1, 0);
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      if (kk + 1 < NKK) {
        fk[kk + 1][0] = la.rowf(kt, 0, kk + 1);
        fk[kk + 1][1] = la.rowf(kt, 1, kk + 1);
      }
      __builtin_amdgcn_sched_barrier(0);
      s0 = mfma(fk[kk][0], qf[kk], s0);
      s1 = mfma(fk[kk][1], qf[kk], s1);
    }
    if (kb >= kb_mask) {
      const int lim = key_limit(p, kb, BN, qg, h, true);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (acc_row0(i) > lim) s0[i] = -INFINITY;
        if (acc_row0(i) + 32 > lim) s1[i] = -INFINITY;
      }
    }
    float mx0 = fmaxf(s0[0], s1[0]), mx1 = fmaxf(s0[1], s1[1]);
#pragma unroll
    for (int i = 2; i < 16; i += 2) {
      mx0 = fmaxf(mx0, fmaxf(s0[i], s1[i]));
      mx1 = fmaxf(mx1, fmaxf(s0[i + 1], s1[i + 1]));
    }
    float mx = fmaxf(mx0, mx1);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mxs = mx * c2;
    if (__any(mxs > m + kRescaleThr)) {  // T13: rare after the first blocks
      const float m_new = fmaxf(m, mxs);
      const float alpha = (m == m_new) ? 1.f : fast_exp2(m - m_new);
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;
      m = m_new;
    }
    const float mu = (m == -INFINITY) ? 0.f : m;
    float r0 = 0.f, r1 = 0.f, r2 = 0.f, r3 = 0.f;
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      s0[i] = fast_exp2(fmaf(s0[i], c2, -mu));
      s1[i] = fast_exp2(fmaf(s1[i], c2, -mu));
      s0[i + 1] = fast_exp2(fmaf(s0[i + 1], c2, -mu));
      s1[i + 1] = fast_exp2(fmaf(s1[i + 1], c2, -mu));
      r0 += s0[i];
      r1 += s1[i];
      r2 += s0[i + 1];
      r3 += s1[i + 1];
    }
    float rs = (r0 + r1) + (r2 + r3);
    rs += __shfl_xor(rs, 32, 64);
    l += rs;
    const bfx8 p00 = acc_frag(s0, 0), p01 = acc_frag(s0, 1), p10 = acc_frag(s1, 0), p11 = acc_frag(s1, 1);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      oacc[dt] = mfma(la.trf(vt, 0, 0, dt), p00, oacc[dt]);
      oacc[dt] = mfma(la.trf(vt, 0, 1, dt), p01, oacc[dt]);
      oacc[dt] = mfma(la.trf(vt, 32, 0, dt), p10, oacc[dt]);
      oacc[dt] = mfma(la.trf(vt, 32, 1, dt), p11, oacc[dt]);
    }
    dma_barrier();
  };
  int kb = 0;  // unconditional pairs (see the dQ kernel)
  for (; kb + 1 < nkb; kb += 2) {
    step(Buf<0>(), kb);
    step(Buf<1>(), kb + 1);
  }
  if (kb < nkb) step(Buf<0>(), kb);

  if (my_q < p.Sq) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16_t* orow = o + (int64_t)b * sob + (int64_t)my_q * sos + (int64_t)hq * soh;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * h;
        uint2 w;
        w.x = pack_bf16x2(oacc[dt][4 * g + 0] * inv, oacc[dt][4 * g + 1] * inv);
        w.y = pack_bf16x2(oacc[dt][4 * g + 2] * inv, oacc[dt][4 * g + 3] * inv);
        *reinterpret_cast<uint2*>(orow + d) = w;
      }
    }
    if (h == 0)
      lse[((int64_t)b * p.H + hq) * p.Sq + my_q] = l > 0.f ? (m * kLn2 + __logf(l)) : -INFINITY;
  }
}

// ============================================================== forward, 8-wave ping-pong
// 256 queries per workgroup in two groups of 4 waves (A = waves 0-3, queries
// 0-127; B = waves 4-7, queries 128-255); wave w and w+4 share a SIMD.  Every key
// block k is split into two phases separated by workgroup barriers:
//   X(k): PV(k-1) MFMAs (P of the previous block against V(k-1)) + S(k) = K(k) Q^T MFMAs
//   Y(k): the softmax of S(k) (VALU / transcendental), P(k) fragments, running max/sum
// Group B starts one barrier late, so on every SIMD one wave runs its MFMA phase
// while its partner runs the softmax phase (MI355X_MICROARCH.md "Two waves per
// SIMD"): the matrix pipe no longer idles during the exp/convert work.  K(k+1)
// and V(k) are DMA'd (LDS-DMA, XOR-swizzled images as in the 4-wave kernel) by
// group B during its softmax phase, into double-buffered slots whose previous
// contents were last read one barrier earlier; they are retired by B's
// vmcnt(0) before the next odd barrier.  Interval i: k = i/2; even i: A X(k), B
// Y(k-1) + DMA; odd i: A Y(k), B X(k).  2*nkb+2 intervals, same barrier count in
// both groups.
template <int D>
__global__ __launch_bounds__(512, 1) void flash_fwd_pp_kernel(AttnParams p, bf16_t* __restrict__ o,
                                                              int64_t sob, int64_t sos, int64_t soh,
                                                              float* __restrict__ lse) {
  constexpr int BM = 256, BG = 128, BN = 64, NKK = D / 16, NDT = D / 32;
  constexpr int TB = BN * D * 2;
  __shared__ __attribute__((aligned(16))) char smem_raw[4 * TB];  // K0 K1 V0 V1
  lds_t* smem = (lds_t*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2, wg = wid & 3;
  const int BH = p.B * p.H, nqt = (p.Sq + BM - 1) / BM, id = blockIdx.x;
  const int qt = p.causal ? nqt - 1 - id / BH : id / BH;
  const int bh = id % BH, b = bh / p.H, hq = bh % p.H, hk = hq / (p.H / p.Hkv);
  const int q0 = qt * BM, g0 = q0 + grp * BG, my_q = g0 + wg * 32 + r;

  const rsrc_t rq = make_rsrc(p.q + (int64_t)b * p.sqb + (int64_t)hq * p.sqh, p.Sq, p.sqs, D);
  const rsrc_t rk = make_rsrc(p.k + (int64_t)b * p.skb + (int64_t)hk * p.skh, p.Sk, p.sks, D);
  const rsrc_t rv = make_rsrc(p.v + (int64_t)b * p.svb + (int64_t)hk * p.svh, p.Sk, p.svs, D);
  bfx8 qf[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk)
    qf[kk] = bload_frag(rq, (uint32_t)my_q * (uint32_t)(p.sqs * 2) + (2 * kk + h) * 16);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): fragments resident before the DMA pipeline
  int nkb, kbm_unused, my_nkb, kb_mask;
  key_blocks<BM, BN>(p, q0, true, nkb, kbm_unused);  // blocks any query of the workgroup sees
  key_blocks<BG, BN>(p, g0, true, my_nkb, kb_mask);   // blocks this group's queries see

  LdsAddr<D> la;
  la.init(lane);
  DmaStager<D, BN> sk, sv;  // group B (4 waves) moves every tile
  sk.init(wg, lane, p.sks);
  sv.init(wg, lane, p.svs);

  f32x16 oacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) oacc[dt] = zero16();
  f32x16 s0 = zero16(), s1 = zero16();
  bfx8 p00 = {}, p01 = {}, p10 = {}, p11 = {};
  float m = -INFINITY, l = 0.f;
  const float c2 = p.scale * kLog2e;
  const int64_t qg = p.q_offset + my_q;

  if (grp == 1 && nkb > 0) sk.load(rk, smem, 0);
  dma_barrier();
  if (grp == 1) __builtin_amdgcn_s_setprio(1);  // the younger half wins arbitration (item 4)

  auto xphase = [&](auto kpar, int k) {
    constexpr int KP = decltype(kpar)::value;
    if (k >= 1 && k - 1 < my_nkb) {  // PV(k-1)
      const lds_t* vt = smem + (2 + (KP ^ 1)) * TB;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        oacc[dt] = mfma(la.trf(vt, 0, 0, dt), p00, oacc[dt]);
        oacc[dt] = mfma(la.trf(vt, 0, 1, dt), p01, oacc[dt]);
        oacc[dt] = mfma(la.trf(vt, 32, 0, dt), p10, oacc[dt]);
        oacc[dt] = mfma(la.trf(vt, 32, 1, dt), p11, oacc[dt]);
      }
    }
    if (k < my_nkb) {  // S(k)
      const lds_t* kt = smem + KP * TB;
      s0 = zero16();
      s1 = zero16();
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        s0 = mfma(la.rowf(kt, 0, kk), qf[kk], s0);
        s1 = mfma(la.rowf(kt, 1, kk), qf[kk], s1);
      }
    }
  };
  auto yphase = [&](int k) {
    if (k < 0 || k >= my_nkb) return;
    if (k >= kb_mask) {
      const int lim = key_limit(p, k, BN, qg, h, true);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (acc_row0(i) > lim) s0[i] = -INFINITY;
        if (acc_row0(i) + 32 > lim) s1[i] = -INFINITY;
      }
    }
    float mx0 = fmaxf(s0[0], s1[0]), mx1 = fmaxf(s0[1], s1[1]);
#pragma unroll
    for (int i = 2; i < 16; i += 2) {
      mx0 = fmaxf(mx0, fmaxf(s0[i], s1[i]));
      mx1 = fmaxf(mx1, fmaxf(s0[i + 1], s1[i + 1]));
    }
    float mx = fmaxf(mx0, mx1);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mxs = mx * c2;
    if (__any(mxs > m + kRescaleThr)) {  // T13
      const float m_new = fmaxf(m, mxs);
      const float alpha = (m == m_new) ? 1.f : fast_exp2(m - m_new);
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;
      m = m_new;
    }
    const float mu = (m == -INFINITY) ? 0.f : m;
    float r0 = 0.f, r1 = 0.f, r2 = 0.f, r3 = 0.f;
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      s0[i] = fast_exp2(fmaf(s0[i], c2, -mu));
      s1[i] = fast_exp2(fmaf(s1[i], c2, -mu));
      s0[i + 1] = fast_exp2(fmaf(s0[i + 1], c2, -mu));
      s1[i + 1] = fast_exp2(fmaf(s1[i + 1], c2, -mu));
      r0 += s0[i];
      r1 += s1[i];
      r2 += s0[i + 1];
      r3 += s1[i + 1];
    }
    float rs = (r0 + r1) + (r2 + r3);
    rs += __shfl_xor(rs, 32, 64);
    l += rs;
    p00 = acc_frag(s0, 0);
    p01 = acc_frag(s0, 1);
    p10 = acc_frag(s1, 0);
    p11 = acc_frag(s1, 1);
  };
  auto bar = [] {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // One key block = two intervals (even, odd); the slot parity of k is a template
  // constant.  Each group runs its own straight-line loop (same barrier count).
  // No lambda captures another lambda: a captured closure object keeps pointers
  // to the accumulators alive and pins them in scratch.
  // A: even X(k) | odd Y(k).   B: even Y(k-1) + DMA K(k+1), V(k) | odd X(k).
  if (grp == 0) {
    for (int k = 0; k <= nkb; k += 2) {
      xphase(Buf<0>(), k);
      bar();
      yphase(k);
      bar();
      if (k + 1 <= nkb) {
        xphase(Buf<1>(), k + 1);
        bar();
        yphase(k + 1);
        bar();
      }
    }
  } else {
    for (int k = 0; k <= nkb; k += 2) {
      if (k + 1 < nkb) sk.load(rk, smem + TB, (k + 1) * BN);
      if (k < nkb) sv.load(rv, smem + 2 * TB, k * BN);
      yphase(k - 1);
      bar();
      xphase(Buf<0>(), k);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // DMAs retired before the odd barrier
      bar();
      if (k + 1 <= nkb) {
        if (k + 2 < nkb) sk.load(rk, smem, (k + 2) * BN);
        if (k + 1 < nkb) sv.load(rv, smem + 3 * TB, (k + 1) * BN);
        yphase(k);
        bar();
        xphase(Buf<1>(), k + 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bar();
      }
    }
  }
  __builtin_amdgcn_s_setprio(0);

  if (my_q < p.Sq) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16_t* orow = o + (int64_t)b * sob + (int64_t)my_q * sos + (int64_t)hq * soh;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * h;
        uint2 w;
        w.x = pack_bf16x2(oacc[dt][4 * g + 0] * inv, oacc[dt][4 * g + 1] * inv);
        w.y = pack_bf16x2(oacc[dt][4 * g + 2] * inv, oacc[dt][4 * g + 3] * inv);
        *reinterpret_cast<uint2*>(orow + d) = w;
      }
    }
    if (h == 0)
      lse[((int64_t)b * p.H + hq) * p.Sq + my_q] = l > 0.f ? (m * kLn2 + __logf(l)) : -INFINITY;
  }
}

// ============================================================== backward: delta
// Per query row: ndelta = -rowsum(dO * O) and nlse2 = -lse * log2(e), the two row
// constants of the backward in the form the dK/dV kernel consumes without VALU work:
// -delta seeds the dP accumulator (dP - delta comes out of the MFMA chain) and
// P = exp2(S c2 + nlse2) is one fma + exp per element.
template <int D>
__global__ __launch_bounds__(256) void flash_bwd_pre_kernel(const bf16_t* __restrict__ o,
                                                            const bf16_t* __restrict__ dout,
                                                            const float* __restrict__ lse,
                                                            float* __restrict__ delta, float* __restrict__ nlse2,
                                                            int B, int S, int H, int64_t sob, int64_t sos,
                                                            int64_t soh, int64_t sdb, int64_t sds,
                                                            int64_t sdh) {
  constexpr int NCH = D / 8;  // lanes per row
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t row = t / NCH;  // row = (b*S + s)*H + h
  const int ch = (int)(t % NCH);
  const int64_t nrows = (int64_t)B * S * H;
  float acc = 0.f;
  int b = 0, s = 0, hh = 0;
  if (row < nrows) {
    hh = (int)(row % H);
    const int64_t bs = row / H;
    s = (int)(bs % S);
    b = (int)(bs / S);
    float x[8], y[8];
    unpack8(ld8(o + b * sob + s * sos + hh * soh + ch * 8), x);
    unpack8(ld8(dout + b * sdb + s * sds + hh * sdh + ch * 8), y);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += x[i] * y[i];
  }
#pragma unroll
  for (int w = NCH / 2; w > 0; w >>= 1) acc += __shfl_xor(acc, w, 64);
  if (row < nrows && ch == 0) {
    const int64_t li = ((int64_t)b * H + hh) * S + s;
    delta[li] = -acc;
    nlse2[li] = -lse[li] * kLog2e;
  }
}

// ============================================================== backward: dQ
// One workgroup = 128 queries of one (b, q-head); iterates the visible key
// blocks.  S^T and dP^T keep the query on the lane, so lse/delta are scalars
// per lane; dQ^T += K^T dS^T feeds dS^T back as the B operand.  Keys past Sk
// read as zero (K = V = 0 => dS^T K^T contributes nothing), so only the causal
// diagonal is masked.
template <int D, int PROBE = 0>  // PROBE 1 (diagnostic library only): softmax / dS VALU skipped, wrong results
__global__ __launch_bounds__(256, 1) void flash_bwd_dq_kernel(AttnParams p,
                                                              const bf16_t* __restrict__ dout,
                                                              int64_t sdb, int64_t sds, int64_t sdh,
                                                              const float* __restrict__ lse,
                                                              const float* __restrict__ delta,
                                                              bf16_t* __restrict__ dq, int nsplit,
                                                              float* __restrict__ part) {
  constexpr int BM = 128, BN = 64, NKK = D / 16, NDT = D / 32;
  constexpr int TB = BN * D * 2;
  __shared__ __attribute__((aligned(16))) char smem_raw[4 * TB];  // K0 K1 V0 V1
  lds_t* smem = (lds_t*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, r = lane & 31, h = lane >> 5;
  const int BH = p.B * p.H, nqt = (p.Sq + BM - 1) / BM, id = blockIdx.x;
  // heaviest query tiles first; each tile's key range may be cut into nsplit workgroups
  // (short causal grids, see st_flash_bwd)
  const int rank = id / (BH * nsplit), sp = (id / BH) % nsplit;
  const int qt = p.causal ? nqt - 1 - rank : rank;
  const int bh = id % BH, b = bh / p.H, hq = bh % p.H, hk = hq / (p.H / p.Hkv);
  const int q0 = qt * BM, my_q = q0 + wid * 32 + r;

  const rsrc_t rq = make_rsrc(p.q + (int64_t)b * p.sqb + (int64_t)hq * p.sqh, p.Sq, p.sqs, D);
  const rsrc_t rdo = make_rsrc(dout + (int64_t)b * sdb + (int64_t)hq * sdh, p.Sq, sds, D);
  const rsrc_t rk = make_rsrc(p.k + (int64_t)b * p.skb + (int64_t)hk * p.skh, p.Sk, p.sks, D);
  const rsrc_t rv = make_rsrc(p.v + (int64_t)b * p.svb + (int64_t)hk * p.svh, p.Sk, p.svs, D);

  bfx8 qf[NKK], df[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    qf[kk] = bload_frag(rq, (uint32_t)my_q * (uint32_t)(p.sqs * 2) + (2 * kk + h) * 16);
    df[kk] = bload_frag(rdo, (uint32_t)my_q * (uint32_t)(sds * 2) + (2 * kk + h) * 16);
  }
  const int64_t li = ((int64_t)b * p.H + hq) * p.Sq + my_q;
  const float lse2 = my_q < p.Sq ? lse[li] * kLog2e : 0.f;
  const float dlt = my_q < p.Sq ? -delta[li] : 0.f;  // the pre kernel stores -delta
  // register fragments resident before the DMA pipeline starts: hipcc's own
  // vmcnt bookkeeping for these loads otherwise lands inside the loop, where
  // (the asm DMAs being invisible to it) a small vmcnt would wait for them
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  const float c2 = p.scale * kLog2e;
  const int64_t qg = p.q_offset + my_q;

  int nkb, kb_mask;
  key_blocks<BM, BN>(p, q0, false, nkb, kb_mask);
  const int kb0 = (int)((int64_t)nkb * sp / nsplit), kb1 = (int)((int64_t)nkb * (sp + 1) / nsplit);

  LdsAddr<D> la;
  la.init(lane);
  DmaStager<D, BN> sk, sv;
  sk.init(wid, lane, p.sks);
  sv.init(wid, lane, p.svs);

  f32x16 dqacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dqacc[dt] = zero16();

  if (kb0 < kb1) {
    sk.load(rk, smem, kb0 * BN);
    sv.load(rv, smem + 2 * TB, kb0 * BN);
  }
  dma_barrier();

  auto step = [&](auto bufc, int kb) {
    constexpr int BUF = decltype(bufc)::value;
    const bool more = kb + 1 < kb1;
    if (more) {
      sk.load(rk, smem + (BUF ^ 1) * TB, (kb + 1) * BN);
      sv.load(rv, smem + (2 + (BUF ^ 1)) * TB, (kb + 1) * BN);
    }
    const lds_t* kt = smem + BUF * TB;
    const lds_t* vt = smem + (2 + BUF) * TB;
    f32x16 s0 = zero16(), s1 = zero16(), d0 = zero16(), d1 = zero16();
    // K/V row fragments one k-step ahead, pinned above the MFMAs (1 wave/SIMD)
    bfx8 fk[NKK][2], fv[NKK][2];
    auto load_k = [&](int kk) {
      fk[kk][0] = la.rowf(kt, 0, kk);
      fk[kk][1] = la.rowf(kt, 1, kk);
      fv[kk][0] = la.rowf(vt, 0, kk);
      fv[kk][1] = la.rowf(vt, 1, kk);
    };
    load_k(0);
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      if (kk + 1 < NKK) load_k(kk + 1);
      __builtin_amdgcn_sched_barrier(0);
      s0 = mfma(fk[kk][0], qf[kk], s0);
      s1 = mfma(fk[kk][1], qf[kk], s1);
      d0 = mfma(fv[kk][0], df[kk], d0);
      d1 = mfma(fv[kk][1], df[kk], d1);
    }
#pragma unroll
    for (int i = 0; i < (PROBE ? 0 : 16); ++i) {
      const float pa = fast_exp2(fmaf(s0[i], c2, -lse2));
      const float pb = fast_exp2(fmaf(s1[i], c2, -lse2));
      s0[i] = pa * (d0[i] - dlt);
      s1[i] = pb * (d1[i] - dlt);
    }
    if (kb >= kb_mask) {
      const int lim = key_limit(p, kb, BN, qg, h, false);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (acc_row0(i) > lim) s0[i] = 0.f;
        if (acc_row0(i) + 32 > lim) s1[i] = 0.f;
      }
    }
    const bfx8 g00 = acc_frag(s0, 0), g01 = acc_frag(s0, 1), g10 = acc_frag(s1, 0), g11 = acc_frag(s1, 1);
    bfx8 tk[NDT][4];
    auto load_t = [&](int dt) {
      tk[dt][0] = la.trf(kt, 0, 0, dt);
      tk[dt][1] = la.trf(kt, 0, 1, dt);
      tk[dt][2] = la.trf(kt, 32, 0, dt);
      tk[dt][3] = la.trf(kt, 32, 1, dt);
    };
    load_t(0);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      if (dt + 1 < NDT) load_t(dt + 1);
      __builtin_amdgcn_sched_barrier(0);
      mfma_acc(dqacc[dt], tk[dt][0], g00);
      mfma_acc(dqacc[dt], tk[dt][1], g01);
      mfma_acc(dqacc[dt], tk[dt][2], g10);
      mfma_acc(dqacc[dt], tk[dt][3], g11);
    }
    dma_barrier();
  };
  // pairs of steps with no branch between them: a conditional second step
  // merges two copies of the AGPR accumulators, and hipcc resolved that merge by
  // parking dQ in VGPRs (64 v_accvgpr copies a pair + spills of Q/dO fragments)
  int kb = kb0;
  for (; kb + 1 < kb1; kb += 2) {
    step(Buf<0>(), kb);
    step(Buf<1>(), kb + 1);
  }
  if (kb < kb1) step(Buf<0>(), kb);

  agpr_fence(dqacc);
  if (nsplit > 1) {
    // fp32 partial [split][B*H][Sq][D], summed in split order by dq_split_reduce_kernel
    if (my_q < p.Sq) {
      float* pq = part + ((int64_t)sp * BH + bh) * p.Sq * D + (int64_t)my_q * D;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(pq + 32 * dt + 8 * g + 4 * h) =
              make_float4(dqacc[dt][4 * g] * p.scale, dqacc[dt][4 * g + 1] * p.scale,
                          dqacc[dt][4 * g + 2] * p.scale, dqacc[dt][4 * g + 3] * p.scale);
    }
    return;
  }
  if (my_q < p.Sq) {
    bf16_t* row = dq +(int64_t)b * p.sxb + (int64_t)my_q * p.sxs + (int64_t)hq * p.sxh;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * h;
        uint2 w;
        w.x = pack_bf16x2(dqacc[dt][4 * g + 0] * p.scale, dqacc[dt][4 * g + 1] * p.scale);
        w.y = pack_bf16x2(dqacc[dt][4 * g + 2] * p.scale, dqacc[dt][4 * g + 3] * p.scale);
        *reinterpret_cast<uint2*>(row + d) = w;
      }
    }
  }
}

// ============================================================== backward: dQ from stored dS
// dS-materialising backward (ST_FLASH_BWD_DS): dQ^T += K^T dS^T over the visible
// key blocks, both operands by transposed LDS reads of LDS-DMA'd tiles (K as in
// the dQ kernel above; dS^T tiles written pre-swizzled by the dK/dV kernel, copied
// linearly).  One MFMA product per tile instead of three and no softmax, so the
// kernel is bound by the bytes it streams into LDS (measured ~14 B/clk/CU with one
// head per workgroup, where every dS tile brought its own copy of the K tile): one
// workgroup now serves GH query heads of one kv head -- each K tile is staged once
// for GH dS tiles and its fragments are read once per wave for GH heads' MFMAs.
// 4 waves x 32 queries; dQ of the GH heads stays in AGPRs (GH x D/32 tiles).
template <int D, int GH>
__global__ __launch_bounds__(256, 1) void flash_bwd_dq_ds_kernel(AttnParams p, const bf16_t* __restrict__ dsw,
                                                                 bf16_t* __restrict__ dq, int nsplit,
                                                                 float* __restrict__ part) {
  constexpr int BM = 128, BN = 64, NDT = D / 32;
  constexpr int TK = BN * D * 2, TS = kDsTile * 2;
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * TK + 2 * GH * TS];  // K0 K1 | dS[buf][head]
  lds_t* smem = (lds_t*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, r = lane & 31, h = lane >> 5;
  const int G = p.H / p.Hkv, NG = G / GH;  // head groups per kv head
  const int BHG = p.B * p.Hkv * NG, nqt = (p.Sq + BM - 1) / BM, id = blockIdx.x;
  const int rank = id / (BHG * nsplit), sp = (id / BHG) % nsplit;
  const int qt = p.causal ? nqt - 1 - rank : rank;
  const int bhg = id % BHG, b = bhg / (p.Hkv * NG), hk = (bhg / NG) % p.Hkv;
  const int hq0 = hk * G + (bhg % NG) * GH;  // first query head of this workgroup
  const int q0 = qt * BM, my_q = q0 + wid * 32 + r;

  const rsrc_t rk = make_rsrc(p.k + (int64_t)b * p.skb + (int64_t)hk * p.skh, p.Sk, p.sks, D);
  const int64_t per_bh = ds_prefix(p.causal, p.Sk, p.q_offset, p.k_offset, nqt);
  // the GH heads' tile regions as rows of 128 bf16 (64 rows a tile); offsets fit 32 bits (host check)
  const rsrc_t rs = make_rsrc(dsw + ((int64_t)b * p.H + hq0) * per_bh * kDsTile, (int)(GH * per_bh * 64), 128, 128);
  const uint32_t t0 = (uint32_t)ds_prefix(p.causal, p.Sk, p.q_offset, p.k_offset, qt);

  int nkb, kb_mask;
  key_blocks<BM, BN>(p, q0, false, nkb, kb_mask);
  const int kb0 = (int)((int64_t)nkb * sp / nsplit), kb1 = (int)((int64_t)nkb * (sp + 1) / nsplit);

  LdsAddr<D> la;
  la.init(lane);
  // transposed-read addresses into a dS^T tile (ds_off layout) for this wave's 32 query
  // columns 32 wid + 16 g + 4 pp + 0..3: read hf of k-step (key half u, s) takes keys
  // 32u + 16s + 8hf + 4h + q (the k order of LdsAddr::trf); queries 16g + 4pp of the 32-query
  // half wid & 1 are fragment piece pp >> 1 of the writer's lane half pp & 1, block s = g
  int sa[2];
  {
    const int g = (lane >> 4) & 1, q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
      sa[hf] = ds_off(8 * hf + 4 * h + q, wid >> 1, wid & 1, g, pp & 1) + 8 * (pp >> 1);
  }
  DmaStager<D, BN> sk;
  sk.init(wid, lane, p.sks);
  // the GH 16 KiB dS^T tiles of key block kb, 4 KiB of each per wave, copied linearly
  uint32_t sv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) sv[i] = (uint32_t)(wid * (TS / 4) + i * 1024 + lane * 16);
  const uint32_t head_stride = (uint32_t)(per_bh * TS);
  auto load_ds = [&](lds_t* dst, int kb) {
    const uint32_t o = (t0 + (uint32_t)kb) * (uint32_t)TS;
#pragma unroll
    for (int j = 0; j < GH; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        lds_dma16_nt(rs, dst + j * TS + wid * (TS / 4) + i * 1024, o + (uint32_t)j * head_stride + sv[i]);
  };

  f32x16 dqacc[GH][NDT];
#pragma unroll
  for (int j = 0; j < GH; ++j)
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) dqacc[j][dt] = zero16();

  if (kb0 < kb1) {
    sk.load(rk, smem, kb0 * BN);
    load_ds(smem + 2 * TK, kb0);
  }
  dma_barrier();

  auto step = [&](auto bufc, int kb) {
    constexpr int BUF = decltype(bufc)::value;
    if (kb + 1 < kb1) {
      sk.load(rk, smem + (BUF ^ 1) * TK, (kb + 1) * BN);
      load_ds(smem + 2 * TK + (BUF ^ 1) * GH * TS, kb + 1);
    }
    const lds_t* kt = smem + BUF * TK;
    const lds_t* st = smem + 2 * TK + BUF * GH * TS;
    // B operands: dS^T columns of this wave's 32 queries per head, k-steps (key half u, s)
    bfx8 g[GH][4];
#pragma unroll
    for (int j = 0; j < GH; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const lds_t* bp = st + j * TS + 8192 * (u >> 1) + 256 * (u & 1);  // keys 32(u>>1) + 16(u&1)
        g[j][u] = lds_tr(bp + sa[0], bp + sa[1]);
      }
    bfx8 tk[NDT][4];
    auto load_t = [&](int dt) {
#pragma unroll
      for (int u = 0; u < 4; ++u) tk[dt][u] = la.trf(kt, 32 * (u >> 1), u & 1, dt);
    };
    load_t(0);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      if (dt + 1 < NDT) load_t(dt + 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < GH; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u) mfma_acc(dqacc[j][dt], tk[dt][u], g[j][u]);
    }
    dma_barrier();
  };
  int kb = kb0;
  for (; kb + 1 < kb1; kb += 2) {
    step(Buf<0>(), kb);
    step(Buf<1>(), kb + 1);
  }
  if (kb < kb1) step(Buf<0>(), kb);

#pragma unroll
  for (int j = 0; j < GH; ++j) agpr_fence(dqacc[j]);
  if (my_q >= p.Sq) return;
#pragma unroll
  for (int j = 0; j < GH; ++j) {
    const int hq = hq0 + j;
    if (nsplit > 1) {
      float* pq = part + ((int64_t)sp * p.B * p.H + (int64_t)b * p.H + hq) * p.Sq * D + (int64_t)my_q * D;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg)
          *reinterpret_cast<float4*>(pq + 32 * dt + 8 * gg + 4 * h) =
              make_float4(dqacc[j][dt][4 * gg] * p.scale, dqacc[j][dt][4 * gg + 1] * p.scale,
                          dqacc[j][dt][4 * gg + 2] * p.scale, dqacc[j][dt][4 * gg + 3] * p.scale);
    } else {
      bf16_t* row = dq + (int64_t)b * p.sxb + (int64_t)my_q * p.sxs + (int64_t)hq * p.sxh;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          const int d = 32 * dt + 8 * gg + 4 * h;
          uint2 w;
          w.x = pack_bf16x2(dqacc[j][dt][4 * gg + 0] * p.scale, dqacc[j][dt][4 * gg + 1] * p.scale);
          w.y = pack_bf16x2(dqacc[j][dt][4 * gg + 2] * p.scale, dqacc[j][dt][4 * gg + 3] * p.scale);
          *reinterpret_cast<uint2*>(row + d) = w;
        }
      }
    }
  }
}

// ============================================================== backward: dK, dV
// One workgroup = 128 keys (4 waves x 32) of one (b, kv-head); iterates every
// query head of the GQA group x query blocks of 64 rows staged in LDS (Q, dO,
// lse, delta), so dK/dV of the kv head are summed in registers and written
// once as bf16.  Rows past Sq read as zero with lse = +inf => P = dS = 0.
// the 4 nlse2 values of query rows `rowo` .. +3 (LDS stats slot)
ST_DEVICE f32x4 dkdv_ldL(const lds_t* st, int rowo) {
  return *reinterpret_cast<const f32x4 __attribute__((address_space(3)))*>(st + 4 * rowo);
}
// dS softmax slice of one accumulator row group (4 registers: query rows
// 8 gq + 4h .. +3 of the half, this lane's key): P = exp2(S c2 + nlse2), dS = P (dP - delta)
// where the dP accumulator was seeded with -delta; P overwrites S in place.  fma + exp +
// mul per element, straight-line (the causal mask is applied afterwards, dkdv_mask).
ST_DEVICE void dkdv_softmax4(f32x16& s, f32x16& dp, const f32x4& L, int gq, float c2) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = 4 * gq + j;
    const float pv = fast_exp2(fmaf(s[i], c2, L[j]));
    s[i] = pv;
    dp[i] = pv * dp[i];
  }
}
// causal diagonal: zero P and dS of the future keys of one 32-query half (register i holds
// half-row acc_row0(i) + 4h; thr = this lane's key - the half's first query - 4h).  A select,
// so an overflowed exp2 of a masked score leaves nothing behind.
ST_DEVICE void dkdv_mask(f32x16& s, f32x16& dp, int thr) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const bool m = acc_row0(i) < thr;
    s[i] = m ? 0.f : s[i];
    dp[i] = m ? 0.f : dp[i];
  }
}

// PROBE 1: softmax / dS VALU skipped; PROBE 2 (with WDS): dS stores skipped (timing
// probes of the diagnostic library, -DST_PROBES; wrong results).
// WDS: also store dS^T tiles into the dS workspace `dsw` (see ds_prefix) for
// flash_bwd_dq_ds_kernel.
template <int D, int PROBE = 0, bool WDS = false>
__global__ __launch_bounds__(256, 1) void flash_bwd_dkdv_kernel(
    AttnParams p, const bf16_t* __restrict__ dout, int64_t sdb, int64_t sds, int64_t sdh,
    const float* __restrict__ nlse2, const float* __restrict__ delta, bf16_t* __restrict__ dk,
    bf16_t* __restrict__ dv, int nsplit, float* __restrict__ part, bf16_t* __restrict__ dsw) {
  constexpr int BKW = 128, BQ = 64, NKK = D / 16, NDT = D / 32;
  constexpr int TB = BQ * D * 2;
  // Q / dO / stats ring: 2 slots, or 3 when storing dS (tiles issued two steps ahead, so
  // the dS stores of a step get a step and a half to retire before a barrier waits on
  // the DMA issued after them -- vmcnt counts stores too, in issue order)
  constexpr int NB = WDS ? 3 : 2;
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * NB * TB + NB * 2 * BQ * 4];
  lds_t* smem = (lds_t*)smem_raw;  // Q[NB] dO[NB] | stats[slot][lse2 | delta][BQ]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, r = lane & 31, h = lane >> 5;
  const int G = p.H / p.Hkv, BHk = p.B * p.Hkv, id = blockIdx.x;
  // causal: early keys are the heaviest -> launched first; a key tile's query work may be
  // cut into nsplit ranges (small grids, see st_flash_bwd), each its own workgroup
  const int kt_i = id / (BHk * nsplit), sp = (id / BHk) % nsplit;
  const int bhk = id % BHk, b = bhk / p.Hkv, hk = bhk % p.Hkv;
  const int k0 = kt_i * BKW, kw = k0 + wid * 32, my_k = kw + r;

  const rsrc_t rk = make_rsrc(p.k + (int64_t)b * p.skb + (int64_t)hk * p.skh, p.Sk, p.sks, D);
  const rsrc_t rv = make_rsrc(p.v + (int64_t)b * p.svb + (int64_t)hk * p.svh, p.Sk, p.svs, D);
  // K^T / V^T as B operands: lane holds K[my_k][16kk + 8h .. +8]
  bfx8 kf[NKK], vf[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    kf[kk] = bload_frag(rk, (uint32_t)my_k * (uint32_t)(p.sks * 2) + (2 * kk + h) * 16);
    vf[kk] = bload_frag(rv, (uint32_t)my_k * (uint32_t)(p.svs * 2) + (2 * kk + h) * 16);
  }
  // register fragments resident before the DMA pipeline starts: hipcc's own
  // vmcnt bookkeeping for these loads otherwise lands inside the loop, where
  // (the asm DMAs being invisible to it) a small vmcnt would wait for them
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  const int64_t kg = p.k_offset + my_k, kgw = p.k_offset + k0 + 32 * __builtin_amdgcn_readfirstlane(wid);
  // kgw: the wave's first key, read into an SGPR so the causal mask test is a scalar branch
  // (not an exec-mask region cutting the MFMA / softmax interleave apart)
  const float c2 = p.scale * kLog2e;

  // query blocks that can see any key of this tile; from qb_full on, every
  // query of the block sees every key of the tile
  int qb0 = 0;
  if (p.causal) {
    const int64_t first_q = p.k_offset + k0 - p.q_offset;
    qb0 = first_q <= 0 ? 0 : (int)((first_q) / BQ);
  }
  // dS workspace: every 128-query tile the dQ kernel reads from this key tile must be
  // written whole, so start at an even 64-query block (a dead block stores zeros)
  if constexpr (WDS) qb0 &= ~1;
  const int nqb = (p.Sq + BQ - 1) / BQ;
  const int nqt128 = (p.Sq + 127) / 128;
  const int64_t ds_per_bh = WDS ? ds_prefix(p.causal, p.Sk, p.q_offset, p.k_offset, nqt128) : 0;
  const int ds_kb = (k0 >> 6) + (wid >> 1), ds_row = (wid & 1) * 32 + r;
  // dS stores are buffer stores into one (batch, q-head)'s workspace region: scalar
  // base + soffset per step, lane-constant VGPR offset, the (u, s2) part an immediate --
  // no per-store address arithmetic.  Chunk c = ch0 + 4u + 2 s2 + h of this lane's key:
  // ds_off = 8192 (k >> 5) + 4096 qh + 2048 u + 1024 s2 + 512 h + 16 ((k & 31) ^ (8 s2 + 4 h)).
  // A step whose tile the dQ kernel never reads stores past the region's end, where
  // buffer stores are dropped -- every step still issues exactly 4 (ring_wait counts).
  const uint32_t ds_region = (uint32_t)(ds_per_bh * kDsTile * 2);
  uint32_t ds_voff[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
    ds_voff[s2] = (uint32_t)ds_off(ds_row, 0, 0, s2, h) - 1024 * s2;  // + 2048 u + 1024 s2 as immediates
  auto ds_store = [&](rsrc_t rs, uint32_t soff, int u, int s2, u32x4 w) {
    if constexpr (PROBE != 2)
      // non-temporal (aux 2): each dS tile is read once, by the dQ pass, long after this
      // kernel -- kept out of L2, whose hit rate on the re-read Q / dO tiles then rises
      // (bench shape: backward 2.87 -> 2.75 ms, cp8 rank-3 chunk 3.85 -> 3.69 ms;
      // profiles/r06/flash/nt_ds/)
      __builtin_amdgcn_raw_buffer_store_b128(w, rs, (int)(ds_voff[s2] + 2048 * u + 1024 * s2), (int)soff, 2);
  };
  const int nq = nqb > qb0 ? nqb - qb0 : 0;
  const int total = G * nq;
  const int it0 = (int)((int64_t)total * sp / nsplit), it1 = (int)((int64_t)total * (sp + 1) / nsplit);

  LdsAddr<D> la;
  la.init(lane);
  DmaStager<D, BQ> sq, sd;
  sq.init(wid, lane, p.sqs);
  sd.init(wid, lane, sds);
  float* stats = (float*)(smem_raw + 2 * NB * TB);
  // WDS: every step issues exactly 4 dS stores per wave (a step whose tile the dQ kernel
  // never reads stores into a dummy tile past the workspace), so the ring's waits are
  // fixed counts: DMA instructions per issue(), and stores per step
  constexpr int kDmaPerIssue = 2 * DmaStager<D, BQ>::NI;  // + 1 (stats) on waves 0, 1

  f32x16 dkacc[NDT], dvacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dkacc[dt] = dvacc[dt] = zero16();

  // Q / dO tiles of step (g, qb) and the block's lse / delta rows DMA'd straight
  // into LDS buffer `buf` (rows past Sq land as zeros: their Q / dO rows are zero
  // too, so P * (dP - delta) vanishes there and they contribute nothing)
  auto issue = [&](int g, int qb, int buf) {
    const int hq = hk * G + g;
    sq.load(make_rsrc(p.q + (int64_t)b * p.sqb + (int64_t)hq * p.sqh, p.Sq, p.sqs, D), smem + buf * TB, qb * BQ);
    sd.load(make_rsrc(dout + (int64_t)b * sdb + (int64_t)hq * sdh, p.Sq, sds, D), smem + (NB + buf) * TB, qb * BQ);
    if (wid < 2) {
      const int64_t row = ((int64_t)b * p.H + hq) * p.Sq;
      lds_dma4(make_rsrc_f32((wid == 0 ? nlse2 : delta) + row, p.Sq),
               (lds_t*)(stats + buf * 2 * BQ + wid * BQ), (uint32_t)((qb * BQ + lane) * 4));
    }
  };
  // iteration order: heads outer, query blocks inner (a reversed, heads-inner sweep that
  // lets concurrent key tiles of one kv head share Q / dO tiles in L2 measured neutral)
  auto advance = [&](int& g, int& qb) {  // next (head, query block) of the iteration
    if (++qb == nqb) {
      qb = qb0;
      ++g;
    }
  };
  // WDS wait at the end of a step: everything but the youngest `N` vector-memory ops
  // (the previous and this step's dS stores, plus the DMA issued two steps ahead when
  // there was one) has landed; then the barrier publishes the tiles and retires reads
  auto ring_wait = [&](bool ahead) {
    if (!ahead) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
    else if (wid < 2) {
      if constexpr (kDmaPerIssue == 8) asm volatile("s_waitcnt vmcnt(17) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(13) lgkmcnt(0)" ::: "memory");
    } else {
      if constexpr (kDmaPerIssue == 8) asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  static_assert(kDmaPerIssue == 8 || kDmaPerIssue == 4, "ring_wait counts");
  int g_c = nq > 0 ? it0 / nq : 0, qb_c = qb0 + (nq > 0 ? it0 % nq : 0);
  if (it0 < it1) issue(g_c, qb_c, 0);
  if constexpr (WDS) {
    int g1 = g_c, qb1 = qb_c;
    advance(g1, qb1);
    if (it0 + 1 < it1) issue(g1, qb1, 1);
    // 8 (dropped, out-of-range) stores standing in for the dS stores that follow a DMA in
    // the steady state (the previous and the current step's), so ring_wait's counts hold
    // from the start
    const rsrc_t rs0 = make_rsrc(dsw, (int)(ds_per_bh * 64), 128, 128);
    const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int c = 0; c < 8; ++c) ds_store(rs0, ds_region, c >> 2, (c >> 1) & 1, z);
    ring_wait(it0 + 1 < it1);  // slot 0 landed; slot 1 may still be in flight
  } else {
    dma_barrier();
  }

  auto step = [&](auto bufc, int it) {
    constexpr int BUF = decltype(bufc)::value;  // ring slot of this step
    int g_n = g_c, qb_n = qb_c;
    advance(g_n, qb_n);
    bool ahead = false;
    if constexpr (WDS) {
      int g2 = g_n, qb2 = qb_n;
      advance(g2, qb2);
      ahead = it + 2 < it1;
      if (ahead) issue(g2, qb2, (BUF + 2) % 3);
    } else {
      if (it + 1 < it1) issue(g_n, qb_n, BUF ^ 1);
    }
    const lds_t* qt = smem + BUF * TB;
    const lds_t* dt_ = smem + (NB + BUF) * TB;
    const lds_t* st = (const lds_t*)(stats + BUF * 2 * BQ);
    const int64_t qstart = p.q_offset + (int64_t)qb_c * BQ;  // global index of the block's row 0
    // this wave's keys vs this query block: skip when every key is in the future
    const bool dead = p.causal && (kgw > qstart + BQ - 1);
    // this wave's dS^T tile: region of (b, q-head), byte offset of the tile's 64-query half
    const rsrc_t ds_rs = make_rsrc(dsw + ((int64_t)b * p.H + hk * G + g_c) * ds_per_bh * kDsTile,
                                   (int)(ds_per_bh * 64), 128, 128);
    uint32_t ds_soff = 0;
    if constexpr (WDS) {
      const int qt = qb_c >> 1;
      ds_soff = ds_kb < ds_nkb(p.causal, p.Sk, p.q_offset, p.k_offset, qt)
                    ? (uint32_t)((ds_prefix(p.causal, p.Sk, p.q_offset, p.k_offset, qt) + ds_kb) * kDsTile * 2 +
                                 4096 * (qb_c & 1))
                    : ds_region;  // never read by the dQ kernel: dropped
      // wave-uniform (ds_kb comes from the wave index): keep it scalar, or hipcc wraps
      // every store in a readfirstlane waterfall loop (T20)
      ds_soff = __builtin_amdgcn_readfirstlane(ds_soff);
      if (dead) {  // 4 stores, as a live step issues (ring_wait counts them)
        const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int c = 0; c < 4; ++c) ds_store(ds_rs, ds_soff, c >> 1, c & 1, z);
      }
    }
    if (!dead) {
      // software-pipelined within the wave (one wave per SIMD: nothing else fills
      // the MFMA pipe while the softmax VALU runs): half 0's softmax is issued
      // between half 1's S/dP MFMAs, half 1's between half 0's dV/dK MFMAs
      const bool need_mask = p.causal && (kgw + 31 > qstart);
      int thr[2] = {0, 0};
      if (need_mask) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int64_t t = kg - qstart - 32 * u - 4 * h;
          thr[u] = t > 64 ? 64 : (int)t;
        }
      }
      f32x16 s[2], dp[2];
      s[0] = s[1] = zero16();

      // dP accumulators seeded with -delta of their query rows (registers 4g .. 4g+3 of half
      // u = rows 32u + 8g + 4h .. +3): the MFMA chain then yields dP - delta directly
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const f32x4 nd =
              *reinterpret_cast<const f32x4 __attribute__((address_space(3)))*>(st + 4 * (BQ + 32 * u + 8 * g4 + 4 * h));
#pragma unroll
          for (int j = 0; j < 4; ++j) dp[u][4 * g4 + j] = nd[j];
        }
      bfx8 qa[2][NKK], da[2][NKK];
      // nlse2 of the next softmax row group, read two MFMAs ahead of its use (read right
      // before it, the wait for it also waited for the operand reads queued in between)
      f32x4 Lc;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        qa[u][0] = la.rowf(qt, u, 0);
        da[u][0] = la.rowf(dt_, u, 0);
        qa[u][1] = la.rowf(qt, u, 1);
        da[u][1] = la.rowf(dt_, u, 1);
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) {
          if (kk + 2 < NKK) {
            qa[u][kk + 2] = la.rowf(qt, u, kk + 2);
            da[u][kk + 2] = la.rowf(dt_, u, kk + 2);
          }
          if (u == 0 && kk == NKK - 1) Lc = dkdv_ldL(st, 4 * h);
          __builtin_amdgcn_sched_barrier(0);
          s[u] = mfma(qa[u][kk], kf[kk], s[u]);
          dp[u] = mfma(da[u][kk], vf[kk], dp[u]);
          if (u == 1 && PROBE != 1) {
#pragma unroll
            for (int gq = 0; gq < 4; ++gq)  // the 4 row groups of half 0 spread over the k-steps
              if (gq * NKK / 4 == kk) {
                dkdv_softmax4(s[0], dp[0], Lc, gq, c2);
                Lc = dkdv_ldL(st, gq < 3 ? 8 * (gq + 1) + 4 * h : 32 + 4 * h);  // half 1's group 0 last
              }
          }
        }
      }
      // wave-uniform (scalar) branch: only blocks on the causal diagonal pay for the mask
      if (need_mask) dkdv_mask(s[0], dp[0], thr[0]);
      bfx8 pf[2][2], gf[2][2];
      pf[0][0] = acc_frag(s[0], 0);
      pf[0][1] = acc_frag(s[0], 1);
      gf[0][0] = acc_frag(dp[0], 0);
      gf[0][1] = acc_frag(dp[0], 1);
      // the dK MFMA's B fragments (k-step s2 of 32-query half u) are stored as they are:
      // one 16-byte store per lane, 1 KiB contiguous per instruction (ds_off)
      auto ds_half = [&](int u) {
        if constexpr (WDS) {
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) ds_store(ds_rs, ds_soff, u, s2, __builtin_bit_cast(u32x4, gf[u][s2]));
        }
      };
      ds_half(0);
      // dV^T += dO^T P, dK^T += Q^T dS: half 0's four dt groups, then half 1's
      constexpr int NG = NDT * 2;
      bfx8 tv[NG][2], tk[NG][2];
      auto load_group = [&](int gidx) {
        const int dt = gidx % NDT, u = gidx / NDT;
        tv[gidx][0] = la.trf(dt_, 32 * u, 0, dt);
        tv[gidx][1] = la.trf(dt_, 32 * u, 1, dt);
        tk[gidx][0] = la.trf(qt, 32 * u, 0, dt);
        tk[gidx][1] = la.trf(qt, 32 * u, 1, dt);
      };
      load_group(0);
#pragma unroll
      for (int gi = 0; gi < NG; ++gi) {
        if (gi + 1 < NG) load_group(gi + 1);
        __builtin_amdgcn_sched_barrier(0);
        const int dt = gi % NDT, u = gi / NDT;
        if (gi == NDT) {
          if (need_mask) dkdv_mask(s[1], dp[1], thr[1]);
          pf[1][0] = acc_frag(s[1], 0);
          pf[1][1] = acc_frag(s[1], 1);
          gf[1][0] = acc_frag(dp[1], 0);
          gf[1][1] = acc_frag(dp[1], 1);
          ds_half(1);
        }
        mfma_acc(dvacc[dt], tv[gi][0], pf[u][0]);
        mfma_acc(dvacc[dt], tv[gi][1], pf[u][1]);
        mfma_acc(dkacc[dt], tk[gi][0], gf[u][0]);
        mfma_acc(dkacc[dt], tk[gi][1], gf[u][1]);
        if (u == 0 && PROBE != 1) {
#pragma unroll
          for (int gq = 0; gq < 4; ++gq)  // half 1's row groups spread over half 0's dt groups
            if (gq * NDT / 4 == dt) {
              dkdv_softmax4(s[1], dp[1], Lc, gq, c2);
              if (gq < 3) Lc = dkdv_ldL(st, 32 + 8 * (gq + 1) + 4 * h);
            }
        }
      }
    }
    if constexpr (WDS) ring_wait(ahead);
    else dma_barrier();
    g_c = g_n;
    qb_c = qb_n;
  };
  int it = it0;  // unconditional groups of steps (see the dQ kernel); the slot is a constant
  if constexpr (WDS) {
    for (; it + 2 < it1; it += 3) {
      step(Buf<0>(), it);
      step(Buf<1>(), it + 1);
      step(Buf<2>(), it + 2);
    }
    if (it < it1) step(Buf<0>(), it);
    if (it + 1 < it1) step(Buf<1>(), it + 1);
  } else {
    for (; it + 1 < it1; it += 2) {
      step(Buf<0>(), it);
      step(Buf<1>(), it + 1);
    }
    if (it < it1) step(Buf<0>(), it);
  }

  agpr_fence(dkacc);
  agpr_fence(dvacc);
  if (nsplit > 1) {
    // fp32 partials [split][B*Hkv][Sk][D] (dK block first, then dV), summed in split
    // order by dkdv_split_reduce_kernel: deterministic
    if (my_k < p.Sk) {
      const int64_t blk = (int64_t)BHk * p.Sk * D;
      float* pk = part + (int64_t)sp * 2 * blk + ((int64_t)bhk * p.Sk + my_k) * D;
      float* pv = pk + blk;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = 32 * dt + 8 * g + 4 * h;
          *reinterpret_cast<float4*>(pk + d) = make_float4(dkacc[dt][4 * g] * p.scale, dkacc[dt][4 * g + 1] * p.scale,
                                                           dkacc[dt][4 * g + 2] * p.scale, dkacc[dt][4 * g + 3] * p.scale);
          *reinterpret_cast<float4*>(pv + d) =
              make_float4(dvacc[dt][4 * g], dvacc[dt][4 * g + 1], dvacc[dt][4 * g + 2], dvacc[dt][4 * g + 3]);
        }
      }
    }
    return;
  }
  if (my_k < p.Sk) {
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * h;
        const int64_t off = (int64_t)b * p.sxb + (int64_t)my_k * p.sxs + (int64_t)hk * p.sxh + d;
        uint2 wk, wv;
        wk.x = pack_bf16x2(dkacc[dt][4 * g] * p.scale, dkacc[dt][4 * g + 1] * p.scale);
        wk.y = pack_bf16x2(dkacc[dt][4 * g + 2] * p.scale, dkacc[dt][4 * g + 3] * p.scale);
        wv.x = pack_bf16x2(dvacc[dt][4 * g], dvacc[dt][4 * g + 1]);
        wv.y = pack_bf16x2(dvacc[dt][4 * g + 2], dvacc[dt][4 * g + 3]);
        *reinterpret_cast<uint2*>(dk + off) = wk;
        *reinterpret_cast<uint2*>(dv + off) = wv;
      }
    }
  }
}

// dK / dV = sum over the query-range splits of the fp32 partials (fixed split order),
// written as bf16 through the output strides.  One thread per 8 elements.
__global__ __launch_bounds__(256) void dkdv_split_reduce_kernel(const float* __restrict__ part, int nsplit,
                                                                int Hkv, int Sk, int D, int64_t total8,
                                                                bf16_t* __restrict__ dk, bf16_t* __restrict__ dv,
                                                                int64_t sxb, int64_t sxs, int64_t sxh) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total8) return;
  const int D8 = D / 8;
  const int c = (int)(t % D8);
  const int64_t row = t / D8;  // (b * Hkv + hk) * Sk + k
  const int k = (int)(row % Sk);
  const int64_t bhk = row / Sk;
  const int hk = (int)(bhk % Hkv), b = (int)(bhk / Hkv);
  const int64_t blk = total8 * 8;
  float ak[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, av[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < nsplit; ++s) {
    const float* pk = part + (int64_t)s * 2 * blk + row * D + c * 8;
    const float4 k0 = ld4f(pk), k1 = ld4f(pk + 4), v0 = ld4f(pk + blk), v1 = ld4f(pk + blk + 4);
    ak[0] += k0.x; ak[1] += k0.y; ak[2] += k0.z; ak[3] += k0.w;
    ak[4] += k1.x; ak[5] += k1.y; ak[6] += k1.z; ak[7] += k1.w;
    av[0] += v0.x; av[1] += v0.y; av[2] += v0.z; av[3] += v0.w;
    av[4] += v1.x; av[5] += v1.y; av[6] += v1.z; av[7] += v1.w;
  }
  const int64_t off = (int64_t)b * sxb + (int64_t)k * sxs + (int64_t)hk * sxh + c * 8;
  st8(dk + off, pack8(ak));
  st8(dv + off, pack8(av));
}

// dQ = sum over the key-range splits of the fp32 partials [split][B*H][Sq][D] (fixed split
// order), written as bf16 through the output strides.  One thread per 8 elements.
__global__ __launch_bounds__(256) void dq_split_reduce_kernel(const float* __restrict__ part, int nsplit, int H,
                                                              int Sq, int D, int64_t total8, bf16_t* __restrict__ dq,
                                                              int64_t sxb, int64_t sxs, int64_t sxh) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total8) return;
  const int D8 = D / 8;
  const int c = (int)(t % D8);
  const int64_t row = t / D8;  // (b * H + hq) * Sq + q
  const int q = (int)(row % Sq);
  const int64_t bh = row / Sq;
  const int hq = (int)(bh % H), b = (int)(bh / H);
  const int64_t blk = total8 * 8;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < nsplit; ++s) {
    const float* pq = part + (int64_t)s * blk + row * D + c * 8;
    const float4 v0 = ld4f(pq), v1 = ld4f(pq + 4);
    a[0] += v0.x; a[1] += v0.y; a[2] += v0.z; a[3] += v0.w;
    a[4] += v1.x; a[5] += v1.y; a[6] += v1.z; a[7] += v1.w;
  }
  st8(dq + (int64_t)b * sxb + (int64_t)q * sxs + (int64_t)hq * sxh + c * 8, pack8(a));
}

// ============================================================== ring-attention merge
__global__ __launch_bounds__(256) void lse_merge_kernel(float* __restrict__ out, float* __restrict__ lse,
                                                        const bf16_t* __restrict__ bout,
                                                        const float* __restrict__ blse, int B, int S,
                                                        int H, int D, int64_t sbb, int64_t sbs,
                                                        int64_t sbh) {
  const int D8 = D / 8;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)B * S * H * D8;
  if (t >= total) return;
  const int c = (int)(t % D8);
  int64_t r = t / D8;
  const int hh = (int)(r % H);
  r /= H;
  const int s = (int)(r % S);
  const int b = (int)(r / S);
  const int64_t li = ((int64_t)b * H + hh) * S + s;
  const float a = lse[li], bl = blse[li];
  const float mx = fmaxf(a, bl);
  float wa, wb, nl;
  if (mx == -INFINITY) { wa = 1.f; wb = 0.f; nl = -INFINITY; }
  else {
    const float ea = __expf(a - mx), eb = __expf(bl - mx);
    nl = mx + __logf(ea + eb);
    wa = __expf(a - nl);
    wb = __expf(bl - nl);
  }
  float* op = out + (((int64_t)b * S + s) * H + hh) * D + c * 8;
  float x[8];
  unpack8(ld8(bout + b * sbb + s * sbs + hh * sbh + c * 8), x);
  float4 o0 = ld4f(op), o1 = ld4f(op + 4);
  o0.x = o0.x * wa + x[0] * wb; o0.y = o0.y * wa + x[1] * wb;
  o0.z = o0.z * wa + x[2] * wb; o0.w = o0.w * wa + x[3] * wb;
  o1.x = o1.x * wa + x[4] * wb; o1.y = o1.y * wa + x[5] * wb;
  o1.z = o1.z * wa + x[6] * wb; o1.w = o1.w * wa + x[7] * wb;
  st4f(op, o0);
  st4f(op + 4, o1);
  // every lane of the row computes nl; the first chunk's lane publishes it
  // after all lanes have read lse[li] (same wave: reads precede this store).
  if (c == 0) lse[li] = nl;
}

AttnParams make_params(const void* q, const void* k, const void* v, int B, int Sq, int Sk, int H,
                       int Hkv, int64_t sqb, int64_t sqs, int64_t sqh, int64_t skb, int64_t sks,
                       int64_t skh, int64_t svb, int64_t svs, int64_t svh, float scale, int causal,
                       int64_t q_offset, int64_t k_offset) {
  AttnParams p;
  p.q = (const bf16_t*)q; p.k = (const bf16_t*)k; p.v = (const bf16_t*)v;
  p.B = B; p.Sq = Sq; p.Sk = Sk; p.H = H; p.Hkv = Hkv;
  p.sqb = sqb; p.sqs = sqs; p.sqh = sqh; p.skb = skb; p.sks = sks; p.skh = skh;
  p.svb = svb; p.svs = svs; p.svh = svh;
  p.scale = scale; p.causal = causal; p.q_offset = q_offset; p.k_offset = k_offset;
  p.sxb = p.sxs = p.sxh = 0;
  return p;
}

// Buffer offsets are 32-bit: every row read (plus one tile of overrun) must
// stay below 2^31 bytes from its (batch, head) base.
bool offsets_fit(int64_t rows, int64_t stride) {
  return (rows + 256) * stride * 2 < (int64_t(1) << 31);
}

}  // namespace

extern "C" {

int st_flash_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int Sq,
                 int Sk, int H, int Hkv, int D, int64_t sqb, int64_t sqs, int64_t sqh, int64_t skb,
                 int64_t sks, int64_t skh, int64_t svb, int64_t svs, int64_t svh, int64_t sob,
                 int64_t sos, int64_t soh, float scale, int causal, int64_t q_offset,
                 int64_t k_offset, hipStream_t st) {
  if (H % Hkv != 0) return -2;
  if (Sq == 0 || B == 0) return 0;
  if (!offsets_fit(Sq, sqs) || !offsets_fit(Sk, sks) || !offsets_fit(Sk, svs)) return -5;
  AttnParams p = make_params(q, k, v, B, Sq, Sk, H, Hkv, sqb, sqs, sqh, skb, sks, skh, svb, svs, svh,
                             scale, causal, q_offset, k_offset);
  const unsigned grid = (unsigned)(((Sq + 127) / 128) * B * H);
  // ST_FLASH_PP=1 selects the 8-wave ping-pong kernel; it measured equal to the
  // 4-wave kernel (0.345 ms both, B2 S4096 H32/8 causal), so the 4-wave one stays default
  // (read per call so tests can switch it; one getenv per launch)
  const char* ppe = std::getenv("ST_FLASH_PP");
  const int pp = ppe ? std::atoi(ppe) : 0;
  const char* xe = std::getenv("ST_FLASH_XCD");  // XCD-aware workgroup order (default on)
  const bool xcd = !xe || std::atoi(xe) != 0;
  // ST_FLASH_FWD_HP=2: two query heads per workgroup sharing each K/V tile in LDS.  Measured
  // equal to one head per workgroup once the XCD-aware order shares K/V in L2 (B6 S4096:
  // 0.852 vs 0.853 ms, profiles/r03/flash_pmc.md), so one head stays the default.
  const char* he = std::getenv("ST_FLASH_FWD_HP");
  const bool hp2 = (H / Hkv) % 2 == 0 && he && std::atoi(he) == 2;
  if (D == 128 && pp) {
    const unsigned grid2 = (unsigned)(((Sq + 255) / 256) * B * H);
    flash_fwd_pp_kernel<128><<<grid2, 512, 0, st>>>(p, (bf16_t*)o, sob, sos, soh, lse);
  } else if (hp2) {
    const unsigned grid2 = grid / 2;
    if (D == 128 && xcd) flash_fwd_kernel<128, true, 2><<<grid2, 512, 0, st>>>(p, (bf16_t*)o, sob, sos, soh, lse);
    else if (D == 128) flash_fwd_kernel<128, false, 2><<<grid2, 512, 0, st>>>(p, (bf16_t*)o, sob, sos, soh, lse);
    else if (D == 64 && xcd) flash_fwd_kernel<64, true, 2><<<grid2, 512, 0, st>>>(p, (bf16_t*)o, sob, sos, soh, lse);
    else if (D == 64) flash_fwd_kernel<64, false, 2><<<grid2, 512, 0, st>>>(p, (bf16_t*)o, sob, sos, soh, lse);
    else return -3;
  } else if (D == 128 && xcd)
    flash_fwd_kernel<128, true><<<grid, 256, 0, st>>>(p, (bf16_t*)o, sob, sos, soh, lse);
  else if (D == 128)
    flash_fwd_kernel<128, false><<<grid, 256, 0, st>>>(p, (bf16_t*)o, sob, sos, soh, lse);
  else if (D == 64 && xcd)
    flash_fwd_kernel<64, true><<<grid, 256, 0, st>>>(p, (bf16_t*)o, sob, sos, soh, lse);
  else if (D == 64)
    flash_fwd_kernel<64, false><<<grid, 256, 0, st>>>(p, (bf16_t*)o, sob, sos, soh, lse);
  else
    return -3;
  return (int)hipGetLastError();
}

int st_flash_bwd_preprocess(const void* o, const void* dout, const float* lse, float* delta, float* nlse2,
                            int B, int S, int H,
                            int D, int64_t sob, int64_t sos, int64_t soh, int64_t sdb, int64_t sds,
                            int64_t sdh, hipStream_t st) {
  const int64_t threads = (int64_t)B * S * H * (D / 8);
  if (threads == 0) return 0;
  const unsigned blocks = (unsigned)((threads + 255) / 256);
  if (D == 128)
    flash_bwd_pre_kernel<128><<<blocks, 256, 0, st>>>((const bf16_t*)o, (const bf16_t*)dout, lse, delta, nlse2, B,
                                                      S, H, sob, sos, soh, sdb, sds, sdh);
  else if (D == 64)
    flash_bwd_pre_kernel<64><<<blocks, 256, 0, st>>>((const bf16_t*)o, (const bf16_t*)dout, lse, delta, nlse2, B, S,
                                                     H, sob, sos, soh, sdb, sds, sdh);
  else
    return -3;
  return (int)hipGetLastError();
}

// Query-range split of the dK/dV kernel.  It runs one workgroup (one wave per SIMD)
// per 128-key tile of each (batch, kv head); under a causal mask tile j carries
// (nqb - j) query blocks, so when the grid is at most one round (Qwen3-0.6B mbs 2 x
// 2048: 256 workgroups on 256 CUs; Qwen3-1.7B 1 x 2048: 128) the kernel lasts as long
// as its heaviest tile, ~2x the mean, or leaves CUs empty.  Cutting every tile's query
// range into nsplit workgroups (~3 rounds) lets the heaviest-first dispatch balance
// them; fp32 partials, reduced in split order (deterministic).
// ST_FLASH_DKDV_SPLIT=N forces N (1 = off).
static int dkdv_nsplit(int B, int Sk, int Hkv, int causal) {
  const char* e = std::getenv("ST_FLASH_DKDV_SPLIT");
  if (e) {
    const int v = std::atoi(e);
    if (v >= 1 && v <= 8) return v;
  }
  const int64_t gk = (int64_t)((Sk + 127) / 128) * B * Hkv;
  // measured (tools/bench_flash_split.py): 128-256 workgroups -24..-41 % backward time,
  // 512 (two rounds, already balanced by the heaviest-first order) +4 %: split <= 1 round
  if (gk > 256) return 1;
  // without a causal mask every key tile carries the same work: a full round needs no split
  // (off-diagonal ring-attention blocks of CP)
  if (!causal && gk > 192) return 1;
  const int64_t want = (768 + gk - 1) / gk;
  return (int)(want > 8 ? 8 : want);
}

// The same key-range split exists for the dQ kernel (one workgroup per 128-query tile of
// each (batch, head); under a causal mask tile i walks i + 1 key tiles) but stays OFF by
// default: on the one short grid it could serve (Qwen3-1.7B 1 x 2048, 256 workgroups) it
// measured 0.144 -> 0.155 ms slower (tools/bench_flash_split.py) -- each split re-loads the
// tile's Q / dO fragments and writes a 128 KiB fp32 partial.  ST_FLASH_DQ_SPLIT=N forces N.
static int dq_nsplit(int B, int Sq, int H, int causal) {
  (void)B, (void)Sq, (void)H, (void)causal;
  const char* e = std::getenv("ST_FLASH_DQ_SPLIT");
  if (e) {
    const int v = std::atoi(e);
    if (v >= 1 && v <= 8) return v;
  }
  return 1;
}

// fp32 partial elements of the dK/dV and dQ splits (one buffer: dK/dV part first)
int64_t st_flash_bwd_part_elems(int B, int Sq, int Sk, int H, int Hkv, int D, int causal) {
  const int n = dkdv_nsplit(B, Sk, Hkv, causal), m = dq_nsplit(B, Sq, H, causal);
  return (n > 1 ? (int64_t)n * 2 * B * Hkv * Sk * D : 0) + (m > 1 ? (int64_t)m * B * H * Sq * D : 0);
}

// bf16 elements of the dS workspace of the dS-materialising backward, 0 when that
// path is off (ST_FLASH_BWD_DS=0) or its per-(b, head) region would not fit the
// 32-bit buffer offsets of flash_bwd_dq_ds_kernel.
int64_t st_flash_bwd_ds_elems(int B, int Sq, int Sk, int H, int D, int causal, int64_t q_offset,
                              int64_t k_offset) {
  const char* e = std::getenv("ST_FLASH_BWD_DS");  // read per call: same-process A/B
  if (e && std::atoi(e) == 0) return 0;
  if (D != 128 && D != 64) return 0;
  const int64_t per_bh = ds_prefix(causal, Sk, q_offset, k_offset, (Sq + 127) / 128);
  // one dQ workgroup addresses up to 4 heads' regions through one buffer descriptor
  if (4 * per_bh * (int64_t)kDsTile * 2 >= (int64_t(1) << 31) - (1 << 20)) return 0;
  return (int64_t)B * H * per_bh * kDsTile;
}

// dq / dk / dv: bf16 outputs with arbitrary (b, s, h) strides (D contiguous) so
// they can be slices of one fused dQKV buffer.  `dsw` (st_flash_bwd_ds_elems bf16
// elements, or null) selects the dS-materialising backward; its `phases` can be run
// separately (bit 0: dK/dV + the dS stores, bit 1: dQ from dS) so a caller can put the
// HBM-bound dQ pass on another stream beside compute-bound work (ops/attention.py).
int st_flash_bwd(const void* q, const void* k, const void* v, const void* dout, const float* lse,
                 const float* delta, const float* nlse2, void* dq, void* dk, void* dv, int B, int Sq, int Sk, int H,
                 int Hkv, int D, int64_t sqb, int64_t sqs, int64_t sqh, int64_t skb, int64_t sks,
                 int64_t skh, int64_t svb, int64_t svs, int64_t svh, int64_t sdb, int64_t sds,
                 int64_t sdh, int64_t sdqb, int64_t sdqs, int64_t sdqh, int64_t sdkb, int64_t sdks,
                 int64_t sdkh, float scale, int causal, int64_t q_offset, int64_t k_offset,
                 float* part, void* dsw, int phases, hipStream_t st) {
  if (H % Hkv != 0) return -2;
  if (B == 0 || Sq == 0 || Sk == 0) return 0;
  if (!offsets_fit(Sq, sqs) || !offsets_fit(Sq, sds) || !offsets_fit(Sk, sks) || !offsets_fit(Sk, svs))
    return -5;
  AttnParams p = make_params(q, k, v, B, Sq, Sk, H, Hkv, sqb, sqs, sqh, skb, sks, skh, svb, svs, svh,
                             scale, causal, q_offset, k_offset);
  AttnParams pq = p, pk = p;
  pq.sxb = sdqb; pq.sxs = sdqs; pq.sxh = sdqh;
  pk.sxb = sdkb; pk.sxs = sdks; pk.sxh = sdkh;
  const int nsplit = part ? dkdv_nsplit(B, Sk, Hkv, causal) : 1;
  const int qsplit = part ? dq_nsplit(B, Sq, H, causal) : 1;
  const unsigned gq = (unsigned)(((Sq + 127) / 128) * B * H * qsplit);
  float* qpart = part ? part + (nsplit > 1 ? (int64_t)nsplit * 2 * B * Hkv * Sk * D : 0) : nullptr;
  const unsigned gk = (unsigned)(((Sk + 127) / 128) * B * Hkv * nsplit);
  const bf16_t* dop = (const bf16_t*)dout;
  if (dsw && (D == 128 || D == 64)) {
    // dK/dV (storing dS^T tiles), then dQ = dS K from the workspace, in stream order
    bf16_t* ds = (bf16_t*)dsw;
    // query heads per dQ workgroup (sharing each staged K tile): 4, 2 or 1
    const int G = H / Hkv, GH = G % 4 == 0 ? 4 : (G % 2 == 0 ? 2 : 1);
    const unsigned gds = (unsigned)(((Sq + 127) / 128) * B * Hkv * (G / GH) * qsplit);
#ifdef ST_PROBES
    const char* pe = std::getenv("ST_FLASH_PROBE");  // diagnostic library only: 2 = dS stores skipped (wrong dQ)
    const bool probe2 = D == 128 && pe && std::atoi(pe) == 2;
#endif
    if (phases & 1) {
#ifdef ST_PROBES
      if (probe2)
        flash_bwd_dkdv_kernel<128, 2, true><<<gk, 256, 0, st>>>(pk, dop, sdb, sds, sdh, nlse2, delta, (bf16_t*)dk,
                                                               (bf16_t*)dv, nsplit, part, ds);
      else
#endif
      if (D == 128)
        flash_bwd_dkdv_kernel<128, 0, true><<<gk, 256, 0, st>>>(pk, dop, sdb, sds, sdh, nlse2, delta, (bf16_t*)dk,
                                                               (bf16_t*)dv, nsplit, part, ds);
      else
        flash_bwd_dkdv_kernel<64, 0, true><<<gk, 256, 0, st>>>(pk, dop, sdb, sds, sdh, nlse2, delta, (bf16_t*)dk,
                                                              (bf16_t*)dv, nsplit, part, ds);
      ST_HIP_CHECK(hipGetLastError());
      if (nsplit > 1) {
        const int64_t total8 = (int64_t)B * Hkv * Sk * (D / 8);
        dkdv_split_reduce_kernel<<<(unsigned)((total8 + 255) / 256), 256, 0, st>>>(
            part, nsplit, Hkv, Sk, D, total8, (bf16_t*)dk, (bf16_t*)dv, sdkb, sdks, sdkh);
      }
    }
    if (phases & 2) {
      if (D == 128) {
        if (GH == 4) flash_bwd_dq_ds_kernel<128, 4><<<gds, 256, 0, st>>>(pq, ds, (bf16_t*)dq, qsplit, qpart);
        else if (GH == 2) flash_bwd_dq_ds_kernel<128, 2><<<gds, 256, 0, st>>>(pq, ds, (bf16_t*)dq, qsplit, qpart);
        else flash_bwd_dq_ds_kernel<128, 1><<<gds, 256, 0, st>>>(pq, ds, (bf16_t*)dq, qsplit, qpart);
      } else {
        if (GH == 4) flash_bwd_dq_ds_kernel<64, 4><<<gds, 256, 0, st>>>(pq, ds, (bf16_t*)dq, qsplit, qpart);
        else if (GH == 2) flash_bwd_dq_ds_kernel<64, 2><<<gds, 256, 0, st>>>(pq, ds, (bf16_t*)dq, qsplit, qpart);
        else flash_bwd_dq_ds_kernel<64, 1><<<gds, 256, 0, st>>>(pq, ds, (bf16_t*)dq, qsplit, qpart);
      }
      ST_HIP_CHECK(hipGetLastError());
      if (qsplit > 1) {
        const int64_t total8 = (int64_t)B * H * Sq * (D / 8);
        dq_split_reduce_kernel<<<(unsigned)((total8 + 255) / 256), 256, 0, st>>>(qpart, qsplit, H, Sq, D, total8,
                                                                                 (bf16_t*)dq, sdqb, sdqs, sdqh);
      }
    }
    return (int)hipGetLastError();
  }
  if (phases != 3) return -6;  // separate phases need the dS workspace
  // the dQ kernel (and its split reduce) runs on a second stream beside dK/dV, so the
  // dispatcher fills each kernel's causal tail with the other's workgroups; joined with an
  // event before returning (same stream order for callers).  Same-process A/B at Llama-3-8B
  // mbs 6: 993.2 vs 996.2 ms/step median, lower in all 4 rounds
  // (profiles/r03/flash_bwd_concurrent_ab.log); ST_FLASH_BWD_CONCURRENT=0 serialises them.
  const char* ce = std::getenv("ST_FLASH_BWD_CONCURRENT");  // read per call: same-process A/B
  const bool concurrent = !ce || std::atoi(ce) != 0;
  hipStream_t sq = st;
  hipEvent_t ev_join = nullptr;
  if (concurrent && D == 128) {
    static hipStream_t side[16] = {};
    static hipEvent_t fork_ev[16] = {}, join_ev[16] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 16) {
      if (!side[dev]) {
        ST_HIP_CHECK(hipStreamCreateWithFlags(&side[dev], hipStreamNonBlocking));
        ST_HIP_CHECK(hipEventCreateWithFlags(&fork_ev[dev], hipEventDisableTiming));
        ST_HIP_CHECK(hipEventCreateWithFlags(&join_ev[dev], hipEventDisableTiming));
      }
      ST_HIP_CHECK(hipEventRecord(fork_ev[dev], st));
      ST_HIP_CHECK(hipStreamWaitEvent(side[dev], fork_ev[dev], 0));
      sq = side[dev];
      ev_join = join_ev[dev];
    }
  }
  if (D == 128) {
#ifdef ST_PROBES
    const char* pe = std::getenv("ST_FLASH_PROBE");  // diagnostic library only: 1 = softmax VALU skipped
    if (pe && std::atoi(pe) == 1) {
      flash_bwd_dq_kernel<128, 1><<<gq, 256, 0, st>>>(pq, dop, sdb, sds, sdh, lse, delta, (bf16_t*)dq, qsplit, qpart);
      flash_bwd_dkdv_kernel<128, 1><<<gk, 256, 0, st>>>(pk, dop, sdb, sds, sdh, nlse2, delta, (bf16_t*)dk,
                                                   (bf16_t*)dv, nsplit, part, nullptr);
      return (int)hipGetLastError();
    }
#endif
    flash_bwd_dq_kernel<128><<<gq, 256, 0, sq>>>(pq, dop, sdb, sds, sdh, lse, delta, (bf16_t*)dq, qsplit, qpart);
    flash_bwd_dkdv_kernel<128><<<gk, 256, 0, st>>>(pk, dop, sdb, sds, sdh, nlse2, delta, (bf16_t*)dk,
                                                 (bf16_t*)dv, nsplit, part, nullptr);
  } else if (D == 64) {
    flash_bwd_dq_kernel<64><<<gq, 256, 0, st>>>(pq, dop, sdb, sds, sdh, lse, delta, (bf16_t*)dq, qsplit, qpart);
    flash_bwd_dkdv_kernel<64><<<gk, 256, 0, st>>>(pk, dop, sdb, sds, sdh, nlse2, delta, (bf16_t*)dk,
                                                  (bf16_t*)dv, nsplit, part, nullptr);
  } else {
    return -3;
  }
  if (qsplit > 1) {
    ST_HIP_CHECK(hipGetLastError());
    const int64_t total8 = (int64_t)B * H * Sq * (D / 8);
    dq_split_reduce_kernel<<<(unsigned)((total8 + 255) / 256), 256, 0, sq>>>(qpart, qsplit, H, Sq, D, total8,
                                                                             (bf16_t*)dq, sdqb, sdqs, sdqh);
  }
  if (ev_join) {  // rejoin: everything after this call on `st` sees dQ
    ST_HIP_CHECK(hipGetLastError());
    ST_HIP_CHECK(hipEventRecord(ev_join, sq));
    ST_HIP_CHECK(hipStreamWaitEvent(st, ev_join, 0));
  }
  if (nsplit > 1) {
    ST_HIP_CHECK(hipGetLastError());
    const int64_t total8 = (int64_t)B * Hkv * Sk * (D / 8);
    dkdv_split_reduce_kernel<<<(unsigned)((total8 + 255) / 256), 256, 0, st>>>(
        part, nsplit, Hkv, Sk, D, total8, (bf16_t*)dk, (bf16_t*)dv, sdkb, sdks, sdkh);
  }
  return (int)hipGetLastError();
}

int st_lse_merge(float* out, float* lse, const void* bout, const float* blse, int B, int S, int H,
                 int D, int64_t sbb, int64_t sbs, int64_t sbh, hipStream_t st) {
  const int64_t total = (int64_t)B * S * H * (D / 8);
  if (total == 0) return 0;
  lse_merge_kernel<<<(unsigned)((total + 255) / 256), 256, 0, st>>>(out, lse, (const bf16_t*)bout, blse,
                                                                     B, S, H, D, sbb, sbs, sbh);
  return (int)hipGetLastError();
}

}  // extern "C"

// Grouped / dense "TN" GEMM for gfx950 with ONE wave per SIMD and a 128 x 128 tile per wave:
//   Y[rows of g] = X[rows of g] @ W[g]^T,  X [T][K], W[g] [N][K] (both K-contiguous)
// (G = 1 is a plain GEMM; the data gradient dX = dY W runs in this layout on the W^T copy the
// optimizer writes, ops/grad.py).  Reference call sites: every F.linear of the models and the
// grouped expert matmul of scaletorch/models/npu_patch.py:94-127.
//
// Why another GEMM: csrc/grouped_gemm.hip's 8 waves x (128 x 64) tiles read 24 KiB of LDS per
// wave per 64-k step; with the 64 KiB DMA fill that is 256 KiB per CU per 2,048 MFMA cycles,
// i.e. LDS-bound at the MFMA rate (57-61 % MFMA busy measured, profiles/r04/grouped_gemm_pmc.md).
// Here 4 waves x (128 x 128) read 128 KiB + write 64 KiB per K-step: 75 % of the LDS port at
// full MFMA rate.  With one wave per SIMD nothing else hides a stall, so:
//   * operands go global -> VGPR (buffer_load_dwordx4, a few issue cycles) -> ds_write_b128, not
//     by LDS-DMA (whose ~60-cycle issue cost lands on the only wave of the SIMD); the loads of
//     K-tile kt + 2 are issued during tile kt, written to LDS during tile kt + 1;
//   * fragment registers are double-buffered: sub-step 0's MFMAs run while sub-step 1's
//     fragments are read and half of the next tile's staged data written, sub-step 1's while
//     the other half is written, the loads of the tile after it issued, and -- after the ONE
//     barrier of the K-tile, a quarter into sub-step 1 -- the next tile's first fragments read;
//   * 256 fp32 accumulators per lane (16x16x32 MFMA: 8 x 8 fragments), 512 registers / lane.
// LDS images: [256 rows][64 k] bf16, 16-byte chunk c of row r at c ^ ((r >> 1) & 7): the
// ds_read_b128 fragment reads and the ds_write_b128 fills are bank-conflict free.
//
// STATUS: measured experiment, not on the model path (docs/PERF.md "one wave per SIMD GEMM").
// On the dense gate|up / down / qkv shapes all variants run 1.16-1.37 PF/s; hipBLASLt's
// MT256x256x64 kernel (the same 4-wave 128 x 128-per-wave structure) runs 1.35-1.58 on the same
// box, and the 8-phase grouped kernel equals variant 0.  PMC (profiles/r05/gemm4w/pmc.md): 0 LDS
// bank conflicts, L2 hit 64 % (78 % XCD-grouped, hipBLASLt 79 %) at the same ~250-cycle mean
// L2 latency; hipBLASLt issues 32 LDS instructions per wave and K-tile (DMA fills) vs 48 here.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"

using namespace st;

namespace {

typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) char lds_t;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int BM = 256, BN = 256, BK = 64, NT = 256;
constexpr int IMG = BM * BK * 2;  // one operand image: 32 KiB
constexpr int STAGE = 2 * IMG;     // A + B images of one K-tile

ST_DEVICE int rsw(int r) { return (r >> 1) & 7; }

ST_DEVICE rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

ST_DEVICE u32x4 gload(rsrc_t rs, uint32_t off) { return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0); }
ST_DEVICE void lds_w128(lds_t* p, u32x4 v) { *reinterpret_cast<u32x4 __attribute__((address_space(3)))*>(p) = v; }
ST_DEVICE bfx8 lds_r128(const lds_t* p) { return *reinterpret_cast<const bfx8 __attribute__((address_space(3)))*>(p); }

// first g with tile_end[g] > s
ST_DEVICE int find_group(const int* __restrict__ tile_end, int G, int s) {
  int lo = 0, hi = G;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (tile_end[mid] <= s) lo = mid + 1; else hi = mid;
  }
  return lo;
}

ST_DEVICE void fence() { __builtin_amdgcn_sched_barrier(0); }

// compile-time loop: f(std::integral_constant<int, i>) for i in [B, E) -- every index a constant
// (a 128-iteration `#pragma unroll` body with several slot tables was left partly rolled by
// hipcc, with the accumulators indexed dynamically through scratch)
template <int B, int E, typename F>
ST_DEVICE void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>());
    static_for<B + 1, E>(f);
  }
}

// work item of this workgroup.  gm == 0: slot-major (N-tile fastest).  gm > 0: XCD-aware --
// each XCD walks its own contiguous range of ids, in groups of gm slots x (N-tiles) with the
// slot fastest, so the ~32 workgroups an XCD runs at once start together on gm X tiles and
// 32 / gm weight tiles and stream the same 64-k slices through its L2 (slot-major spreads a
// weight tile's readers over time: each streams its own copy from the Infinity Cache / HBM).
ST_DEVICE void tile_of(int gm, int nbn, int& slot, int& nt) {
  if (gm <= 0) {
    slot = (int)blockIdx.x / nbn;
    nt = (int)blockIdx.x % nbn;
    return;
  }
  const int nslots = (int)gridDim.x / nbn;
  const int id = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  const int per = gm * nbn, grp = id / per, in = id % per;
  const int gsz = min(gm, nslots - grp * gm);
  slot = grp * gm + in % gsz;
  nt = in / gsz;
}

// tile_of for a persistent workgroup's virtual tile id vb of nv
ST_DEVICE void tile_of_v(int gm, int nbn, int vb, int nv, int& slot, int& nt) {
  if (gm <= 0) {
    slot = vb / nbn;
    nt = vb % nbn;
    return;
  }
  const int nslots = nv / nbn;
  const int id = xcd_remap(vb, nv);
  const int per = gm * nbn, grp = id / per, in = id % per;
  const int gsz = min(gm, nslots - grp * gm);
  slot = grp * gm + in % gsz;
  nt = in / gsz;
}

// PROBE (timing probes, wrong results): 1 = no fragment reads in the loop, 2 = no staging
// (loads + LDS writes) in the loop, 3 = no barrier in the loop, 4 = MFMAs only, 5 = no LDS
// writes (loads kept), 6 = no loads (LDS writes of stale registers kept)
template <int EPI, int PROBE = 0>
__global__ __launch_bounds__(NT, 1) void gemm4w_kernel(const bf16_t* __restrict__ X, int64_t ldx,
                                                       const bf16_t* __restrict__ W, int64_t ldw, int64_t strideW,
                                                       bf16_t* __restrict__ Y, int64_t ldy,
                                                       const int* __restrict__ offs, const int* __restrict__ tile_end,
                                                       int G, int N, int K, int gm) {
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * STAGE];
  lds_t* smem = (lds_t*)smem_raw;
  const int t = threadIdx.x, lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wid >> 1, wn = wid & 1;  // 2 x 2 waves of 128 x 128
  const int nbn = N / BN;
  int slot, nt;
  tile_of(gm, nbn, slot, nt);
  const int total_slots = tile_end[G - 1];
  if (slot >= total_slots) return;  // uniform over the workgroup: no barrier reached yet
  const int g = find_group(tile_end, G, slot);
  const int first_slot = g ? tile_end[g - 1] : 0;
  const int row0 = (g ? offs[g - 1] : 0) + (slot - first_slot) * BM;
  const int rows = min(BM, offs[g] - row0);
  const int n0 = nt * BN;

  // descriptors: X rows past the group's end read as zeros; W rows n0 .. n0 + 255 of W[g]
  const rsrc_t rsX = make_rsrc(X + (int64_t)row0 * ldx, (uint32_t)(((int64_t)(rows - 1) * ldx + K) * 2));
  const rsrc_t rsW = make_rsrc(W + (int64_t)g * strideW + (int64_t)n0 * ldw, (uint32_t)(((int64_t)(BN - 1) * ldw + K) * 2));

  // global -> VGPR staging: thread t loads 16-B chunk (t & 7) of rows (t >> 3) + 32 i, i < 8,
  // for A and for B; its LDS destination is that row's swizzled chunk
  const int gr = t >> 3, gc = t & 7;
  const uint32_t ga = (uint32_t)gr * (uint32_t)(ldx * 2) + (uint32_t)gc * 16;
  const uint32_t gb = (uint32_t)gr * (uint32_t)(ldw * 2) + (uint32_t)gc * 16;
  const uint32_t sxa = (uint32_t)(32 * ldx * 2), sxb = (uint32_t)(32 * ldw * 2);
  const int wlds = gr * 128 + ((gc ^ rsw(gr)) * 16);  // + 32 rows * 128 B per i (same swizzle)
  // staging registers roll: right after row i of the staged tile kt+1 is written to LDS, the
  // same registers receive row i of tile kt+2, which is written one K-tile (64 MFMAs, ~1,000
  // cycles) later.  (Loading tile kt+2 only after ALL of tile kt+1 was written left ~50 MFMAs
  // for the loads and every LDS write waited on them: 1.13 vs 1.55 PF/s in the probes.)
  // (a second register set, loading two K-tiles ahead, needs ~250 VGPRs and spilled)
  const int KT = K / BK;
  u32x4 sa[8], sb[8];
  auto load_a = [&](int kt, int i) { sa[i] = gload(rsX, ga + i * sxa + (uint32_t)(kt * BK * 2)); };
  auto load_b = [&](int kt, int i) { sb[i] = gload(rsW, gb + i * sxb + (uint32_t)(kt * BK * 2)); };
  auto write_a = [&](lds_t* st, int i) { lds_w128(st + wlds + i * 32 * 128, sa[i]); };
  auto write_b = [&](lds_t* st, int i) { lds_w128(st + IMG + wlds + i * 32 * 128, sb[i]); };

  // fragment reads: A rows wm*128 + 16 f + (lane & 15), B rows wn*128 + 16 f + (lane & 15);
  // lane group q = lane >> 4 holds k 8q .. 8q+7 of sub-step ks (chunk 4 ks + q)
  const int q = lane >> 4, rl = lane & 15;
  int foff[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) foff[ks] = rl * 128 + (((4 * ks + q) ^ rsw(rl)) * 16);
  const int abase = wm * 128 * 128, bbase = IMG + wn * 128 * 128;
  // A fragments roll (row i's register is refilled for the next sub-step as soon as row i's 8
  // MFMAs are issued), B fragments are double-buffered: 96 fragment VGPRs instead of 128
  bfx8 fa[8], fb[2][8];
  auto read_a = [&](const lds_t* st, int ks, int f) { fa[f] = lds_r128(st + abase + f * 16 * 128 + foff[ks]); };
  auto read_b = [&](const lds_t* st, int set, int ks, int f) { fb[set][f] = lds_r128(st + bbase + f * 16 * 128 + foff[ks]); };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the 256 accumulators are pinned to the AGPR file by inline-asm MFMAs (a builtin MFMA left
  // hipcc free to re-home them per unrolled copy: ~400 v_accvgpr moves per K-tile, 40 % MFMA busy)
  auto mfma = [&](int set, int idx) {
    const int i = idx >> 3, j = idx & 7;
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(fa[i]), "v"(fb[set][j]));
  };

  // prologue: tile 0 staged and written, tile 1 in flight, sub-step 0 of tile 0 read
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    load_a(0, i);
    load_b(0, i);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    write_a(smem, i);
    write_b(smem, i);
  }
  if (KT > 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      load_a(1, i);
      load_b(1, i);
    }
  }
  __syncthreads();
#pragma unroll
  for (int f = 0; f < 8; ++f) read_b(smem, 0, 0, f);
#pragma unroll
  for (int f = 0; f < 8; ++f) read_a(smem, 0, f);

  auto step = [&](auto more_c, auto more2_c, int kt) {
    constexpr bool more = decltype(more_c)::value, more2 = decltype(more2_c)::value;
    const lds_t* cur = smem + (kt & 1) * STAGE;
    lds_t* nxt = smem + ((kt + 1) & 1) * STAGE;
    __builtin_amdgcn_s_setprio(1);
    // ---- sub-step 0 (k 0..31): MFMAs on fb[0] and the rolling A fragments.  Set 1's B
    // fragments read one per 4 MFMAs (m = 1, 5, ..); row i's A register refilled with its
    // k 32..63 fragment right after row i's 8 MFMAs; half of the staged tile kt+1 (A rows)
    // written to nxt (free since the previous tile's barrier), one write per 8 MFMAs, each
    // followed by the load of the same row of tile kt+2
#pragma unroll
    for (int m = 0; m < 64; ++m) {
      mfma(0, m);
      if ((m & 7) == 1) {
        fence();
        if (PROBE != 1 && PROBE != 4) read_b(cur, 1, 1, m >> 3);
        fence();
      }
      if ((m & 7) == 7) {
        fence();
        if (PROBE != 1 && PROBE != 4) read_a(cur, 1, m >> 3);
        fence();
      }
      if (more && (m & 7) == 4) {
        fence();
        if (PROBE != 2 && PROBE != 4 && PROBE != 5) write_a(nxt, m >> 3);
        if (more2 && PROBE != 2 && PROBE != 4 && PROBE != 6) load_a(kt + 2, m >> 3);
        fence();
      }
    }
    // ---- sub-step 1 (k 32..63): MFMAs on fb[1].  The staged B rows written (MFMAs 0-15),
    // each followed by the load of the same row of tile kt+2 into its register, the barrier
    // that publishes tile kt+1 (MFMA 24), then its sub-step-0 fragments read: A rows 0-2 at
    // once, row i >= 3 after its MFMAs, B one per 4 MFMAs
#pragma unroll
    for (int m = 0; m < 64; ++m) {
      mfma(1, m);
      if (more && m < 16 && (m & 1) == 1) {
        fence();
        if (PROBE != 2 && PROBE != 4 && PROBE != 5) write_b(nxt, m >> 1);
        if (more2 && PROBE != 2 && PROBE != 4 && PROBE != 6) load_b(kt + 2, m >> 1);
        fence();
      }
      if (more && m == 24) {
        fence();
        __builtin_amdgcn_s_setprio(0);
        if (PROBE != 3 && PROBE != 4) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
        if (PROBE != 1 && PROBE != 4) {
          read_a(nxt, 0, 0);
          read_a(nxt, 0, 1);
          read_a(nxt, 0, 2);
        }
        fence();
      }
      if (more && m >= 31 && (m & 7) == 7) {
        fence();
        if (PROBE != 1 && PROBE != 4) read_a(nxt, 0, m >> 3);
        fence();
      }
      if (more && m >= 26 && m <= 54 && (m & 3) == 2) {
        fence();
        if (PROBE != 1 && PROBE != 4) read_b(nxt, 0, 0, (m - 26) >> 2);
        fence();
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  using T1 = std::true_type;
  using F0 = std::false_type;
  int kt = 0;
  for (; kt + 2 < KT; ++kt) step(T1(), T1(), kt);
  if (kt + 1 < KT) step(T1(), F0(), kt++);
  step(F0(), F0(), kt);

  // the last MFMAs' results must land before VALU reads the AGPRs (>= 12 wait states)
  asm volatile("s_nop 15\n\ts_nop 3" ::: "memory");
  // ---- epilogue: acc[i][j] reg r = row wm*128 + 16 i + 4 q + r, column wn*128 + 16 j + rl
  bf16_t* yb = Y + (int64_t)row0 * ldy + n0 + wn * 128 + rl;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = wm * 128 + 16 * i + 4 * q + r;
      if (m < rows) {
#pragma unroll
        for (int j = 0; j < 8; ++j) yb[(int64_t)m * ldy + 16 * j] = f2bf(acc[i][j][r]);
      }
    }
}

// ---- "1 x 4" variant: each wave owns 256 rows x 64 columns.  Only X goes through LDS (written
// once, read by all four waves); the wave's 64 weight columns are loaded straight from global
// memory into MFMA B-operand registers (lane (rl, q) of fragment j: row 16 j + rl, 16 bytes at
// k 8 q of the sub-step -- one buffer_load_dwordx4, no LDS round trip), NS - 1 K-tiles ahead.
// Per CU and 64-k step: LDS 32 KiB written + 128 KiB read (vs 64 + 128), global 64 KiB (same),
// 8 ds_write_b128 per wave instead of 16 -- the LDS store transfer was the largest single cost
// of the 2 x 2 layout (probe 5: 1.27 -> 1.71 PF/s without it).
// The last steps re-load / re-stage the final K-tile into free buffers (clamped indices) instead
// of branching inside the MFMA stream.
template <int NS, int PROBE = 0>
__global__ __launch_bounds__(NT, 1) void gemm4b_kernel(const bf16_t* __restrict__ X, int64_t ldx,
                                                       const bf16_t* __restrict__ W, int64_t ldw, int64_t strideW,
                                                       bf16_t* __restrict__ Y, int64_t ldy,
                                                       const int* __restrict__ offs, const int* __restrict__ tile_end,
                                                       int G, int N, int K, int gm) {
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * IMG];
  lds_t* smem = (lds_t*)smem_raw;
  const int t = threadIdx.x, lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nbn = N / BN;
  int slot, nt;
  tile_of(gm, nbn, slot, nt);
  const int total_slots = tile_end[G - 1];
  if (slot >= total_slots) return;  // uniform over the workgroup: no barrier reached yet
  const int g = find_group(tile_end, G, slot);
  const int first_slot = g ? tile_end[g - 1] : 0;
  const int row0 = (g ? offs[g - 1] : 0) + (slot - first_slot) * BM;
  const int rows = min(BM, offs[g] - row0);
  const int n0 = nt * BN + wid * 64;  // this wave's columns

  const rsrc_t rsX = make_rsrc(X + (int64_t)row0 * ldx, (uint32_t)(((int64_t)(rows - 1) * ldx + K) * 2));
  const rsrc_t rsW = make_rsrc(W + (int64_t)g * strideW + (int64_t)n0 * ldw, (uint32_t)((63 * ldw + K) * 2));
  const int KT = K / BK;

  // X staging (as the 2 x 2 kernel): thread t holds chunk (t & 7) of rows (t >> 3) + 32 i
  const int gr = t >> 3, gc = t & 7;
  const uint32_t ga = (uint32_t)gr * (uint32_t)(ldx * 2) + (uint32_t)gc * 16;
  const uint32_t sxa = (uint32_t)(32 * ldx * 2);
  const int wlds = gr * 128 + ((gc ^ rsw(gr)) * 16);
  u32x4 sa[8];
  auto load_a = [&](int kt, int i) { sa[i] = gload(rsX, ga + i * sxa + (uint32_t)(min(kt, KT - 1) * BK * 2)); };
  auto write_a = [&](lds_t* st, int i) { lds_w128(st + wlds + i * 32 * 128, sa[i]); };

  const int q = lane >> 4, rl = lane & 15;
  // weight fragments straight from memory: slot s holds K-tile kt = s (mod NS)
  const uint32_t gbw = (uint32_t)rl * (uint32_t)(ldw * 2) + (uint32_t)q * 16;
  const uint32_t sbj = (uint32_t)(16 * ldw * 2);
  bfx8 fb[NS][2][4];
  auto load_b = [&](int s, int kt, int ks, int j) {
    fb[s][ks][j] = __builtin_bit_cast(bfx8, gload(rsW, gbw + j * sbj + (uint32_t)(min(kt, KT - 1) * BK * 2 + ks * 64)));
  };

  int foff[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) foff[ks] = rl * 128 + (((4 * ks + q) ^ rsw(rl)) * 16);
  bfx8 fa[16];
  auto read_a = [&](const lds_t* st, int ks, int i) { fa[i] = lds_r128(st + i * 16 * 128 + foff[ks]); };

  f32x4 acc[16][4];
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfma = [&](int s, int ks, int m) {
    const int i = m >> 2, j = m & 3;
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(fa[i]), "v"(fb[s][ks][j]));
  };

  // prologue: weight tiles 0 .. NS-2 in flight, X tile 0 staged + written, X tile 1 in flight
#pragma unroll
  for (int i = 0; i < 8; ++i) load_a(0, i);
#pragma unroll
  for (int s = 0; s + 1 < NS; ++s)
#pragma unroll
    for (int e = 0; e < 8; ++e) load_b(s, s, e >> 2, e & 3);
#pragma unroll
  for (int i = 0; i < 8; ++i) write_a(smem, i);
#pragma unroll
  for (int i = 0; i < 8; ++i) load_a(1, i);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) read_a(smem, 0, i);

  auto step = [&](auto s_c, int kt) {
    constexpr int S = decltype(s_c)::value, SL = (S + NS - 1) % NS;
    const lds_t* cur = smem + (kt & 1) * IMG;
    lds_t* nxt = smem + ((kt + 1) & 1) * IMG;
    __builtin_amdgcn_s_setprio(1);
    // sub-step 0 (k 0..31): row i's register refilled with its k 32..63 fragment after its 4
    // MFMAs; X tile kt+1 written (one row-piece per 8 MFMAs, each followed by the load of the
    // same piece of tile kt+2); weight tile kt+NS-1 loaded into the slot tile kt-1 freed
#pragma unroll
    for (int m = 0; m < 64; ++m) {
      mfma(S, 0, m);
      if ((m & 3) == 3) {
        fence();
        if (PROBE != 1 && PROBE != 4) read_a(cur, 1, m >> 2);
        fence();
      }
      if ((m & 7) == 5) {
        fence();
        if (PROBE != 2 && PROBE != 4 && PROBE != 5) write_a(nxt, m >> 3);
        if (PROBE != 2 && PROBE != 4 && PROBE != 6) load_a(kt + 2, m >> 3);
        fence();
      }
      if ((m & 7) == 1) {
        fence();
        if (PROBE != 2 && PROBE != 4 && PROBE != 6) load_b(SL, kt + NS - 1, (m >> 3) & 1, m >> 4);
        fence();
      }
    }
    // sub-step 1 (k 32..63): the barrier that publishes X tile kt+1 after row 3's MFMAs, then
    // its k 0..31 fragments: rows 0-3 at once, row i >= 4 after its MFMAs
#pragma unroll
    for (int m = 0; m < 64; ++m) {
      mfma(S, 1, m);
      if (m == 15) {
        fence();
        __builtin_amdgcn_s_setprio(0);
        if (PROBE != 3 && PROBE != 4) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
        if (PROBE != 1 && PROBE != 4) {
#pragma unroll
          for (int i = 0; i < 4; ++i) read_a(nxt, 0, i);
        }
        fence();
      }
      if (m >= 19 && (m & 3) == 3) {
        fence();
        if (PROBE != 1 && PROBE != 4) read_a(nxt, 0, m >> 2);
        fence();
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  int kt = 0;
  for (; kt + NS <= KT; kt += NS) {
    step(std::integral_constant<int, 0>(), kt);
    step(std::integral_constant<int, 1>(), kt + 1);
    if constexpr (NS == 3) step(std::integral_constant<int, 2>(), kt + 2);
  }
  if (kt < KT) step(std::integral_constant<int, 0>(), kt);
  if constexpr (NS == 3)
    if (kt + 1 < KT) step(std::integral_constant<int, 1>(), kt + 1);

  asm volatile("s_nop 15\n\ts_nop 3" ::: "memory");
  // epilogue: acc[i][j] reg r = row 16 i + 4 q + r, column 16 j + rl of the wave's 64
  bf16_t* yb = Y + (int64_t)row0 * ldy + n0 + rl;
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 16 * i + 4 * q + r;
      if (m < rows) {
#pragma unroll
        for (int j = 0; j < 4; ++j) yb[(int64_t)m * ldy + 16 * j] = f2bf(acc[i][j][r]);
      }
    }
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved: nothing else in this kernel uses it
// one 1-KiB LDS-DMA piece: lane L's 16 bytes land at lds_base + 16 L
ST_DEVICE void dma16(rsrc_t rs, uint32_t lds_base, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(lds_base), "v"(voff), "s"(rs)
               : "memory", "m0");
}
// the same with the K-tile advance in the instruction's scalar offset: the lane offsets stay
// loop-invariant VGPRs, no VALU address arithmetic ahead of a piece
ST_DEVICE void dma16s(rsrc_t rs, uint32_t lds_base, uint32_t voff, uint32_t soff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :
               : "s"(lds_base), "v"(voff), "s"(rs), "s"(soff)
               : "memory", "m0");
}
#pragma clang diagnostic pop

// ---- "2 x 2, LDS-DMA" variant: the 2 x 2 kernel's per-wave tile and fragment schedule, with
// both operands copied global -> LDS by buffer_load ... lds (no staging VGPRs, no ds_write:
// per CU and K-tile 64 LDS instructions fewer -- 32 ds_read_b128 per wave remain).  The
// source address carries the swizzle (lane L of piece q writes row 8 q + L / 8, physical
// chunk L % 8, so it reads logical chunk (L % 8) ^ rsw(row)).  Two LDS stages: tile kt+1's 16
// pieces per wave go out half right after the barrier of tile kt-1 (the buffer's last readers
// are past it), half during sub-step 0 of tile kt; its barrier waits for them (vmcnt(0)).
template <int EPI, int PROBE = 0>
__global__ __launch_bounds__(NT, 1) void gemm4d_kernel(const bf16_t* __restrict__ X, int64_t ldx,
                                                       const bf16_t* __restrict__ W, int64_t ldw, int64_t strideW,
                                                       bf16_t* __restrict__ Y, int64_t ldy,
                                                       const int* __restrict__ offs, const int* __restrict__ tile_end,
                                                       int G, int N, int K, int gm) {
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * STAGE];
  lds_t* smem = (lds_t*)smem_raw;
  const int t = threadIdx.x, lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int nbn = N / BN;
  int slot, nt;
  tile_of(gm, nbn, slot, nt);
  const int total_slots = tile_end[G - 1];
  if (slot >= total_slots) return;  // uniform over the workgroup: no barrier reached yet
  const int g = find_group(tile_end, G, slot);
  const int first_slot = g ? tile_end[g - 1] : 0;
  const int row0 = (g ? offs[g - 1] : 0) + (slot - first_slot) * BM;
  const int rows = min(BM, offs[g] - row0);
  const int n0 = nt * BN;
  const rsrc_t rsX = make_rsrc(X + (int64_t)row0 * ldx, (uint32_t)(((int64_t)(rows - 1) * ldx + K) * 2));
  const rsrc_t rsW = make_rsrc(W + (int64_t)g * strideW + (int64_t)n0 * ldw, (uint32_t)(((int64_t)(BN - 1) * ldw + K) * 2));
  const int KT = K / BK;

  // wave w copies pieces w*8 .. w*8+7 of each image (piece q = image rows 8q .. 8q+7)
  uint32_t voa[8], vob[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int pr = (wid * 8 + i) * 8 + (lane >> 3), pc = lane & 7;
    voa[i] = (uint32_t)pr * (uint32_t)(ldx * 2) + (uint32_t)((pc ^ rsw(pr)) * 16);
    vob[i] = (uint32_t)pr * (uint32_t)(ldw * 2) + (uint32_t)((pc ^ rsw(pr)) * 16);
  }
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem + (uint32_t)(wid * 8 * 1024));
  auto dma_a = [&](int buf, int kt, int i) {
    if (PROBE != 2 && PROBE != 4) dma16(rsX, lbase + buf * STAGE + i * 1024, voa[i] + (uint32_t)(kt * BK * 2));
  };
  auto dma_b = [&](int buf, int kt, int i) {
    if (PROBE != 2 && PROBE != 4) dma16(rsW, lbase + buf * STAGE + IMG + i * 1024, vob[i] + (uint32_t)(kt * BK * 2));
  };

  const int q = lane >> 4, rl = lane & 15;
  int foff[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) foff[ks] = rl * 128 + (((4 * ks + q) ^ rsw(rl)) * 16);
  const int abase = wm * 128 * 128, bbase = IMG + wn * 128 * 128;
  bfx8 fa[8], fb[2][8];
  auto read_a = [&](const lds_t* st, int ks, int f) { fa[f] = lds_r128(st + abase + f * 16 * 128 + foff[ks]); };
  auto read_b = [&](const lds_t* st, int set, int ks, int f) { fb[set][f] = lds_r128(st + bbase + f * 16 * 128 + foff[ks]); };
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfma = [&](int set, int idx) {
    const int i = idx >> 3, j = idx & 7;
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(fa[i]), "v"(fb[set][j]));
  };

  // prologue: tile 0 copied and published; the X half of tile 1 in flight
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    dma_a(0, 0, i);
    dma_b(0, 0, i);
  }
  if (KT > 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) dma_a(1, 1, i);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
#pragma unroll
  for (int f = 0; f < 8; ++f) read_b(smem, 0, 0, f);
#pragma unroll
  for (int f = 0; f < 8; ++f) read_a(smem, 0, f);

  auto step = [&](auto more_c, auto more2_c, int kt) {
    constexpr bool more = decltype(more_c)::value, more2 = decltype(more2_c)::value;
    const lds_t* cur = smem + (kt & 1) * STAGE;
    const lds_t* nxt = smem + ((kt + 1) & 1) * STAGE;
    __builtin_amdgcn_s_setprio(1);
    // sub-step 0: set 1's B fragments and row i's k 32..63 A fragment read as in the 2 x 2
    // kernel; the weight half of tile kt+1 copied (one piece per 8 MFMAs)
#pragma unroll
    for (int m = 0; m < 64; ++m) {
      mfma(0, m);
      if ((m & 7) == 1) {
        fence();
        if (PROBE != 1 && PROBE != 4) read_b(cur, 1, 1, m >> 3);
        fence();
      }
      if ((m & 7) == 7) {
        fence();
        if (PROBE != 1 && PROBE != 4) read_a(cur, 1, m >> 3);
        fence();
      }
      if (more && (m & 7) == 4) {
        fence();
        dma_b((kt + 1) & 1, kt + 1, m >> 3);
        fence();
      }
    }
    // sub-step 1: barrier publishing tile kt+1 after MFMA 24 (own pieces landed, own reads of
    // cur done), its first fragments read, and the X half of tile kt+2 copied into cur
#pragma unroll
    for (int m = 0; m < 64; ++m) {
      mfma(1, m);
      if (more && m == 24) {
        fence();
        __builtin_amdgcn_s_setprio(0);
        if (PROBE != 3 && PROBE != 4) {
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
        if (PROBE != 1 && PROBE != 4) {
          read_a(nxt, 0, 0);
          read_a(nxt, 0, 1);
          read_a(nxt, 0, 2);
        }
        fence();
      }
      if (more && m >= 31 && (m & 7) == 7) {
        fence();
        if (PROBE != 1 && PROBE != 4) read_a(nxt, 0, m >> 3);
        fence();
      }
      if (more && m >= 26 && m <= 54 && (m & 3) == 2) {
        fence();
        if (PROBE != 1 && PROBE != 4) read_b(nxt, 0, 0, (m - 26) >> 2);
        fence();
      }
      if (more2 && m >= 28 && m <= 63 && (m & 3) == 0 && m != 60) {
        fence();
        dma_a(kt & 1, kt + 2, (m - 28) >> 2);
        fence();
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  using T1 = std::true_type;
  using F0 = std::false_type;
  int kt = 0;
  for (; kt + 2 < KT; ++kt) step(T1(), T1(), kt);
  if (kt + 1 < KT) step(T1(), F0(), kt++);
  step(F0(), F0(), kt);

  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 15\n\ts_nop 3" ::: "memory");
  bf16_t* yb = Y + (int64_t)row0 * ldy + n0 + wn * 128 + rl;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = wm * 128 + 16 * i + 4 * q + r;
      if (m < rows) {
#pragma unroll
        for (int j = 0; j < 8; ++j) yb[(int64_t)m * ldy + 16 * j] = f2bf(acc[i][j][r]);
      }
    }
}

// ---- "2 x 2, LDS-DMA, whole-tile fragments" variant.  The K-tile's fragments of BOTH 32-k
// sub-steps live in registers (fa / fb [ks][8]: 128 VGPRs), so a stage of LDS is dead once its
// sub-step-1 fragments are read -- 40 % into the tile -- instead of at its end:
//   phase 0 (MFMAs 0-63, sub-step 0 operands): sub-step 1's fragments read (one per 2 MFMAs);
//   MFMA 44: s_waitcnt vmcnt(0) lgkmcnt(0) + the tile's ONE barrier -- every wave holds all of
//   tile kt (its stage is free) and has landed its pieces of tile kt+1 (published);
//   then tile kt+2's 16 DMA pieces per wave into the freed stage, spread over MFMAs 45-103,
//   and (phase 1, MFMAs 64-127 on sub-step 1 operands) tile kt+1's sub-step-0 fragments read
//   into the registers phase 0 released.
// The DMA of a tile is issued ~1 tile before its barrier (vs ~0.4 in variant 4).
template <int EPI, int PROBE = 0, int SCHED = 0>
__global__ __launch_bounds__(NT, 1) void gemm4e_kernel(const bf16_t* __restrict__ X, int64_t ldx,
                                                       const bf16_t* __restrict__ W, int64_t ldw, int64_t strideW,
                                                       bf16_t* __restrict__ Y, int64_t ldy,
                                                       const int* __restrict__ offs, const int* __restrict__ tile_end,
                                                       int G, int N, int K, int gm, bf16_t* __restrict__ Y2,
                                                       int64_t ldy2, int I, int Tdense, int nvirt) {
  static_assert(EPI == 0 || EPI == 1, "EPI 0: plain, 1: gate|up + SwiGLU");
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * STAGE];
  lds_t* smem = (lds_t*)smem_raw;
  const int t = threadIdx.x, lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int nbn = N / BN;
  // persistent: the workgroup walks virtual tiles vb = blockIdx.x, + gridDim.x, ... (one launch
  // of #CU workgroups holds the chip for the whole GEMM, so a side-stream kernel cannot wedge
  // into a CU between two tiles); nvirt == 0: one tile per workgroup
  const int nv = nvirt ? nvirt : (int)gridDim.x;
  for (int vb = (int)blockIdx.x; vb < nv; vb += (nvirt ? (int)gridDim.x : nv)) {
  if (vb != (int)blockIdx.x) __syncthreads();  // every wave is past the previous tile's LDS reads
  int slot, nt;
  tile_of_v(gm, nbn, vb, nv, slot, nt);
  int g = 0, row0, rows;
  if (tile_end == nullptr) {  // dense: Tdense rows, one weight
    if (slot >= (Tdense + BM - 1) / BM) continue;  // uniform over the workgroup
    row0 = slot * BM;
    rows = min(BM, Tdense - row0);
  } else {
    const int total_slots = tile_end[G - 1];
    if (slot >= total_slots) continue;  // uniform over the workgroup
    g = find_group(tile_end, G, slot);
    const int first_slot = g ? tile_end[g - 1] : 0;
    row0 = (g ? offs[g - 1] : 0) + (slot - first_slot) * BM;
    rows = min(BM, offs[g] - row0);
  }
  const int n0 = nt * BN;
  const rsrc_t rsX = make_rsrc(X + (int64_t)row0 * ldx, (uint32_t)(((int64_t)(rows - 1) * ldx + K) * 2));
  // EPI 1: the descriptor spans the whole [2I, K] weight (the tile's rows are gathered)
  const rsrc_t rsW = EPI == 1
      ? make_rsrc(W + (int64_t)g * strideW, (uint32_t)(((int64_t)(N - 1) * ldw + K) * 2))
      : make_rsrc(W + (int64_t)g * strideW + (int64_t)n0 * ldw, (uint32_t)(((int64_t)(BN - 1) * ldw + K) * 2));
  const int KT = K / BK;

  // wave w copies pieces w*8 .. w*8+7 of each image (piece q = image rows 8q .. 8q+7)
  uint32_t voa[8], vob[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int pr = (wid * 8 + i) * 8 + (lane >> 3), pc = lane & 7;
    voa[i] = (uint32_t)pr * (uint32_t)(ldx * 2) + (uint32_t)((pc ^ rsw(pr)) * 16);
    // EPI 1: image row pr of N-tile nt -> wave column wn = pr / 128 holds 64 gate rows then the
    // 64 matching up rows, so a lane's acc[.][j] and acc[.][j + 4] are gate and up of ONE feature
    int wrow = pr;
    if (EPI == 1) {
      const int loc = pr & 127;
      wrow = ((loc & 64) ? I : 0) + nt * 128 + (pr >> 7) * 64 + (loc & 63);
    }
    vob[i] = (uint32_t)wrow * (uint32_t)(ldw * 2) + (uint32_t)((pc ^ rsw(pr)) * 16);
  }
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem + (uint32_t)(wid * 8 * 1024));
  // piece p < 8: X piece p, else W piece p - 8
  auto dma = [&](int buf, int kt, int p) {
    if (PROBE == 2 || PROBE == 4) return;
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(kt * BK * 2));
    if (p < 8) dma16s(rsX, lbase + buf * STAGE + p * 1024, voa[p], so);
    else dma16s(rsW, lbase + buf * STAGE + IMG + (p - 8) * 1024, vob[p - 8], so);
  };

  const int q = lane >> 4, rl = lane & 15;
  int foff[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) foff[ks] = rl * 128 + (((4 * ks + q) ^ rsw(rl)) * 16);
  const int abase = wm * 128 * 128, bbase = IMG + wn * 128 * 128;
  bfx8 fa[2][8], fb[2][8];
  // fragment read r < 8: A row-block r, else B column-block r - 8
  auto read = [&](const lds_t* st, int ks, int r) {
    if (PROBE == 1 || PROBE == 4) return;
    if (r < 8) fa[ks][r] = lds_r128(st + abase + r * 16 * 128 + foff[ks]);
    else fb[ks][r - 8] = lds_r128(st + bbase + (r - 8) * 16 * 128 + foff[ks]);
  };
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // operands swapped (weight fragment as A): acc[i][j] reg r = C[row 16 i + rl][col 16 j + 4 q + r],
  // so a lane holds 4 CONSECUTIVE output columns of one row -- 8-byte epilogue stores
  auto mfma = [&](int ks, int idx) {
    const int i = idx >> 3, j = idx & 7;
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(fb[ks][j]), "v"(fa[ks][i]));
  };

  // prologue: tiles 0 and 1 requested, tile 0 published, its sub-step-0 fragments read
#pragma unroll
  for (int p = 0; p < 16; ++p) dma(0, 0, p);
  if (KT > 1) {
#pragma unroll
    for (int p = 0; p < 16; ++p) dma(1, 1, p);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) read(smem, 0, r);

  // slot tables (MFMA index of each operation).  SCHED bit 1: sub-step 1 reads spread over
  // MFMAs 0-42 and the next tile's sub-step 0 reads over 64-124 (else packed into 0-30 / 64-94);
  // bit 0: M0 of a piece written two MFMAs before its DMA (else right before it).
  // bit 2 (SPLIT): the X region of a stage is released after its sub-step-1 reads (barrier at
  // MFMA 20, lgkmcnt(3)) and gets tile kt+2's X pieces at MFMAs 21-56; the W region and the
  // publication of tile kt+1 share one barrier at MFMA 63 (vmcnt(8): all but this step's X
  // pieces); W pieces at 64-120 -- the pieces spread over the whole tile (hipBLASLt's DTL
  // kernels release their stage in parts too)
  constexpr bool SPREAD = SCHED & 2, M0AHEAD = SCHED & 1, SPLIT = SCHED & 4;
  constexpr int BAR = SPLIT ? 63 : (SPREAD ? 46 : 44), DMA0 = BAR + 1, BARA = 20;
  constexpr auto rd1_slot = [](int m) constexpr -> int {  // read index of tile kt's sub-step 1 after MFMA m
    if (SPREAD) {
      for (int r = 0; r < 16; ++r)
        if (m == (r * 42) / 15) return r;
      return -1;
    }
    return m < 32 && (m & 1) == 0 ? m >> 1 : -1;
  };
  constexpr auto rd0_slot = [](int m) constexpr -> int {  // read index of tile kt+1's sub-step 0
    if (SPREAD) return m >= 64 && m <= 124 && (m & 3) == 0 ? (m - 64) >> 2 : -1;
    return m >= 64 && m < 96 && (m & 1) == 0 ? (m - 64) >> 1 : -1;
  };
  constexpr auto dma_slot = [](int m) constexpr -> int {
    if (SPLIT) {
      if (m >= 21 && m <= 56 && (m - 21) % 5 == 0) return (m - 21) / 5;          // X pieces
      if (m >= 64 && m <= 120 && ((m - 64) & 7) == 0) return 8 + ((m - 64) >> 3);  // W pieces
      return -1;
    }
    return m >= DMA0 && m <= DMA0 + 60 && ((m - DMA0) & 3) == 0 ? (m - DMA0) >> 2 : -1;
  };
  auto piece_m0 = [&](int buf, int p) {
    return lbase + buf * STAGE + (p < 8 ? p * 1024 : IMG + (p - 8) * 1024);
  };
  auto set_m0 = [&](uint32_t v) { asm volatile("s_mov_b32 m0, %0" : : "s"(v) : "m0"); };
  auto dma_nom0 = [&](int kt, int p) {  // M0 already holds the piece's LDS address
    if (PROBE == 2 || PROBE == 4) return;
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(kt * BK * 2));
    if (p < 8)
      asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" : : "v"(voa[p]), "s"(rsX), "s"(so) : "memory");
    else
      asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" : : "v"(vob[p - 8]), "s"(rsW), "s"(so) : "memory");
  };
  // PROBE 7 (diagnostic build): shader-cycle stamps per segment of the steady-state step,
  // summed per wave and written over the output (tools/_g4stamps.py reads them)
  uint64_t seg[4] = {0, 0, 0, 0};
  uint64_t ts[5];
  auto stamp = [&](int k) {
    if constexpr (PROBE == 7) {
      fence();
      ts[k] = __builtin_amdgcn_s_memtime();
      fence();
    }
  };
  auto step = [&](auto more_c, auto more2_c, int kt) {
    constexpr bool more = decltype(more_c)::value, more2 = decltype(more2_c)::value;
    const lds_t* cur = smem + (kt & 1) * STAGE;
    const lds_t* nxt = smem + ((kt + 1) & 1) * STAGE;
    __builtin_amdgcn_s_setprio(1);
    if constexpr (more2) stamp(0);
    static_for<0, 128>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      mfma(m >> 6, m & 63);
      constexpr int r1 = rd1_slot(m), r0 = rd0_slot(m), pd = dma_slot(m), pn = dma_slot(m + 2);
      if constexpr (r1 >= 0) {  // sub-step 1 fragments of tile kt
        fence();
        read(cur, 1, r1);
        fence();
      }
      if constexpr (SPLIT && m == BARA && more2) {  // X region of cur: every wave's reads done
        fence();
        if (PROBE != 3 && PROBE != 4) {
          asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
        asm volatile("" ::: "memory");
        fence();
      }
      if constexpr (m == BAR && more) {
        fence();
        if constexpr (more2) stamp(1);
        __builtin_amdgcn_s_setprio(0);
        if (PROBE != 3 && PROBE != 4) {
          if constexpr (SPLIT && more2) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
        if constexpr (more2) stamp(2);
        fence();
      }
      if constexpr (m == (SPLIT ? 100 : 63) && more2) stamp(3);
      if constexpr (more2 && M0AHEAD && pn >= 0 && PROBE != 2 && PROBE != 4) {
        fence();
        set_m0(piece_m0(kt & 1, pn));
        fence();
      }
      if constexpr (more2 && pd >= 0) {
        fence();
        if constexpr (M0AHEAD) dma_nom0(kt + 2, pd);
        else dma(kt & 1, kt + 2, pd);
        fence();
      }
      if constexpr (more && r0 >= 0) {  // sub-step 0 fragments of tile kt+1
        fence();
        read(nxt, 0, r0);
        fence();
      }
    });
    if constexpr (more2 && PROBE == 7) {
      stamp(4);
      for (int k = 0; k < 4; ++k) seg[k] += ts[k + 1] - ts[k];
    }
    __builtin_amdgcn_s_setprio(0);
  };
  using T1 = std::true_type;
  using F0 = std::false_type;
  int kt = 0;
  for (; kt + 2 < KT; ++kt) step(T1(), T1(), kt);
  if (kt + 1 < KT) step(T1(), F0(), kt++);
  step(F0(), F0(), kt);

  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 15\n\ts_nop 3" ::: "memory");
  if constexpr (PROBE == 7) {  // lane 0 of each wave: 4 x u64 segment sums + step count at row 4 w + lane
    if (lane == 0) {
      uint64_t* d = reinterpret_cast<uint64_t*>(Y + (int64_t)(row0 + wid) * ldy + n0);
      for (int k = 0; k < 4; ++k) d[k] = seg[k];
      d[4] = (uint64_t)(KT - 2);
    }
    continue;
  }
  auto pk4 = [](float a, float b, float c, float d) {
    uint2 v;
    v.x = (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
    v.y = (uint32_t)f2bf(c) | ((uint32_t)f2bf(d) << 16);
    return v;
  };
  if constexpr (EPI == 1) {
    // gu [T, 2I]: gate feature c at column c, up at I + c; h [T, I] = silu(gate) * up of the
    // bf16-rounded gate / up (what csrc/swiglu.hip computes from the stored gu)
    const int c0 = nt * 128 + wn * 64 + 4 * q;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = wm * 128 + 16 * i + rl;
      if (m < rows) {
        bf16_t* gb = Y + (int64_t)(row0 + m) * ldy + c0;
        bf16_t* hb = Y2 + (int64_t)(row0 + m) * ldy2 + c0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 gv = acc[i][j], uv = acc[i][j + 4];
          const uint2 gp = pk4(gv[0], gv[1], gv[2], gv[3]), up = pk4(uv[0], uv[1], uv[2], uv[3]);
          *reinterpret_cast<uint2*>(gb + 16 * j) = gp;
          *reinterpret_cast<uint2*>(gb + I + 16 * j) = up;
          float hv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t gw = r < 2 ? gp.x : gp.y, uw = r < 2 ? up.x : up.y;
            const float gq = __uint_as_float((r & 1) ? (gw & 0xffff0000u) : (gw << 16));
            const float uq = __uint_as_float((r & 1) ? (uw & 0xffff0000u) : (uw << 16));
            hv[r] = silu(gq) * uq;
          }
          *reinterpret_cast<uint2*>(hb + 16 * j) = pk4(hv[0], hv[1], hv[2], hv[3]);
        }
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = wm * 128 + 16 * i + rl;
      if (m < rows) {
        bf16_t* yb = Y + (int64_t)(row0 + m) * ldy + n0 + wn * 128 + 4 * q;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const f32x4 v = acc[i][j];
          *reinterpret_cast<uint2*>(yb + 16 * j) = pk4(v[0], v[1], v[2], v[3]);
        }
      }
    }
  }
  }  // tile loop
}


// ---- gemm4f: the kind-5 tile (whole-tile fragments, split stage release, M0 set ahead) in a
// PERSISTENT workgroup that treats its tiles as ONE stream of K-tiles: the DMA two steps ahead
// runs into the next tile's first K-tiles while this tile's last steps and epilogue run, and
// the next tile's first fragments are read in the last step -- no per-tile prologue, no launch
// gaps, and (one workgroup per CU for the whole GEMM) no side-stream kernel wedged between
// tiles.  K must hold >= 2 K-tiles.
template <int EPI>
__global__ __launch_bounds__(NT, 1) void gemm4f_kernel(const bf16_t* __restrict__ X, int64_t ldx,
                                                       const bf16_t* __restrict__ W, int64_t ldw, int64_t strideW,
                                                       bf16_t* __restrict__ Y, int64_t ldy,
                                                       const int* __restrict__ offs, const int* __restrict__ tile_end,
                                                       int G, int N, int K, int gm, bf16_t* __restrict__ Y2,
                                                       int64_t ldy2, int I, int Tdense, int nvirt) {
  static_assert(EPI == 0 || EPI == 1, "EPI 0: plain, 1: gate|up + SwiGLU");
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * STAGE];
  lds_t* smem = (lds_t*)smem_raw;
  const int t = threadIdx.x, lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int nbn = N / BN, KT = K / BK, stride = (int)gridDim.x;

  struct Tile {
    int vb, g, row0, rows, nt;
    rsrc_t rsX, rsW;
  };
  // the first live virtual tile at or after vb (vb == nvirt: none)
  auto find = [&](int vb, Tile& tl) -> bool {
    for (; vb < nvirt; vb += stride) {
      int slot, nt;
      tile_of_v(gm, nbn, vb, nvirt, slot, nt);
      int g = 0, row0, rows;
      if (tile_end == nullptr) {
        if (slot >= (Tdense + BM - 1) / BM) continue;
        row0 = slot * BM;
        rows = min(BM, Tdense - row0);
      } else {
        if (slot >= tile_end[G - 1]) continue;
        g = find_group(tile_end, G, slot);
        const int first_slot = g ? tile_end[g - 1] : 0;
        row0 = (g ? offs[g - 1] : 0) + (slot - first_slot) * BM;
        rows = min(BM, offs[g] - row0);
      }
      tl.vb = vb;
      tl.g = g;
      tl.row0 = row0;
      tl.rows = rows;
      tl.nt = nt;
      tl.rsX = make_rsrc(X + (int64_t)row0 * ldx, (uint32_t)(((int64_t)(rows - 1) * ldx + K) * 2));
      // EPI 1: base at the tile's first gate row, the up rows I further (lane offsets tile-free)
      tl.rsW = EPI == 1 ? make_rsrc(W + (int64_t)g * strideW + (int64_t)nt * 128 * ldw,
                                    (uint32_t)(((int64_t)(I + 127) * ldw + K) * 2))
                        : make_rsrc(W + (int64_t)g * strideW + (int64_t)nt * BN * ldw,
                                    (uint32_t)(((int64_t)(BN - 1) * ldw + K) * 2));
      return true;
    }
    return false;
  };

  uint32_t voa[8], vob[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int pr = (wid * 8 + i) * 8 + (lane >> 3), pc = lane & 7;
    voa[i] = (uint32_t)pr * (uint32_t)(ldx * 2) + (uint32_t)((pc ^ rsw(pr)) * 16);
    int wrow = pr;
    if (EPI == 1) {
      const int loc = pr & 127;
      wrow = ((loc & 64) ? I : 0) + (pr >> 7) * 64 + (loc & 63);
    }
    vob[i] = (uint32_t)wrow * (uint32_t)(ldw * 2) + (uint32_t)((pc ^ rsw(pr)) * 16);
  }
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem + (uint32_t)(wid * 8 * 1024));
  auto piece_m0 = [&](int buf, int p) { return lbase + buf * STAGE + (p < 8 ? p * 1024 : IMG + (p - 8) * 1024); };
  auto set_m0 = [&](uint32_t v) { asm volatile("s_mov_b32 m0, %0" : : "s"(v) : "m0"); };
  auto dma_nom0 = [&](rsrc_t dX, rsrc_t dW, uint32_t so, int p) {  // M0 holds the piece's LDS address
    if (p < 8)
      asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" : : "v"(voa[p]), "s"(dX), "s"(so) : "memory");
    else
      asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" : : "v"(vob[p - 8]), "s"(dW), "s"(so) : "memory");
  };
  auto dma = [&](int buf, rsrc_t dX, rsrc_t dW, int kt, int p) {
    set_m0(piece_m0(buf, p));
    dma_nom0(dX, dW, __builtin_amdgcn_readfirstlane((uint32_t)(kt * BK * 2)), p);
  };

  const int q = lane >> 4, rl = lane & 15;
  int foff[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) foff[ks] = rl * 128 + (((4 * ks + q) ^ rsw(rl)) * 16);
  const int abase = wm * 128 * 128, bbase = IMG + wn * 128 * 128;
  bfx8 fa[2][8], fb[2][8];
  auto read = [&](const lds_t* st, int ks, int r) {
    if (r < 8) fa[ks][r] = lds_r128(st + abase + r * 16 * 128 + foff[ks]);
    else fb[ks][r - 8] = lds_r128(st + bbase + (r - 8) * 16 * 128 + foff[ks]);
  };

  Tile cur, nxt;
  if (!find((int)blockIdx.x, cur)) return;  // uniform: no barrier reached
  bool has_nxt = find(cur.vb + stride, nxt);

  // prologue: K-tiles 0 and 1 of the first tile requested, 0 published, its sub-step-0 read
#pragma unroll
  for (int p = 0; p < 16; ++p) dma(0, cur.rsX, cur.rsW, 0, p);
#pragma unroll
  for (int p = 0; p < 16; ++p) dma(1, cur.rsX, cur.rsW, 1, p);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) read(smem, 0, r);

  // slot tables (SCHED 5 of gemm4e): sub-step 1 reads at MFMAs 0-30; X stage region released
  // at 20 and refilled at 21-56; publication + W region at 63; W pieces at 64-120; the next
  // step's sub-step 0 reads at 64-94
  constexpr auto dslot = [](int m) constexpr -> int {
    if (m >= 21 && m <= 56 && (m - 21) % 5 == 0) return (m - 21) / 5;
    if (m >= 64 && m <= 120 && ((m - 64) & 7) == 0) return 8 + ((m - 64) >> 3);
    return -1;
  };
  // gs: global step (buffer parity); d / kd: the tile and K-tile two steps ahead
  auto mfma = [&](f32x4 (&acc)[8][8], int ks, int idx) {
    const int i = idx >> 3, j = idx & 7;
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(fb[ks][j]), "v"(fa[ks][i]));
  };
  auto step = [&](f32x4 (&acc)[8][8], auto more_c, auto more2_c, int gs, rsrc_t dX, rsrc_t dW, uint32_t so) {
    constexpr bool more = decltype(more_c)::value, more2 = decltype(more2_c)::value;
    const lds_t* cs = smem + (gs & 1) * STAGE;
    const lds_t* ns = smem + ((gs + 1) & 1) * STAGE;
    __builtin_amdgcn_s_setprio(1);
    static_for<0, 128>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      mfma(acc, m >> 6, m & 63);
      constexpr int pd = dslot(m), pn = dslot(m + 2);
      if constexpr (m < 32 && (m & 1) == 0) {
        fence();
        read(cs, 1, m >> 1);
        fence();
      }
      if constexpr (m == 20 && more2) {  // X region of this stage: every wave's reads done
        fence();
        asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        fence();
      }
      if constexpr (m == 63 && more) {  // next step's K-tile published, W region free
        fence();
        __builtin_amdgcn_s_setprio(0);
        if constexpr (more2) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
        fence();
      }
      if constexpr (more2 && pn >= 0) {
        fence();
        set_m0(piece_m0(gs & 1, pn));
        fence();
      }
      if constexpr (more2 && pd >= 0) {
        fence();
        dma_nom0(dX, dW, so, pd);
        fence();
      }
      if constexpr (more && m >= 64 && m < 96 && (m & 1) == 0) {
        fence();
        read(ns, 0, (m - 64) >> 1);
        fence();
      }
    });
    __builtin_amdgcn_s_setprio(0);
  };
  auto pk4 = [](float a, float b, float c, float dd) {
    uint2 v;
    v.x = (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
    v.y = (uint32_t)f2bf(c) | ((uint32_t)f2bf(dd) << 16);
    return v;
  };
  using T1 = std::true_type;
  using F0 = std::false_type;
  int gs = 0;
  for (;;) {
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // steps whose K-tile two ahead exists (this tile's, or the next tile's first two): all of
    // them when a next tile follows, else all but the last two (the stream's tail)
    const int kfull = has_nxt ? KT : KT - 2;
    int kt = 0;
    for (; kt < kfull; ++kt, ++gs) {
      const bool in_cur = kt + 2 < KT;
      const rsrc_t dX = in_cur ? cur.rsX : nxt.rsX, dW = in_cur ? cur.rsW : nxt.rsW;
      const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)((in_cur ? kt + 2 : kt + 2 - KT) * BK * 2));
      step(acc, T1(), T1(), gs, dX, dW, so);
    }
    if (!has_nxt) {
      step(acc, T1(), F0(), gs++, cur.rsX, cur.rsW, 0u);
      step(acc, F0(), F0(), gs++, cur.rsX, cur.rsW, 0u);
    }
    asm volatile("s_nop 15\n\ts_nop 3" ::: "memory");
    // epilogue of `cur` (the next tile's first K-tiles are in flight meanwhile)
    if constexpr (EPI == 1) {
      const int c0 = cur.nt * 128 + wn * 64 + 4 * q;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = wm * 128 + 16 * i + rl;
        if (m < cur.rows) {
          bf16_t* gb = Y + (int64_t)(cur.row0 + m) * ldy + c0;
          bf16_t* hb = Y2 + (int64_t)(cur.row0 + m) * ldy2 + c0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4 gv = acc[i][j], uv = acc[i][j + 4];
            const uint2 gp = pk4(gv[0], gv[1], gv[2], gv[3]), up = pk4(uv[0], uv[1], uv[2], uv[3]);
            *reinterpret_cast<uint2*>(gb + 16 * j) = gp;
            *reinterpret_cast<uint2*>(gb + I + 16 * j) = up;
            float hv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const uint32_t gw = r < 2 ? gp.x : gp.y, uw = r < 2 ? up.x : up.y;
              const float gq = __uint_as_float((r & 1) ? (gw & 0xffff0000u) : (gw << 16));
              const float uq = __uint_as_float((r & 1) ? (uw & 0xffff0000u) : (uw << 16));
              hv[r] = silu(gq) * uq;
            }
            *reinterpret_cast<uint2*>(hb + 16 * j) = pk4(hv[0], hv[1], hv[2], hv[3]);
          }
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = wm * 128 + 16 * i + rl;
        if (m < cur.rows) {
          bf16_t* yb = Y + (int64_t)(cur.row0 + m) * ldy + cur.nt * BN + wn * 128 + 4 * q;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const f32x4 v = acc[i][j];
            *reinterpret_cast<uint2*>(yb + 16 * j) = pk4(v[0], v[1], v[2], v[3]);
          }
        }
      }
    }
    if (!has_nxt) break;
    cur = nxt;
    has_nxt = find(cur.vb + stride, nxt);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

// compute units of the current device (persistent grids)
static int cu_count() {
  static int cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

static bool persist_on() {
  const char* e = std::getenv("ST_GEMM4W_PERSIST");  // 0: one tile per workgroup (A/B)
  return !e || std::atoi(e) != 0;
}

extern "C" {

// M-tile slots for T rows in G groups (upper bound of sum_g ceil(n_g / 256)).
int64_t st_gemm4w_slots(int T, int G) { return (int64_t)(T + BM - 1) / BM + G; }

// Y[rows of g] = X[rows of g] @ W[g]^T; W[g] [N][K]; offs / tile_end int32 [G] device
// (tile_end = inclusive prefix of ceil(n_g / 256)).  0 on success, -2 unsupported shape.
int st_gemm4w(const void* X, int64_t ldx, const void* W, int64_t ldw, int64_t strideW, void* Y, int64_t ldy,
              const int* offs, const int* tile_end, int T, int G, int N, int K, hipStream_t st) {
  if (T <= 0 || G <= 0 || N <= 0 || K <= 0) return -2;
  if (K % BK || N % BN) return -2;
  if (ldx % 8 || ldw % 8 || ldy % 8 || ldx < K || ldw < K || ldy < N) return -2;
  if (((uintptr_t)X | (uintptr_t)W | (uintptr_t)Y) % 16) return -2;
  if (((int64_t)(BM + 32) * ldx) * 2 >= (int64_t)1 << 32) return -2;  // 32-bit buffer offsets per tile
  if (((int64_t)BN * ldw) * 2 >= (int64_t)1 << 32) return -2;
  const int64_t grid = st_gemm4w_slots(T, G) * (N / BN);
  if (grid >= (1LL << 31)) return -2;
  const char* pe = std::getenv("ST_GEMM4W_PROBE");  // timing probes (wrong results)
  const int probe = pe ? std::atoi(pe) : 0;
  const char* ke = std::getenv("ST_GEMM4W_KIND");  // 0: 2 x 2 waves, 1 / 2: 1 x 4 (NS 2 / 3), 4 / 5: 2 x 2 LDS-DMA (rolling / whole-tile fragments)
  const int kind = ke ? std::atoi(ke) : 5;
  const char* oe = std::getenv("ST_GEMM4W_ORDER");  // slots per XCD group (0: slot-major)
  const int gm = oe ? std::atoi(oe) : 0;
#define G4ARGS (const bf16_t*)X, ldx, (const bf16_t*)W, ldw, strideW, (bf16_t*)Y, ldy, offs, tile_end, G, N, K, gm
#define G4LAUNCH(KERN, ...)                                                            \
  do {                                                                                 \
    if (probe == 1) KERN, 1 __VA_ARGS__><<<(unsigned)grid, NT, 0, st>>>(G4ARGS);       \
    else if (probe == 2) KERN, 2 __VA_ARGS__><<<(unsigned)grid, NT, 0, st>>>(G4ARGS);  \
    else if (probe == 3) KERN, 3 __VA_ARGS__><<<(unsigned)grid, NT, 0, st>>>(G4ARGS);  \
    else if (probe == 4) KERN, 4 __VA_ARGS__><<<(unsigned)grid, NT, 0, st>>>(G4ARGS);  \
    else if (probe == 5) KERN, 5 __VA_ARGS__><<<(unsigned)grid, NT, 0, st>>>(G4ARGS);  \
    else if (probe == 6) KERN, 6 __VA_ARGS__><<<(unsigned)grid, NT, 0, st>>>(G4ARGS);  \
    else KERN, 0 __VA_ARGS__><<<(unsigned)grid, NT, 0, st>>>(G4ARGS);                  \
  } while (0)
  if (kind == 0) G4LAUNCH(gemm4w_kernel<0);
  else if (kind == 4) G4LAUNCH(gemm4d_kernel<0);
  else if (kind == 6 && K / BK >= 2) {
    const int64_t lg = std::min<int64_t>(grid, cu_count());
    gemm4f_kernel<0><<<(unsigned)lg, NT, 0, st>>>((const bf16_t*)X, ldx, (const bf16_t*)W, ldw, strideW,
                                                  (bf16_t*)Y, ldy, offs, tile_end, G, N, K, gm, nullptr, 0, 0, 0,
                                                  (int)grid);
  } else if (kind == 5 || kind == 6) {
    const int64_t vt = grid;  // virtual tiles
    const int pv = persist_on() ? (int)vt : 0;
    const int64_t grid = pv ? std::min<int64_t>(vt, cu_count()) : vt;  // persistent: one workgroup per CU
#undef G4ARGS
#define G4ARGS (const bf16_t*)X, ldx, (const bf16_t*)W, ldw, strideW, (bf16_t*)Y, ldy, offs, tile_end, G, N, K, gm, \
               (bf16_t*)nullptr, (int64_t)0, 0, 0, pv
    const char* se = std::getenv("ST_GEMM4W_SCHED");
    const int sched = se ? std::atoi(se) : 5;
    if (probe == 7 && sched == 4) gemm4e_kernel<0, 7, 4><<<(unsigned)grid, NT, 0, st>>>(G4ARGS);
    else if (probe == 7) gemm4e_kernel<0, 7><<<(unsigned)grid, NT, 0, st>>>(G4ARGS);
    else if (sched == 1) G4LAUNCH(gemm4e_kernel<0, , 1);
    else if (sched == 2) G4LAUNCH(gemm4e_kernel<0, , 2);
    else if (sched == 3) G4LAUNCH(gemm4e_kernel<0, , 3);
    else if (sched == 4) G4LAUNCH(gemm4e_kernel<0, , 4);
    else if (sched == 5) G4LAUNCH(gemm4e_kernel<0, , 5);
    else G4LAUNCH(gemm4e_kernel<0);
#undef G4ARGS
#define G4ARGS (const bf16_t*)X, ldx, (const bf16_t*)W, ldw, strideW, (bf16_t*)Y, ldy, offs, tile_end, G, N, K, gm
  }
  else if (kind == 2) G4LAUNCH(gemm4b_kernel<3);
  else G4LAUNCH(gemm4b_kernel<2);
#undef G4LAUNCH
#undef G4ARGS
  return (int)hipGetLastError();
}

// Grouped form of st_gemm4w_swiglu: rows [offs[g-1], offs[g]) use W[g] ([2I, K], gate rows then
// up rows, stride strideW); tile_end = inclusive prefix of ceil(n_g / 256) (device).  Rows past
// offs[G-1] are not written.  0 on success, -2 unsupported shape.
int st_gemm4w_swiglu_grouped(const void* X, int64_t ldx, const void* W, int64_t ldw, int64_t strideW, void* GU,
                             int64_t ldgu, void* H, int64_t ldh, const int* offs, const int* tile_end, int T, int G,
                             int I, int K, hipStream_t st) {
  if (T <= 0 || G <= 0 || I <= 0 || K <= 0 || K % BK || I % 128) return -2;
  if (ldx % 8 || ldw % 8 || ldgu % 8 || ldh % 8 || strideW % 8 || ldx < K || ldw < K || ldgu < 2 * I || ldh < I)
    return -2;
  if (((uintptr_t)X | (uintptr_t)W | (uintptr_t)GU | (uintptr_t)H) % 16) return -2;
  if (((int64_t)(BM + 32) * ldx) * 2 >= (int64_t)1 << 32) return -2;
  if (((int64_t)2 * I * ldw) * 2 >= (int64_t)1 << 32) return -2;
  const int N = 2 * I;
  const int64_t grid = st_gemm4w_slots(T, G) * (N / BN);
  if (grid >= (1LL << 31)) return -2;
  const char* oe = std::getenv("ST_GEMM4W_ORDER");
  const int gm = oe ? std::atoi(oe) : 0;
  const int pv = persist_on() ? (int)grid : 0;
  const int64_t lg = pv ? std::min<int64_t>(grid, cu_count()) : grid;
  gemm4e_kernel<1, 0, 5><<<(unsigned)lg, NT, 0, st>>>((const bf16_t*)X, ldx, (const bf16_t*)W, ldw, strideW,
                                                      (bf16_t*)GU, ldgu, offs, tile_end, G, N, K, gm, (bf16_t*)H, ldh,
                                                      I, T, pv);
  return (int)hipGetLastError();
}

// gu [T, 2I] = X @ W^T and h [T, I] = silu(gate) * up in ONE launch (dense, W [2I, K] = gate
// rows then up rows).  0 on success, -2 unsupported shape.
int st_gemm4w_swiglu(const void* X, int64_t ldx, const void* W, int64_t ldw, void* GU, int64_t ldgu, void* H,
                     int64_t ldh, int T, int I, int K, hipStream_t st) {
  if (T <= 0 || I <= 0 || K <= 0 || K % BK || I % 128) return -2;
  if (ldx % 8 || ldw % 8 || ldgu % 8 || ldh % 8 || ldx < K || ldw < K || ldgu < 2 * I || ldh < I) return -2;
  if (((uintptr_t)X | (uintptr_t)W | (uintptr_t)GU | (uintptr_t)H) % 16) return -2;
  if (((int64_t)(BM + 32) * ldx) * 2 >= (int64_t)1 << 32) return -2;
  if (((int64_t)2 * I * ldw) * 2 >= (int64_t)1 << 32) return -2;
  const int N = 2 * I;
  const int64_t grid = (int64_t)((T + BM - 1) / BM) * (N / BN);
  if (grid >= (1LL << 31)) return -2;
  const char* oe = std::getenv("ST_GEMM4W_ORDER");
  const int gm = oe ? std::atoi(oe) : 4;
  // e (default): kind 5 (1.39-1.42 PF/s at gate|up), f: the stream-persistent kind 6 (1.08-1.16;
  // profiles/r05/gemm4w/kind5_persistent_vs_kind6_stream.log)
  const char* ke = std::getenv("ST_GEMM4W_SWIGLU_KERNEL");
  if (K / BK >= 2 && ke && ke[0] == 'f') {
    const int64_t lg = std::min<int64_t>(grid, cu_count());
    gemm4f_kernel<1><<<(unsigned)lg, NT, 0, st>>>((const bf16_t*)X, ldx, (const bf16_t*)W, ldw, 0, (bf16_t*)GU, ldgu,
                                                  nullptr, nullptr, 1, N, K, gm, (bf16_t*)H, ldh, I, T, (int)grid);
    return (int)hipGetLastError();
  }
  const int pv = persist_on() ? (int)grid : 0;
  const int64_t lg = pv ? std::min<int64_t>(grid, cu_count()) : grid;
  gemm4e_kernel<1, 0, 5><<<(unsigned)lg, NT, 0, st>>>((const bf16_t*)X, ldx, (const bf16_t*)W, ldw, 0, (bf16_t*)GU,
                                                      ldgu, nullptr, nullptr, 1, N, K, gm, (bf16_t*)H, ldh, I, T, pv);
  return (int)hipGetLastError();
}

}  // extern "C"

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
// STATUS: on the model path for the MoE long-K expert GEMMs (forward gate|up + SwiGLU epilogue,
// down; models/moe.py), where it beats the grouped kernel by 8-12 %.  On the dense gate|up /
// down / qkv shapes it runs 1.39-1.46 PF/s against hipBLASLt's MT256x256x64 kernel (the same
// 4-wave 128 x 128-per-wave structure) at 1.55-1.57, so the dense GEMMs stay on hipBLASLt.  PMC (profiles/r05/gemm4w/pmc.md): 0 LDS
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

// work item of a persistent workgroup's virtual tile id vb of nv.  gm == 0: slot-major (N-tile
// fastest).  gm > 0: XCD-aware -- each XCD walks its own contiguous range of ids, in groups of gm
// slots x (N-tiles) with the slot fastest, so the ~32 workgroups an XCD runs at once start
// together on gm X tiles and 32 / gm weight tiles and stream the same 64-k slices through its L2
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


#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved: nothing else in this kernel uses it
// one 1-KiB LDS-DMA piece (lane L's 16 bytes land at lds_base + 16 L), the K-tile advance in the
// instruction's scalar offset: the lane offsets stay
// loop-invariant VGPRs, no VALU address arithmetic ahead of a piece
ST_DEVICE void dma16s(rsrc_t rs, uint32_t lds_base, uint32_t voff, uint32_t soff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :
               : "s"(lds_base), "v"(voff), "s"(rs), "s"(soff)
               : "memory", "m0");
}
#pragma clang diagnostic pop


// ---- the kernel: 2 x 2 waves of 128 x 128, both operands by LDS-DMA, whole-tile fragments.
// The K-tile's fragments of BOTH 32-k sub-steps live in registers (fa / fb [ks][8]: 128 VGPRs),
// so a stage of LDS is released in parts as soon as its fragments are read:
//   MFMAs 0-31 read tile kt's sub-step-1 fragments (one per 2 MFMAs); at MFMA 20 a barrier
//   (lgkmcnt(3)) releases the stage's X region, which takes tile kt+2's 8 X pieces over MFMAs
//   21-56; at MFMA 63 one barrier (vmcnt(8): all but this step's X pieces) releases the W region
//   and publishes tile kt+1; tile kt+2's 8 W pieces go out over MFMAs 64-120 and tile kt+1's
//   sub-step-0 fragments are read over MFMAs 64-94.  M0 of each piece is written two MFMAs
//   ahead of its DMA.  (Variants with one barrier per tile, register staging, 1 x 4 waves or a
//   stream-persistent K-tile walk lost their A/Bs and were removed; logs: profiles/r05/gemm4w/.)
// PROBE (diagnostic library only, -DST_PROBES; wrong results): 1 = no fragment reads,
// 2 = no DMA, 3 = no barriers, 4 = MFMAs only, 7 = shader-cycle stamps per segment.
template <int EPI, int PROBE = 0>
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

  // slot tables: the MFMA index after which each operation issues (see the header)
  constexpr int BAR = 63, BARA = 20;
  constexpr auto rd1_slot = [](int m) constexpr -> int {  // read index of tile kt's sub-step 1 after MFMA m
    return m < 32 && (m & 1) == 0 ? m >> 1 : -1;
  };
  constexpr auto rd0_slot = [](int m) constexpr -> int {  // read index of tile kt+1's sub-step 0
    return m >= 64 && m < 96 && (m & 1) == 0 ? (m - 64) >> 1 : -1;
  };
  constexpr auto dma_slot = [](int m) constexpr -> int {
    if (m >= 21 && m <= 56 && (m - 21) % 5 == 0) return (m - 21) / 5;          // X pieces
    if (m >= 64 && m <= 120 && ((m - 64) & 7) == 0) return 8 + ((m - 64) >> 3);  // W pieces
    return -1;
  };
  auto piece_m0 = [&](int buf, int p) {
    return lbase + buf * STAGE + (p < 8 ? p * 1024 : IMG + (p - 8) * 1024);
  };
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved: nothing else in this kernel uses it
  auto set_m0 = [&](uint32_t v) { asm volatile("s_mov_b32 m0, %0" : : "s"(v) : "m0"); };
#pragma clang diagnostic pop
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
      if constexpr (m == BARA && more2) {  // X region of cur: every wave's reads done
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
          if constexpr (more2) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
        if constexpr (more2) stamp(2);
        fence();
      }
      if constexpr (m == 100 && more2) stamp(3);
      if constexpr (more2 && pn >= 0 && PROBE != 2 && PROBE != 4) {
        fence();
        set_m0(piece_m0(kt & 1, pn));
        fence();
      }
      if constexpr (more2 && pd >= 0) {
        fence();
        dma_nom0(kt + 2, pd);
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

// one launch of #CU persistent workgroups (ST_GEMM4W_PERSIST=0: one tile per workgroup, A/B)
static bool persist_on() {
  const char* e = std::getenv("ST_GEMM4W_PERSIST");
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
  const char* oe = std::getenv("ST_GEMM4W_ORDER");  // slots per XCD group (0: slot-major)
  const int gm = oe ? std::atoi(oe) : 0;
  const int pv = persist_on() ? (int)grid : 0;
  const int64_t lg = pv ? std::min<int64_t>(grid, cu_count()) : grid;
#define G4ARGS (const bf16_t*)X, ldx, (const bf16_t*)W, ldw, strideW, (bf16_t*)Y, ldy, offs, tile_end, G, N, K, gm, \
               (bf16_t*)nullptr, (int64_t)0, 0, 0, pv
#ifdef ST_PROBES
  // timing probes of the diagnostic library (wrong results): ST_GEMM4W_PROBE=1..4, 7
  const char* pe = std::getenv("ST_GEMM4W_PROBE");
  switch (pe ? std::atoi(pe) : 0) {
    case 1: gemm4e_kernel<0, 1><<<(unsigned)lg, NT, 0, st>>>(G4ARGS); return (int)hipGetLastError();
    case 2: gemm4e_kernel<0, 2><<<(unsigned)lg, NT, 0, st>>>(G4ARGS); return (int)hipGetLastError();
    case 3: gemm4e_kernel<0, 3><<<(unsigned)lg, NT, 0, st>>>(G4ARGS); return (int)hipGetLastError();
    case 4: gemm4e_kernel<0, 4><<<(unsigned)lg, NT, 0, st>>>(G4ARGS); return (int)hipGetLastError();
    case 7: gemm4e_kernel<0, 7><<<(unsigned)lg, NT, 0, st>>>(G4ARGS); return (int)hipGetLastError();
    default: break;
  }
#endif
  gemm4e_kernel<0><<<(unsigned)lg, NT, 0, st>>>(G4ARGS);
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
  gemm4e_kernel<1><<<(unsigned)lg, NT, 0, st>>>((const bf16_t*)X, ldx, (const bf16_t*)W, ldw, strideW,
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
  const int pv = persist_on() ? (int)grid : 0;
  const int64_t lg = pv ? std::min<int64_t>(grid, cu_count()) : grid;
  gemm4e_kernel<1><<<(unsigned)lg, NT, 0, st>>>((const bf16_t*)X, ldx, (const bf16_t*)W, ldw, 0, (bf16_t*)GU,
                                                      ldgu, nullptr, nullptr, 1, N, K, gm, (bf16_t*)H, ldh, I, T, pv);
  return (int)hipGetLastError();
}

}  // extern "C"

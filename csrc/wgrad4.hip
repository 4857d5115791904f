// Weight-gradient GEMM, one wave per SIMD: C[M,N] (fp32) = beta * C + sum_t A[t,m] * B[t,n]
// (dW = dY^T X with both bf16 operands TOKEN-major, the reduction index the strided one).
// Reference call site: the wgrad of LinearWithAsyncAllReduce,
// scaletorch/parallel/tensor_parallel/tp_comms.py:288-311, and autograd's F.linear backward.
//
// The schedule of csrc/gemm4w.hip's kind-5 kernel (docs/PERF.md round 5) on csrc/wgrad_gemm.hip's
// operand handling:
//   * 256 x 256 output tile, 4 waves of 128 x 128 (16x16x32 MFMAs, 256 AGPR accumulators) --
//     half the LDS bytes per MFMA of the 8-wave wgrad8 kernel;
//   * K-tiles of 64 tokens staged by LDS-DMA exactly as stored (rows = tokens, 256-B rows of
//     128 features, XOR-swizzled on the source address) and read with ds_read_b64_tr_b16, which
//     puts the token index down a lane's fragment (two reads per 16 x 32 fragment);
//   * both 32-token sub-steps' fragments of a K-tile held in registers: the A images of a stage
//     are released after their sub-step-1 reads (barrier at MFMA 20), the B images with the
//     publication of the next K-tile (barrier at MFMA 63, vmcnt(8)); the next-but-one K-tile's
//     16 pieces per wave spread over MFMAs 21-120, M0 written two MFMAs ahead of each;
//   * operands swapped in the MFMA so a lane holds 4 consecutive output columns: the fp32
//     epilogue (beta: read-add-write) moves 16 B per lane;
//   * persistent: one workgroup per CU walks the tiles (XCD-grouped order optional).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"

using namespace st;

namespace {

typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
typedef __bf16 bfx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_t;
typedef uint32_t srd_t __attribute__((ext_vector_type(4)));  // buffer descriptor words (SGPR quad)

constexpr int BT = 256, BK = 64, NT = 256;  // output tile BT x BT, K-tile of 64 tokens
constexpr int RB = 256;                     // bytes per image row: 128 bf16 features
constexpr int IMGW = BK * RB;               // one [64 tokens][128 features] image: 16 KiB
constexpr int STAGE = 4 * IMGW;             // A0 A1 B0 B1

// 256-B rows, 16-B chunks: the transposed reads and the DMA fill are bank-conflict free
ST_DEVICE int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
ST_DEVICE int lds_off(int row, int ch) { return row * RB + 16 * (ch ^ swz(row)); }

ST_DEVICE bfx8 lds_tr(const lds_t* p0, const lds_t* p1) {
  bfx4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bfx4 __attribute__((address_space(3)))*)p0);
  bfx4 b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((bfx4 __attribute__((address_space(3)))*)p1);
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// Buffer descriptor as four explicitly wave-uniform words (what __builtin_amdgcn_make_buffer_rsrc
// emits: base lo, base hi[15:0] with stride 0, num_records, flags 0x20000).  The DMA asm takes
// them through an "s" constraint, so every word is a readfirstlane result: uniform to the compiler
// at any optimisation level, not only where -O3's uniformity analysis proves it.
ST_DEVICE srd_t make_srd(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  srd_t w;
  w[0] = __builtin_amdgcn_readfirstlane((uint32_t)a);
  w[1] = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) & 0xffffu;
  w[2] = __builtin_amdgcn_readfirstlane(bytes);
  w[3] = 0x00020000u;
  return w;
}

ST_DEVICE void fence() { __builtin_amdgcn_sched_barrier(0); }

template <int B, int E, typename F>
ST_DEVICE void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>());
    static_for<B + 1, E>(f);
  }
}

// virtual tile vb of nv -> (row block bm, column block bn); gm > 0: XCD-aware groups of gm
// row blocks (the ~32 tiles an XCD runs at once share their token slices in its L2)
ST_DEVICE void tile_of(int gm, int nbm, int nbn, int vb, int nv, int& bm, int& bn) {
  if (gm <= 0) {
    bm = vb / nbn;
    bn = vb % nbn;
    return;
  }
  const int id = xcd_remap(vb, nv);
  const int per = gm * nbn, grp = id / per, in = id % per;
  const int gsz = min(gm, nbm - grp * gm);
  bm = grp * gm + in % gsz;
  bn = in / gsz;
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved: nothing else in this kernel uses it
// PROBE 7 (diagnostic build, ST_WGRAD4_PROBE=7): shader-cycle stamps per segment of every
// steady-state K-tile step, summed per wave and written over C (tools/_w4stamps.py reads them)
// KDESC: the K-tile offset lives in per-K-tile descriptors (ragged token counts, grouped
// experts); else in soffset over one descriptor per unit (T a multiple of 64, fewer scalar ops)
// (A variant reading the fragment halves one transposed read at a time lost its A/B and was
// removed; profiles/r05/wgrad4/.)  PROBE != 0 exists only in the diagnostic library (-DST_PROBES).
template <int PROBE = 0, bool KDESC = true>
__global__ __launch_bounds__(NT, 1) void wgrad4_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                       const bf16_t* __restrict__ B, int64_t ldb,
                                                       float* __restrict__ C, int64_t ldc, int M, int N, int T,
                                                       int beta, int gm, int nfull, int splits,
                                                       float* __restrict__ ws, const int* __restrict__ offs,
                                                       int64_t strideC) {
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * STAGE];
  lds_t* smem = (lds_t*)smem_raw;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  // offs != null: grouped (MoE experts) -- unit u is (expert u / tiles, tile u % tiles), expert g's
  // tokens are rows [offs[g-1], offs[g]) of A / B and its output C + g strideC
  const int nbm = M / BT, nbn = N / BT, tiles = nbm * nbn;
  const int nv = offs ? 0 : tiles;
  const uint32_t sa = (uint32_t)(lda * 2), sb = (uint32_t)(ldb * 2);

  // DMA: wave w fills rows 16 w .. 16 w + 15 of every image, 4 pieces (4 rows, 1 KiB) each;
  // piece p < 8 is an A image's (A0, A1), p >= 8 a B image's
  uint32_t voff[16];
#pragma unroll
  for (int p = 0; p < 16; ++p) {
    const int img = p >> 2, i = p & 3;
    const int row = 16 * wid + 4 * i + (lane >> 4), pos = lane & 15;
    const uint32_t col = (uint32_t)((img & 1) * 256 + 16 * (pos ^ swz(row)));
    voff[p] = (uint32_t)row * (img < 2 ? sa : sb) + col;
  }
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem + (uint32_t)(wid * 4 * 1024));
  auto piece_m0 = [&](int buf, int p) { return lbase + buf * STAGE + (p >> 2) * IMGW + (p & 3) * 1024; };
  auto set_m0 = [&](uint32_t v) {
    asm volatile("s_mov_b32 m0, %0" : : "s"(__builtin_amdgcn_readfirstlane(v)) : "m0");
  };
  // descriptors over K-tile kt onward of an operand slice: base advanced by kt * 64 rows, range
  // = the rows left, so a ragged last K-tile reads zeros past the token count (the range check
  // covers the VGPR offset only -- the K offset lives in the base, not in soffset)
  struct Krs {
    srd_t a, b;
    uint32_t soa, sob;
  };
  srd_t unit_a = make_srd(A, 0u), unit_b = make_srd(B, 0u);  // !KDESC: the unit's whole-operand descriptors
  auto krs = [&](const bf16_t* abase, const bf16_t* bbase, int rows, int kt) {
    if constexpr (KDESC) {
      const int left = rows - kt * BK;
      const uint32_t ba = left > 0 ? (uint32_t)(((int64_t)(left - 1) * lda + BT) * 2) : 0u;
      const uint32_t bb = left > 0 ? (uint32_t)(((int64_t)(left - 1) * ldb + BT) * 2) : 0u;
      return Krs{make_srd(abase + (int64_t)kt * BK * lda, ba), make_srd(bbase + (int64_t)kt * BK * ldb, bb), 0u,
                 0u};
    } else {
      return Krs{unit_a, unit_b, (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)kt * (uint32_t)BK * sa),
                 (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)kt * (uint32_t)BK * sb)};
    }
  };
  auto dma_nom0 = [&](const Krs& k, int p) {
    if (p < 8)
      asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds"
                   : : "v"(voff[p]), "s"(k.a), "s"(__builtin_amdgcn_readfirstlane(k.soa)) : "memory");
    else
      asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds"
                   : : "v"(voff[p]), "s"(k.b), "s"(__builtin_amdgcn_readfirstlane(k.sob)) : "memory");
  };

  // fragment reads (16 features x 32 tokens, natural k order permuted the same way for both
  // operands): lane group G = lane >> 4 reads token rows 8 G + 4 hf + q of 16 feature columns,
  // lane 4 q + p addressing columns 4 p .. 4 p + 3 (csrc/wgrad_gemm.hip's plan)
  const int G = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  int aoff[8][2], boff[8][2];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf)
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      const int o = lds_off(8 * G + 4 * hf + q, 2 * f + (pp >> 1)) + 8 * (pp & 1);
      aoff[f][hf] = wm * IMGW + o;
      boff[f][hf] = (2 + wn) * IMGW + o;
    }
  bfx8 fa[2][8], fb[2][8];
  // read r < 8: A fragment r, else B fragment r - 8, of sub-step ks
  auto read = [&](const lds_t* st, int ks, int r) {
    if (r < 8) fa[ks][r] = lds_tr(st + aoff[r][0] + ks * 32 * RB, st + aoff[r][1] + ks * 32 * RB);
    else fb[ks][r - 8] = lds_tr(st + boff[r - 8][0] + ks * 32 * RB, st + boff[r - 8][1] + ks * 32 * RB);
  };
  // operands swapped: acc[i][j] reg r = C[row 16 i + (lane & 15)][col 16 j + 4 G + r]
  auto mfma = [&](f32x4 (&acc)[8][8], int ks, int idx) {
    const int i = idx >> 3, j = idx & 7;
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(fb[ks][j]), "v"(fa[ks][i]));
  };
  // slots: sub-step-1 fragments (2 tr reads each) at even MFMAs 0-30, A images released at 20
  // (lgkmcnt(6): B fragments 8-10 may still be in flight), next-but-one K-tile's A pieces at
  // 21-56, publication at 63, B pieces at 64-120, the next K-tile's sub-step-0 reads at 64-94
  constexpr auto dslot = [](int m) constexpr -> int {
    if (m >= 21 && m <= 56 && (m - 21) % 5 == 0) return (m - 21) / 5;
    if (m >= 64 && m <= 120 && ((m - 64) & 7) == 0) return 8 + ((m - 64) >> 3);
    return -1;
  };
  uint64_t seg[5] = {0, 0, 0, 0, 0}, nst = 0;
  uint64_t ts[6];
  auto stamp = [&](int k) {
    if constexpr (PROBE == 7) {
      fence();
      ts[k] = __builtin_amdgcn_s_memtime();
      fence();
    }
  };
  auto step = [&](f32x4 (&acc)[8][8], auto more_c, auto more2_c, int kt, const bf16_t* abase, const bf16_t* bbase,
                  int rows) {
    constexpr bool more = decltype(more_c)::value, more2 = decltype(more2_c)::value;
    Krs k2{};
    if constexpr (decltype(more2_c)::value) k2 = krs(abase, bbase, rows, kt + 2);
    const lds_t* cs = smem + (kt & 1) * STAGE;
    const lds_t* ns = smem + ((kt + 1) & 1) * STAGE;
    __builtin_amdgcn_s_setprio(1);
    if constexpr (more2) stamp(0);
    static_for<0, 128>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      mfma(acc, m >> 6, m & 63);
      constexpr int pd = dslot(m), pn = dslot(m + 2);
      if constexpr (m < 32 && (m & 1) == 0 && PROBE != 2) {  // fragment r = m / 2 (A 0-7, then B)
        fence();
        read(cs, 1, m >> 1);
        fence();
      }
      if constexpr (m == 20 && more2 && PROBE != 3) {
        stamp(1);
        fence();
        asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");  // B fragments 8-10 may be in flight
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        fence();
        stamp(2);
      }
      if constexpr (m == 63 && more) {
        if constexpr (more2) stamp(3);
        fence();
        __builtin_amdgcn_s_setprio(0);
        if constexpr (more2) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        if constexpr (PROBE != 3) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
        fence();
        if constexpr (more2) stamp(4);
      }
      if constexpr (more2 && pn >= 0) {
        fence();
        set_m0(piece_m0(kt & 1, pn));
        fence();
      }
      if constexpr (more2 && pd >= 0 && PROBE != 1) {
        fence();
        dma_nom0(k2, pd);
        fence();
      }
      if constexpr (more && m >= 64 && m < 96 && (m & 1) == 0 && PROBE != 2) {
        fence();
        read(ns, 0, (m - 64) >> 1);
        fence();
      }
    });
    if constexpr (more2 && PROBE == 7) {
      stamp(5);
      for (int k = 0; k < 5; ++k) seg[k] += ts[k + 1] - ts[k];
      ++nst;
    }
    __builtin_amdgcn_s_setprio(0);
  };

  // work units: tiles 0 .. nfull - 1 whole, then the tail tiles as `splits` K ranges each
  // (split-major); range 0 lands in C, range s > 0 in workspace tile (s - 1, tl), added in order
  // by wgrad4_tail_reduce
  const int nu = offs ? nfull : nfull + (nv - nfull) * splits, tail = nv - nfull;
  for (int u = (int)blockIdx.x; u < nu; u += (int)gridDim.x) {
    if (u != (int)blockIdx.x) __syncthreads();  // every wave past the previous tile's LDS reads
    const bf16_t* Ag = A;
    const bf16_t* Bg = B;
    float* Cg = C;
    int Tg = T, vb = u;
    if (offs) {
      const int g = u / tiles, k0 = g ? offs[g - 1] : 0;
      vb = u % tiles;
      Tg = offs[g] - k0;
      Ag += (int64_t)k0 * lda;
      Bg += (int64_t)k0 * ldb;
      Cg += (int64_t)g * strideC;
      if (Tg <= 0) {  // no tokens: C_g unchanged, or zeros for beta 0
        if (!beta) {
          int bm, bn;
          tile_of(gm, nbm, nbn, vb, tiles, bm, bn);
          float* cz = Cg + (int64_t)(bm * BT) * ldc + bn * BT;
          for (int e = threadIdx.x * 4; e < BT * BT; e += NT * 4)
            *reinterpret_cast<f32x4*>(cz + (int64_t)(e / BT) * ldc + e % BT) = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        continue;
      }
    }
    const int KT = (Tg + BK - 1) / BK;
    int kb = 0, ke = KT, sidx = 0, tl = 0;
    if (u >= nfull) {
      const int t = u - nfull;
      sidx = t / tail;
      tl = t % tail;
      vb = nfull + tl;
      kb = sidx * KT / splits;
      ke = (sidx + 1) * KT / splits;
    }
    int bm, bn;
    tile_of(gm, nbm, nbn, vb, tiles, bm, bn);
    const int m0 = bm * BT, n0 = bn * BT;
    const bf16_t* abase = Ag + m0;
    const bf16_t* bbase = Bg + n0;
    if constexpr (!KDESC) {
      unit_a = make_srd(abase, (uint32_t)(((int64_t)(Tg - 1) * lda + BT) * 2));
      unit_b = make_srd(bbase, (uint32_t)(((int64_t)(Tg - 1) * ldb + BT) * 2));
    }
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // prologue: K-tiles kb and kb + 1 requested, kb published, its sub-step-0 fragments read
    const Krs k0 = krs(abase, bbase, Tg, kb);
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      set_m0(piece_m0(kb & 1, p));
      dma_nom0(k0, p);
    }
    if (ke - kb > 1) {
      const Krs k1 = krs(abase, bbase, Tg, kb + 1);
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        set_m0(piece_m0((kb + 1) & 1, p));
        dma_nom0(k1, p);
      }
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) read(smem + (kb & 1) * STAGE, 0, r);
    using T1 = std::true_type;
    using F0 = std::false_type;
    int kt = kb;
    for (; kt + 2 < ke; ++kt) step(acc, T1(), T1(), kt, abase, bbase, Tg);
    if (kt + 1 < ke) step(acc, T1(), F0(), kt++, abase, bbase, Tg);
    step(acc, F0(), F0(), kt, abase, bbase, Tg);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 15\n\ts_nop 3" ::: "memory");
    if constexpr (PROBE == 7) continue;  // the stamps go over C below: no tile stores
    // epilogue: lane (row 16 i + (lane & 15), cols 16 j + 4 G .. +3) -- 16-B fp32 accesses
    float* cb = sidx ? ws + ((int64_t)(sidx - 1) * tail + tl) * (BT * BT) : Cg + (int64_t)m0 * ldc + n0;
    const int64_t ld = sidx ? BT : ldc;
    const bool acc_c = beta && !sidx;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float* cr = cb + (int64_t)(wm * 128 + 16 * i + (lane & 15)) * ld + wn * 128 + 4 * G;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        f32x4* p = reinterpret_cast<f32x4*>(cr + 16 * j);
        f32x4 v = acc[i][j];
        if (acc_c) v += *p;
        *p = v;
      }
    }
  }
  if constexpr (PROBE == 7) {  // lane 0 of each wave: 5 x u64 segment sums + step count, row 4 b + w
    __syncthreads();
    if (lane == 0) {
      uint64_t* d = reinterpret_cast<uint64_t*>(C + (int64_t)(blockIdx.x * 4 + wid) * ldc);
      for (int k = 0; k < 5; ++k) d[k] = seg[k];
      d[5] = nst;
    }
  }
}

// C tile (row-major tail tile tl) += workspace partials 1 .. splits - 1, in order (bitwise
// repeatable); 4 elements per lane
__global__ __launch_bounds__(256) void wgrad4_tail_reduce(float* __restrict__ C, int64_t ldc,
                                                          const float* __restrict__ ws, int nbn, int nfull,
                                                          int tail, int splits) {
  const int tl = blockIdx.y, vb = nfull + tl;
  const int e = (blockIdx.x * 256 + threadIdx.x) * 4;
  const int r = e / BT, c = e % BT;
  f32x4* pc = reinterpret_cast<f32x4*>(C + (int64_t)((vb / nbn) * BT + r) * ldc + (vb % nbn) * BT + c);
  f32x4 acc = *pc;
  for (int s = 1; s < splits; ++s)
    acc += *reinterpret_cast<const f32x4*>(ws + ((int64_t)(s - 1) * tail + tl) * (BT * BT) + e);
  *pc = acc;
}
#pragma clang diagnostic pop

int cu_count() {
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

int wgrad4_order() {
  const char* oe = std::getenv("ST_WGRAD4_ORDER");  // row blocks per XCD group (0: row-major)
  return oe ? std::atoi(oe) : 0;
}

// The last, partial round of tiles (fewer than one per CU) is split along K so it fills the
// chip: splits * tail <= CUs, each range >= 4 K-tiles; row-major tile order only (the tail tiles
// are then the trailing ones).  ST_WGRAD4_SPLIT caps the ranges per tile (1: off).
struct Split {
  int nfull, tail, splits;
};
Split wgrad4_split(int M, int N, int T, int gm) {
  const int64_t nv = (int64_t)(M / BT) * (N / BT);
  const int cus = cu_count(), KT = (T + BK - 1) / BK;
  const char* se = std::getenv("ST_WGRAD4_SPLIT");
  const int smax = se ? std::atoi(se) : 4;
  const int tail = (int)(nv % cus);
  int splits = 1;
  if (gm <= 0 && tail > 0)
    while (splits < smax && (splits + 1) * tail <= cus && KT / (splits + 1) >= 4) ++splits;
  return Split{(int)(nv - tail), tail, splits};
}

}  // namespace

extern "C" {

// fp32 workspace elements a launch of this shape needs (0: no tail split).
int64_t st_wgrad4_ws_elems(int M, int N, int T) {
  if (M <= 0 || N <= 0 || T <= 0 || M % BT || N % BT) return 0;
  const Split sp = wgrad4_split(M, N, T, wgrad4_order());
  return sp.splits > 1 ? (int64_t)(sp.splits - 1) * sp.tail * BT * BT : 0;
}

// C[M,N] fp32 (+)= A[T,M]^T B[T,N] (bf16, token-major) on the one-wave-per-SIMD kernel.
// ws: st_wgrad4_ws_elems(M, N, T) fp32 elements (null when that is 0).
// 0 on success, -2: shape not supported (caller falls back).
int st_wgrad4(const void* A, int64_t lda, const void* B, int64_t ldb, float* C, int64_t ldc, int M, int N, int T,
              int beta, float* ws, hipStream_t st) {
  // any T: the K-tile offset is range checked, a ragged last K-tile reads zeros past row T
  if (M <= 0 || N <= 0 || T <= 0 || M % BT || N % BT) return -2;
  if (lda % 8 || ldb % 8 || ldc % 4 || lda < M || ldb < N || ldc < N) return -2;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16) return -2;
  // 32-bit buffer offsets: every row a K-tile addresses (up to T + 63) below 2^32 bytes
  if (((int64_t)(T + BK) * lda + M) * 2 >= (int64_t)1 << 32) return -2;
  if (((int64_t)(T + BK) * ldb + N) * 2 >= (int64_t)1 << 32) return -2;
  const int64_t nv = (int64_t)(M / BT) * (N / BT);
  if (nv >= (1LL << 31)) return -2;
  const int gm = wgrad4_order();
  Split sp = wgrad4_split(M, N, T, gm);
  if (ws == nullptr) sp.splits = 1;
  const int nbn = N / BT;
  const int nfull = sp.splits > 1 ? sp.nfull : (int)nv;
  const int64_t nu = nfull + (int64_t)(nv - nfull) * sp.splits;
  const int64_t grid = std::min<int64_t>(nu, cu_count());
  // whole K-tiles: K offsets in soffset (ST_WGRAD4_KDESC=1 forces the per-K-tile descriptors)
  const char* ke = std::getenv("ST_WGRAD4_KDESC");
  const bool kdesc = T % BK != 0 || (ke && std::atoi(ke) == 1);
#define W4ARGS (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, ldc, M, N, T, beta ? 1 : 0, gm, nfull, sp.splits, ws, \
               nullptr, (int64_t)0
#ifdef ST_PROBES
  // diagnostic library only (wrong results): 7 = cycle stamps over C; 1 / 2 / 3 = no K-loop DMA /
  // no fragment reads / no barriers
  const char* pe = std::getenv("ST_WGRAD4_PROBE");
  const int pv = pe ? std::atoi(pe) : 0;
  if (pv) {
    if (pv == 1 && !kdesc) wgrad4_kernel<1, false><<<(unsigned)grid, NT, 0, st>>>(W4ARGS);
    else if (pv == 2 && !kdesc) wgrad4_kernel<2, false><<<(unsigned)grid, NT, 0, st>>>(W4ARGS);
    else if (pv == 3 && !kdesc) wgrad4_kernel<3, false><<<(unsigned)grid, NT, 0, st>>>(W4ARGS);
    else if (pv == 7 && grid * 4 <= M && ldc >= 12 && kdesc) wgrad4_kernel<7, true><<<(unsigned)grid, NT, 0, st>>>(W4ARGS);
    else if (pv == 7 && grid * 4 <= M && ldc >= 12) wgrad4_kernel<7, false><<<(unsigned)grid, NT, 0, st>>>(W4ARGS);
    else return -2;
    return (int)hipGetLastError();
  }
#endif
  if (kdesc) wgrad4_kernel<0, true><<<(unsigned)grid, NT, 0, st>>>(W4ARGS);
  else wgrad4_kernel<0, false><<<(unsigned)grid, NT, 0, st>>>(W4ARGS);
#undef W4ARGS
  if (sp.splits > 1) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    wgrad4_tail_reduce<<<dim3(BT * BT / 1024, (unsigned)sp.tail), 256, 0, st>>>(C, ldc, ws, nbn, sp.nfull, sp.tail,
                                                                               sp.splits);
  }
  return (int)hipGetLastError();
}

// Grouped weight gradient on the same kernel (MoE experts): C[g] = beta C[g] + A[rows of g]^T
// B[rows of g], rows of g = [offs[g-1], offs[g]) (int32 device prefix sums, never read by the
// host), C[g] at C + g strideC.  Units expert-major, so the ~256 tiles in flight belong to one
// or two experts (csrc/wgrad_gemm.hip st_wgrad_grouped's order).  T_total bounds every
// expert's rows.  -2: shape not supported.
int st_wgrad4_grouped(const void* A, int64_t lda, const void* B, int64_t ldb, float* C, int64_t ldc,
                      int64_t strideC, int M, int N, int G, const int* offs, int T_total, int beta, hipStream_t st) {
  if (M <= 0 || N <= 0 || G <= 0 || T_total < 0 || M % BT || N % BT) return -2;
  if (lda % 8 || ldb % 8 || ldc % 4 || strideC % 4 || lda < M || ldb < N || ldc < N) return -2;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16) return -2;
  if (((int64_t)(T_total + BK) * lda + M) * 2 >= (int64_t)1 << 32) return -2;
  if (((int64_t)(T_total + BK) * ldb + N) * 2 >= (int64_t)1 << 32) return -2;
  const int64_t nu = (int64_t)G * (M / BT) * (N / BT);
  if (nu >= (1LL << 31)) return -2;
  // ST_WGRAD4_GROUPED_PERSIST=0: one unit per workgroup (A/B against the persistent grid)
  const char* pe = std::getenv("ST_WGRAD4_GROUPED_PERSIST");
  const bool persist = !pe || std::atoi(pe) != 0;
  const int64_t grid = persist ? std::min<int64_t>(nu, cu_count()) : nu;
  wgrad4_kernel<<<(unsigned)grid, NT, 0, st>>>((const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, ldc, M, N, 0,
                                               beta ? 1 : 0, wgrad4_order(), (int)nu, 1, nullptr, offs, strideC);
  return (int)hipGetLastError();
}

}  // extern "C"

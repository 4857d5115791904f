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
//   * one LDS image per K/V (or Q/dO) tile, XOR-swizzled so both the 16-byte
//     row reads and the transposed reads are bank-conflict free (T10 (b)).
//   * register-staged double buffering (T14): the next tile's global loads are
//     issued before the MFMAs of the current tile and written to the other LDS
//     buffer after them -- one barrier per tile.
//   * online softmax in base 2 with the scale folded into one multiply.
//   * backward = 3 kernels: delta = rowsum(dO*O); dQ (per 128-query tile,
//     iterating keys); dK/dV (per 128-key tile x query head, iterating
//     queries) -- no atomics anywhere, bitwise deterministic; GQA groups are
//     summed by a final bandwidth-bound pass.
//   * causal: workgroups are launched heaviest-first and skip blocks that are
//     entirely masked; only diagonal blocks evaluate the mask.
#include "common.h"

using namespace st;

namespace {

typedef __bf16 bfx8 __attribute__((ext_vector_type(8)));
typedef __bf16 bfx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) char lds_t;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// ---- LDS tile geometry: rows of D bf16, 16-byte chunks, XOR swizzle ----
template <int D>
ST_DEVICE int lds_off(int row, int ch) {
  if constexpr (D == 128) {
    return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
  } else {
    return row * 128 + 16 * (ch ^ ((row >> 1) & 7));
  }
}

// 8 contiguous bf16 of row `row`, chunk `ch` (MFMA A or B fragment, natural k order).
template <int D>
ST_DEVICE bfx8 row_frag(const lds_t* tile, int row, int ch) {
  return *reinterpret_cast<const bfx8 __attribute__((address_space(3)))*>(tile + lds_off<D>(row, ch));
}

// Transposed fragment: element j of lane (r = lane&31, h = lane>>5) is
//   tile[rbase + 16 s + 8 (j>>2) + 4 h + (j&3)][32 dt + r]
// i.e. the operand whose k index runs over tile ROWS, permuted to match an
// accumulator fed back as the other operand.
template <int D>
ST_DEVICE bfx8 tr_frag(const lds_t* tile, int rbase, int s, int dt, int lane) {
  const int h = lane >> 5, g = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
  const int col = 32 * dt + 16 * g + 4 * p;
  const int row0 = rbase + 16 * s + 4 * h + q;
  const int ch = col >> 3, sub = (col & 7) * 2;
  bfx4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (bfx4 __attribute__((address_space(3)))*)(tile + lds_off<D>(row0, ch) + sub));
  bfx4 b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (bfx4 __attribute__((address_space(3)))*)(tile + lds_off<D>(row0 + 8, ch) + sub));
  bfx8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

ST_DEVICE f32x16 mfma(bfx8 a, bfx8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

ST_DEVICE f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// registers 8s..8s+7 of an accumulator -> bf16 fragment for k-step s
ST_DEVICE bfx8 acc_frag(const f32x16& a, int s) {
  bfx8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = static_cast<__bf16>(a[8 * s + j]);
  return r;
}

// accumulator register -> row index inside the 32x32 C tile
ST_DEVICE int acc_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// Global 16-byte row chunk of a [rows, D] tile starting at `row0`, zero past `nrows`.
ST_DEVICE BF8 ld_chunk(const bf16_t* base, int64_t row_stride, int row, int ch, int nrows) {
  if (row < nrows) return ld8(base + (int64_t)row * row_stride + ch * 8);
  return BF8{{0u, 0u, 0u, 0u}};
}

template <int D>
ST_DEVICE void st_chunk(lds_t* tile, int row, int ch, const BF8& v) {
  u32x4 w;
  w[0] = v.w[0]; w[1] = v.w[1]; w[2] = v.w[2]; w[3] = v.w[3];
  *reinterpret_cast<u32x4 __attribute__((address_space(3)))*>(tile + lds_off<D>(row, ch)) = w;
}

// Cooperative tile staging: ROWS x D bf16 by 256 threads, register-staged.
template <int D, int ROWS>
struct Stage {
  static constexpr int NCH = D / 8;
  static constexpr int N = ROWS * NCH / 256;  // 16-byte chunks per thread
  BF8 r[N];
  ST_DEVICE void load(const bf16_t* base, int64_t row_stride, int row0, int nrows, int tid) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int c = tid + 256 * i, row = c / NCH, ch = c % NCH;
      r[i] = ld_chunk(base, row_stride, row0 + row, ch, nrows);
    }
  }
  ST_DEVICE void store(lds_t* tile, int tid) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int c = tid + 256 * i, row = c / NCH, ch = c % NCH;
      st_chunk<D>(tile, row, ch, r[i]);
    }
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

// ============================================================== forward
template <int D>
__global__ __launch_bounds__(256, 2) void flash_fwd_kernel(AttnParams p, bf16_t* __restrict__ o,
                                                           int64_t sob, int64_t sos, int64_t soh,
                                                           float* __restrict__ lse) {
  constexpr int BM = 128, BN = 64, NKK = D / 16, NDT = D / 32;
  constexpr int TILE = BN * D * 2;
  __shared__ __attribute__((aligned(16))) char smem_raw[4 * TILE];
  lds_t* smem = (lds_t*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, r = lane & 31, h = lane >> 5;
  const int nqt = gridDim.x;
  const int qt = p.causal ? (nqt - 1 - (int)blockIdx.x) : (int)blockIdx.x;
  const int bh = blockIdx.y, b = bh / p.H, hq = bh % p.H, hk = hq / (p.H / p.Hkv);
  const int q0 = qt * BM, qw = q0 + wid * 32, my_q = qw + r;

  const bf16_t* qbase = p.q + (int64_t)b * p.sqb + (int64_t)hq * p.sqh;
  const bf16_t* kbase = p.k + (int64_t)b * p.skb + (int64_t)hk * p.skh;
  const bf16_t* vbase = p.v + (int64_t)b * p.svb + (int64_t)hk * p.svh;

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[my_q][16kk + 8h .. +8]
  bfx8 qf[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    BF8 c = ld_chunk(qbase, p.sqs, my_q, 2 * kk + h, p.Sq);
    qf[kk] = __builtin_bit_cast(bfx8, c);
  }

  // key blocks this query tile needs
  int nkb = (p.Sk + BN - 1) / BN;
  if (p.causal) {
    const int64_t last_key = p.q_offset + q0 + BM - 1 - p.k_offset;  // local index of last visible key
    const int64_t lim = last_key < 0 ? 0 : last_key / BN + 1;
    if (lim < nkb) nkb = (int)lim;
  }

  f32x16 oacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) oacc[dt] = zero16();
  float m = -INFINITY, l = 0.f;
  const float c2 = p.scale * kLog2e;
  const int64_t qg = p.q_offset + my_q;

  Stage<D, BN> sk, sv;
  if (nkb > 0) {
    sk.load(kbase, p.sks, 0, p.Sk, tid);
    sv.load(vbase, p.svs, 0, p.Sk, tid);
    sk.store(smem, tid);
    sv.store(smem + 2 * TILE, tid);
  }
  __syncthreads();
  int cur = 0;
  for (int kb = 0; kb < nkb; ++kb) {
    const bool more = kb + 1 < nkb;
    if (more) {
      sk.load(kbase, p.sks, (kb + 1) * BN, p.Sk, tid);
      sv.load(vbase, p.svs, (kb + 1) * BN, p.Sk, tid);
    }
    const lds_t* kt = smem + cur * TILE;
    const lds_t* vt = smem + 2 * TILE + cur * TILE;
    // S^T tiles: rows = keys 32t + acc_row, col = query (lane)
    f32x16 s0 = zero16(), s1 = zero16();
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      s0 = mfma(row_frag<D>(kt, r, 2 * kk + h), qf[kk], s0);
      s1 = mfma(row_frag<D>(kt, 32 + r, 2 * kk + h), qf[kk], s1);
    }
    const int kbase_l = kb * BN;
    const bool need_mask =
        (kbase_l + BN > p.Sk) || (p.causal && (p.k_offset + kbase_l + BN - 1 > p.q_offset + q0));
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float a = s0[i] * c2, bb = s1[i] * c2;
      if (need_mask) {
        const int k0 = kbase_l + acc_row(i, h), k1 = k0 + 32;
        if (k0 >= p.Sk || (p.causal && p.k_offset + k0 > qg)) a = -INFINITY;
        if (k1 >= p.Sk || (p.causal && p.k_offset + k1 > qg)) bb = -INFINITY;
      }
      s0[i] = a;
      s1[i] = bb;
      mx = fmaxf(mx, fmaxf(a, bb));
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m, mx);
    const float m_use = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = exp2f(m - m_use);
    float rs = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      s0[i] = exp2f(s0[i] - m_use);
      s1[i] = exp2f(s1[i] - m_use);
      rs += s0[i] + s1[i];
    }
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    m = m_new;
    if (alpha != 1.f) {
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;
    }
    const bfx8 p00 = acc_frag(s0, 0), p01 = acc_frag(s0, 1), p10 = acc_frag(s1, 0), p11 = acc_frag(s1, 1);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      oacc[dt] = mfma(tr_frag<D>(vt, 0, 0, dt, lane), p00, oacc[dt]);
      oacc[dt] = mfma(tr_frag<D>(vt, 0, 1, dt, lane), p01, oacc[dt]);
      oacc[dt] = mfma(tr_frag<D>(vt, 32, 0, dt, lane), p10, oacc[dt]);
      oacc[dt] = mfma(tr_frag<D>(vt, 32, 1, dt, lane), p11, oacc[dt]);
    }
    if (more) {
      sk.store(smem + (cur ^ 1) * TILE, tid);
      sv.store(smem + 2 * TILE + (cur ^ 1) * TILE, tid);
    }
    __syncthreads();
    cur ^= 1;
  }

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
template <int D>
__global__ __launch_bounds__(256) void flash_bwd_pre_kernel(const bf16_t* __restrict__ o,
                                                            const bf16_t* __restrict__ dout,
                                                            float* __restrict__ delta, int B, int S,
                                                            int H, int64_t sob, int64_t sos,
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
  if (row < nrows && ch == 0) delta[((int64_t)b * H + hh) * S + s] = acc;
}

// ============================================================== backward: dQ
// One workgroup = 128 queries of one (b, q-head); iterates the visible key
// blocks.  S^T and dP^T keep the query on the lane, so lse/delta are scalars
// per lane; dQ^T += K^T dS^T feeds dS^T back as the B operand.
template <int D>
__global__ __launch_bounds__(256, 1) void flash_bwd_dq_kernel(AttnParams p,
                                                              const bf16_t* __restrict__ dout,
                                                              int64_t sdb, int64_t sds, int64_t sdh,
                                                              const float* __restrict__ lse,
                                                              const float* __restrict__ delta,
                                                              bf16_t* __restrict__ dq) {
  constexpr int BM = 128, BN = 64, NKK = D / 16, NDT = D / 32;
  constexpr int TILE = BN * D * 2;
  __shared__ __attribute__((aligned(16))) char smem_raw[4 * TILE];
  lds_t* smem = (lds_t*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, r = lane & 31, h = lane >> 5;
  const int nqt = gridDim.x;
  const int qt = p.causal ? (nqt - 1 - (int)blockIdx.x) : (int)blockIdx.x;
  const int bh = blockIdx.y, b = bh / p.H, hq = bh % p.H, hk = hq / (p.H / p.Hkv);
  const int q0 = qt * BM, qw = q0 + wid * 32, my_q = qw + r;

  const bf16_t* qbase = p.q + (int64_t)b * p.sqb + (int64_t)hq * p.sqh;
  const bf16_t* dobase = dout + (int64_t)b * sdb + (int64_t)hq * sdh;
  const bf16_t* kbase = p.k + (int64_t)b * p.skb + (int64_t)hk * p.skh;
  const bf16_t* vbase = p.v + (int64_t)b * p.svb + (int64_t)hk * p.svh;

  bfx8 qf[NKK], df[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    qf[kk] = __builtin_bit_cast(bfx8, ld_chunk(qbase, p.sqs, my_q, 2 * kk + h, p.Sq));
    df[kk] = __builtin_bit_cast(bfx8, ld_chunk(dobase, sds, my_q, 2 * kk + h, p.Sq));
  }
  const int64_t li = ((int64_t)b * p.H + hq) * p.Sq + my_q;
  const float lse2 = my_q < p.Sq ? lse[li] * kLog2e : 0.f;
  const float dlt = my_q < p.Sq ? delta[li] : 0.f;
  const float c2 = p.scale * kLog2e;
  const int64_t qg = p.q_offset + my_q;

  int nkb = (p.Sk + BN - 1) / BN;
  if (p.causal) {
    const int64_t last_key = p.q_offset + q0 + BM - 1 - p.k_offset;
    const int64_t lim = last_key < 0 ? 0 : last_key / BN + 1;
    if (lim < nkb) nkb = (int)lim;
  }

  f32x16 dqacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dqacc[dt] = zero16();

  Stage<D, BN> sk, sv;
  if (nkb > 0) {
    sk.load(kbase, p.sks, 0, p.Sk, tid);
    sv.load(vbase, p.svs, 0, p.Sk, tid);
    sk.store(smem, tid);
    sv.store(smem + 2 * TILE, tid);
  }
  __syncthreads();
  int cur = 0;
  for (int kb = 0; kb < nkb; ++kb) {
    const bool more = kb + 1 < nkb;
    if (more) {
      sk.load(kbase, p.sks, (kb + 1) * BN, p.Sk, tid);
      sv.load(vbase, p.svs, (kb + 1) * BN, p.Sk, tid);
    }
    const lds_t* kt = smem + cur * TILE;
    const lds_t* vt = smem + 2 * TILE + cur * TILE;
    f32x16 s0 = zero16(), s1 = zero16(), d0 = zero16(), d1 = zero16();
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      s0 = mfma(row_frag<D>(kt, r, 2 * kk + h), qf[kk], s0);
      s1 = mfma(row_frag<D>(kt, 32 + r, 2 * kk + h), qf[kk], s1);
      d0 = mfma(row_frag<D>(vt, r, 2 * kk + h), df[kk], d0);
      d1 = mfma(row_frag<D>(vt, 32 + r, 2 * kk + h), df[kk], d1);
    }
    const int kbase_l = kb * BN;
    const bool need_mask =
        (kbase_l + BN > p.Sk) || (p.causal && (p.k_offset + kbase_l + BN - 1 > p.q_offset + q0));
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float pa = exp2f(s0[i] * c2 - lse2), pb = exp2f(s1[i] * c2 - lse2);
      if (need_mask) {
        const int k0 = kbase_l + acc_row(i, h), k1 = k0 + 32;
        if (k0 >= p.Sk || (p.causal && p.k_offset + k0 > qg)) pa = 0.f;
        if (k1 >= p.Sk || (p.causal && p.k_offset + k1 > qg)) pb = 0.f;
      }
      s0[i] = pa * (d0[i] - dlt);
      s1[i] = pb * (d1[i] - dlt);
    }
    const bfx8 g00 = acc_frag(s0, 0), g01 = acc_frag(s0, 1), g10 = acc_frag(s1, 0), g11 = acc_frag(s1, 1);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      dqacc[dt] = mfma(tr_frag<D>(kt, 0, 0, dt, lane), g00, dqacc[dt]);
      dqacc[dt] = mfma(tr_frag<D>(kt, 0, 1, dt, lane), g01, dqacc[dt]);
      dqacc[dt] = mfma(tr_frag<D>(kt, 32, 0, dt, lane), g10, dqacc[dt]);
      dqacc[dt] = mfma(tr_frag<D>(kt, 32, 1, dt, lane), g11, dqacc[dt]);
    }
    if (more) {
      sk.store(smem + (cur ^ 1) * TILE, tid);
      sv.store(smem + 2 * TILE + (cur ^ 1) * TILE, tid);
    }
    __syncthreads();
    cur ^= 1;
  }
  if (my_q < p.Sq) {
    bf16_t* row = dq + (int64_t)b * p.sxb + (int64_t)my_q * p.sxs + (int64_t)hq * p.sxh;
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

// ============================================================== backward: dK, dV
// One workgroup = 128 keys (4 waves x 32) of one (b, q-head); iterates query
// blocks of 32 rows staged in LDS (Q, dO, lse, delta).  Output is this query
// head's contribution, fp32 [B, Sk, H, D] (summed over the GQA group later)
// or bf16 directly when H == Hkv.
template <int D, bool DIRECT>
__global__ __launch_bounds__(256, 1) void flash_bwd_dkdv_kernel(
    AttnParams p, const bf16_t* __restrict__ dout, int64_t sdb, int64_t sds, int64_t sdh,
    const float* __restrict__ lse, const float* __restrict__ delta, void* __restrict__ dk_out,
    void* __restrict__ dv_out) {
  constexpr int BKW = 128, BQ = 32, NKK = D / 16, NDT = D / 32;
  constexpr int TILE = BQ * D * 2;
  __shared__ __attribute__((aligned(16))) char smem_raw[4 * TILE + 4 * BQ * 4];
  lds_t* smem = (lds_t*)smem_raw;
  float* stats = (float*)(smem_raw + 4 * TILE);  // [2 buf][lse2 | delta][BQ]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, r = lane & 31, h = lane >> 5;
  const int nkt = gridDim.x;
  const int kt_i = p.causal ? (int)blockIdx.x : (int)blockIdx.x;  // early keys = heaviest (causal)
  (void)nkt;
  const int bh = blockIdx.y, b = bh / p.H, hq = bh % p.H, hk = hq / (p.H / p.Hkv);
  const int k0 = kt_i * BKW, kw = k0 + wid * 32, my_k = kw + r;

  const bf16_t* qbase = p.q + (int64_t)b * p.sqb + (int64_t)hq * p.sqh;
  const bf16_t* dobase = dout + (int64_t)b * sdb + (int64_t)hq * sdh;
  const bf16_t* kbase = p.k + (int64_t)b * p.skb + (int64_t)hk * p.skh;
  const bf16_t* vbase = p.v + (int64_t)b * p.svb + (int64_t)hk * p.svh;
  const float* lse_row = lse + ((int64_t)b * p.H + hq) * p.Sq;
  const float* dlt_row = delta + ((int64_t)b * p.H + hq) * p.Sq;

  // K^T / V^T as B operands: lane holds K[my_k][16kk + 8h .. +8]
  bfx8 kf[NKK], vf[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    kf[kk] = __builtin_bit_cast(bfx8, ld_chunk(kbase, p.sks, my_k, 2 * kk + h, p.Sk));
    vf[kk] = __builtin_bit_cast(bfx8, ld_chunk(vbase, p.svs, my_k, 2 * kk + h, p.Sk));
  }
  const int64_t kg = p.k_offset + my_k;
  const float c2 = p.scale * kLog2e;

  // query blocks that can see any key of this tile
  int qb0 = 0;
  if (p.causal) {
    const int64_t first_q = p.k_offset + k0 - p.q_offset;  // local query index of first visible row
    qb0 = first_q <= 0 ? 0 : (int)(first_q / BQ);
  }
  const int nqb = (p.Sq + BQ - 1) / BQ;

  f32x16 dkacc[NDT], dvacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dkacc[dt] = dvacc[dt] = zero16();

  // staging: Q and dO tiles (32 x D each = 256 threads x N chunks), stats by threads < 64
  Stage<D, BQ> sq, sd;
  float st_v = 0.f;
  auto load_stats = [&](int qb) {
    if (tid < 2 * BQ) {
      const int qi = qb * BQ + (tid & (BQ - 1));
      if (tid < BQ) st_v = qi < p.Sq ? lse_row[qi] * kLog2e : INFINITY;
      else st_v = qi < p.Sq ? dlt_row[qi] : 0.f;
    }
  };
  auto store_stats = [&](int buf) {
    if (tid < 2 * BQ) stats[buf * 2 * BQ + tid] = st_v;
  };
  if (qb0 < nqb) {
    sq.load(qbase, p.sqs, qb0 * BQ, p.Sq, tid);
    sd.load(dobase, sds, qb0 * BQ, p.Sq, tid);
    load_stats(qb0);
    sq.store(smem, tid);
    sd.store(smem + 2 * TILE, tid);
    store_stats(0);
  }
  __syncthreads();
  int cur = 0;
  for (int qb = qb0; qb < nqb; ++qb) {
    const bool more = qb + 1 < nqb;
    if (more) {
      sq.load(qbase, p.sqs, (qb + 1) * BQ, p.Sq, tid);
      sd.load(dobase, sds, (qb + 1) * BQ, p.Sq, tid);
      load_stats(qb + 1);
    }
    const lds_t* qt = smem + cur * TILE;
    const lds_t* dt_ = smem + 2 * TILE + cur * TILE;
    const float* lse2 = stats + cur * 2 * BQ;
    const float* dl = lse2 + BQ;
    const int qbase_l = qb * BQ;
    // this wave's keys vs this query block: skip when every key is in the future
    const bool wave_dead = p.causal && (p.k_offset + kw > p.q_offset + qbase_l + BQ - 1);
    if (!wave_dead) {
      // S = Q K^T, dP = dO V^T : rows = queries (acc_row), col = key (lane)
      f32x16 s = zero16(), dp = zero16();
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        s = mfma(row_frag<D>(qt, r, 2 * kk + h), kf[kk], s);
        dp = mfma(row_frag<D>(dt_, r, 2 * kk + h), vf[kk], dp);
      }
      const bool need_mask = (qbase_l + BQ > p.Sq) || (my_k >= p.Sk) ||
                             (p.causal && (p.k_offset + kw + 31 > p.q_offset + qbase_l));
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qi = acc_row(i, h);
        float pv = exp2f(s[i] * c2 - lse2[qi]);
        if (need_mask) {
          const int64_t qgl = p.q_offset + qbase_l + qi;
          if (qbase_l + qi >= p.Sq || my_k >= p.Sk || (p.causal && kg > qgl)) pv = 0.f;
        }
        s[i] = pv;
        dp[i] = pv * (dp[i] - dl[qi]);
      }
      const bfx8 p0 = acc_frag(s, 0), p1 = acc_frag(s, 1);
      const bfx8 g0 = acc_frag(dp, 0), g1 = acc_frag(dp, 1);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        dvacc[dt] = mfma(tr_frag<D>(dt_, 0, 0, dt, lane), p0, dvacc[dt]);
        dvacc[dt] = mfma(tr_frag<D>(dt_, 0, 1, dt, lane), p1, dvacc[dt]);
        dkacc[dt] = mfma(tr_frag<D>(qt, 0, 0, dt, lane), g0, dkacc[dt]);
        dkacc[dt] = mfma(tr_frag<D>(qt, 0, 1, dt, lane), g1, dkacc[dt]);
      }
    }
    if (more) {
      sq.store(smem + (cur ^ 1) * TILE, tid);
      sd.store(smem + 2 * TILE + (cur ^ 1) * TILE, tid);
      store_stats(cur ^ 1);
    }
    __syncthreads();
    cur ^= 1;
  }
  if (my_k < p.Sk) {
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * h;
        if (DIRECT) {
          const int64_t off = (int64_t)b * p.sxb + (int64_t)my_k * p.sxs + (int64_t)hk * p.sxh + d;
          uint2 wk, wv;
          wk.x = pack_bf16x2(dkacc[dt][4 * g] * p.scale, dkacc[dt][4 * g + 1] * p.scale);
          wk.y = pack_bf16x2(dkacc[dt][4 * g + 2] * p.scale, dkacc[dt][4 * g + 3] * p.scale);
          wv.x = pack_bf16x2(dvacc[dt][4 * g], dvacc[dt][4 * g + 1]);
          wv.y = pack_bf16x2(dvacc[dt][4 * g + 2], dvacc[dt][4 * g + 3]);
          *reinterpret_cast<uint2*>((bf16_t*)dk_out + off) = wk;
          *reinterpret_cast<uint2*>((bf16_t*)dv_out + off) = wv;
        } else {
          const int64_t off = (((int64_t)b * p.Sk + my_k) * p.H + hq) * D + d;
          st4f((float*)dk_out + off,
               make_float4(dkacc[dt][4 * g] * p.scale, dkacc[dt][4 * g + 1] * p.scale,
                           dkacc[dt][4 * g + 2] * p.scale, dkacc[dt][4 * g + 3] * p.scale));
          st4f((float*)dv_out + off,
               make_float4(dvacc[dt][4 * g], dvacc[dt][4 * g + 1], dvacc[dt][4 * g + 2],
                           dvacc[dt][4 * g + 3]));
        }
      }
    }
  }
}

// Sum the per-query-head fp32 dK/dV partials over each GQA group -> bf16.
// in: [B*Sk, H, D] fp32, out: [B, Sk, Hkv, D] with strides (bf16).
__global__ __launch_bounds__(256) void gqa_reduce_kernel(const float* __restrict__ in,
                                                         bf16_t* __restrict__ out, int64_t rows,
                                                         int H, int Hkv, int D, int64_t sob,
                                                         int64_t sos, int64_t soh, int Sk) {
  const int G = H / Hkv, D8 = D / 8;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = rows * Hkv * D8;
  if (t >= total) return;
  const int c = (int)(t % D8);
  const int64_t rh = t / D8;
  const int hk = (int)(rh % Hkv);
  const int64_t row = rh / Hkv;  // b*Sk + s
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int g = 0; g < G; ++g) {
    const float* src = in + (row * H + hk * G + g) * D + c * 8;
    float4 a = ld4f(src), bq = ld4f(src + 4);
    acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
    acc[4] += bq.x; acc[5] += bq.y; acc[6] += bq.z; acc[7] += bq.w;
  }
  const int64_t b = row / Sk, s = row % Sk;
  st8(out + b * sob + s * sos + hk * soh + c * 8, pack8(acc));
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

}  // namespace

extern "C" {

int st_flash_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int Sq,
                 int Sk, int H, int Hkv, int D, int64_t sqb, int64_t sqs, int64_t sqh, int64_t skb,
                 int64_t sks, int64_t skh, int64_t svb, int64_t svs, int64_t svh, int64_t sob,
                 int64_t sos, int64_t soh, float scale, int causal, int64_t q_offset,
                 int64_t k_offset, hipStream_t st) {
  if (H % Hkv != 0) return -2;
  if (Sq == 0 || B == 0) return 0;
  AttnParams p = make_params(q, k, v, B, Sq, Sk, H, Hkv, sqb, sqs, sqh, skb, sks, skh, svb, svs, svh,
                             scale, causal, q_offset, k_offset);
  dim3 grid((Sq + 127) / 128, B * H);
  if (D == 128)
    flash_fwd_kernel<128><<<grid, 256, 0, st>>>(p, (bf16_t*)o, sob, sos, soh, lse);
  else if (D == 64)
    flash_fwd_kernel<64><<<grid, 256, 0, st>>>(p, (bf16_t*)o, sob, sos, soh, lse);
  else
    return -3;
  return (int)hipGetLastError();
}

int st_flash_bwd_preprocess(const void* o, const void* dout, float* delta, int B, int S, int H,
                            int D, int64_t sob, int64_t sos, int64_t soh, int64_t sdb, int64_t sds,
                            int64_t sdh, hipStream_t st) {
  const int64_t threads = (int64_t)B * S * H * (D / 8);
  if (threads == 0) return 0;
  const unsigned blocks = (unsigned)((threads + 255) / 256);
  if (D == 128)
    flash_bwd_pre_kernel<128><<<blocks, 256, 0, st>>>((const bf16_t*)o, (const bf16_t*)dout, delta, B,
                                                      S, H, sob, sos, soh, sdb, sds, sdh);
  else if (D == 64)
    flash_bwd_pre_kernel<64><<<blocks, 256, 0, st>>>((const bf16_t*)o, (const bf16_t*)dout, delta, B, S,
                                                     H, sob, sos, soh, sdb, sds, sdh);
  else
    return -3;
  return (int)hipGetLastError();
}

// dq / dk / dv: bf16 outputs with arbitrary (b, s, h) strides (D contiguous) so
// they can be slices of one fused dQKV buffer.  `work` must hold
// 2*B*Sk*H*D floats when H != Hkv (per-query-head partials of the GQA sum).
int st_flash_bwd(const void* q, const void* k, const void* v, const void* dout, const float* lse,
                 const float* delta, void* dq, void* dk, void* dv, float* work, int B, int Sq,
                 int Sk, int H, int Hkv, int D, int64_t sqb, int64_t sqs, int64_t sqh, int64_t skb,
                 int64_t sks, int64_t skh, int64_t svb, int64_t svs, int64_t svh, int64_t sdb,
                 int64_t sds, int64_t sdh, int64_t sdqb, int64_t sdqs, int64_t sdqh, int64_t sdkb,
                 int64_t sdks, int64_t sdkh, float scale, int causal, int64_t q_offset,
                 int64_t k_offset, hipStream_t st) {
  if (H % Hkv != 0) return -2;
  if (B == 0 || Sq == 0 || Sk == 0) return 0;
  AttnParams p = make_params(q, k, v, B, Sq, Sk, H, Hkv, sqb, sqs, sqh, skb, sks, skh, svb, svs, svh,
                             scale, causal, q_offset, k_offset);
  AttnParams pq = p, pk = p;
  pq.sxb = sdqb; pq.sxs = sdqs; pq.sxh = sdqh;
  pk.sxb = sdkb; pk.sxs = sdks; pk.sxh = sdkh;
  dim3 gq((Sq + 127) / 128, B * H);
  dim3 gk((Sk + 127) / 128, B * H);
  const bool direct = (H == Hkv);
  if (!direct && work == nullptr) return -4;
  float* wk = work;
  float* wv = direct ? nullptr : work + (int64_t)B * Sk * H * D;
  const bf16_t* dop = (const bf16_t*)dout;
  if (D == 128) {
    flash_bwd_dq_kernel<128><<<gq, 256, 0, st>>>(pq, dop, sdb, sds, sdh, lse, delta, (bf16_t*)dq);
    if (direct)
      flash_bwd_dkdv_kernel<128, true><<<gk, 256, 0, st>>>(pk, dop, sdb, sds, sdh, lse, delta, dk, dv);
    else
      flash_bwd_dkdv_kernel<128, false><<<gk, 256, 0, st>>>(pk, dop, sdb, sds, sdh, lse, delta, wk, wv);
  } else if (D == 64) {
    flash_bwd_dq_kernel<64><<<gq, 256, 0, st>>>(pq, dop, sdb, sds, sdh, lse, delta, (bf16_t*)dq);
    if (direct)
      flash_bwd_dkdv_kernel<64, true><<<gk, 256, 0, st>>>(pk, dop, sdb, sds, sdh, lse, delta, dk, dv);
    else
      flash_bwd_dkdv_kernel<64, false><<<gk, 256, 0, st>>>(pk, dop, sdb, sds, sdh, lse, delta, wk, wv);
  } else {
    return -3;
  }
  if (!direct) {
    const int64_t rows = (int64_t)B * Sk;
    const int64_t total = rows * Hkv * (D / 8);
    const unsigned blocks = (unsigned)((total + 255) / 256);
    gqa_reduce_kernel<<<blocks, 256, 0, st>>>(wk, (bf16_t*)dk, rows, H, Hkv, D, sdkb, sdks, sdkh, Sk);
    gqa_reduce_kernel<<<blocks, 256, 0, st>>>(wv, (bf16_t*)dv, rows, H, Hkv, D, sdkb, sdks, sdkh, Sk);
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

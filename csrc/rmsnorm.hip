// RMSNorm forward / backward for gfx950, optionally fused with the residual add
// that precedes every pre-norm in a Llama/Qwen3 decoder layer.
//
// Reference semantics: scaletorch/models/attention_utils.py:247-271 (fp32
// variance, rsqrt, scale by weight) and the residual adds in
// scaletorch/models/llama.py:320-379.  The MI355X design:
//   * one wave64 owns one row; the whole row lives in VGPRs (h <= 8192), so the
//     sum of squares is a pure register + DPP/shuffle reduction with no LDS and
//     no barrier;
//   * 16-byte (8 x bf16) loads/stores per lane: a wave touches 1 KiB per access;
//   * the residual add is fused: s = x + r is rounded to bf16 once, written as
//     the new residual stream and normalised from the rounded value, so the
//     fused path is bit-compatible with the unfused bf16 graph;
//   * backward recomputes xhat from s and rstd (fp32, saved by forward), emits
//     ds (+ an optional incoming residual-stream gradient) and per-block fp32
//     partial sums of dy*xhat that a second pass reduces into dweight.
#include <cstdlib>

#include "common.h"

using namespace st;

namespace {

constexpr int kRowsPerBlock = 4;  // 4 waves = 256 threads

template <int NCH, bool RES>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ res, const bf16_t* __restrict__ w,
    bf16_t* __restrict__ y, bf16_t* __restrict__ sum_out, float* __restrict__ rstd_out, int rows,
    int h, float eps) {
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const size_t base = (size_t)row * h;
  float v[NCH][8];
  float ss = 0.f;
  // every load of the row is issued before the first store (hipcc otherwise keeps
  // the residual-sum store of chunk c ahead of chunk c+1's loads: 2 loads in flight)
  BF8 xa[NCH], ra[RES ? NCH : 1];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < h) {
      xa[c] = ld8(x + base + col);
      if (RES) ra[RES ? c : 0] = ld8(res + base + col);
    }
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < h) {
      unpack8(xa[c], v[c]);
      if (RES) {
        float r[8];
        unpack8(ra[RES ? c : 0], r);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[c][i] = bf2f(f2bf(v[c][i] + r[i]));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[c][i] * v[c][i];
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[c][i] = 0.f;
    }
  }
  // the weight (L2-resident) is requested before any store, so waiting for it does
  // not also wait for the row's stores (vmcnt counts both)
  BF8 wa[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < h) wa[c] = ld8(w + col);
  }
  if (RES) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < h) st8(sum_out + base + col, pack8(v[c]));
    }
  }
  ss = wave_sum(ss);
  const float rs = rsqrtf(ss / (float)h + eps);
  if (lane == 0) rstd_out[row] = rs;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < h) {
      float wf[8], o[8];
      unpack8(wa[c], wf);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = v[c][i] * rs * wf[i];
      st8(y + base + col, pack8(o));
    }
  }
}

// grid-stride over rows; each wave accumulates its dweight partial in
// registers; the 4 waves of a block fold them through LDS in a fixed order
// (3->1, 2->0, then 1->0: deterministic) and wave 0 writes one row of
// partial[block, h].  The row operands are kept packed (bf16) in registers to
// bound VGPR use at h = 8192.  Dynamic LDS: 2 * NCH * 512 fp32, lane-major
// (element i of lane L in chunk c at c*512 + i*64 + L: bank-conflict free).
template <int NCH, bool DRES, bool PF = false>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ s, const bf16_t* __restrict__ w,
    const float* __restrict__ rstd, const bf16_t* __restrict__ dres, bf16_t* __restrict__ ds,
    float* __restrict__ partial, int rows, int h) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  const int nw = gridDim.x * kRowsPerBlock;
  BF8 wp[NCH];
  float dwp[NCH][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) dwp[c][i] = 0.f;
    if (col < h) wp[c] = ld8(w + col);
    else wp[c] = BF8{{0u, 0u, 0u, 0u}};
  }
  // PF: the operands of the wave's NEXT row are requested before this row's math and
  // stores (ST_RMSNORM_BWD_PF=1), so loads stay in flight across the row boundary
  // instead of each row waiting for the previous row's stores (vmcnt counts both)
  BF8 sp[NCH], dp[NCH], rp[DRES ? NCH : 1];
  float rs = 0.f;
#define ST_RMS_LOAD_ROW(R, S_, D_, Q_)                                        \
  do {                                                                        \
    const size_t b_ = (size_t)(R) * h;                                        \
    _Pragma("unroll") for (int c = 0; c < NCH; ++c) {                         \
      const int col = c * 512 + lane * 8;                                     \
      if (col < h) {                                                          \
        S_[c] = ld8(s + b_ + col);                                            \
        D_[c] = ld8(dy + b_ + col);                                           \
        if (DRES) Q_[DRES ? c : 0] = ld8(dres + b_ + col);                    \
      } else {                                                                \
        S_[c] = BF8{{0u, 0u, 0u, 0u}};                                        \
        D_[c] = BF8{{0u, 0u, 0u, 0u}};                                        \
        if (DRES) Q_[DRES ? c : 0] = BF8{{0u, 0u, 0u, 0u}};                   \
      }                                                                       \
    }                                                                         \
  } while (0)
  if (PF && gw < rows) {
    ST_RMS_LOAD_ROW(gw, sp, dp, rp);
    rs = rstd[gw];
  }
  for (int row = gw; row < rows; row += nw) {
    const size_t base = (size_t)row * h;
    BF8 sn[PF ? NCH : 1], dn[PF ? NCH : 1], rn[(PF && DRES) ? NCH : 1];
    float rsn = 0.f;
    if (PF) {
      if (row + nw < rows) {
        ST_RMS_LOAD_ROW(row + nw, sn, dn, rn);
        rsn = rstd[row + nw];
      }
    } else {
      // every operand of the row (incl. the residual-stream gradient) is issued
      // before the reduction, so a wave has 2-3 x NCH 16-byte loads in flight
      ST_RMS_LOAD_ROW(row, sp, dp, rp);
      rs = rstd[row];
    }
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      float sv[8], dv[8], wf[8];
      unpack8(sp[c], sv);
      unpack8(dp[c], dv);
      unpack8(wp[c], wf);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xh = sv[i] * rs;
        dot += dv[i] * wf[i] * xh;
        dwp[c][i] += dv[i] * xh;
      }
    }
    dot = wave_sum(dot) / (float)h;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < h) {
        float sv[8], dv[8], wf[8], o[8];
        unpack8(sp[c], sv);
        unpack8(dp[c], dv);
        unpack8(wp[c], wf);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = rs * (dv[i] * wf[i] - sv[i] * rs * dot);
        if (DRES) {
          float r[8];
          unpack8(rp[DRES ? c : 0], r);
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] += r[i];
        }
        st8(ds + base + col, pack8(o));
      }
    }
    if (PF) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        sp[c] = sn[PF ? c : 0];
        dp[c] = dn[PF ? c : 0];
        if (DRES) rp[DRES ? c : 0] = rn[(PF && DRES) ? c : 0];
      }
      rs = rsn;
    }
  }
#undef ST_RMS_LOAD_ROW
  extern __shared__ float red_lds[];  // [2][NCH * 512]
  constexpr int kSlab = NCH * 512;
  const int wid = threadIdx.x >> 6;
  // step 1: waves 2,3 park their partials; waves 0,1 add them
  if (wid >= 2) {
    float* dst = red_lds + (wid - 2) * kSlab;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < h) {
#pragma unroll
        for (int i = 0; i < 8; ++i) dst[c * 512 + i * 64 + lane] = dwp[c][i];
      }
    }
  }
  __syncthreads();
  if (wid < 2) {
    const float* src = red_lds + wid * kSlab;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < h) {
#pragma unroll
        for (int i = 0; i < 8; ++i) dwp[c][i] += src[c * 512 + i * 64 + lane];
      }
    }
  }
  __syncthreads();
  // step 2: wave 1 parks, wave 0 adds and writes the block's partial row
  if (wid == 1) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < h) {
#pragma unroll
        for (int i = 0; i < 8; ++i) red_lds[c * 512 + i * 64 + lane] = dwp[c][i];
      }
    }
  }
  __syncthreads();
  if (wid == 0) {
    float* pr = partial + (size_t)blockIdx.x * h;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < h) {
#pragma unroll
        for (int i = 0; i < 8; ++i) dwp[c][i] += red_lds[c * 512 + i * 64 + lane];
        st4f(pr + col, make_float4(dwp[c][0], dwp[c][1], dwp[c][2], dwp[c][3]));
        st4f(pr + col + 4, make_float4(dwp[c][4], dwp[c][5], dwp[c][6], dwp[c][7]));
      }
    }
  }
}

// dw[col] (+)= sum_p partial[p, col], deterministically: a block owns 64 columns
// (16 lanes x float4) and splits the partial rows over 16 row groups (p = g, g+16,
// ...); the 16 group sums fold through LDS in group order and one thread per column
// quad adds them to dw (the only writer of those columns: no atomics, so the
// dweight -- and with it the whole step -- is bitwise repeatable).
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ partial,
                                                     float* __restrict__ out, int P, int h) {
  __shared__ float4 red[16][16];
  const int q = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int col = blockIdx.x * 64 + q * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col < h) {
    for (int p = g; p < P; p += 16) {
      float4 v = ld4f(partial + (size_t)p * h + col);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  red[g][q] = acc;
  __syncthreads();
  if (g == 0 && col < h) {
    float4 t = red[0][q];
#pragma unroll
    for (int k = 1; k < 16; ++k) {
      t.x += red[k][q].x; t.y += red[k][q].y; t.z += red[k][q].z; t.w += red[k][q].w;
    }
    // scalar: dw may be any fp32 view into the main_grad arena (4-byte aligned)
    out[col + 0] += t.x;
    out[col + 1] += t.y;
    out[col + 2] += t.z;
    out[col + 3] += t.w;
  }
}

template <bool RES>
int launch_fwd(const void* x, const void* res, const void* w, void* y, void* sum_out, float* rstd,
               int rows, int h, float eps, hipStream_t st) {
  const int nch = (h + 511) / 512;
  dim3 grid((rows + kRowsPerBlock - 1) / kRowsPerBlock), block(256);
#define ST_RMS_FWD(N)                                                                      \
  rmsnorm_fwd_kernel<N, RES><<<grid, block, 0, st>>>(                                      \
      (const bf16_t*)x, (const bf16_t*)res, (const bf16_t*)w, (bf16_t*)y, (bf16_t*)sum_out, \
      rstd, rows, h, eps)
  if (nch <= 1) ST_RMS_FWD(1);
  else if (nch <= 2) ST_RMS_FWD(2);
  else if (nch <= 4) ST_RMS_FWD(4);
  else if (nch <= 8) ST_RMS_FWD(8);
  else if (nch <= 10) ST_RMS_FWD(10);
  else if (nch <= 16) ST_RMS_FWD(16);
  else return -1;
#undef ST_RMS_FWD
  return (int)hipGetLastError();
}

template <bool DRES>
int launch_bwd(const void* dy, const void* s, const void* w, const float* rstd, const void* dres,
               void* ds, float* partial, int nblocks, int rows, int h, hipStream_t st) {
  const int nch = (h + 511) / 512;
  dim3 grid(nblocks), block(256);
#define ST_RMS_BWD(N)                                                                       \
  rmsnorm_bwd_kernel<N, DRES><<<grid, block, 2 * (N) * 512 * sizeof(float), st>>>(        \
      (const bf16_t*)dy, (const bf16_t*)s, (const bf16_t*)w, rstd, (const bf16_t*)dres,     \
      (bf16_t*)ds, partial, rows, h)
  // prefetching body at h <= 4096 (default on; ST_RMSNORM_BWD_PF=0 for the A/B): isolated at
  // the bench shape 0.1776-0.1779 -> 0.1701-0.1725 ms (profiles/r04/rmsnorm_bwd_prefetch.log)
  const char* pfe = std::getenv("ST_RMSNORM_BWD_PF");  // read per call: same-process A/B
  const bool pf = !pfe || std::atoi(pfe) == 1;
  if (pf && nch > 4 && nch <= 8)
    rmsnorm_bwd_kernel<8, DRES, true><<<grid, block, 2 * 8 * 512 * sizeof(float), st>>>(
        (const bf16_t*)dy, (const bf16_t*)s, (const bf16_t*)w, rstd, (const bf16_t*)dres, (bf16_t*)ds, partial,
        rows, h);
  else if (nch <= 1) ST_RMS_BWD(1);
  else if (nch <= 2) ST_RMS_BWD(2);
  else if (nch <= 4) ST_RMS_BWD(4);
  else if (nch <= 8) ST_RMS_BWD(8);
  else if (nch <= 10) ST_RMS_BWD(10);
  else if (nch <= 16) ST_RMS_BWD(16);
  else return -1;
#undef ST_RMS_BWD
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {

// Number of dweight partial rows the backward writes (one per block; the
// partial buffer must hold nwaves*h fp32).  Name kept for the binding.
// Block cap: enough waves per SIMD across 256 CUs to hide HBM latency; the
// fp32 partial buffer (blocks x h) that colsum re-reads grows with it.
// ST_RMSNORM_BWD_BLOCKS overrides it (A/B only).
static int rmsnorm_bwd_block_cap() {
  static int cap = [] {
    const char* e = getenv("ST_RMSNORM_BWD_BLOCKS");
    int v = e ? atoi(e) : 0;
    return (v >= 64 && v <= 4096) ? v : 256;
  }();
  return cap;
}

int st_rmsnorm_bwd_nwaves(int rows) {
  int blocks = (rows + kRowsPerBlock - 1) / kRowsPerBlock;
  if (blocks > rmsnorm_bwd_block_cap()) blocks = rmsnorm_bwd_block_cap();
  if (blocks < 1) blocks = 1;
  return blocks;
}

int st_rmsnorm_fwd(const void* x, const void* res, const void* w, void* y, void* sum_out,
                   float* rstd, int rows, int h, float eps, hipStream_t st) {
  if (h % 8 != 0) return -2;
  if (res) return launch_fwd<true>(x, res, w, y, sum_out, rstd, rows, h, eps, st);
  return launch_fwd<false>(x, nullptr, w, y, nullptr, rstd, rows, h, eps, st);
}

// dw_out (fp32, length h) is ACCUMULATED into (caller zeroes it or passes a
// main_grad view).
int st_rmsnorm_bwd(const void* dy, const void* s, const void* w, const float* rstd,
                   const void* dres, void* ds, float* partial, float* dw_out, int rows, int h,
                   hipStream_t st) {
  if (h % 8 != 0) return -2;
  const int nw = st_rmsnorm_bwd_nwaves(rows);
  int rc = dres ? launch_bwd<true>(dy, s, w, rstd, dres, ds, partial, nw, rows, h, st)
                : launch_bwd<false>(dy, s, w, rstd, nullptr, ds, partial, nw, rows, h, st);
  if (rc) return rc;
  colsum_kernel<<<(h + 63) / 64, 256, 0, st>>>(partial, dw_out, nw, h);
  return (int)hipGetLastError();
}

}  // extern "C"

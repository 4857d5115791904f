// Custom intra-node collectives over xGMI peer memory: all-reduce (one-shot /
// two-shot), all-gather and reduce-scatter (the sequence-parallel / CP K/V
// collectives), on one flag protocol.
//
// Reference: the TP all-reduces of scaletorch (ReduceFromModelParallelRegion,
// RowParallelLinear and the async grad-input all-reduce,
// scaletorch/parallel/tensor_parallel/tp_comms.py:117-166, :229-320) which go
// through NCCL/HCCL for every message size.  SURVEY.md §2.2 "custom transport".
//
// Why: a TP all-reduce of one activation ([b, S, h] bf16, 1-32 MiB) is
// latency/launch bound on RCCL's ring at small sizes and per-link bound at
// large ones.  An MI355X node is fully connected (every GPU has a direct xGMI
// link to each of the 7 others), so a rank can READ all peers' buffers at once:
//   * one-shot: every rank copies its input into its IPC-shared buffer, signals,
//     then reads the same slice from all W buffers and sums (fp32) -- one
//     round trip, W-1 links busy in parallel; best for small messages.
//   * two-shot: reduce-scatter (rank p sums partition p from all buffers into
//     its result area), signal, all-gather (every rank copies partition p from
//     rank p's result area) -- 2 (W-1)/W of the bytes per rank, for large ones.
// Buffers are plain device allocations; coherence is explicit: every load and
// store of a shared area carries the system-coherence bits (sc0 sc1: written
// through / re-fetched past the non-coherent XCD L2s), flags are system-scope
// atomics, the writer retires its stores (vmcnt(0)) before the release flag
// store and the reader acquires before loading.  (An "uncached" allocation
// alone was not enough: order-dependent stale slices were observed with it.)
//
// Synchronisation is per BLOCK, not per grid: block b of every rank owns the
// same slice of the message, so block b only waits for block b of its peers
// (flags[phase][b][rank], written into the PEER's buffer).  Each call has an
// epoch (host counter, identical on every rank); data areas are double-buffered
// by epoch parity, which with the per-call handshake guarantees no rank
// overwrites a slice a slower peer may still be reading.  Every spin is
// bounded (s_memrealtime, 100 MHz): a dead peer sets the error word and the
// kernel exits instead of hanging the GPU.
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <vector>

#include "common.h"

using namespace st;

namespace {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 256;  // one 512-thread block per CU at most: every block co-resident
constexpr int kThreads = 512;
constexpr int64_t kFlagBytes = 2 * kMaxBlocks * kMaxRanks * 4;  // [phase][block][rank] uint32
constexpr int64_t kHeader = 16384;                              // flags padded to 16 KiB
static_assert(kFlagBytes <= kHeader, "flag area");

struct Peers {
  char* buf[kMaxRanks];
};

// What one rank contributes; a launch normally carries one job (gridDim.y = 1).
// The in-process simulation launches every rank's job as blockIdx.y of ONE grid,
// so all simulated ranks are co-resident by construction.
struct Job {
  const void* in;
  void* out;
  int rank;
  int* err;
  uint64_t timeout;  // spin bound in s_memrealtime ticks (100 MHz)
  int partner;       // pair collectives (modes 5, 6): the other rank of the pair
};
struct Jobs {
  Job j[kMaxRanks];
};

ST_DEVICE uint32_t* flag_ptr(char* base, int phase, int block, int rank) {
  return reinterpret_cast<uint32_t*>(base) + ((phase * kMaxBlocks + block) * kMaxRanks + rank);
}

// Per-block cross-rank barrier: tell every peer "my block b reached phase p of
// epoch e", then wait until every peer told me the same.  Returns false on timeout.
ST_DEVICE bool block_barrier(const Peers& P, int rank, int world, int phase, uint32_t epoch, int* err,
                             uint64_t timeout) {
  // Every wave retires its own data stores first: __syncthreads() is only a
  // workgroup-scope fence and does NOT wait for global stores to complete, and the
  // flag thread's system release below only covers its own wave's stores.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bool ok = true;
  if (threadIdx.x < (unsigned)world) {
    __threadfence_system();
    __hip_atomic_store(flag_ptr(P.buf[threadIdx.x], phase, blockIdx.x, rank), epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = flag_ptr(P.buf[rank], phase, blockIdx.x, threadIdx.x);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {  // default 2 s at 100 MHz
        atomicExch(err, 1);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  // every wave acquires (invalidates its CU's vector L1 / non-coherent L2 lines)
  // before reading what the peers published
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return ok;
}

// The same handshake between the two ranks of a pair only (flags in each other's header).
ST_DEVICE bool pair_barrier(const Peers& P, int rank, int partner, int phase, uint32_t epoch, int* err,
                            uint64_t timeout) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(flag_ptr(P.buf[partner], phase, blockIdx.x, rank), epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = flag_ptr(P.buf[rank], phase, blockIdx.x, partner);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
        atomicExch(err, 1);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return ok;
}

// ---- shared-area access: 16 B per lane through a buffer descriptor with the
// system-coherence bits (sc0 sc1) on EVERY load and store, so no XCD's L2 (and
// no CU's L1) serves or keeps a stale copy of another rank's bytes -- neither
// within one GPU (XCD L2s are not coherent with each other) nor across xGMI.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr int kSys = 1 | 16;  // cache policy: sc0 | sc1

ST_DEVICE rsrc_t buf_rsrc(const char* base, int64_t cap) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)(uint32_t)(kHeader + 4 * cap), 0x00020000);
}
ST_DEVICE u32x4 sh_load(rsrc_t rs, uint32_t off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kSys));
}
ST_DEVICE void sh_store(rsrc_t rs, uint32_t off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, off, 0, kSys);
}
// byte offset of 8-element vector v of area (which, parity)
template <typename T>
ST_DEVICE uint32_t area_off(int which, int parity, int64_t cap, int64_t v) {
  return (uint32_t)(kHeader + (int64_t)(which * 2 + parity) * cap + v * 8 * (int64_t)sizeof(T));
}

// 8 elements <-> fp32 (T = bf16: one 16-B vector; T = fp32: two)
template <typename T>
ST_DEVICE void sh_load8(rsrc_t rs, uint32_t off, float (&f)[8]) {
  if constexpr (sizeof(T) == 2) {
    const u32x4 v = sh_load(rs, off);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __uint_as_float(v[i] << 16);
      f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
    }
  } else {
    const u32x4 a = sh_load(rs, off), b = sh_load(rs, off + 16);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[i] = __uint_as_float(a[i]);
      f[4 + i] = __uint_as_float(b[i]);
    }
  }
}
template <typename T>
ST_DEVICE void sh_store8(rsrc_t rs, uint32_t off, const float (&f)[8]) {
  if constexpr (sizeof(T) == 2) {
    u32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
    sh_store(rs, off, v);
  } else {
    u32x4 a, b;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i] = __float_as_uint(f[i]);
      b[i] = __float_as_uint(f[4 + i]);
    }
    sh_store(rs, off, a);
    sh_store(rs, off + 16, b);
  }
}
// plain local tensor -> shared area (raw bytes)
template <typename T>
ST_DEVICE void put8(rsrc_t rs, uint32_t off, const T* src) {
  const u32x4* p = reinterpret_cast<const u32x4*>(src);
  sh_store(rs, off, p[0]);
  if constexpr (sizeof(T) == 4) sh_store(rs, off + 16, p[1]);
}
// shared area -> plain local tensor (raw bytes)
template <typename T>
ST_DEVICE void get8(rsrc_t rs, uint32_t off, T* dst) {
  u32x4* p = reinterpret_cast<u32x4*>(dst);
  p[0] = sh_load(rs, off);
  if constexpr (sizeof(T) == 4) p[1] = sh_load(rs, off + 16);
}
template <typename T>
ST_DEVICE void store_local8(T* p, const float (&f)[8]) {
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<BF8*>(p) = pack8(f);
  } else {
    reinterpret_cast<float4*>(p)[0] = make_float4(f[0], f[1], f[2], f[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(f[4], f[5], f[6], f[7]);
  }
}

// n8: number of 8-element vectors.  One-shot: block b owns vectors [lo, hi).
template <typename T>
__global__ __launch_bounds__(kThreads) void oneshot_kernel(Peers P, Jobs J, int world, int64_t n8, int64_t cap,
                                                           uint32_t epoch) {
  const Job& jb = J.j[blockIdx.y];
  const int rank = jb.rank;
  const T* __restrict__ in = (const T*)jb.in;
  T* __restrict__ out = (T*)jb.out;
  int* err = jb.err;
  const int parity = epoch & 1;
  const int64_t per = (n8 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = blockIdx.x * per, hi = min(n8, lo + per);
  const rsrc_t mine = buf_rsrc(P.buf[rank], cap);
  for (int64_t v = lo + threadIdx.x; v < hi; v += blockDim.x) put8<T>(mine, area_off<T>(0, parity, cap, v), in + v * 8);
  if (!block_barrier(P, rank, world, 0, epoch, err, jb.timeout)) return;
  for (int64_t v = lo + threadIdx.x; v < hi; v += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < world; ++r) {  // fixed rank order: bitwise identical on every rank
      float f[8];
      sh_load8<T>(buf_rsrc(P.buf[r], cap), area_off<T>(0, parity, cap, v), f);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += f[i];
    }
    store_local8<T>(out + v * 8, acc);
  }
}

// Two-shot: partition p = vectors [p*P8, (p+1)*P8); block b owns slice b of every partition.
template <typename T>
__global__ __launch_bounds__(kThreads) void twoshot_kernel(Peers P, Jobs J, int world, int64_t n8, int64_t cap,
                                                           uint32_t epoch) {
  const Job& jb = J.j[blockIdx.y];
  const int rank = jb.rank;
  const T* __restrict__ in = (const T*)jb.in;
  T* __restrict__ out = (T*)jb.out;
  int* err = jb.err;
  const int parity = epoch & 1;
  const int64_t P8 = (n8 + world - 1) / world;
  const int64_t per = (P8 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = blockIdx.x * per, hi = min(P8, lo + per);
  const rsrc_t mine = buf_rsrc(P.buf[rank], cap);
  for (int p = 0; p < world; ++p) {
    const int64_t e = min(n8, (p + 1) * P8);
    for (int64_t v = p * P8 + lo + threadIdx.x; v < min(e, p * P8 + hi); v += blockDim.x)
      put8<T>(mine, area_off<T>(0, parity, cap, v), in + v * 8);
  }
  if (!block_barrier(P, rank, world, 0, epoch, err, jb.timeout)) return;
  // reduce-scatter: my partition, my slice
  const int64_t pe = min(n8, (rank + 1) * P8);
  for (int64_t v = rank * P8 + lo + threadIdx.x; v < min(pe, rank * P8 + hi); v += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < world; ++r) {
      float f[8];
      sh_load8<T>(buf_rsrc(P.buf[r], cap), area_off<T>(0, parity, cap, v), f);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += f[i];
    }
    sh_store8<T>(mine, area_off<T>(1, parity, cap, v), acc);
  }
  if (!block_barrier(P, rank, world, 1, epoch, err, jb.timeout)) return;
  // all-gather: partition p from rank p's result area
  for (int p = 0; p < world; ++p) {
    const rsrc_t src = buf_rsrc(P.buf[p], cap);
    const int64_t e = min(n8, (p + 1) * P8);
    for (int64_t v = p * P8 + lo + threadIdx.x; v < min(e, p * P8 + hi); v += blockDim.x)
      get8<T>(src, area_off<T>(1, parity, cap, v), out + v * 8);
  }
}

// All-gather: every rank contributes n8 vectors; out = [rank 0 | rank 1 | ...] (n8 each).
// Block b owns slice b of the contribution; after the handshake it copies slice b
// of every peer's contribution over xGMI (all W-1 links busy at once).
template <typename T>
__global__ __launch_bounds__(kThreads) void allgather_kernel(Peers P, Jobs J, int world, int64_t n8, int64_t cap,
                                                             uint32_t epoch) {
  const Job& jb = J.j[blockIdx.y];
  const int rank = jb.rank;
  const T* __restrict__ in = (const T*)jb.in;
  T* __restrict__ out = (T*)jb.out;
  const int parity = epoch & 1;
  const int64_t per = (n8 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = blockIdx.x * per, hi = min(n8, lo + per);
  const rsrc_t mine = buf_rsrc(P.buf[rank], cap);
  for (int64_t v = lo + threadIdx.x; v < hi; v += blockDim.x) put8<T>(mine, area_off<T>(0, parity, cap, v), in + v * 8);
  if (!block_barrier(P, rank, world, 0, epoch, jb.err, jb.timeout)) return;
  for (int r = 0; r < world; ++r) {
    const rsrc_t src = buf_rsrc(P.buf[r], cap);
    for (int64_t v = lo + threadIdx.x; v < hi; v += blockDim.x)
      get8<T>(src, area_off<T>(0, parity, cap, v), out + ((int64_t)r * n8 + v) * 8);
  }
}

// Reduce-scatter: every rank contributes W * n8 vectors; rank r keeps the fp32 sum
// (fixed rank order) of partition r = vectors [r n8, (r+1) n8) -> out (n8 vectors).
template <typename T>
__global__ __launch_bounds__(kThreads) void reducescatter_kernel(Peers P, Jobs J, int world, int64_t n8,
                                                                 int64_t cap, uint32_t epoch) {
  const Job& jb = J.j[blockIdx.y];
  const int rank = jb.rank;
  const T* __restrict__ in = (const T*)jb.in;
  T* __restrict__ out = (T*)jb.out;
  const int parity = epoch & 1;
  const int64_t per = (n8 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = blockIdx.x * per, hi = min(n8, lo + per);
  const rsrc_t mine = buf_rsrc(P.buf[rank], cap);
  for (int p = 0; p < world; ++p)
    for (int64_t v = lo + threadIdx.x; v < hi; v += blockDim.x)
      put8<T>(mine, area_off<T>(0, parity, cap, (int64_t)p * n8 + v), in + ((int64_t)p * n8 + v) * 8);
  if (!block_barrier(P, rank, world, 0, epoch, jb.err, jb.timeout)) return;
  for (int64_t v = lo + threadIdx.x; v < hi; v += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < world; ++r) {
      float f[8];
      sh_load8<T>(buf_rsrc(P.buf[r], cap), area_off<T>(0, parity, cap, (int64_t)rank * n8 + v), f);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += f[i];
    }
    store_local8<T>(out + v * 8, acc);
  }
}

// All-to-all (equal splits): every rank contributes W chunks of n8 vectors (chunk d for
// rank d); out = [from rank 0 | from rank 1 | ...].  PUSH: block b writes slice b of
// chunk d straight into rank d's area at slot [my rank] over the d-link (all W-1 links
// busy at once, posted writes), then the per-block handshake, then every rank copies
// its own area out.  The EP token dispatch / combine and the Ulysses head exchange.
template <typename T>
__global__ __launch_bounds__(kThreads) void alltoall_kernel(Peers P, Jobs J, int world, int64_t n8, int64_t cap,
                                                            uint32_t epoch) {
  const Job& jb = J.j[blockIdx.y];
  const int rank = jb.rank;
  const T* __restrict__ in = (const T*)jb.in;
  T* __restrict__ out = (T*)jb.out;
  const int parity = epoch & 1;
  const int64_t per = (n8 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = blockIdx.x * per, hi = min(n8, lo + per);
  for (int i = 0; i < world; ++i) {
    const int d = (rank + i) % world;  // start with a different peer on every rank: spread the links
    const rsrc_t dst = buf_rsrc(P.buf[d], cap);
    for (int64_t v = lo + threadIdx.x; v < hi; v += blockDim.x)
      put8<T>(dst, area_off<T>(0, parity, cap, (int64_t)rank * n8 + v), in + ((int64_t)d * n8 + v) * 8);
  }
  if (!block_barrier(P, rank, world, 0, epoch, jb.err, jb.timeout)) return;
  const rsrc_t mine = buf_rsrc(P.buf[rank], cap);
  for (int r = 0; r < world; ++r)
    for (int64_t v = lo + threadIdx.x; v < hi; v += blockDim.x)
      get8<T>(mine, area_off<T>(0, parity, cap, (int64_t)r * n8 + v), out + ((int64_t)r * n8 + v) * 8);
}

// ---- pair collectives over MULTIPLE paths (a 2-rank TP group on one node has ONE direct
// xGMI link; the other W-2 GPUs' links are idle for it).  Block b's slice takes path
// b % (1 + nrelay): path 0 = written straight into the partner's area over the direct
// link, path i = written into relay R[i-1]'s memory (slot [my rank]) and read from there
// by the partner -- two hops, through links the direct path does not use.  The relay GPU
// runs nothing: its memory is only a staging area.  Relays = every other rank, in rank
// order (both partners agree).  Only the pair synchronises (flags in each other's
// header); relay slots are disjoint per source rank.
ST_DEVICE int relay_of(int i, int rank, int partner) {  // i-th rank that is neither
  const int lo = min(rank, partner), hi = max(rank, partner);
  int r = i;
  if (r >= lo) ++r;
  if (r >= hi) ++r;
  return r;
}

// where block b's slice of `src`'s message lives after the write: (buffer rank, byte offset)
template <typename T>
ST_DEVICE void pair_loc(int world, int src, int dst, int64_t per, int64_t cap, int parity, int& owner,
                        uint32_t& base) {
  const int npath = world - 1;  // direct + (world - 2) relays
  const int path = blockIdx.x % npath;
  if (path == 0) {
    owner = dst;
    base = area_off<T>(0, parity, cap, (int64_t)blockIdx.x * per);
  } else {
    owner = relay_of(path - 1, src, dst);
    const int64_t slot = cap / kMaxRanks;  // bytes per source rank in a relay's area 1
    const int64_t lb = blockIdx.x / npath;  // compacted block index on this path
    base = (uint32_t)(kHeader + (int64_t)(2 + parity) * cap + (int64_t)src * slot +
                      lb * per * 8 * (int64_t)sizeof(T));
  }
}

// Pair all-gather: each of the two ranks contributes n8 vectors; out = [lower rank's |
// higher rank's].
template <typename T>
__global__ __launch_bounds__(kThreads) void pair_allgather_kernel(Peers P, Jobs J, int world, int64_t n8,
                                                                  int64_t cap, uint32_t epoch) {
  const Job& jb = J.j[blockIdx.y];
  const int rank = jb.rank, partner = jb.partner;
  const T* __restrict__ in = (const T*)jb.in;
  T* __restrict__ out = (T*)jb.out;
  const int parity = epoch & 1;
  const int64_t per = (n8 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = blockIdx.x * per, hi = min(n8, lo + per);
  const int me = rank < partner ? 0 : 1;
  int owner;
  uint32_t base;
  pair_loc<T>(world, rank, partner, per, cap, parity, owner, base);  // where my slice goes
  const rsrc_t dst = buf_rsrc(P.buf[owner], cap);
  for (int64_t v = lo + threadIdx.x; v < hi; v += blockDim.x) {
    put8<T>(dst, base + (uint32_t)((v - lo) * 8 * sizeof(T)), in + v * 8);
    *reinterpret_cast<u32x4*>(out + ((int64_t)me * n8 + v) * 8) = *reinterpret_cast<const u32x4*>(in + v * 8);
    if constexpr (sizeof(T) == 4)
      *reinterpret_cast<u32x4*>(out + ((int64_t)me * n8 + v) * 8 + 4) = *reinterpret_cast<const u32x4*>(in + v * 8 + 4);
  }
  if (!pair_barrier(P, rank, partner, 0, epoch, jb.err, jb.timeout)) return;
  pair_loc<T>(world, partner, rank, per, cap, parity, owner, base);  // where the partner's slice is
  const rsrc_t src = buf_rsrc(P.buf[owner], cap);
  for (int64_t v = lo + threadIdx.x; v < hi; v += blockDim.x)
    get8<T>(src, base + (uint32_t)((v - lo) * 8 * sizeof(T)), out + ((int64_t)(1 - me) * n8 + v) * 8);
}

// Pair reduce-scatter: each rank contributes 2 x n8 vectors ([chunk of the lower rank |
// chunk of the higher rank]); out = the sum of both ranks' chunk for me (fp32, lower
// rank's term first: bitwise the same on both).
template <typename T>
__global__ __launch_bounds__(kThreads) void pair_reducescatter_kernel(Peers P, Jobs J, int world, int64_t n8,
                                                                      int64_t cap, uint32_t epoch) {
  const Job& jb = J.j[blockIdx.y];
  const int rank = jb.rank, partner = jb.partner;
  const T* __restrict__ in = (const T*)jb.in;
  T* __restrict__ out = (T*)jb.out;
  const int parity = epoch & 1;
  const int64_t per = (n8 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = blockIdx.x * per, hi = min(n8, lo + per);
  const int me = rank < partner ? 0 : 1;
  int owner;
  uint32_t base;
  pair_loc<T>(world, rank, partner, per, cap, parity, owner, base);  // the partner's chunk goes out
  const rsrc_t dst = buf_rsrc(P.buf[owner], cap);
  for (int64_t v = lo + threadIdx.x; v < hi; v += blockDim.x)
    put8<T>(dst, base + (uint32_t)((v - lo) * 8 * sizeof(T)), in + ((int64_t)(1 - me) * n8 + v) * 8);
  if (!pair_barrier(P, rank, partner, 0, epoch, jb.err, jb.timeout)) return;
  pair_loc<T>(world, partner, rank, per, cap, parity, owner, base);
  const rsrc_t src = buf_rsrc(P.buf[owner], cap);
  for (int64_t v = lo + threadIdx.x; v < hi; v += blockDim.x) {
    float a[8], b[8];
    sh_load8<T>(src, base + (uint32_t)((v - lo) * 8 * sizeof(T)), b);  // partner's term
    const T* mine = in + ((int64_t)me * n8 + v) * 8;
    if constexpr (sizeof(T) == 2) {
      BF8 x = *reinterpret_cast<const BF8*>(mine);
      unpack8(x, a);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = mine[i];
    }
    float s[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = me == 0 ? a[i] + b[i] : b[i] + a[i];
    store_local8<T>(out + v * 8, s);
  }
}


// ---- expert-parallel token exchange with DEVICE-SIDE counts (dropless, no host sync).
// M[s][g] = rows source rank s routes to global expert g (identical on every rank: the
// [E] count rows are all-gathered first).  Source s holds its rows sorted by global
// expert ("sorted" layout, P[s][g] = first row of expert g); owner d = g / El holds its
// local experts' rows EXPERT-MAJOR: expert g's rows = [from source 0 | source 1 | ...],
// i.e. row (s, i) of expert g sits at q(s, i) = EO[g] + SO[s][g] + (i - P[s][g]) with
// EO[g] = rows of the owner's earlier experts, SO[s][g] = rows of g from sources < s.
// dir 0 (dispatch): sorted rows of every source -> expert-major rows of every owner.
// dir 1 (combine): the reverse.  Block b of every rank moves the rows of block b of each
// SOURCE's sorted range (a fixed split of that source's rows), so after the per-block
// handshake block b reads exactly what the peers' block b wrote.  Every index is checked
// against the area / output sizes the host passed: a count that would overflow sets
// the error word (2) and is skipped, never written out of bounds.
constexpr int kMaxExperts = 256;
struct EpArgs {
  const int* M;      // [world, E] int32, device
  int E, El, row8, dir;
  int64_t in_rows;    // rows of `in`
  int64_t out_rows;   // rows of `out`
  int64_t area_rows;  // rows one data area holds
};

ST_DEVICE int ep_find(const int* Ps, int E, int i) {  // g with Ps[g] <= i < Ps[g + 1]
  int lo = 0, hi = E - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (Ps[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void ep_exchange_kernel(Peers P, Jobs J, int world, EpArgs A, int64_t cap,
                                                               uint32_t epoch) {
  __shared__ int sP[kMaxRanks][kMaxExperts + 1];
  __shared__ int sSO[kMaxRanks][kMaxExperts];
  __shared__ int sEO[kMaxExperts];
  const Job& jb = J.j[blockIdx.y];
  const int me = jb.rank;
  const T* __restrict__ in = (const T*)jb.in;
  T* __restrict__ out = (T*)jb.out;
  const int parity = epoch & 1;
  const int E = A.E, El = A.El, row8 = A.row8;
  for (int x = threadIdx.x; x < world * E; x += blockDim.x) sSO[x / E][x % E] = max(0, A.M[x]);
  __syncthreads();
  if (threadIdx.x < (unsigned)world) {  // P: per-source prefix over experts
    const int s = threadIdx.x;
    int acc = 0;
    for (int g = 0; g < E; ++g) {
      sP[s][g] = acc;
      acc += sSO[s][g];
    }
    sP[s][E] = acc;
  }
  __syncthreads();
  for (int g = threadIdx.x; g < E; g += blockDim.x) {  // SO: per-expert prefix over sources
    int acc = 0;
    for (int s = 0; s < world; ++s) {
      const int m = sSO[s][g];
      sSO[s][g] = acc;
      acc += m;
    }
    sEO[g] = acc;  // total rows of expert g (turned into EO below)
  }
  __syncthreads();
  if (threadIdx.x < (unsigned)world) {  // EO: per-owner prefix over its local experts
    const int d = threadIdx.x;
    int acc = 0;
    for (int e = 0; e < El; ++e) {
      const int tot = sEO[d * El + e];
      sEO[d * El + e] = acc;
      acc += tot;
    }
  }
  __syncthreads();
  const int64_t rowb = (int64_t)row8;  // 8-element vectors per row
  // block b's share of source s's sorted rows
  auto range = [&](int s, int64_t& lo, int64_t& hi) {
    const int64_t Ts = sP[s][E];
    const int64_t per = (Ts + gridDim.x - 1) / gridDim.x;
    lo = min(Ts, (int64_t)blockIdx.x * per);
    hi = min(Ts, lo + per);
  };
  auto qpos = [&](int s, int64_t i, int g) -> int64_t { return (int64_t)sEO[g] + sSO[s][g] + (i - sP[s][g]); };
  const rsrc_t mine = buf_rsrc(P.buf[me], cap);
  if (A.dir == 0) {
    // phase 1, as a source: push my block's sorted rows to their owners' areas (expert-major
    // slots), owner by owner -- the buffer descriptor of the destination must be
    // wave-uniform (buf_rsrc reads the base from lane 0), so one pass per owner
    int64_t lo, hi;
    range(me, lo, hi);
    for (int d = 0; d < world; ++d) {
      const int64_t a = max(lo, (int64_t)sP[me][d * El]), z = min(hi, (int64_t)sP[me][(d + 1) * El]);
      if (z <= a) continue;  // uniform: a, z come from LDS tables and block-uniform bounds
      const rsrc_t dst = buf_rsrc(P.buf[d], cap);
      for (int64_t v = threadIdx.x; v < (z - a) * rowb; v += blockDim.x) {
        const int64_t i = a + v / rowb, c = v % rowb;
        const int64_t q = qpos(me, i, ep_find(sP[me], E, (int)i));
        if (q >= A.area_rows || i >= A.in_rows) {
          atomicExch(jb.err, 2);
          continue;
        }
        put8<T>(dst, area_off<T>(0, parity, cap, q * rowb + c), in + (i * rowb + c) * 8);
      }
    }
    if (!block_barrier(P, me, world, 0, epoch, jb.err, jb.timeout)) return;
    // phase 2, as the owner: copy out the rows block b of every source wrote into my area
    for (int s = 0; s < world; ++s) {
      int64_t a, z;
      range(s, a, z);
      a = max(a, (int64_t)sP[s][me * El]);
      z = min(z, (int64_t)sP[s][(me + 1) * El]);
      for (int64_t v = threadIdx.x; v < max((int64_t)0, z - a) * rowb; v += blockDim.x) {
        const int64_t i = a + v / rowb, c = v % rowb;
        const int64_t q = qpos(s, i, ep_find(sP[s], E, (int)i));
        if (q >= A.out_rows || q >= A.area_rows) {
          atomicExch(jb.err, 2);
          continue;
        }
        get8<T>(mine, area_off<T>(0, parity, cap, q * rowb + c), out + (q * rowb + c) * 8);
      }
    }
  } else {
    // phase 1, as the owner: send every source its rows of my experts (expert-major in -> its sorted slots)
    for (int s = 0; s < world; ++s) {
      int64_t a, z;
      range(s, a, z);
      a = max(a, (int64_t)sP[s][me * El]);
      z = min(z, (int64_t)sP[s][(me + 1) * El]);
      const rsrc_t dst = buf_rsrc(P.buf[s], cap);
      for (int64_t v = threadIdx.x; v < max((int64_t)0, z - a) * rowb; v += blockDim.x) {
        const int64_t i = a + v / rowb, c = v % rowb;
        const int64_t q = qpos(s, i, ep_find(sP[s], E, (int)i));
        if (i >= A.area_rows || q >= A.in_rows) {
          atomicExch(jb.err, 2);
          continue;
        }
        put8<T>(dst, area_off<T>(0, parity, cap, i * rowb + c), in + (q * rowb + c) * 8);
      }
    }
    if (!block_barrier(P, me, world, 0, epoch, jb.err, jb.timeout)) return;
    // phase 2, as a source: my block's sorted rows have arrived in my area
    int64_t lo, hi;
    range(me, lo, hi);
    for (int64_t v = threadIdx.x; v < (hi - lo) * rowb; v += blockDim.x) {
      const int64_t i = lo + v / rowb, c = v % rowb;
      if (i >= A.out_rows || i >= A.area_rows) {
        atomicExch(jb.err, 2);
        continue;
      }
      get8<T>(mine, area_off<T>(0, parity, cap, i * rowb + c), out + (i * rowb + c) * 8);
    }
  }
}

struct Comm {
  int rank = 0, world = 1;
  int64_t cap = 0;  // bytes per data area
  char* local = nullptr;
  Peers peers{};
  bool opened[kMaxRanks] = {};
  int* err = nullptr;
  uint32_t epoch = 0;
  int device = 0;
  uint64_t timeout = 200000000ull;  // 2 s of s_memrealtime ticks
};

// mode: 0 one-shot all-reduce, 1 two-shot all-reduce, 2 all-gather, 3 reduce-scatter,
// 4 all-to-all, 5 pair all-gather, 6 pair reduce-scatter.
// n = elements of the per-rank CONTRIBUTION (all-gather, pair all-gather) / of the OUTPUT
// (reduce-scatter, pair reduce-scatter) / of one chunk (all-to-all) / of the tensor (all-reduce).
template <typename T>
static void launch_t(const Peers& P, const Jobs& J, dim3 grid, int world, int64_t n8, int64_t cap, int mode,
                     uint32_t epoch, hipStream_t st) {
  switch (mode) {
    case 0: oneshot_kernel<T><<<grid, kThreads, 0, st>>>(P, J, world, n8, cap, epoch); break;
    case 1: twoshot_kernel<T><<<grid, kThreads, 0, st>>>(P, J, world, n8, cap, epoch); break;
    case 2: allgather_kernel<T><<<grid, kThreads, 0, st>>>(P, J, world, n8, cap, epoch); break;
    case 3: reducescatter_kernel<T><<<grid, kThreads, 0, st>>>(P, J, world, n8, cap, epoch); break;
    case 4: alltoall_kernel<T><<<grid, kThreads, 0, st>>>(P, J, world, n8, cap, epoch); break;
    case 5: pair_allgather_kernel<T><<<grid, kThreads, 0, st>>>(P, J, world, n8, cap, epoch); break;
    default: pair_reducescatter_kernel<T><<<grid, kThreads, 0, st>>>(P, J, world, n8, cap, epoch); break;
  }
}


std::mutex g_mu;
std::vector<Comm*> g_comms;

Comm* get(int64_t id) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (id < 0 || id >= (int64_t)g_comms.size()) return nullptr;
  return g_comms[id];
}

}  // namespace

extern "C" {

int st_xgmi_header_bytes() { return (int)kHeader; }
int st_xgmi_max_ranks() { return kMaxRanks; }

// Allocate this rank's shared buffer (header + 4 data areas of `cap` bytes) on
// the current device; returns an id >= 0 or a negative hip error.
// `epoch_base`: first epoch - 1.  Must be identical on every rank of the group and
// larger than any epoch an earlier communicator reached, so a flag word left over
// at a reused address (or seen through a stale cache line) can never satisfy a
// new communicator's wait (dist/xgmi.py passes (creation serial) << 24).
int64_t st_xgmi_create(int rank, int world, int64_t cap, int64_t epoch_base) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || cap <= 0 || cap % 256) return -2;
  if (kHeader + 4 * cap >= ((int64_t)1 << 32)) return -2;  // 32-bit buffer offsets
  Comm* c = new Comm();
  c->rank = rank;
  c->world = world;
  c->cap = cap;
  c->epoch = (uint32_t)epoch_base;
  (void)hipGetDevice(&c->device);
  const int64_t bytes = kHeader + 4 * cap;
  hipError_t e = hipMalloc((void**)&c->local, bytes);
  if (e != hipSuccess) {
    delete c;
    return -(int64_t)e;
  }
  (void)hipMemset(c->local, 0xff, kHeader + 4 * cap);  // data areas poisoned (NaN): a stale read cannot pass
  (void)hipMemset(c->local, 0, kHeader);
  (void)hipDeviceSynchronize();
  hipMalloc((void**)&c->err, sizeof(int));
  hipMemset(c->err, 0, sizeof(int));
  hipDeviceSynchronize();
  c->peers.buf[rank] = c->local;
  c->opened[rank] = false;
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(c);
  return (int64_t)g_comms.size() - 1;
}

// 64-byte IPC handle of this rank's buffer.
int st_xgmi_handle(int64_t id, void* out64) {
  Comm* c = get(id);
  if (!c) return -2;
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, c->local);
  if (e != hipSuccess) return (int)e;
  static_assert(sizeof(h) <= 64, "ipc handle size");
  std::memset(out64, 0, 64);
  std::memcpy(out64, &h, sizeof(h));
  return 0;
}

// Map peer r's buffer from its IPC handle (not for r == own rank).
int st_xgmi_open(int64_t id, int r, const void* handle64) {
  Comm* c = get(id);
  if (!c || r < 0 || r >= c->world || r == c->rank) return -2;
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle64, sizeof(h));
  void* p = nullptr;
  hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) return (int)e;
  c->peers.buf[r] = (char*)p;
  c->opened[r] = true;
  return 0;
}

// Same-process wiring (tests / single-process multi-stream simulation): peer r's
// buffer is comm `peer_id`'s local buffer.
int st_xgmi_set_peer(int64_t id, int r, int64_t peer_id) {
  Comm* c = get(id);
  Comm* p = get(peer_id);
  if (!c || !p || r < 0 || r >= c->world) return -2;
  c->peers.buf[r] = p->local;
  return 0;
}

static int launch(const Peers& P, const Jobs& J, int njobs, int world, int64_t n, int64_t cap, int dtype,
                  int mode, int blocks, uint32_t epoch, hipStream_t st) {
  const dim3 grid(blocks, njobs);
  if (dtype == 0) launch_t<bf16_t>(P, J, grid, world, n / 8, cap, mode, epoch, st);
  else launch_t<float>(P, J, grid, world, n / 8, cap, mode, epoch, st);
  return (int)hipGetLastError();
}

// bytes of one data area a collective of n elements needs on each rank
static int64_t area_bytes(int mode, int world, int64_t n, int64_t elt) {
  if (mode == 3 || mode == 4) return (int64_t)world * n * elt;
  if (mode == 5 || mode == 6) return n * elt * kMaxRanks;  // a relay slot (cap / 8) must hold a path's share
  return n * elt;
}

// Collective of n elements (dtype 0 = bf16, 1 = fp32); mode 0 = one-shot all-reduce,
// 1 = two-shot all-reduce (in place allowed), 2 = all-gather (n per rank, out holds
// world * n), 3 = reduce-scatter (in holds world * n, out n).  n must be a multiple
// of 8 and fit the data area (cap bytes).
int st_xgmi_all_reduce(int64_t id, const void* in, void* out, int64_t n, int dtype, int mode, int blocks,
                       hipStream_t st) {
  Comm* c = get(id);
  if (!c || mode < 0 || mode > 4) return -2;
  const int64_t elt = dtype == 0 ? 2 : 4;
  if (n % 8 || area_bytes(mode, c->world, n, elt) > c->cap || ((uintptr_t)in | (uintptr_t)out) % 16) return -2;
  for (int r = 0; r < c->world; ++r)
    if (!c->peers.buf[r]) return -3;
  if (n == 0) return 0;
  if (blocks <= 0 || blocks > kMaxBlocks) blocks = kMaxBlocks;
  Jobs J{};
  J.j[0] = Job{in, out, c->rank, c->err, c->timeout};
  return launch(c->peers, J, 1, c->world, n, c->cap, dtype, mode, blocks, ++c->epoch, st);
}

// Pair collective (mode 5 all-gather / 6 reduce-scatter) between this rank and `partner`
// over the direct link plus 2-hop paths through every other rank's memory.  Both
// partners must call it in the same order; the other ranks need not call anything.
int st_xgmi_pair(int64_t id, const void* in, void* out, int64_t n, int dtype, int mode, int partner, int blocks,
                 hipStream_t st) {
  Comm* c = get(id);
  if (!c || (mode != 5 && mode != 6) || partner < 0 || partner >= c->world || partner == c->rank) return -2;
  const int64_t elt = dtype == 0 ? 2 : 4;
  if (n % 8 || area_bytes(mode, c->world, n, elt) > c->cap || ((uintptr_t)in | (uintptr_t)out) % 16) return -2;
  for (int r = 0; r < c->world; ++r)
    if (!c->peers.buf[r]) return -3;
  if (n == 0) return 0;
  if (blocks <= 0 || blocks > kMaxBlocks) blocks = kMaxBlocks;
  Jobs J{};
  J.j[0] = Job{in, out, c->rank, c->err, c->timeout, partner};
  return launch(c->peers, J, 1, c->world, n, c->cap, dtype, mode, blocks, ++c->epoch, st);
}


// Expert-parallel exchange (dispatch dir 0 / combine dir 1) with device counts M
// ([world, E] int32, the same tensor content on every rank); rows of row_elems
// elements; `in_rows` / `out_rows` = rows of in / out (every rank's, in the simulation); `area_rows_needed` = the most
// rows one data area must hold (host bound: dispatch R_max, combine this rank's rows).
int st_xgmi_ep_exchange(int64_t id, const void* in, void* out, const int* M, int E, int El, int64_t row_elems,
                        int64_t in_rows, int64_t out_rows, int64_t area_rows_needed, int dtype, int dir, int blocks,
                        hipStream_t st) {
  Comm* c = get(id);
  if (!c || E < 1 || E > kMaxExperts || El < 1 || E != El * c->world || row_elems % 8 || (dir != 0 && dir != 1))
    return -2;
  const int64_t elt = dtype == 0 ? 2 : 4;
  const int64_t rowbytes = row_elems * elt;
  if (area_rows_needed * rowbytes > c->cap || ((uintptr_t)in | (uintptr_t)out) % 16) return -2;
  for (int r = 0; r < c->world; ++r)
    if (!c->peers.buf[r]) return -3;
  if (blocks <= 0 || blocks > kMaxBlocks) blocks = kMaxBlocks;
  Jobs J{};
  J.j[0] = Job{in, out, c->rank, c->err, c->timeout};
  EpArgs A{M, E, El, (int)(row_elems / 8), dir, in_rows, out_rows, c->cap / rowbytes};
  const dim3 grid(blocks, 1);
  const uint32_t epoch = ++c->epoch;
  if (dtype == 0) ep_exchange_kernel<bf16_t><<<grid, kThreads, 0, st>>>(c->peers, J, c->world, A, c->cap, epoch);
  else ep_exchange_kernel<float><<<grid, kThreads, 0, st>>>(c->peers, J, c->world, A, c->cap, epoch);
  return (int)hipGetLastError();
}

// Simulation of the exchange across ids[0..world) in ONE launch (rank = blockIdx.y).
int st_xgmi_ep_exchange_sim(const int64_t* ids, const void* const* ins, void* const* outs, const int* M, int world,
                            int E, int El, int64_t row_elems, int64_t in_rows, int64_t out_rows,
                            int64_t area_rows_needed, int dtype, int dir, int blocks, hipStream_t st) {
  if (world < 1 || world > kMaxRanks || E < 1 || E > kMaxExperts || El < 1 || E != El * world || row_elems % 8 ||
      (dir != 0 && dir != 1))
    return -2;
  Comm* c0 = get(ids[0]);
  if (!c0 || c0->world != world) return -2;
  const int64_t elt = dtype == 0 ? 2 : 4;
  const int64_t rowbytes = row_elems * elt;
  if (area_rows_needed * rowbytes > c0->cap) return -2;
  if (blocks <= 0 || blocks > kMaxBlocks) blocks = kMaxBlocks;
  Jobs J{};
  uint32_t epoch = 0;
  for (int r = 0; r < world; ++r) {
    Comm* c = get(ids[r]);
    if (!c || c->rank != r || c->world != world || c->cap != c0->cap) return -2;
    if (((uintptr_t)ins[r] | (uintptr_t)outs[r]) % 16) return -2;
    J.j[r] = Job{ins[r], outs[r], r, c->err, c->timeout};
    epoch = ++c->epoch;
  }
  EpArgs A{M, E, El, (int)(row_elems / 8), dir, in_rows, out_rows, c0->cap / rowbytes};
  const dim3 grid(blocks, world);
  if (dtype == 0) ep_exchange_kernel<bf16_t><<<grid, kThreads, 0, st>>>(c0->peers, J, world, A, c0->cap, epoch);
  else ep_exchange_kernel<float><<<grid, kThreads, 0, st>>>(c0->peers, J, world, A, c0->cap, epoch);
  return (int)hipGetLastError();
}

int st_xgmi_world(int64_t id) {
  Comm* c = get(id);
  return c ? c->world : -2;
}

// Bound (seconds) on every cross-rank wait of this communicator's kernels.
int st_xgmi_set_timeout(int64_t id, double seconds) {
  Comm* c = get(id);
  if (!c || !(seconds > 0)) return -2;
  c->timeout = (uint64_t)(seconds * 1e8);
  return 0;
}

// Simulation: comms ids[0..world) (wired with st_xgmi_set_peer, one process)
// all-reduce ins[r] -> outs[r] in ONE launch (rank r = blockIdx.y).
int st_xgmi_collective_sim(const int64_t* ids, const void* const* ins, void* const* outs, const int* partners,
                           int world, int64_t n, int dtype, int mode, int blocks, hipStream_t st);

int st_xgmi_all_reduce_sim(const int64_t* ids, const void* const* ins, void* const* outs, int world, int64_t n,
                           int dtype, int mode, int blocks, hipStream_t st) {
  return st_xgmi_collective_sim(ids, ins, outs, nullptr, world, n, dtype, mode, blocks, st);
}

// Simulation of any mode; partners[r] = rank r's pair partner (modes 5 / 6; every rank in a
// pair), may be null otherwise.
int st_xgmi_collective_sim(const int64_t* ids, const void* const* ins, void* const* outs, const int* partners,
                           int world, int64_t n, int dtype, int mode, int blocks, hipStream_t st) {
  if (world < 1 || world > kMaxRanks) return -2;
  Jobs J{};
  Comm* c0 = get(ids[0]);
  if (!c0 || c0->world != world) return -2;
  const int64_t elt = dtype == 0 ? 2 : 4;
  if (mode < 0 || mode > 6 || n % 8 || area_bytes(mode, world, n, elt) > c0->cap) return -2;
  if ((mode == 5 || mode == 6) && partners == nullptr) return -2;
  if (blocks <= 0 || blocks > kMaxBlocks) blocks = kMaxBlocks;
  uint32_t epoch = 0;
  for (int r = 0; r < world; ++r) {
    Comm* c = get(ids[r]);
    if (!c || c->rank != r || c->world != world || c->cap != c0->cap) return -2;
    if (((uintptr_t)ins[r] | (uintptr_t)outs[r]) % 16) return -2;
    const int partner = partners ? partners[r] : -1;
    if ((mode == 5 || mode == 6) && (partner < 0 || partner >= world || partner == r || partners[partner] != r))
      return -2;
    J.j[r] = Job{ins[r], outs[r], r, c->err, c->timeout, partner};
    epoch = ++c->epoch;  // every comm advances together
  }
  if (n == 0) return 0;
  return launch(c0->peers, J, world, world, n, c0->cap, dtype, mode, blocks, epoch, st);
}

// 1 if any kernel of this comm timed out waiting for a peer (host sync).
int st_xgmi_error(int64_t id) {
  Comm* c = get(id);
  if (!c) return -2;
  int v = 0;
  hipMemcpy(&v, c->err, sizeof(int), hipMemcpyDeviceToHost);
  return v;
}

int st_xgmi_destroy(int64_t id) {
  Comm* c = get(id);
  if (!c) return -2;
  hipDeviceSynchronize();
  for (int r = 0; r < c->world; ++r)
    if (c->opened[r]) hipIpcCloseMemHandle(c->peers.buf[r]);
  hipFree(c->local);
  hipFree(c->err);
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms[id] = nullptr;
  delete c;
  return 0;
}

}  // extern "C"

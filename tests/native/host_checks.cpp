// Host-side launch planning / validation of the HIP kernels, built with
// -Xarch_host -fsanitize=address,undefined (tests/test_host_sanitizers.py) and run on
// the CPU: every entry point here returns before any kernel launch, so no GPU is
// touched.  Exercises the arithmetic that sizes grids and workspaces (wgrad tail
// split, flash dK/dV split, RMSNorm partial rows) over a sweep of shapes, plus the
// early-return validation of the launchers, for overflow / UB / out-of-bounds.
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include <hip/hip_runtime.h>

extern "C" {
int64_t st_wgrad_ws_elems(int M, int N, int T, int variant);
int st_wgrad_gemm(const void* A, int64_t lda, const void* B, int64_t ldb, float* C, int64_t ldc, int M, int N,
                  int T, int beta, int variant, float* ws, hipStream_t st);
int64_t st_flash_bwd_part_elems(int B, int Sq, int Sk, int H, int Hkv, int D, int causal);
int64_t st_flash_bwd_ds_elems(int B, int Sq, int Sk, int H, int D, int causal, int64_t q_offset, int64_t k_offset);
int st_rmsnorm_bwd_nwaves(int rows);
int st_rmsnorm_fwd(const void* x, const void* res, const void* w, void* y, void* sum_out, float* rstd, int rows,
                   int h, float eps, hipStream_t st);
}

static int fails = 0;
#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                       \
    }                                                                \
  } while (0)

int main() {
  const int dims[] = {128, 256, 384, 1024, 2048, 3072, 4096, 6144, 7168, 14336, 28672, 128256};
  const int toks[] = {32, 64, 96, 4096, 8192, 16384, 24576, 32768};
  int64_t total = 0;
  for (int M : dims)
    for (int N : dims)
      for (int T : toks)
        for (int v : {0, 1, 2, 17, 18}) {
          const int64_t e = st_wgrad_ws_elems(M, N, T, v);
          CHECK(e >= 0);
          // at most (split - 1) <= 7 partial copies of the last partial round (< 256 tiles)
          CHECK(e <= (int64_t)7 * 256 * 256 * 256);
          if (v >= 16) CHECK(e == 0);
          total += e;
        }
  // shapes the kernels do not tile are declined before any launch
  CHECK(st_wgrad_gemm(nullptr, 200, nullptr, 192, nullptr, 192, 200, 192, 64, 0, 1, nullptr, nullptr) == -2);
  CHECK(st_wgrad_gemm(nullptr, 256, nullptr, 256, nullptr, 256, 256, 256, 0, 0, 1, nullptr, nullptr) == -2);
  CHECK(st_wgrad_gemm(nullptr, 256, nullptr, 200, nullptr, 256, 256, 256, 64, 0, 2, nullptr, nullptr) == -2);
  for (int B : {1, 2, 4, 6, 16})
    for (int Sk : {1, 127, 128, 2048, 4096, 32768, 131072})
      for (int Hkv : {1, 2, 8, 32})
        for (int D : {64, 128}) {
          const int64_t e = st_flash_bwd_part_elems(B, Sk, Sk, 4 * Hkv, Hkv, D, (B + Sk) & 1);
          CHECK(e >= 0);
          CHECK(e <= (int64_t)8 * 2 * B * Hkv * Sk * D + (int64_t)8 * B * 4 * Hkv * Sk * D);
          total += e;
        }
  // dS workspace of the dS-materialising flash backward: the closed-form tile count equals
  // the sum over 128-query tiles of the visible 64-key blocks (key_blocks' causal limit)
  for (int Sq : {1, 64, 127, 128, 320, 4096})
    for (int Sk : {1, 64, 200, 384, 4096})
      for (int64_t qo : {0, 32, 96, 300, 1000})
        for (int64_t ko : {0, 32, 160, 5000})
          for (int causal : {0, 1}) {
            const int NKB = (Sk + 63) / 64;
            int64_t want = 0;
            for (int t = 0; t < (Sq + 127) / 128; ++t) {
              int64_t n = NKB;
              if (causal) {
                const int64_t last = qo + 128 * t + 127 - ko;
                const int64_t lim = last < 0 ? 0 : last / 64 + 1;
                n = lim < n ? lim : n;
              }
              want += n;
            }
            const int64_t e = st_flash_bwd_ds_elems(2, Sq, Sk, 8, 128, causal, qo, ko);
            CHECK(e == 2 * 8 * want * 64 * 128);
            total += e;
          }
  for (int rows : {0, 1, 3, 4, 5, 1000, 24576, 1 << 20}) {
    const int nw = st_rmsnorm_bwd_nwaves(rows);
    CHECK(nw >= 1 && nw <= 4096);
  }
  CHECK(st_rmsnorm_fwd(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 4, 100, 1e-5f, nullptr) == -2);
  std::printf("host checks: %d failures (sum %lld)\n", fails, (long long)total);
  return fails ? 1 : 0;
}

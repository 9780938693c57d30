// Minimal repro of the rocprofv3 --pmc crash (rc 139 inside hipLaunchKernel) on the batched-row
// GEMV launches: one GEMV entry point of _lljamd.so called directly (no Python), so the crash can be
// bisected by argv under `rocprofv3 --pmc FETCH_SIZE -- ./pmc_repro <op> <M> <N> <K>`.
//   op: i8 (llj_linear, LLM.int8, workspace from llj_i8_stats), i8q (llj_i8_linear_resid),
//       w4 (llj_linear, int4 W4P), i8swiglu (llj_norm_swiglu wfmt 2), prep (llj_i8_norm_stats),
//       qw (llj_i8_quant_weight of an M x K bf16 matrix), gemm_i8 (llj_i8_stats + llj_gemm_i8_linear),
//       atti8 (llj_attention_i8: M rows, N = n_embd, a K-slot cache)
// Build: hipcc --offload-arch=gfx950 -O2 pmc_repro.cpp -I../../include -L../../lit-llama-ja_amd/lit_llama
//        -l:_lljamd.so -Wl,-rpath,'$ORIGIN/../../lit-llama-ja_amd/lit_llama' -o pmc_repro
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "lit_llama_amd.h"

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 2;                                                            \
    }                                                                      \
  } while (0)

static void* dev_rand(size_t bytes, unsigned seed, int kind) {
  std::vector<unsigned char> h(bytes);
  srand(seed);
  if (kind == 0) {  // bf16 values around N(0, 1): random sign/mantissa, exponent near 127
    for (size_t i = 0; i + 1 < bytes; i += 2) {
      const unsigned short v = (unsigned short)(((rand() & 1) << 15) | ((126 + rand() % 3) << 7) | (rand() & 127));
      memcpy(&h[i], &v, 2);
    }
  } else if (kind == 1) {  // fp32 scales
    for (size_t i = 0; i + 3 < bytes; i += 4) {
      const float v = 0.5f + (rand() % 1000) * 1e-3f;
      memcpy(&h[i], &v, 4);
    }
  } else {
    for (auto& b : h) b = (unsigned char)rand();
  }
  void* d = nullptr;
  if (hipMalloc(&d, bytes) != hipSuccess) return nullptr;
  hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice);
  return d;
}

int main(int argc, char** argv) {
  const char* op = argc > 1 ? argv[1] : "i8";
  const int M = argc > 2 ? atoi(argv[2]) : 8, N = argc > 3 ? atoi(argv[3]) : 4096, K = argc > 4 ? atoi(argv[4]) : 4096;
  const int reps = argc > 5 ? atoi(argv[5]) : 3;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  void* A = dev_rand((size_t)M * K * 2, 1, 0);
  void* W = dev_rand((size_t)N * K, 2, 2);
  void* W2 = dev_rand((size_t)N * K, 3, 2);
  void* sz = dev_rand((size_t)N * 8, 4, 1);
  void* x = dev_rand((size_t)M * N * 2, 5, 0);
  void* C = dev_rand((size_t)M * N * 2, 6, 0);
  void* ws = nullptr;
  CK(hipMalloc(&ws, llj_i8_ws_bytes(M, K > N ? K : N)));
  void* st = nullptr;
  CK(hipMalloc(&st, llj_i8_rowstats_bytes(K)));
  {  // a realistic hand-off block: SCA 4.0 for rows 0..7 in slot 0, ~K/40 outlier columns (i8ws.h layout)
    std::vector<uint32_t> w(llj_i8_rowstats_bytes(K) / 4, 0u);
    const float sca = 4.f;
    uint32_t sbits;
    memcpy(&sbits, &sca, 4);
    for (int m = 0; m < 8; ++m) w[16 + m] = sbits;
    srand(7);
    for (int i = 0; i < K / 40; ++i) {
      const int k = rand() % K;
      w[16 + 8 * 64 + k / 32] |= 1u << (k % 32);
    }
    CK(hipMemcpy(st, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  }
  int rc = 0;
  for (int r = 0; r < reps && rc == 0; ++r) {
    if (!strcmp(op, "i8")) {
      rc = llj_i8_stats(A, K, M, K, 6.f, ws, s);
      if (!rc) rc = llj_linear(2, A, K, W, sz, nullptr, C, N, M, N, K, ws, 0, nullptr, s);
    } else if (!strcmp(op, "i8q")) {
      rc = llj_i8_linear_resid(A, K, W, sz, x, N, M, N, K, st, s);
    } else if (!strcmp(op, "i8swiglu")) {
      rc = llj_i8_stats(A, K, M, K, 6.f, ws, s);
      if (!rc) rc = llj_norm_swiglu(2, A, nullptr, 1e-5f, W, sz, W2, sz, C, M, N, K, ws, 0, nullptr, nullptr, 0, s);
    } else if (!strcmp(op, "prep")) {  // RMSNorm + LLM.int8 statistics, one launch (the rms_1 / rms_2 prep)
      rc = llj_i8_norm_stats(A, x, 1e-5f, C, M, K, 6.f, ws, s);
    } else if (!strcmp(op, "qw")) {  // weight quantization (model build)
      rc = llj_i8_quant_weight(A, 1, W, sz, M, K, s);
    } else if (!strcmp(op, "gemm_i8")) {  // prefill: statistics of M rows + the LLM.int8 GEMM
      rc = llj_i8_stats(A, K, M, K, 6.f, ws, s);
      if (!rc) rc = llj_gemm_i8_linear(A, K, W, sz, ws, nullptr, nullptr, 0, C, N, M, N, K, s);
    } else if (!strcmp(op, "atti8")) {  // decode attention of M rows over a K-slot cache, LLM.int8 statistics of y
      // (N = n_embd, 128-dim heads; the cache holds positions 0..K-1, the rows attend at position K/2)
      // (its own q (M x N), y statistics block for N columns and caches: the shared buffers are sized by K)
      static void *kc = nullptr, *vc = nullptr, *pos = nullptr, *q = nullptr, *yst = nullptr;
      const int nh = N / 128, S = K;
      if (!kc) {
        q = dev_rand((size_t)M * N * 2, 10, 0);
        CK(hipMalloc(&yst, llj_i8_rowstats_bytes(N)));
        CK(hipMemset(yst, 0, llj_i8_rowstats_bytes(N)));
        kc = dev_rand((size_t)M * nh * S * 128 * 2, 8, 0);
        vc = dev_rand((size_t)M * nh * S * 128 * 2, 9, 0);
        std::vector<int> hp(M, S / 2);
        CK(hipMalloc(&pos, M * sizeof(int)));
        CK(hipMemcpy(pos, hp.data(), M * sizeof(int), hipMemcpyHostToDevice));
      }
      if (N % 128 || M > 8) { fprintf(stderr, "atti8: N %% 128 == 0, M <= 8\n"); return 2; }
      rc = llj_attention_i8(q, kc, vc, C, (const int*)pos, M, 1, nh, 128, S, 1, nullptr, yst, nullptr, 0, 6.f, s);
    } else if (!strcmp(op, "w4")) {
      rc = llj_linear(0, A, K, W, sz, nullptr, C, N, M, N, K, nullptr, 0, nullptr, s);
    } else {
      fprintf(stderr, "unknown op %s\n", op);
      return 2;
    }
    fprintf(stderr, "[pmc_repro] %s M=%d N=%d K=%d rep %d rc %d\n", op, M, N, K, r, rc);
  }
  CK(hipStreamSynchronize(s));
  printf("pmc_repro %s M=%d N=%d K=%d done rc=%d\n", op, M, N, K, rc);
  return rc;
}

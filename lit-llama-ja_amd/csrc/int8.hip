// LLM.int8() helpers (reference lit_llama/quantization.py:36-75 over bitsandbytes,
// has_fp16_weights=False, threshold=6.0): weight row quantization (load time) and the
// activation statistics the int8 GEMV (gemv.hip, WF_I8) needs.
//
// bitsandbytes is absent from the image and un-vendored in the reference, so this follows
// the published algorithm (Dettmers et al. 2022) as restated in oracle/llama_np.py:
//   weight:      W16 = W.half(); SCB[n] = max_k |W16[n,k]|; CB = round(W16 * 127 / SCB)
//   activation:  A16 = A.half(); outlier columns = {k : any row |A16[m,k]| >= threshold};
//                SCA[m] = max over the row's elements with |A16| < threshold
#include "common.h"

namespace llj {

constexpr int kNSB = 32;  // statistics blocks (k-ranges)

struct I8Ws {
  int mtot, K, nsb, kb;
};

static inline int i8_kb(int K) { return ((K + kNSB - 1) / kNSB + 15) & ~15; }

__device__ __forceinline__ float to_f16f(float x) { return (float)(_Float16)x; }

__global__ __launch_bounds__(256) void i8_stats_kernel(const bf16_t* __restrict__ A, int lda, int M, int K,
                                                       float thr, char* __restrict__ ws, int kb) {
  __shared__ int flag[1024];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* part = reinterpret_cast<float*>(ws + 16);
  int* cnt = reinterpret_cast<int*>(part + (size_t)kNSB * M);
  int* list = cnt + kNSB;
  if (b == 0 && tid == 0) *reinterpret_cast<I8Ws*>(ws) = I8Ws{M, K, kNSB, kb};
  const int k0 = b * kb;
  const int k1 = min(K, k0 + kb);
  for (int i = tid; i < kb; i += 256) flag[i] = 0;
  __syncthreads();
  for (int m = wave; m < M; m += 4) {
    float mx = 0.f;
    for (int k = k0 + lane; k < k1; k += 64) {
      const float a = fabsf(to_f16f(bf2f(A[(size_t)m * lda + k])));
      if (a >= thr) flag[k - k0] = 1;
      else mx = fmaxf(mx, a);
    }
    mx = wave_max(mx);
    if (lane == 0) part[(size_t)b * M + m] = mx;
  }
  __syncthreads();
  if (tid == 0) {
    int c = 0;
    for (int i = 0; i < k1 - k0; ++i)
      if (flag[i]) list[b * kb + c++] = k0 + i;
    cnt[b] = c;
  }
}

__global__ __launch_bounds__(256) void i8_quant_weight_kernel(const void* __restrict__ W, int dtype,
                                                              int8_t* __restrict__ CB, float* __restrict__ SCB, int K) {
  __shared__ float red[4];
  const int n = blockIdx.x, tid = threadIdx.x;
  auto ld = [&](int k) -> float {
    const size_t i = (size_t)n * K + k;
    float v = dtype == 0 ? ((const float*)W)[i] : dtype == 1 ? bf2f(((const bf16_t*)W)[i])
                                                              : (float)((const _Float16*)W)[i];
    return to_f16f(v);
  };
  float mx = 0.f;
  for (int k = tid; k < K; k += 256) mx = fmaxf(mx, fabsf(ld(k)));
  mx = wave_max(mx);
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float inv = mx > 0.f ? 127.f / mx : 0.f;
  for (int k = tid; k < K; k += 256)
    CB[(size_t)n * K + k] = (int8_t)fminf(fmaxf(rintf(ld(k) * inv), -127.f), 127.f);
  if (tid == 0) SCB[n] = mx;
}

}  // namespace llj

using namespace llj;

extern "C" {

// Bytes of the statistics workspace for an (M, K) activation.
size_t llj_i8_ws_bytes(int M, int K) {
  return 16 + sizeof(float) * (size_t)kNSB * M + sizeof(int) * kNSB + sizeof(int) * (size_t)kNSB * i8_kb(K);
}

int llj_i8_stats(const void* A, int lda, int M, int K, float threshold, void* ws, void* stream) {
  LLJ_REQUIRE(M > 0 && K > 0 && i8_kb(K) <= 1024);
  hipLaunchKernelGGL(i8_stats_kernel, dim3(kNSB), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)A, lda, M, K,
                     threshold, (char*)ws, i8_kb(K));
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_i8_quant_weight(const void* W, int dtype, void* CB, void* SCB, int N, int K, void* stream) {
  LLJ_REQUIRE(N > 0 && K > 0 && dtype >= 0 && dtype <= 2);
  hipLaunchKernelGGL(i8_quant_weight_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, W, dtype, (int8_t*)CB,
                     (float*)SCB, K);
  LLJ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

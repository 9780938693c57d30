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
#include "i8ws.h"

namespace llj {

__device__ __forceinline__ float to_f16f(float x) { return (float)(_Float16)x; }

// Pass 1, one block per k-range: outlier columns (any row |A16| >= thr) as flags and an
// ascending list, and per-row absmax of the other elements.
__global__ __launch_bounds__(256) void i8_stats_kernel(const bf16_t* __restrict__ A, int lda, int M, int K,
                                                       float thr, char* __restrict__ ws, int kb) {
  __shared__ int flag[1024];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const I8Layout L = i8_layout(ws, M, K);
  if (b == 0 && tid == 0) *reinterpret_cast<I8WsHeader*>(ws) = I8WsHeader{M, K, kNSB, kb};
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
    if (lane == 0) L.part[(size_t)b * M + m] = mx;
  }
  __syncthreads();
  for (int k = k0 + tid; k < k1; k += 256) L.flag[k] = (uint8_t)flag[k - k0];
  if (wave == 0) {  // compact the flags into the list, 64 columns per ballot
    int c = 0;
    for (int i0 = 0; i0 < k1 - k0; i0 += 64) {
      const bool f = i0 + lane < k1 - k0 && flag[i0 + lane];
      const unsigned long long bal = __ballot(f);
      if (f) L.list[b * kb + c + __popcll(bal & ((1ull << lane) - 1ull))] = k0 + i0 + lane;
      c += __popcll(bal);
    }
    if (lane == 0) L.cnt[b] = c;
  }
}

// q = round(A16 * 127 / SCA) clamped to +-127, outlier columns 0, for 8 columns
__device__ __forceinline__ uint2 quant8(uint4 x, uint2 fl, float inv) {
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
  const uint32_t fw[2] = {fl.x, fl.y};
  uint32_t o[2] = {0, 0};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = to_f16f(bflo(w[i])), bb = to_f16f(bfhi(w[i]));
    int qa = (int)fminf(fmaxf(rintf(a * inv), -127.f), 127.f);
    int qb = (int)fminf(fmaxf(rintf(bb * inv), -127.f), 127.f);
    if ((fw[i >> 1] >> (16 * (i & 1))) & 0xFF) qa = 0;
    if ((fw[i >> 1] >> (16 * (i & 1) + 8)) & 0xFF) qb = 0;
    o[i >> 1] |= ((uint32_t)(qa & 0xFF) | ((uint32_t)(qb & 0xFF) << 8)) << (16 * (i & 1));
  }
  return make_uint2(o[0], o[1]);
}

// Pass 2, one block per row: SCA = max over the k-blocks, then the row quantized once (outlier
// columns 0: their contribution is the fp16 side product). The row and its flags (up to QV
// vectors of 8 per thread, K <= 8 * 256 * QV) are loaded BEFORE the k-block maxima are reduced, so
// both reads share one memory latency.
constexpr int QV = 8;
__global__ __launch_bounds__(256) void i8_quant_act_kernel(const bf16_t* __restrict__ A, int lda, int M, int K,
                                                           char* __restrict__ ws) {
  __shared__ float s_sca;
  const int m = blockIdx.x, tid = threadIdx.x;
  const I8Layout L = i8_layout(ws, M, K);
  const bf16_t* ar = A + (size_t)m * lda;
  int8_t* qr = L.aq + (size_t)m * K;
  const int nv = K / 8;
  uint4 xs[QV];
  uint2 fs[QV];
  const bool pre = nv <= QV * 256;
  const int jn = (nv + 255) / 256;  // uniform
  if (pre) {
#pragma unroll
    for (int j = 0; j < QV; ++j) {
      if (j < jn) {
        const int v = tid + 256 * j < nv ? tid + 256 * j : nv - 1;  // clamped: always valid
        xs[j] = *reinterpret_cast<const uint4*>(ar + 8 * v);
        fs[j] = *reinterpret_cast<const uint2*>(L.flag + 8 * v);
      }
    }
  }
  if (tid < 64) {
    float mx = tid < kNSB ? L.part[(size_t)tid * M + m] : 0.f;
    mx = wave_max(mx);
    if (tid == 0) {
      s_sca = mx;
      L.sca[m] = mx;
    }
  }
  __syncthreads();
  const float s = s_sca;
  const float inv = s > 0.f ? 127.f / s : 0.f;
  if (pre) {
#pragma unroll
    for (int j = 0; j < QV; ++j) {
      const int v = tid + 256 * j;
      if (j < jn && v < nv) *reinterpret_cast<uint2*>(qr + 8 * v) = quant8(xs[j], fs[j], inv);
    }
    return;
  }
  for (int v = tid; v < nv; v += 256) {
    const uint4 x = *reinterpret_cast<const uint4*>(ar + 8 * v);
    const uint2 fl = *reinterpret_cast<const uint2*>(L.flag + 8 * v);
    *reinterpret_cast<uint2*>(qr + 8 * v) = quant8(x, fl, inv);
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
size_t llj_i8_ws_bytes(int M, int K) { return i8_offsets(M, K).total; }

int llj_i8_stats(const void* A, int lda, int M, int K, float threshold, void* ws, void* stream) {
  LLJ_REQUIRE(M > 0 && K > 0 && K % 16 == 0 && lda % 8 == 0 && i8_kb(K) <= 1024);
  hipLaunchKernelGGL(i8_stats_kernel, dim3(kNSB), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)A, lda, M, K,
                     threshold, (char*)ws, i8_kb(K));
  LLJ_CHECK_LAUNCH();
  hipLaunchKernelGGL(i8_quant_act_kernel, dim3(M), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)A, lda, M, K,
                     (char*)ws);
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

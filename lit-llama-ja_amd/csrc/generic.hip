// The any-shape path: LLaMA configurations the streaming kernels do not tile -- n_embd % 128 != 0
// or a head size other than 64 / 128. The JA fork's own 125M config (n_embd 780, head 78; reference
// lit_llama/model.py:48-51) and the reference test's n_embd 32 / head 2 (tests/test_model.py:108-112)
// run here. Plain kernels: one output per wave (linear) or per thread, fp32 accumulation, the
// reference's bf16 rounding points (the same ones the fast kernels keep). Slower by design: these
// shapes are small models, and none of them is the headline workload.
#include "common.h"
#include "lit_llama_amd.h"

namespace llj {

// ---- RMSNorm (model.py:276-283 on bf16 tensors): one block per row, any C
__global__ __launch_bounds__(256) void g_rmsnorm_kernel(const bf16_t* __restrict__ x, int ldx, const bf16_t* __restrict__ w,
                                                        float eps, bf16_t* __restrict__ y, int ldy, int C) {
  __shared__ float red[4];
  const int m = blockIdx.x, tid = threadIdx.x;
  const bf16_t* xr = x + (size_t)m * ldx;
  float ss = 0.f;
  for (int k = tid; k < C; k += 256) {
    const float v = bf2f(xr[k]);
    ss += round_bf(v * v);  // x * x in bf16 (model.py:281)
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float r = round_bf(rsqrtf(round_bf(round_bf(tot / (float)C) + eps)));
  bf16_t* yr = y + (size_t)m * ldy;
  for (int k = tid; k < C; k += 256) yr[k] = f2bf(round_bf(bf2f(w[k]) * round_bf(bf2f(xr[k]) * r)));
}

// ---- y[m, n] = bf16(sum_k x[m, k] W[n, k]) or, with resid, bf16(resid[m, n] + that) (the residual
// adds of model.py:172-173). WK 1: dense bf16 W (N, K) row-major (F.linear). WK 0: the reference's
// ColBlockQuantizedLinear buffers untouched -- codes in quant_weight's column-major storage (byte
// (n, j) at j N + n, 8 / bits codes per byte, code of k = j epb + r at bits r * bits), per-group
// fp32 scales / zeros (N, G), group = tile_cols (K for -1); the weight element is the Triton path's
// (q - zero) * scale in fp32 (quantization.py:250-267, 390-409). One wave per output column, lanes
// over k, up to 8 rows per wave.
constexpr int GL_ROWS = 8;
template <int WK>
__global__ __launch_bounds__(256) void g_linear_kernel(const bf16_t* __restrict__ x, int ldx, int M, int K,
                                                       const void* __restrict__ W, const float* __restrict__ sc,
                                                       const float* __restrict__ zr, int bits, int group, int N,
                                                       bf16_t* __restrict__ y, int ldy, const bf16_t* resid, int ldr) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  const int m0 = blockIdx.y * GL_ROWS;
  const int mr = M - m0 < GL_ROWS ? M - m0 : GL_ROWS;
  const int G = (K + group - 1) / group;
  const int epb = 8 / bits;
  const uint32_t mask = (1u << bits) - 1u;
  float acc[GL_ROWS];
#pragma unroll
  for (int r = 0; r < GL_ROWS; ++r) acc[r] = 0.f;
  for (int k = lane; k < K; k += 64) {
    float wv;
    if (WK == 1) {
      wv = bf2f(reinterpret_cast<const bf16_t*>(W)[(size_t)n * K + k]);
    } else {
      const int j = k / epb, sh = (k - j * epb) * bits;
      const uint32_t q = ((uint32_t)reinterpret_cast<const unsigned char*>(W)[(size_t)j * N + n] >> sh) & mask;
      const int g = k / group;
      wv = ((float)q - zr[(size_t)n * G + g]) * sc[(size_t)n * G + g];
    }
#pragma unroll
    for (int r = 0; r < GL_ROWS; ++r)
      if (r < mr) acc[r] += bf2f(x[(size_t)(m0 + r) * ldx + k]) * wv;
  }
#pragma unroll
  for (int r = 0; r < GL_ROWS; ++r) {
    const float s = wave_sum(acc[r]);
    if (lane == r && r < mr) {
      const size_t m = (size_t)(m0 + r);
      float v = round_bf(s);
      if (resid) v = round_bf(bf2f(resid[m * ldr + n]) + v);
      y[m * ldy + n] = f2bf(v);
    }
  }
}

// ---- q / k / v split of c_attn's output (model.py:204), apply_rope on q and k in fp32
// (model.py:312-329), k / v of the token at position p into cache slot p % S. Block (row, head).
__global__ __launch_bounds__(64) void g_rope_kv_kernel(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ q_out,
                                                       bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,
                                                       const float* __restrict__ rope, const int* __restrict__ pos,
                                                       int T, int C, int nh, int S) {
  const int m = blockIdx.x, h = blockIdx.y;
  const int hs = C / nh, b = m / T, t = m - b * T;
  const int p = pos[t], slot = p % S;
  const bf16_t* row = qkv + (size_t)m * 3 * C + h * hs;
  const size_t cbase = (((size_t)b * nh + h) * S + slot) * hs;
  for (int i = threadIdx.x; i < hs / 2; i += 64) {
    const float c = rope[((size_t)p * (hs / 2) + i) * 2], s = rope[((size_t)p * (hs / 2) + i) * 2 + 1];
    const float q0 = bf2f(row[2 * i]), q1 = bf2f(row[2 * i + 1]);
    const float k0 = bf2f(row[C + 2 * i]), k1 = bf2f(row[C + 2 * i + 1]);
    q_out[(size_t)m * C + h * hs + 2 * i] = f2bf(q0 * c - q1 * s);
    q_out[(size_t)m * C + h * hs + 2 * i + 1] = f2bf(q1 * c + q0 * s);
    kc[cbase + 2 * i] = f2bf(k0 * c - k1 * s);
    kc[cbase + 2 * i + 1] = f2bf(k1 * c + k0 * s);
    vc[cbase + 2 * i] = row[2 * C + 2 * i];
    vc[cbase + 2 * i + 1] = row[2 * C + 2 * i + 1];
  }
}

// ---- causal attention (model.py:237, the tril mask rows): row m at position p attends cache
// slots [0, p] (all S slots once p >= S: the ring holds the last S positions). Scores in LDS,
// fp32 softmax, y = bf16(P V / sum). Block (row, head); LDS: S + hs floats.
__global__ __launch_bounds__(256) void g_attention_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc,
                                                          const bf16_t* __restrict__ vc, bf16_t* __restrict__ y,
                                                          const int* __restrict__ pos, int T, int C, int nh, int S) {
  extern __shared__ float g_att_lds[];
  __shared__ float red[4];
  const int m = blockIdx.x, h = blockIdx.y, tid = threadIdx.x;
  const int hs = C / nh, b = m / T, t = m - b * T;
  const int p = pos[t];
  const int nvis = p < S ? p + 1 : S;
  float* sc = g_att_lds;       // [S]
  float* sq = g_att_lds + S;   // [hs]
  const float scale = 1.f / sqrtf((float)hs);
  for (int d = tid; d < hs; d += 256) sq[d] = bf2f(q[(size_t)m * C + h * hs + d]) * scale;
  __syncthreads();
  const size_t kb = ((size_t)b * nh + h) * S * hs;
  float mx = -INFINITY;
  for (int j = tid; j < nvis; j += 256) {
    const bf16_t* kr = kc + kb + (size_t)j * hs;
    float s = 0.f;
    for (int d = 0; d < hs; ++d) s += sq[d] * bf2f(kr[d]);
    sc[j] = s;
    mx = fmaxf(mx, s);
  }
  // block max
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float l = 0.f;
  for (int j = tid; j < nvis; j += 256) {
    const float e = __expf(sc[j] - mx);
    sc[j] = e;
    l += e;
  }
  l = wave_sum(l);
  if ((tid & 63) == 0) red[tid >> 6] = l;
  __syncthreads();
  l = red[0] + red[1] + red[2] + red[3];
  const float inv = 1.f / l;
  for (int d = tid; d < hs; d += 256) {
    float o = 0.f;
    for (int j = 0; j < nvis; ++j) o += sc[j] * bf2f(vc[kb + (size_t)j * hs + d]);
    y[(size_t)m * C + h * hs + d] = f2bf(o * inv);
  }
}

// ---- h = bf16(bf16(silu(a1)) * a2) (model.py:258-259 on bf16 tensors)
__global__ __launch_bounds__(256) void g_silu_mul_kernel(const bf16_t* __restrict__ a1, const bf16_t* __restrict__ a2,
                                                         bf16_t* __restrict__ h, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const float a = bf2f(a1[i]);
    h[i] = f2bf(round_bf(a / (1.f + __expf(-a))) * bf2f(a2[i]));
  }
}

}  // namespace llj

using namespace llj;

extern "C" {
LLJ_TRACE_EXPORT(generic)

int llj_g_rmsnorm(const void* x, int ldx, const void* w, float eps, void* y, int ldy, int M, int C, void* stream) {
  LLJ_REQUIRE(x && w && y && M > 0 && C > 0 && ldx >= C && ldy >= C);
  hipLaunchKernelGGL(g_rmsnorm_kernel, dim3(M), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, ldx, (const bf16_t*)w,
                     eps, (bf16_t*)y, ldy, C);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_g_linear(int wkind, const void* x, int ldx, int M, int K, const void* W, const float* scales, const float* zeros,
                 int bits, int group, int N, void* y, int ldy, const void* resid, int ldr, void* stream) {
  LLJ_REQUIRE(x && W && y && M > 0 && K > 0 && N > 0 && ldx >= K && ldy >= N && (!resid || ldr >= N));
  LLJ_REQUIRE(wkind == 1 || (wkind == 0 && scales && zeros && (bits == 2 || bits == 4 || bits == 8) && group > 0 &&
                             K % (8 / bits) == 0));
  const dim3 grid((N + 3) / 4, (M + GL_ROWS - 1) / GL_ROWS);
  if (wkind == 1)
    hipLaunchKernelGGL(g_linear_kernel<1>, grid, dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, ldx, M, K, W, scales,
                       zeros, 16, K, N, (bf16_t*)y, ldy, (const bf16_t*)resid, ldr);
  else
    hipLaunchKernelGGL(g_linear_kernel<0>, grid, dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, ldx, M, K, W, scales,
                       zeros, bits, group, N, (bf16_t*)y, ldy, (const bf16_t*)resid, ldr);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_g_rope_kv(const void* qkv, void* q_out, void* kcache, void* vcache, const float* rope, const int* pos, int B, int T,
                  int C, int n_head, int S, void* stream) {
  LLJ_REQUIRE(qkv && q_out && kcache && vcache && rope && pos && B > 0 && T > 0 && n_head > 0 && C % n_head == 0 &&
              (C / n_head) % 2 == 0 && S > 0);
  hipLaunchKernelGGL(g_rope_kv_kernel, dim3(B * T, n_head), dim3(64), 0, (hipStream_t)stream, (const bf16_t*)qkv,
                     (bf16_t*)q_out, (bf16_t*)kcache, (bf16_t*)vcache, rope, pos, T, C, n_head, S);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_g_attention(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T, int C,
                    int n_head, int S, void* stream) {
  LLJ_REQUIRE(q && kcache && vcache && y && pos && B > 0 && T > 0 && n_head > 0 && C % n_head == 0 && S > 0);
  const size_t lds = (size_t)(S + C / n_head) * 4;
  LLJ_REQUIRE(lds <= 64 * 1024);
  hipLaunchKernelGGL(g_attention_kernel, dim3(B * T, n_head), dim3(256), lds, (hipStream_t)stream, (const bf16_t*)q,
                     (const bf16_t*)kcache, (const bf16_t*)vcache, (bf16_t*)y, pos, T, C, n_head, S);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_g_silu_mul(const void* a1, const void* a2, void* h, size_t n, void* stream) {
  LLJ_REQUIRE(a1 && a2 && h && n > 0);
  const size_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(g_silu_mul_kernel, dim3(blocks < 4096 ? (unsigned)blocks : 4096u), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)a1, (const bf16_t*)a2, (bf16_t*)h, n);
  LLJ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

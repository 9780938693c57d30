// The any-shape path: LLaMA configurations the streaming kernels do not tile -- n_embd % 128 != 0
// or a head size other than 64 / 128. The JA fork's own 125M config (n_embd 780, head 78; reference
// lit_llama/model.py:48-51) and the reference test's n_embd 32 / head 2 (tests/test_model.py:108-112)
// run here. Plain kernels: one output per wave (linear) or per thread, fp32 accumulation, the
// reference's bf16 rounding points (the same ones the fast kernels keep). Slower by design: these
// shapes are small models, and none of them is the headline workload.
// Every kernel also runs in fp32 (dt = 1: activations, dense weights, KV cache and logits fp32, no
// bf16 rounding -- the reference's float32 model, e.g. evaluate/full.py's default dtype and the
// CPU config of generate.py:121): LLaMA.forward routes an fp32 model here whatever its shape.
#include "common.h"
#include "lit_llama_amd.h"

namespace llj {

// element access of the activation type: bf16 (the reference's rounding points) or fp32 (none)
template <typename T>
__device__ __forceinline__ float ldv(const T* p, size_t i) {
  if constexpr (sizeof(T) == 2) return bf2f(p[i]);
  else return p[i];
}
template <typename T>
__device__ __forceinline__ void stv(T* p, size_t i, float v) {
  if constexpr (sizeof(T) == 2) p[i] = f2bf(v);
  else p[i] = v;
}
template <typename T>
__device__ __forceinline__ float rnd(float v) {
  if constexpr (sizeof(T) == 2) return round_bf(v);
  else return v;
}

// ---- embedding (model.py:110), any C, optionally bumping the device-side decode position
template <typename T>
__global__ __launch_bounds__(256) void g_embedding_kernel(const int* __restrict__ idx, const T* __restrict__ wte,
                                                          T* __restrict__ out, int C, int* pos_inc) {
  const int m = blockIdx.x;
  const size_t r = (size_t)idx[m];
  for (int v = threadIdx.x; v < C; v += blockDim.x) out[(size_t)m * C + v] = wte[r * C + v];
  if (pos_inc && m == 0 && threadIdx.x == 0) *pos_inc += 1;
}

// ---- RMSNorm (model.py:276-283; on bf16 tensors every op rounds): one block per row, any C
template <typename T>
__global__ __launch_bounds__(256) void g_rmsnorm_kernel(const T* __restrict__ x, int ldx, const T* __restrict__ w,
                                                        float eps, T* __restrict__ y, int ldy, int C) {
  __shared__ float red[4];
  const int m = blockIdx.x, tid = threadIdx.x;
  const T* xr = x + (size_t)m * ldx;
  float ss = 0.f;
  for (int k = tid; k < C; k += 256) {
    const float v = ldv(xr, k);
    ss += rnd<T>(v * v);  // x * x (model.py:281)
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float r = rnd<T>(rsqrtf(rnd<T>(rnd<T>(tot / (float)C) + eps)));
  T* yr = y + (size_t)m * ldy;
  for (int k = tid; k < C; k += 256) stv(yr, k, ldv(w, k) * rnd<T>(ldv(xr, k) * r));
}

// ---- y[m, n] = bf16(sum_k x[m, k] W[n, k]) or, with resid, bf16(resid[m, n] + that) (the residual
// adds of model.py:172-173). WK 1: dense bf16 W (N, K) row-major (F.linear). WK 0: the reference's
// ColBlockQuantizedLinear buffers untouched -- codes in quant_weight's column-major storage (byte
// (n, j) at j N + n, 8 / bits codes per byte, code of k = j epb + r at bits r * bits), per-group
// fp32 scales / zeros (N, G), group = tile_cols (K for -1); the weight element is the Triton path's
// (q - zero) * scale in fp32 (quantization.py:250-267, 390-409). One wave per output column, lanes
// over k, up to 8 rows per wave. T: activation (and dense weight) type.
constexpr int GL_ROWS = 8;
template <int WK, typename T>
__global__ __launch_bounds__(256) void g_linear_kernel(const T* __restrict__ x, int ldx, int M, int K,
                                                       const void* __restrict__ W, const float* __restrict__ sc,
                                                       const float* __restrict__ zr, int bits, int group, int N,
                                                       T* __restrict__ y, int ldy, const T* resid, int ldr) {
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
      wv = ldv(reinterpret_cast<const T*>(W), (size_t)n * K + k);
    } else {
      const int j = k / epb, sh = (k - j * epb) * bits;
      const uint32_t q = ((uint32_t)reinterpret_cast<const unsigned char*>(W)[(size_t)j * N + n] >> sh) & mask;
      const int g = k / group;
      wv = ((float)q - zr[(size_t)n * G + g]) * sc[(size_t)n * G + g];
    }
#pragma unroll
    for (int r = 0; r < GL_ROWS; ++r)
      if (r < mr) acc[r] += ldv(x, (size_t)(m0 + r) * ldx + k) * wv;
  }
#pragma unroll
  for (int r = 0; r < GL_ROWS; ++r) {
    const float s = wave_sum(acc[r]);
    if (lane == r && r < mr) {
      const size_t m = (size_t)(m0 + r);
      float v = rnd<T>(s);
      if (resid) v = ldv(resid, m * ldr + n) + v;
      stv(y, m * ldy + n, v);
    }
  }
}

// ---- q / k / v split of c_attn's output (model.py:204), apply_rope on q and k in fp32
// (model.py:312-329), k / v of the token at position p into cache slot p % S. Block (row, head).
template <typename TT>
__global__ __launch_bounds__(64) void g_rope_kv_kernel(const TT* __restrict__ qkv, TT* __restrict__ q_out,
                                                       TT* __restrict__ kc, TT* __restrict__ vc,
                                                       const float* __restrict__ rope, const int* __restrict__ pos,
                                                       int T, int C, int nh, int S) {
  const int m = blockIdx.x, h = blockIdx.y;
  const int hs = C / nh, b = m / T, t = m - b * T;
  const int p = pos[t], slot = p % S;
  const TT* row = qkv + (size_t)m * 3 * C + h * hs;
  const size_t cbase = (((size_t)b * nh + h) * S + slot) * hs;
  for (int i = threadIdx.x; i < hs / 2; i += 64) {
    const float c = rope[((size_t)p * (hs / 2) + i) * 2], s = rope[((size_t)p * (hs / 2) + i) * 2 + 1];
    const float q0 = ldv(row, 2 * i), q1 = ldv(row, 2 * i + 1);
    const float k0 = ldv(row, C + 2 * i), k1 = ldv(row, C + 2 * i + 1);
    stv(q_out, (size_t)m * C + h * hs + 2 * i, q0 * c - q1 * s);
    stv(q_out, (size_t)m * C + h * hs + 2 * i + 1, q1 * c + q0 * s);
    stv(kc, cbase + 2 * i, k0 * c - k1 * s);
    stv(kc, cbase + 2 * i + 1, k1 * c + k0 * s);
    vc[cbase + 2 * i] = row[2 * C + 2 * i];
    vc[cbase + 2 * i + 1] = row[2 * C + 2 * i + 1];
  }
}

// ---- causal attention (model.py:237, the tril mask rows): row m at position p attends cache
// slots [0, p] (all S slots once p >= S: the ring holds the last S positions). Scores in LDS,
// fp32 softmax, y = P V / sum (rounded to bf16 on the bf16 path). Block (row, head); LDS: S + hs floats.
template <typename TT>
__global__ __launch_bounds__(256) void g_attention_kernel(const TT* __restrict__ q, const TT* __restrict__ kc,
                                                          const TT* __restrict__ vc, TT* __restrict__ y,
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
  for (int d = tid; d < hs; d += 256) sq[d] = ldv(q, (size_t)m * C + h * hs + d) * scale;
  __syncthreads();
  const size_t kb = ((size_t)b * nh + h) * S * hs;
  float mx = -INFINITY;
  for (int j = tid; j < nvis; j += 256) {
    const TT* kr = kc + kb + (size_t)j * hs;
    float s = 0.f;
    for (int d = 0; d < hs; ++d) s += sq[d] * ldv(kr, d);
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
    for (int j = 0; j < nvis; ++j) o += sc[j] * ldv(vc, kb + (size_t)j * hs + d);
    stv(y, (size_t)m * C + h * hs + d, o * inv);
  }
}

// ---- h = silu(a1) * a2 (model.py:258-259; bf16: bf16(bf16(silu(a1)) * a2))
template <typename T>
__global__ __launch_bounds__(256) void g_silu_mul_kernel(const T* __restrict__ a1, const T* __restrict__ a2,
                                                         T* __restrict__ h, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const float a = ldv(a1, i);
    stv(h, i, rnd<T>(a / (1.f + expf(-a))) * ldv(a2, i));
  }
}

// ---- greedy next token over fp32 logits (lowest index on ties), as llj_argmax for bf16 ones
__global__ __launch_bounds__(1024) void g_argmax_kernel(const float* __restrict__ logits, int ldl, int V,
                                                        int* __restrict__ out_idx, int* __restrict__ tokens_out,
                                                        int tok_stride, const int* __restrict__ pos) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const int m = blockIdx.x, tid = threadIdx.x;
  const float* lr = logits + (size_t)m * ldl;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int v = tid; v < V; v += 1024) {
    const float x = lr[v];
    if (x > best || (x == best && v < bi)) { best = x; bi = v; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
  }
  if ((tid & 63) == 0) { sv[tid >> 6] = best; si[tid >> 6] = bi; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < 16; ++w)
      if (sv[w] > best || (sv[w] == best && si[w] < bi)) { best = sv[w]; bi = si[w]; }
    if (bi == 0x7fffffff) bi = 0;  // all-NaN row
    out_idx[m] = bi;
    if (tokens_out) tokens_out[(size_t)m * tok_stride + pos[0] + 1] = bi;
  }
}

}  // namespace llj

using namespace llj;

// ---- LLM.int8() for any K (Linear8bitLt outside the streaming tiling, e.g. the 125M's K = 780):
// the restated bnb MatMul8bitLt (oracle/llama_np.py int8_linear, reference quantization.py:36-75):
// A16 = f16(A); outlier columns = {k : any row |A16[m, k]| >= thr}; SCA[m] = max |A16[m, k]| < thr; CA = rint(A16 * (127 / SCA)); y = f16(f16(sum_k CA CB (int32) * SCA SCB / 127^2)
// + sum_{outliers} A16 f16(CB SCB / 127)), cast to bf16. ws: K flag bytes, then M fp32 SCA.
// T: the activation type. bitsandbytes' MatMul8bitLt casts its input to fp16 (A16) whatever it is
// and casts the fp16 result back to the input dtype, so a float32 model's Linear8bitLt computes on
// f16(x) and returns fp32 holding fp16 values (no bf16 rounding, fp32 residual add).
template <typename T>
__global__ __launch_bounds__(256) void g_i8_flags_kernel(const T* __restrict__ x, int ldx, int M, int K, float thr,
                                                         unsigned char* __restrict__ flags) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  bool o = false;
  for (int m = 0; m < M; ++m) o |= fabsf((float)(_Float16)ldv(x, (size_t)m * ldx + k)) >= thr;
  flags[k] = o ? 1 : 0;
}
// SCA[m]: max |A16| over the row's elements below the threshold (element-wise, as double_quant's row
// statistics; an element under it in an outlier column still counts, its code is then dropped)
template <typename T>
__global__ __launch_bounds__(256) void g_i8_sca_kernel(const T* __restrict__ x, int ldx, int K, float thr,
                                                       float* __restrict__ sca) {
  __shared__ float red[4];
  const int m = blockIdx.x, tid = threadIdx.x;
  float mx = 0.f;
  for (int k = tid; k < K; k += 256) {
    const float a = fabsf((float)(_Float16)ldv(x, (size_t)m * ldx + k));
    if (a < thr) mx = fmaxf(mx, a);
  }
  mx = wave_max(mx);
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  if (tid == 0) sca[m] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}
template <typename T>
__global__ __launch_bounds__(256) void g_i8_linear_kernel(const T* __restrict__ x, int ldx, int M, int K,
                                                          const int8_t* __restrict__ CB, const float* __restrict__ SCB,
                                                          const unsigned char* __restrict__ flags,
                                                          const float* __restrict__ sca, int N, T* __restrict__ y,
                                                          int ldy, const T* resid, int ldr) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  const int m0 = blockIdx.y * GL_ROWS;
  const int mr = M - m0 < GL_ROWS ? M - m0 : GL_ROWS;
  const float scb = SCB[n];
  float qs[GL_ROWS];
#pragma unroll
  for (int r = 0; r < GL_ROWS; ++r) {
    const float sa = r < mr ? sca[m0 + r] : 1.f;
    qs[r] = 127.f / (sa == 0.f ? 1.f : sa);
  }
  int acc[GL_ROWS];
  float side[GL_ROWS];
#pragma unroll
  for (int r = 0; r < GL_ROWS; ++r) {
    acc[r] = 0;
    side[r] = 0.f;
  }
  for (int k = lane; k < K; k += 64) {
    const int cb = CB[(size_t)n * K + k];
    const bool o = flags[k] != 0;
    const float w16 = (float)(_Float16)((float)cb * (scb / 127.f));
#pragma unroll
    for (int r = 0; r < GL_ROWS; ++r) {
      if (r < mr) {
        const float a16 = (float)(_Float16)ldv(x, (size_t)(m0 + r) * ldx + k);
        if (o) side[r] += a16 * w16;
        else acc[r] += (int)rintf(fminf(fmaxf(a16 * qs[r], -127.f), 127.f)) * cb;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < GL_ROWS; ++r) {
    int a = acc[r];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    const float sd = wave_sum(side[r]);
    if (lane == r && r < mr) {
      const size_t m = (size_t)(m0 + r);
      const float sa = sca[m];
      float v = (float)a * (sa * scb * (1.f / (127.f * 127.f)));
      v = (float)(_Float16)((float)(_Float16)v + sd);
      v = rnd<T>(v);
      if (resid) v = ldv(resid, m * ldr + n) + v;
      stv(y, m * ldy + n, v);
    }
  }
}

#define LLJ_DT(dt, CALL_BF16, CALL_F32) \
  do {                                 \
    if ((dt) == 0) CALL_BF16;          \
    else CALL_F32;                     \
  } while (0)

extern "C" {
LLJ_TRACE_EXPORT(generic)

int llj_g_embedding(const int* idx, const void* wte, void* out, int M, int C, int* pos_inc, int dt, void* stream) {
  LLJ_REQUIRE(idx && wte && out && M > 0 && C > 0 && (dt == 0 || dt == 1));
  hipStream_t s = (hipStream_t)stream;
  LLJ_DT(dt, hipLaunchKernelGGL(g_embedding_kernel<bf16_t>, dim3(M), dim3(256), 0, s, idx, (const bf16_t*)wte, (bf16_t*)out, C, pos_inc),
         hipLaunchKernelGGL(g_embedding_kernel<float>, dim3(M), dim3(256), 0, s, idx, (const float*)wte, (float*)out, C, pos_inc));
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_g_rmsnorm(const void* x, int ldx, const void* w, float eps, void* y, int ldy, int M, int C, int dt, void* stream) {
  LLJ_REQUIRE(x && w && y && M > 0 && C > 0 && ldx >= C && ldy >= C && (dt == 0 || dt == 1));
  hipStream_t s = (hipStream_t)stream;
  LLJ_DT(dt, hipLaunchKernelGGL(g_rmsnorm_kernel<bf16_t>, dim3(M), dim3(256), 0, s, (const bf16_t*)x, ldx, (const bf16_t*)w, eps, (bf16_t*)y, ldy, C),
         hipLaunchKernelGGL(g_rmsnorm_kernel<float>, dim3(M), dim3(256), 0, s, (const float*)x, ldx, (const float*)w, eps, (float*)y, ldy, C));
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_g_linear(int wkind, const void* x, int ldx, int M, int K, const void* W, const float* scales, const float* zeros,
                 int bits, int group, int N, void* y, int ldy, const void* resid, int ldr, int dt, void* stream) {
  LLJ_REQUIRE(x && W && y && M > 0 && K > 0 && N > 0 && ldx >= K && ldy >= N && (!resid || ldr >= N) && (dt == 0 || dt == 1));
  LLJ_REQUIRE(wkind == 1 || (wkind == 0 && scales && zeros && (bits == 2 || bits == 4 || bits == 8) && group > 0 &&
                             K % (8 / bits) == 0));
  const dim3 grid((N + 3) / 4, (M + GL_ROWS - 1) / GL_ROWS);
  hipStream_t s = (hipStream_t)stream;
#define LLJ_GL(WK, T) \
  hipLaunchKernelGGL((g_linear_kernel<WK, T>), grid, dim3(256), 0, s, (const T*)x, ldx, M, K, W, scales, zeros, \
                     WK == 1 ? 16 : bits, WK == 1 ? K : group, N, (T*)y, ldy, (const T*)resid, ldr)
  if (wkind == 1) LLJ_DT(dt, LLJ_GL(1, bf16_t), LLJ_GL(1, float));
  else LLJ_DT(dt, LLJ_GL(0, bf16_t), LLJ_GL(0, float));
#undef LLJ_GL
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_g_rope_kv(const void* qkv, void* q_out, void* kcache, void* vcache, const float* rope, const int* pos, int B, int T,
                  int C, int n_head, int S, int dt, void* stream) {
  LLJ_REQUIRE(qkv && q_out && kcache && vcache && rope && pos && B > 0 && T > 0 && n_head > 0 && C % n_head == 0 &&
              (C / n_head) % 2 == 0 && S > 0 && (dt == 0 || dt == 1));
  hipStream_t s = (hipStream_t)stream;
  LLJ_DT(dt, hipLaunchKernelGGL(g_rope_kv_kernel<bf16_t>, dim3(B * T, n_head), dim3(64), 0, s, (const bf16_t*)qkv, (bf16_t*)q_out,
                                (bf16_t*)kcache, (bf16_t*)vcache, rope, pos, T, C, n_head, S),
         hipLaunchKernelGGL(g_rope_kv_kernel<float>, dim3(B * T, n_head), dim3(64), 0, s, (const float*)qkv, (float*)q_out,
                            (float*)kcache, (float*)vcache, rope, pos, T, C, n_head, S));
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_g_attention(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T, int C,
                    int n_head, int S, int dt, void* stream) {
  LLJ_REQUIRE(q && kcache && vcache && y && pos && B > 0 && T > 0 && n_head > 0 && C % n_head == 0 && S > 0 &&
              (dt == 0 || dt == 1));
  const size_t lds = (size_t)(S + C / n_head) * 4;
  LLJ_REQUIRE(lds <= 64 * 1024);
  hipStream_t s = (hipStream_t)stream;
  LLJ_DT(dt, hipLaunchKernelGGL(g_attention_kernel<bf16_t>, dim3(B * T, n_head), dim3(256), lds, s, (const bf16_t*)q,
                                (const bf16_t*)kcache, (const bf16_t*)vcache, (bf16_t*)y, pos, T, C, n_head, S),
         hipLaunchKernelGGL(g_attention_kernel<float>, dim3(B * T, n_head), dim3(256), lds, s, (const float*)q,
                            (const float*)kcache, (const float*)vcache, (float*)y, pos, T, C, n_head, S));
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_g_silu_mul(const void* a1, const void* a2, void* h, size_t n, int dt, void* stream) {
  LLJ_REQUIRE(a1 && a2 && h && n > 0 && (dt == 0 || dt == 1));
  const size_t blocks = (n + 255) / 256;
  const unsigned g = blocks < 4096 ? (unsigned)blocks : 4096u;
  hipStream_t s = (hipStream_t)stream;
  LLJ_DT(dt, hipLaunchKernelGGL(g_silu_mul_kernel<bf16_t>, dim3(g), dim3(256), 0, s, (const bf16_t*)a1, (const bf16_t*)a2, (bf16_t*)h, n),
         hipLaunchKernelGGL(g_silu_mul_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)a1, (const float*)a2, (float*)h, n));
  LLJ_CHECK_LAUNCH();
  return 0;
}

size_t llj_g_i8_ws_bytes(int M, int K) { return (((size_t)K + 15) & ~(size_t)15) + (size_t)M * 4; }

int llj_g_i8_linear(const void* x, int ldx, int M, int K, const void* CB, const float* SCB, float threshold, void* ws, int N,
                    void* y, int ldy, const void* resid, int ldr, int dt, void* stream) {
  LLJ_REQUIRE(x && CB && SCB && ws && y && M > 0 && K > 0 && N > 0 && ldx >= K && ldy >= N && (!resid || ldr >= N) &&
              (dt == 0 || dt == 1));
  hipStream_t s = (hipStream_t)stream;
  unsigned char* flags = (unsigned char*)ws;
  float* sca = (float*)((char*)ws + (((size_t)K + 15) & ~(size_t)15));
  const dim3 grid((N + 3) / 4, (M + GL_ROWS - 1) / GL_ROWS);
#define LLJ_GI8(T)                                                                                                   \
  do {                                                                                                                \
    hipLaunchKernelGGL(g_i8_flags_kernel<T>, dim3((K + 255) / 256), dim3(256), 0, s, (const T*)x, ldx, M, K, threshold, \
                       flags);                                                                                        \
    hipLaunchKernelGGL(g_i8_sca_kernel<T>, dim3(M), dim3(256), 0, s, (const T*)x, ldx, K, threshold, sca);            \
    hipLaunchKernelGGL(g_i8_linear_kernel<T>, grid, dim3(256), 0, s, (const T*)x, ldx, M, K, (const int8_t*)CB, SCB,  \
                       flags, sca, N, (T*)y, ldy, (const T*)resid, ldr);                                              \
  } while (0)
  LLJ_DT(dt, LLJ_GI8(bf16_t), LLJ_GI8(float));
#undef LLJ_GI8
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_g_argmax(const float* logits, int ldl, int M, int V, int* out_idx, int* tokens_out, int tok_stride, const int* pos,
                 void* stream) {
  LLJ_REQUIRE(logits && out_idx && M > 0 && V > 0 && ldl >= V && (!tokens_out || pos));
  hipLaunchKernelGGL(g_argmax_kernel, dim3(M), dim3(1024), 0, (hipStream_t)stream, logits, ldl, V, out_idx, tokens_out,
                     tok_stride, pos);
  LLJ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

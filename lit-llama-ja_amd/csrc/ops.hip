// Decode-step ops around the weight-streaming GEMVs: token embedding, standalone RMSNorm
// (prefill rows beyond the fused-LDS limit), causal attention over the KV cache, and the
// greedy (top_k = 1) next-token selection.
#include "common.h"
#include "attention.h"
#include "lit_llama_amd.h"

namespace llj {

// ---- embedding: out[m] = wte[idx[m]]  (reference model.py:110). Optionally bumps the
// device-side decode position (*pos_inc += 1) so a captured decode step is self-advancing.
__global__ __launch_bounds__(256) void embedding_kernel(const int* __restrict__ idx, const uint4* __restrict__ wte,
                                                        uint4* __restrict__ out, int C8, int* pos_inc) {
  const int m = blockIdx.x;
  const size_t r = (size_t)idx[m];
  for (int v = threadIdx.x; v < C8; v += blockDim.x) out[(size_t)m * C8 + v] = wte[r * C8 + v];
  if (pos_inc && m == 0 && threadIdx.x == 0) *pos_inc += 1;
}

// ---- RMSNorm with the bf16 rounding points of model.py:281-283 on bf16 tensors. One block
// per row; rows up to 8192 wide are loaded once into registers (x and the scale together,
// before any use), so the kernel is one memory round trip.
__device__ __forceinline__ uint32_t norm_pair(uint32_t a, uint32_t g, float r) {
  return pack2bf(round_bf(bflo(g) * round_bf(bflo(a) * r)), round_bf(bfhi(g) * round_bf(bfhi(a) * r)));
}

__global__ __launch_bounds__(256) void rmsnorm_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                      float eps, bf16_t* __restrict__ y, int C,
                                                      float* __restrict__ rowsum) {
  constexpr int MAXV = 4;  // 16-byte vectors per thread held in registers
  __shared__ float red[8];
  const int m = blockIdx.x, tid = threadIdx.x;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)m * C);
  const uint4* g4 = reinterpret_cast<const uint4*>(w);
  uint4* yr = reinterpret_cast<uint4*>(y + (size_t)m * C);
  const int nvec = C >> 3;
  const bool regs = nvec <= MAXV * 256;
  uint4 xa[MAXV], ga[MAXV];
  float ss = 0.f;
  if (regs) {
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      const int v = tid + 256 * j, vv = v < nvec ? v : 0;
      xa[j] = xr[vv];
      ga[j] = g4[vv];
    }
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      if (tid + 256 * j < nvec) {
        const uint32_t aw[4] = {xa[j].x, xa[j].y, xa[j].z, xa[j].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) ss += round_bf(bflo(aw[i]) * bflo(aw[i])) + round_bf(bfhi(aw[i]) * bfhi(aw[i]));
      }
    }
  } else {
    for (int v = tid; v < nvec; v += 256) {
      const uint4 a = xr[v];
      const uint32_t aw[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) ss += round_bf(bflo(aw[i]) * bflo(aw[i])) + round_bf(bfhi(aw[i]) * bfhi(aw[i]));
    }
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float r = round_bf(rsqrtf(round_bf(round_bf(tot / (float)C) + eps)));
  float rsum = 0.f;
  auto emit = [&](int v, uint4 a, uint4 g) {
    const uint32_t o0 = norm_pair(a.x, g.x, r), o1 = norm_pair(a.y, g.y, r), o2 = norm_pair(a.z, g.z, r),
                   o3 = norm_pair(a.w, g.w, r);
    rsum += bflo(o0) + bfhi(o0) + bflo(o1) + bfhi(o1) + bflo(o2) + bfhi(o2) + bflo(o3) + bfhi(o3);
    yr[v] = make_uint4(o0, o1, o2, o3);
  };
  if (regs) {
#pragma unroll
    for (int j = 0; j < MAXV; ++j)
      if (tid + 256 * j < nvec) emit(tid + 256 * j, xa[j], ga[j]);
  } else {
    for (int v = tid; v < nvec; v += 256) emit(v, xr[v], g4[v]);
  }
  if (rowsum) {  // sum of the normalized bf16 row: the int4 GEMV's offset term (gemv.hip header)
    rsum = wave_sum(rsum);
    if ((tid & 63) == 0) red[4 + (tid >> 6)] = rsum;
    __syncthreads();
    if (tid == 0) rowsum[m] = red[4] + red[5] + red[6] + red[7];
  }
}

// ---- attention (attention.h): one block per (head, query row)
#ifndef LLJ_ATT_NTH
#define LLJ_ATT_NTH 256  // threads per (row, head) block
#endif
#ifndef LLJ_ATT_U
#define LLJ_ATT_U 8  // keys per 16-lane group per pass
#endif
template <int HS, int U, int NTH>
__global__ __launch_bounds__(NTH) void attention_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc,
                                                        const bf16_t* __restrict__ vc, bf16_t* __restrict__ y,
                                                        const int* __restrict__ pos, int T, int S, int nh,
                                                        float scale_log2) {
  __shared__ float lds[attention_lds_floats<HS, NTH>()];
  attention_body<HS, U, NTH>(q, kc, vc, y, pos, T, S, nh, scale_log2, blockIdx.x, blockIdx.y, lds);
}

// split-K attention over the keys (long contexts): block (head, row, split) -> partial
template <int HS, int U, int NTH>
__global__ __launch_bounds__(NTH) void attention_part_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc,
                                                             const bf16_t* __restrict__ vc, const int* __restrict__ pos,
                                                             int T, int S, int nh, float scale_log2, int nsplit,
                                                             float* __restrict__ part) {
  __shared__ float lds[attention_lds_floats<HS, NTH>()];
  attention_body<HS, U, NTH, true>(q, kc, vc, nullptr, pos, T, S, nh, scale_log2, blockIdx.x, blockIdx.y, lds, nsplit,
                                   blockIdx.z, part);
}

// ---- greedy next token: argmax over bf16 logits (lowest index on ties). Reference
// generate.py:66-74 with top_k = 1 (multinomial over the kept maximum).
__global__ __launch_bounds__(1024) void argmax_kernel(const bf16_t* __restrict__ logits, int ldl, int V,
                                                      int* __restrict__ out_idx, int* __restrict__ tokens_out,
                                                      int tok_stride, const int* __restrict__ pos) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const int m = blockIdx.x, tid = threadIdx.x;
  const bf16_t* lr = logits + (size_t)m * ldl;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  auto take = [&](float x, int v) {
    if (x > best || (x == best && v < bi)) { best = x; bi = v; }
  };
  if ((V & 7) == 0 && (ldl & 7) == 0 && (reinterpret_cast<uintptr_t>(lr) & 15) == 0) {
    // 16-byte loads, 4 in flight per thread before any compare (V <= 32768 in one round)
    const uint4* l4 = reinterpret_cast<const uint4*>(lr);
    const int nv = V >> 3;
    for (int v0 = tid; v0 < nv; v0 += 4 * 1024) {
      uint4 r[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int v = v0 + 1024 * u;
        r[u] = l4[v < nv ? v : v0];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int v = v0 + 1024 * u;
        if (v < nv) {
          const uint32_t w[4] = {r[u].x, r[u].y, r[u].z, r[u].w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            take(bflo(w[i]), 8 * v + 2 * i);
            take(bfhi(w[i]), 8 * v + 2 * i + 1);
          }
        }
      }
    }
  } else {
    for (int v = tid; v < V; v += 1024) take(bf2f(lr[v]), v);
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

extern "C" {
LLJ_TRACE_EXPORT(ops)

int llj_embedding(const int* idx, const void* wte, void* out, int M, int C, int* pos_inc, void* stream) {
  LLJ_REQUIRE(M > 0 && C % 8 == 0);
  hipLaunchKernelGGL(embedding_kernel, dim3(M), dim3(256), 0, (hipStream_t)stream, idx, (const uint4*)wte,
                     (uint4*)out, C / 8, pos_inc);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_rmsnorm(const void* x, const void* w, float eps, void* y, int M, int C, void* stream) {
  return llj_rmsnorm_rows(x, w, eps, y, nullptr, M, C, stream);
}

int llj_rmsnorm_rows(const void* x, const void* w, float eps, void* y, float* rowsum, int M, int C, void* stream) {
  LLJ_REQUIRE(M > 0 && C % 8 == 0);
  hipLaunchKernelGGL(rmsnorm_kernel, dim3(M), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                     (const bf16_t*)w, eps, (bf16_t*)y, C, rowsum);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_attention(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T,
                  int n_head, int head_size, int S, void* stream) {
  LLJ_REQUIRE(B > 0 && T > 0 && n_head > 0 && S > 0);
  const float sl2 = 1.4426950408889634f / sqrtf((float)head_size);
  dim3 grid(n_head, B * T);
  if (head_size == 128) {
    hipLaunchKernelGGL((attention_kernel<128, LLJ_ATT_U, LLJ_ATT_NTH>), grid, dim3(LLJ_ATT_NTH), 0, (hipStream_t)stream, (const bf16_t*)q,
                       (const bf16_t*)kcache, (const bf16_t*)vcache, (bf16_t*)y, pos, T, S, n_head, sl2);
  } else if (head_size == 64) {
    hipLaunchKernelGGL((attention_kernel<64, LLJ_ATT_U, LLJ_ATT_NTH>), grid, dim3(LLJ_ATT_NTH), 0, (hipStream_t)stream, (const bf16_t*)q,
                       (const bf16_t*)kcache, (const bf16_t*)vcache, (bf16_t*)y, pos, T, S, n_head, sl2);
  } else {
    return LLJ_EINVAL;
  }
  LLJ_CHECK_LAUNCH();
  return 0;
}

size_t llj_attention_ws_bytes(int rows, int n_head, int head_size, int nsplit) {
  return (size_t)rows * n_head * (nsplit < 1 ? 1 : nsplit) * (head_size + 2) * sizeof(float);
}

int llj_attention_split(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T,
                        int n_head, int head_size, int S, int nsplit, void* part_ws, void* stream) {
  if (nsplit <= 1) return llj_attention(q, kcache, vcache, y, pos, B, T, n_head, head_size, S, stream);
  LLJ_REQUIRE(B > 0 && T > 0 && n_head > 0 && S > 0 && part_ws && nsplit <= 1024);
  const float sl2 = 1.4426950408889634f / sqrtf((float)head_size);
  const dim3 grid(n_head, B * T, nsplit), cgrid(n_head, B * T);
  hipStream_t st = (hipStream_t)stream;
  if (head_size == 128) {
    hipLaunchKernelGGL((attention_part_kernel<128, LLJ_ATT_U, LLJ_ATT_NTH>), grid, dim3(LLJ_ATT_NTH), 0, st,
                       (const bf16_t*)q, (const bf16_t*)kcache, (const bf16_t*)vcache, pos, T, S, n_head, sl2, nsplit,
                       (float*)part_ws);
    LLJ_CHECK_LAUNCH();
    hipLaunchKernelGGL((attention_combine_kernel<128>), cgrid, dim3(128), 0, st, (const float*)part_ws, (bf16_t*)y,
                       n_head, nsplit);
  } else if (head_size == 64) {
    hipLaunchKernelGGL((attention_part_kernel<64, LLJ_ATT_U, LLJ_ATT_NTH>), grid, dim3(LLJ_ATT_NTH), 0, st,
                       (const bf16_t*)q, (const bf16_t*)kcache, (const bf16_t*)vcache, pos, T, S, n_head, sl2, nsplit,
                       (float*)part_ws);
    LLJ_CHECK_LAUNCH();
    hipLaunchKernelGGL((attention_combine_kernel<64>), cgrid, dim3(64), 0, st, (const float*)part_ws, (bf16_t*)y,
                       n_head, nsplit);
  } else {
    return LLJ_EINVAL;
  }
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_argmax(const void* logits, int ldl, int M, int V, int* out_idx, int* tokens_out, int tok_stride,
               const int* pos, void* stream) {
  LLJ_REQUIRE(M > 0 && V > 0 && (!tokens_out || pos));
  hipLaunchKernelGGL(argmax_kernel, dim3(M), dim3(1024), 0, (hipStream_t)stream, (const bf16_t*)logits, ldl, V,
                     out_idx, tokens_out, tok_stride, pos);
  LLJ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

// Decode-step ops around the weight-streaming GEMVs: token embedding, standalone RMSNorm
// (prefill rows beyond the fused-LDS limit), causal attention over the KV cache, and the
// greedy (top_k = 1) next-token selection.
#include <cstdlib>

#include "common.h"
#include "attention.h"
#ifndef LLJ_NORM_SC1
#define LLJ_NORM_SC1 0
#endif
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

// any C (the any-shape path, csrc/generic.hip): bf16 elements
__global__ __launch_bounds__(256) void embedding_any_kernel(const int* __restrict__ idx, const bf16_t* __restrict__ wte,
                                                            bf16_t* __restrict__ out, int C, int* pos_inc) {
  const int m = blockIdx.x;
  const size_t r = (size_t)idx[m];
  for (int v = threadIdx.x; v < C; v += blockDim.x) out[(size_t)m * C + v] = wte[r * C + v];
  if (pos_inc && m == 0 && threadIdx.x == 0) *pos_inc += 1;
}

// ---- RMSNorm with the bf16 rounding points of model.py:281-283 on bf16 tensors. One block
// per row; rows up to 8192 wide are loaded once into registers (x and the scale together,
// before any use), so the kernel is one memory round trip.
// (norm_pair: common.h)

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
#if LLJ_NORM_SC1  // write-through (sc1) 8-byte stores, as the GEMV epilogues (A/B)
    unsigned long long* d8 = reinterpret_cast<unsigned long long*>(yr + v);
    __hip_atomic_store(d8, (unsigned long long)o0 | ((unsigned long long)o1 << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(d8 + 1, (unsigned long long)o2 | ((unsigned long long)o3 << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    yr[v] = make_uint4(o0, o1, o2, o3);
#endif
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
// 512 x 4 (128 keys per pass, half the serial score / softmax chain per lane of 256 x 8): 7B
// gptq.int4 decode-only at position ~80, bs=1 847.4 -> 857.8 tok/s, bs=8 4321 -> 4355
// (profiles/r04_attention_block_ab.json; 512 x 8 and 1024 x 2 in between)
#ifndef LLJ_ATT_NTH
#define LLJ_ATT_NTH 512  // threads per (row, head) block
#endif
#ifndef LLJ_ATT_SPEC_BATCH
#define LLJ_ATT_SPEC_BATCH 0  // half speculative pass at any grid size (A/B: option LLJ_OPT_ATT_SPEC_BATCH)
#endif
#ifndef LLJ_ATT_U
#define LLJ_ATT_U 4  // keys per 16-lane group per pass
#endif
template <int HS, int U, int NTH, int SPECU>
__global__ __launch_bounds__(NTH) void attention_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc,
                                                        const bf16_t* __restrict__ vc, bf16_t* __restrict__ y,
                                                        const int* __restrict__ pos, int T, int S, int nh,
                                                        float scale_log2, uint32_t* st, float thr, uint32_t* clr,
                                                        int clr_words, int spec_ok) {
  __shared__ float lds[attention_lds_floats<HS, NTH>()];
  attention_body<HS, U, NTH, false, SPECU>(q, kc, vc, y, pos, T, S, nh, scale_log2, blockIdx.x, blockIdx.y, lds, 1, 0,
                                           nullptr, st, thr, clr, clr_words, spec_ok != 0);
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

// interleaved key splits of a short cache (attention.h ILV), partials merged by the consumer
template <int HS, int U, int NTH, int SPECU>
__global__ __launch_bounds__(NTH) void attention_ilv_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc,
                                                            const bf16_t* __restrict__ vc, const int* __restrict__ pos,
                                                            int T, int S, int nh, float scale_log2, int nsplit,
                                                            float* __restrict__ part, int spec_ok) {
  __shared__ float lds[attention_lds_floats<HS, NTH>()];
  attention_body<HS, U, NTH, true, SPECU, true>(q, kc, vc, nullptr, pos, T, S, nh, scale_log2, blockIdx.x, blockIdx.y,
                                                lds, nsplit, blockIdx.z, part, nullptr, 0.f, nullptr, 0,
                                                spec_ok != 0);
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


// ---- sampled next token (generate.py:66-74 with top_k > 1 / None and a temperature):
//   x = bf16(logits * (1 / temperature)) (a bf16 tensor divided by a scalar on the device),
//   keep x >= the top_k-th largest x (torch.topk + where(x < v[-1], -inf): ties at the
//   threshold are kept), probs = bf16(softmax(x)) (fp32 inside), then one draw from probs.
// The draw is the inverse CDF over the kept probabilities in index order at a uniform u in
// [0, 1): the first index whose running sum exceeds u * sum(probs). torch.multinomial draws
// from the same distribution with its own generator (exponential race); u is either given
// (u_in, tests) or a counter-based hash of (seed, decode position, row), so a captured decode
// graph samples a fresh u every step without the host.
// One 1024-thread block per row. The top_k threshold is an exact radix select on the 16-bit
// order-preserving keys of the bf16 values (a 2048-bin histogram of key >> 5, then a 32-bin one
// inside the selected bin, each walked with a block suffix scan), so no sort is needed.
__device__ __forceinline__ uint32_t bf_key(uint32_t b) { return (b & 0x8000u) ? (~b & 0xFFFFu) : (b | 0x8000u); }
__device__ __forceinline__ float key_bf(uint32_t k) {
  const uint32_t b = (k & 0x8000u) ? (k & 0x7FFFu) : (~k & 0xFFFFu);
  return bf2f((bf16_t)b);
}
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

constexpr int kSampNT = 1024;
// Exclusive suffix sum over the block (thread order): sum of v over threads > tid.
__device__ __forceinline__ uint32_t block_suffix_excl(uint32_t v, uint32_t* wsum) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_down((int)x, o, 64);
    if (lane + o < 64) x += y;
  }
  if (lane == 0) wsum[wv] = x;
  __syncthreads();
  uint32_t above = 0;
  for (int w = wv + 1; w < kSampNT / 64; ++w) above += wsum[w];
  __syncthreads();
  return x - v + above;
}

// The logits type of the sampler: bf16 (the reference's GPU precision: x = bf16(logits * (1/T)),
// probabilities rounded to bf16; 16-bit keys selected in passes of 11 + 5 bits) or fp32 (its
// float32 model: x = logits / T, fp32 softmax; 32-bit keys in passes of 11 + 11 + 10 bits).
template <typename T>
struct SampTraits;
template <>
struct SampTraits<bf16_t> {
  static constexpr int NP = 2;
  static constexpr int SH[3] = {5, 0, 0}, W[3] = {11, 5, 0};
  __device__ static uint32_t key(const bf16_t* l, int i, float inv_t, float) { return bf_key(f2bf(bf2f(l[i]) * inv_t)); }
  __device__ static float val(uint32_t k) { return key_bf(k); }
  __device__ static float ex(float d) { return __expf(d); }
  __device__ static float prob(float e) { return bf2f(f2bf(e)); }
};
__device__ __forceinline__ uint32_t f_key(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float key_f(uint32_t k) { return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k); }
template <>
struct SampTraits<float> {
  static constexpr int NP = 3;
  static constexpr int SH[3] = {21, 10, 0}, W[3] = {11, 11, 10};
  __device__ static uint32_t key(const float* l, int i, float, float t) { return f_key(l[i] / t); }
  __device__ static float val(uint32_t k) { return key_f(k); }
  __device__ static float ex(float d) { return expf(d); }
  __device__ static float prob(float e) { return e; }
};

template <typename T>
__global__ __launch_bounds__(kSampNT) void sample_kernel(const T* __restrict__ logits, int ldl, int V, float inv_t,
                                                        float temp, int top_k, const float* __restrict__ u_in,
                                                        uint64_t seed, int* __restrict__ out_idx,
                                                        int* __restrict__ tokens_out, int tok_stride,
                                                        const int* __restrict__ pos) {
  using Tr = SampTraits<T>;
  constexpr int HB = 2048;  // the widest pass: 11 bits
  __shared__ uint32_t hist[HB];
  __shared__ float fred[kSampNT / 64];
  __shared__ uint32_t ured[kSampNT / 64];
  __shared__ float chunk_excl[kSampNT];
  __shared__ uint32_t sel[4];
  const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const T* lr = logits + (size_t)m * ldl;
  auto xkey = [&](int i) -> uint32_t { return Tr::key(lr, i, inv_t, temp); };
  const int k = top_k < 1 || top_k > V ? V : top_k;
  // ---- radix select: thr = the k-th largest key; keep key >= thr
  uint32_t prefix = 0, want = (uint32_t)k;
#pragma unroll
  for (int pass = 0; pass < Tr::NP; ++pass) {
    const int sh = Tr::SH[pass], nbins = 1 << Tr::W[pass];
    for (int b = tid; b < HB; b += kSampNT) hist[b] = 0;
    __syncthreads();
    for (int i = tid; i < V; i += kSampNT) {
      const uint32_t key = xkey(i);
      if (pass == 0 || (key >> (sh + Tr::W[pass])) == prefix) atomicAdd(&hist[(key >> sh) & (nbins - 1)], 1u);
    }
    __syncthreads();
    // thread t owns bins [b0, b0 + nb): counts above them by a suffix scan
    const int nb = nbins >= kSampNT ? nbins / kSampNT : (tid < nbins ? 1 : 0);
    const int b0 = nbins >= kSampNT ? nb * tid : tid;
    uint32_t c = 0;
    for (int q = 0; q < nb; ++q) c += hist[b0 + q];
    const uint32_t above = block_suffix_excl(c, ured);
    if (above < want && want <= above + c) {  // exactly one thread
      uint32_t a = above;
      int b = b0 + nb - 1;
      for (; b > b0; --b) {
        if (a + hist[b] >= want) break;
        a += hist[b];
      }
      sel[0] = (uint32_t)b;
      sel[1] = want - a;
    }
    __syncthreads();
    prefix = pass == 0 ? sel[0] : (prefix << Tr::W[pass]) | sel[0];
    want = sel[1];
    __syncthreads();
  }
  const uint32_t thr = prefix;
  // ---- max and sum of exp over the kept values (fp32, fixed reduction order)
  uint32_t kmax = 0;
  for (int i = tid; i < V; i += kSampNT) kmax = max(kmax, xkey(i));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o, 64));
  if (lane == 0) ured[wv] = kmax;
  __syncthreads();
  if (tid == 0) {
    uint32_t mk = 0;
    for (int w = 0; w < kSampNT / 64; ++w) mk = max(mk, ured[w]);
    sel[2] = mk;
  }
  __syncthreads();
  const float xmax = Tr::val(sel[2]);
  // each thread owns a contiguous index range (the CDF is taken in index order)
  const int per = (V + kSampNT - 1) / kSampNT;
  const int i0 = tid * per, i1 = min(V, i0 + per);
  float esum = 0.f;
  for (int i = i0; i < i1; ++i) {
    const uint32_t key = xkey(i);
    if (key >= thr) esum += Tr::ex(Tr::val(key) - xmax);
  }
  float t = wave_sum(esum);
  if (lane == 0) fred[wv] = t;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int w = 0; w < kSampNT / 64; ++w) tot += fred[w];
  const float rinv = 1.f / tot;
  // probabilities, chunk sums, exclusive scan over the chunks (thread order = index order)
  float csum = 0.f;
  for (int i = i0; i < i1; ++i) {
    const uint32_t key = xkey(i);
    if (key >= thr) csum += Tr::prob(Tr::ex(Tr::val(key) - xmax) * rinv);
  }
  chunk_excl[tid] = csum;
  __syncthreads();
  if (tid == 0) {  // sequential scan of 1024 chunk sums: deterministic
    float run = 0.f;
    for (int c = 0; c < kSampNT; ++c) {
      const float v = chunk_excl[c];
      chunk_excl[c] = run;
      run += v;
    }
    float u;
    if (u_in) {  // row m of the uniforms of this position (or of the only position without pos)
      u = u_in[(size_t)(pos ? pos[0] + 1 : 0) * gridDim.x + m];
    } else {
      const uint64_t h = splitmix64(seed ^ ((uint64_t)(pos ? pos[0] + 1 : 0) << 20) ^ (uint64_t)m);
      u = (float)(h >> 40) * (1.0f / 16777216.0f);
    }
    fred[0] = u * run;
    sel[3] = 0xFFFFFFFFu;
  }
  __syncthreads();
  const float target = fred[0];
  const float base = chunk_excl[tid];
  const float next = tid + 1 < kSampNT ? chunk_excl[tid + 1] : 3.4e38f;
  if (i0 < i1 && base <= target && target < next) {
    float run = base;
    int pick = -1, last = -1;
    for (int i = i0; i < i1; ++i) {
      const uint32_t key = xkey(i);
      if (key < thr) continue;
      last = i;
      run += Tr::prob(Tr::ex(Tr::val(key) - xmax) * rinv);
      if (run > target) { pick = i; break; }
    }
    if (pick < 0) pick = last;
    if (pick >= 0) atomicMin(&sel[3], (uint32_t)pick);
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t pick = sel[3];
    if (pick == 0xFFFFFFFFu) {  // u * sum at the very end (rounding): the last kept index
      for (int i = V - 1; i >= 0; --i)
        if (xkey(i) >= thr) { pick = (uint32_t)i; break; }
    }
    out_idx[m] = (int)pick;
    if (tokens_out) tokens_out[(size_t)m * tok_stride + pos[0] + 1] = (int)pick;
  }
}

// Streaming read of n16 16-byte words (the achievable HBM read rate the decode kernels are priced
// against): grid-stride, 4 non-temporal loads in flight per thread, one float per workgroup out so
// the loads stay live.
__global__ __launch_bounds__(256) void stream_read_kernel(const uint4* __restrict__ p, size_t n16, float* out) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u* q = reinterpret_cast<const v4u*>(p);
  uint32_t acc = 0;
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const v4u a = __builtin_nontemporal_load(q + i), b = __builtin_nontemporal_load(q + i + stride);
    const v4u c = __builtin_nontemporal_load(q + i + 2 * stride), d = __builtin_nontemporal_load(q + i + 3 * stride);
    acc ^= a.x ^ b.y ^ c.z ^ d.w;
  }
  for (; i < n16; i += stride) acc ^= __builtin_nontemporal_load(q + i).x;
  __shared__ uint32_t r[256];
  r[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int k = 0; k < 256; ++k) t ^= r[k];
    out[blockIdx.x] = (float)(t & 0xFFu);
  }
}

}  // namespace llj

using namespace llj;

extern "C" {
LLJ_TRACE_EXPORT(ops)

int llj_stream_read(const void* p, size_t bytes, float* out, int grid, void* stream) {
  LLJ_REQUIRE(p && out && bytes % 16 == 0 && grid > 0);
  hipLaunchKernelGGL(stream_read_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint4*)p, bytes / 16, out);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_embedding(const int* idx, const void* wte, void* out, int M, int C, int* pos_inc, void* stream) {
  LLJ_REQUIRE(M > 0 && C > 0);
  if (C % 8) {
    hipLaunchKernelGGL(embedding_any_kernel, dim3(M), dim3(256), 0, (hipStream_t)stream, idx, (const bf16_t*)wte,
                       (bf16_t*)out, C, pos_inc);
    LLJ_CHECK_LAUNCH();
    return 0;
  }
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

// decode attention, optionally with the LLM.int8 statistics of y (int8 c_proj) and a block to zero
static int attention_run(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T,
                         int n_head, int head_size, int S, uint32_t* st, float thr, uint32_t* clr, int clr_words,
                         void* stream) {
  LLJ_REQUIRE(B > 0 && T > 0 && n_head > 0 && S > 0);
  const float sl2 = 1.4426950408889634f / sqrtf((float)head_size);
  dim3 grid(n_head, B * T);
  // keys loaded before the position is known at small grids: half a pass (default) or a whole one
  // (option LLJ_OPT_ATT_SPEC_FULL: one memory latency less, more K / V rows read past the position)
  const bool full = opt(LLJ_OPT_ATT_SPEC_FULL) == 1;
  const int sb = opt(LLJ_OPT_ATT_SPEC_BATCH);
  const int spec_ok = (int)grid.x * (int)grid.y <= 64 || (!full && (sb < 0 ? LLJ_ATT_SPEC_BATCH : sb) != 0);
  hipStream_t st_ = (hipStream_t)stream;
#define LLJ_ATT_LAUNCH(HS_, SU_)                                                                                   \
  hipLaunchKernelGGL((attention_kernel<HS_, LLJ_ATT_U, LLJ_ATT_NTH, SU_>), grid, dim3(LLJ_ATT_NTH), 0, st_,         \
                     (const bf16_t*)q, (const bf16_t*)kcache, (const bf16_t*)vcache, (bf16_t*)y, pos, T, S, n_head, sl2, \
                     st, thr, clr, clr_words, spec_ok)
  if (head_size == 128) {
    if (full) LLJ_ATT_LAUNCH(128, LLJ_ATT_U); else LLJ_ATT_LAUNCH(128, LLJ_ATT_U / 2);
  } else if (head_size == 64) {
    if (full) LLJ_ATT_LAUNCH(64, LLJ_ATT_U); else LLJ_ATT_LAUNCH(64, LLJ_ATT_U / 2);
  } else {
    return LLJ_EINVAL;
  }
#undef LLJ_ATT_LAUNCH
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_attention(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T,
                  int n_head, int head_size, int S, void* stream) {
  return attention_run(q, kcache, vcache, y, pos, B, T, n_head, head_size, S, nullptr, 0.f, nullptr, 0, stream);
}

size_t llj_attention_ws_bytes(int rows, int n_head, int head_size, int nsplit) {
  return (size_t)rows * n_head * (nsplit < 1 ? 1 : nsplit) * (head_size + 4) * sizeof(float);  // kAttPart
}

static int attention_split_run(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B,
                               int T, int n_head, int head_size, int S, int nsplit, void* part_ws, uint32_t* st,
                               float thr, uint32_t* clr, int clr_words, void* stream) {
  if (nsplit <= 1)
    return attention_run(q, kcache, vcache, y, pos, B, T, n_head, head_size, S, st, thr, clr, clr_words, stream);
  LLJ_REQUIRE(B > 0 && T > 0 && n_head > 0 && S > 0 && part_ws && nsplit <= 1024);
  const float sl2 = 1.4426950408889634f / sqrtf((float)head_size);
  const dim3 grid(n_head, B * T, nsplit), cgrid(n_head, B * T);
  hipStream_t s = (hipStream_t)stream;
  if (head_size == 128) {
    hipLaunchKernelGGL((attention_part_kernel<128, LLJ_ATT_U, LLJ_ATT_NTH>), grid, dim3(LLJ_ATT_NTH), 0, s,
                       (const bf16_t*)q, (const bf16_t*)kcache, (const bf16_t*)vcache, pos, T, S, n_head, sl2, nsplit,
                       (float*)part_ws);
    LLJ_CHECK_LAUNCH();
    hipLaunchKernelGGL((attention_combine_kernel<128>), cgrid, dim3(128), 0, s, (const float*)part_ws, (bf16_t*)y,
                       n_head, nsplit, st, thr, clr, clr_words);
  } else if (head_size == 64) {
    hipLaunchKernelGGL((attention_part_kernel<64, LLJ_ATT_U, LLJ_ATT_NTH>), grid, dim3(LLJ_ATT_NTH), 0, s,
                       (const bf16_t*)q, (const bf16_t*)kcache, (const bf16_t*)vcache, pos, T, S, n_head, sl2, nsplit,
                       (float*)part_ws);
    LLJ_CHECK_LAUNCH();
    hipLaunchKernelGGL((attention_combine_kernel<64>), cgrid, dim3(64), 0, s, (const float*)part_ws, (bf16_t*)y,
                       n_head, nsplit, st, thr, clr, clr_words);
  } else {
    return LLJ_EINVAL;
  }
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_attention_split(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T,
                        int n_head, int head_size, int S, int nsplit, void* part_ws, void* stream) {
  return attention_split_run(q, kcache, vcache, y, pos, B, T, n_head, head_size, S, nsplit, part_ws, nullptr, 0.f,
                             nullptr, 0, stream);
}

// Decode attention (one-block or split over nsplit key ranges) that also writes the LLM.int8
// statistics of y for the int8 c_proj (i8ws.h; y_stats zeroed beforehand, B * T <= 8 rows) and zeroes
// clr_words words at clr (the previous layer's mlp.c_proj statistics block).
// Decode attention as nsplit interleaved key splits per (row, head) (block s takes the key groups
// s * NG + NG * nsplit * i: a fixed set, loaded before the position is known at small grids), each writing
// its unnormalized partial to part_ws; no combine launch -- llj_linear_resid_attn merges them in its prologue.
int llj_attention_part(const void* q, const void* kcache, const void* vcache, const int* pos, int B, int T,
                       int n_head, int head_size, int S, int nsplit, void* part_ws, void* stream) {
  LLJ_REQUIRE(B > 0 && T > 0 && n_head > 0 && S > 0 && part_ws && nsplit >= 1 && nsplit <= 64);
  const float sl2 = 1.4426950408889634f / sqrtf((float)head_size);
  const dim3 grid(n_head, B * T, nsplit);
  const int spec_ok = (int)(grid.x * grid.y * grid.z) <= 256;
  hipStream_t s = (hipStream_t)stream;
  if (head_size == 128)
    hipLaunchKernelGGL((attention_ilv_kernel<128, LLJ_ATT_U, LLJ_ATT_NTH, LLJ_ATT_U / 2>), grid, dim3(LLJ_ATT_NTH), 0, s,
                       (const bf16_t*)q, (const bf16_t*)kcache, (const bf16_t*)vcache, pos, T, S, n_head, sl2, nsplit,
                       (float*)part_ws, spec_ok);
  else if (head_size == 64)
    hipLaunchKernelGGL((attention_ilv_kernel<64, LLJ_ATT_U, LLJ_ATT_NTH, LLJ_ATT_U / 2>), grid, dim3(LLJ_ATT_NTH), 0, s,
                       (const bf16_t*)q, (const bf16_t*)kcache, (const bf16_t*)vcache, pos, T, S, n_head, sl2, nsplit,
                       (float*)part_ws, spec_ok);
  else
    return LLJ_EINVAL;
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_attention_i8(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T,
                     int n_head, int head_size, int S, int nsplit, void* part_ws, void* y_stats, void* clr,
                     int clr_words, float threshold, void* stream) {
  LLJ_REQUIRE(y_stats && B * T <= 8 && clr_words >= 0 && (!clr_words || clr));
  return attention_split_run(q, kcache, vcache, y, pos, B, T, n_head, head_size, S, nsplit, part_ws,
                             (uint32_t*)y_stats, threshold, (uint32_t*)clr, clr_words, stream);
}

int llj_sample(const void* logits, int ldl, int M, int V, float temperature, int top_k, const float* u,
               unsigned long long seed, int* out_idx, int* tokens_out, int tok_stride, const int* pos, void* stream) {
  LLJ_REQUIRE(M > 0 && V > 0 && temperature > 0.f && (!tokens_out || pos) && (u || pos));
  hipLaunchKernelGGL(sample_kernel<bf16_t>, dim3(M), dim3(kSampNT), 0, (hipStream_t)stream, (const bf16_t*)logits, ldl,
                     V, 1.f / temperature, temperature, top_k, u, (uint64_t)seed, out_idx, tokens_out, tok_stride, pos);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_g_sample(const float* logits, int ldl, int M, int V, float temperature, int top_k, const float* u,
                 unsigned long long seed, int* out_idx, int* tokens_out, int tok_stride, const int* pos, void* stream) {
  LLJ_REQUIRE(logits && out_idx && M > 0 && V > 0 && ldl >= V && temperature > 0.f && (!tokens_out || pos) && (u || pos));
  hipLaunchKernelGGL(sample_kernel<float>, dim3(M), dim3(kSampNT), 0, (hipStream_t)stream, logits, ldl, V,
                     1.f / temperature, temperature, top_k, u, (uint64_t)seed, out_idx, tokens_out, tok_stride, pos);
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

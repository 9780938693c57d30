// Decode attention over the KV cache (device code of the launches in ops.hip).
//
// Query rows m = b*T + t against cache slots of sequence b. Reference semantics
// (model.py:101-104, 218-237): the query at absolute position p attends the slots holding
// tokens <= p; once p >= S (sliding window after the roll) it attends all S slots. Slots are a
// ring (token p lives at p % S): the same key set as the reference's roll-by-one, so the
// softmax is identical up to summation order.
// 16 lanes per key (HS/16 dims each); NG = NTH/16 key groups, U keys per group per pass, so one
// pass has NG*U keys in flight, all loads of a pass issued before any use. Per-group online
// softmax; the groups of a wave merge through lane swaps, the waves through LDS.
#pragma once
#include "common.h"
#include "i8ws.h"

namespace llj {

template <int HS, int NTH>
constexpr int attention_lds_floats() {
  constexpr int NWV = NTH / 64;  // waves: one (max, sum, HS outputs) partial each
  return 2 * NWV + NWV * HS;
}

// LLM.int8() statistics of attention output rows for the int8 c_proj (i8ws.h): the calling wave
// holds 64 consecutive output columns col0 .. col0 + 63 of row m (bf16 bits in ob). Row maximum of
// |f16(y)| below the threshold (atomicMax on the float bits, SCA slot `slot`) and the outlier columns
// (atomicOr); both order-independent.
__device__ __forceinline__ void i8_emit_stats64(uint32_t* st, float thr, int m, int col0, uint32_t ob, int slot) {
  const float a16 = fabsf(f16r(bflo(ob)));
  const bool big = a16 >= thr;
  const float mx = wave_max(big ? 0.f : a16);
  const unsigned long long bal = __ballot(big);
  if ((threadIdx.x & 63) == 0) {
    atomicMax(st + kI8StSca + 8 * (slot % kI8StSlots) + m, __float_as_uint(mx));
    if ((uint32_t)bal) atomicOr(st + kI8StFlags + (col0 >> 5), (uint32_t)bal);
    if ((uint32_t)(bal >> 32)) atomicOr(st + kI8StFlags + (col0 >> 5) + 1, (uint32_t)(bal >> 32));
  }
}

// Merge two online-softmax partials (running max, sum, outputs) of the same dims: the lanes
// holding `lo` and `hi` compute the same expression, so both end bitwise equal.
template <int DPL>
__device__ __forceinline__ void softmax_merge(float& mx, float& l, float* o, const float mx_lo, const float mx_hi,
                                              const float l_lo, const float l_hi, const float* o_lo,
                                              const float* o_hi) {
  const float M = fmaxf(mx_lo, mx_hi);
  const float f_lo = mx_lo == -INFINITY ? 0.f : exp2f(mx_lo - M);
  const float f_hi = mx_hi == -INFINITY ? 0.f : exp2f(mx_hi - M);
  mx = M;
  l = l_lo * f_lo + l_hi * f_hi;
#pragma unroll
  for (int i = 0; i < DPL; ++i) o[i] = o_lo[i] * f_lo + o_hi[i] * f_hi;
}

// PART: split-K over the keys (long contexts): this block takes key range `split` of `nsplit`
// equal ranges (>= one pass of NG * U keys each) of the valid keys and writes its unnormalized partial (outputs, running max,
// sum) to part[((m * nh + h) * nsplit + split) * kAttPart<HS>]; attention_combine_kernel merges.
// ILV (with PART): interleaved splits for short caches -- block `split` takes the key groups
// j = split * NG + kg + NG * nsplit * i (a fixed set whatever the position, so its first pass can be
// loaded before the position is known); the partials are merged in the consumer's prologue (the
// attn.c_proj GEMV, gemv_impl.h apart) instead of a combine launch.
template <int HS>
constexpr int kAttPart = HS + 4;  // floats per partial record: HS outputs, max, sum, 2 pad (16-byte records)

template <int HS, int U, int NTH, bool PART = false, int SPECU = U / 2, bool ILV = false>
__device__ __forceinline__ void attention_body(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc,
                                               const bf16_t* __restrict__ vc, bf16_t* __restrict__ y,
                                               const int* __restrict__ pos, int T, int S, int nh, float scale_log2,
                                               int h, int m, float* lds, int nsplit = 1,
                                               int split = 0, float* __restrict__ part = nullptr,
                                               uint32_t* __restrict__ st = nullptr, float thr = 0.f,
                                               uint32_t* __restrict__ clr = nullptr, int clr_words = 0,
                                               bool spec_ok = false) {
  constexpr int DPL = HS / 16;
  constexpr int NG = NTH / 16;
  constexpr int NWV = NTH / 64;
  float* s_m = lds;                     // [NWV]
  float* s_l = s_m + NWV;               // [NWV]
  float* s_o = s_l + NWV;               // [NWV][HS]
  LLJ_STAMP(0);
  if (clr && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0)  // a statistics block to zero (int8 decode)
    for (int i = threadIdx.x; i < clr_words; i += NTH) clr[i] = 0u;
  const int b = m / T, t = m % T;
  const int sub = threadIdx.x & 15, kg = threadIdx.x >> 4;
  const int C = nh * HS;
  const size_t base = ((size_t)(b * nh + h) * S) * HS + sub * DPL;  // elements
  // K/V rows of one pass (U keys of this group): every load first, rows clamped into the cache
  // keys u in [u0, u1) of a pass; past jlim: row 0 (an L2 hit after the first pass, never used)
  const int KS = ILV ? NG * nsplit : NG;  // key stride between a group's keys of one pass
  auto load_pass = [&](int j0, int jlim, uint32_t (&kw)[U][DPL / 2], uint32_t (&vw)[U][DPL / 2], int u0 = 0,
                       int u1 = U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u < u0 || u >= u1) continue;
      const int j = j0 + KS * u < jlim ? j0 + KS * u : 0;
      const size_t eo = base + (size_t)j * HS;
      if constexpr (DPL == 8) {
        const uint4 a = *reinterpret_cast<const uint4*>(kc + eo);
        const uint4 c = *reinterpret_cast<const uint4*>(vc + eo);
        kw[u][0] = a.x; kw[u][1] = a.y; kw[u][2] = a.z; kw[u][3] = a.w;
        vw[u][0] = c.x; vw[u][1] = c.y; vw[u][2] = c.z; vw[u][3] = c.w;
      } else {
        const uint2 a = *reinterpret_cast<const uint2*>(kc + eo);
        const uint2 c = *reinterpret_cast<const uint2*>(vc + eo);
        kw[u][0] = a.x; kw[u][1] = a.y;
        vw[u][0] = c.x; vw[u][1] = c.y;
      }
    }
  };
  uint32_t kw[U][DPL / 2], vw[U][DPL / 2];
  // the first half of the first pass (keys kg + NG u, u < U / 2: slots 0 .. NG U / 2 - 1) is
  // loaded before the position is known: the cache rows exist whatever p is, and keys past the
  // valid range are masked below, so the position read and the first K/V reads are one memory
  // latency instead of two; the second half waits for the position and reads only valid rows
  // (a whole speculative pass read 128 rows at p = 80: 1.6x the K/V bytes the step uses). spec_ok
  // (host): small grids (bs = 1: 32 blocks), where the launch is latency-bound, and -- option
  // LLJ_OPT_ATT_SPEC_BATCH -- half passes at any grid; a whole pass over many blocks read more rows
  // past p than the latency saved (7B bs=8: 1.79 -> 1.87 ms)
  const bool spec = (!PART || ILV) && spec_ok;
  if (spec) load_pass((ILV ? split * NG : 0) + kg, S, kw, vw, 0, SPECU);
  const int ps = pos[t];
  const int nvalid = ps < S ? ps + 1 : S;
  // key range of this block (the whole valid range unless split)
  int jbeg = 0, jend = nvalid;
  if constexpr (ILV) {
    jbeg = split * NG;
  } else if constexpr (PART) {  // ranges of at least one full pass (NG * U keys); the rest stay empty
    const int chunk = max((nvalid + nsplit - 1) / nsplit, NG * U);
    jbeg = split * chunk;
    jend = min(nvalid, jbeg + chunk);
  }
  float qf[DPL];
  {
    const size_t qo = (size_t)m * C + h * HS + sub * DPL;
    if constexpr (DPL == 8) {
      const uint4 a = *reinterpret_cast<const uint4*>(q + qo);
      const uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        qf[2 * i] = bflo(w[i]) * scale_log2;
        qf[2 * i + 1] = bfhi(w[i]) * scale_log2;
      }
    } else {
      const uint2 a = *reinterpret_cast<const uint2*>(q + qo);
      qf[0] = bflo(a.x) * scale_log2;
      qf[1] = bfhi(a.x) * scale_log2;
      qf[2] = bflo(a.y) * scale_log2;
      qf[3] = bfhi(a.y) * scale_log2;
    }
  }
  LLJ_STAMP(2);
  float mx = -INFINITY, l = 0.f, o[DPL];
#pragma unroll
  for (int i = 0; i < DPL; ++i) o[i] = 0.f;

  bool first = spec;
  for (int j0 = jbeg + kg; j0 < jend; j0 += KS * U) {
    if (!first) load_pass(j0, jend, kw, vw);
    else if (SPECU < U) load_pass(j0, jend, kw, vw, SPECU, U);  // the speculative pass's second half
    first = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < DPL / 2; ++i) s += qf[2 * i] * bflo(kw[u][i]) + qf[2 * i + 1] * bfhi(kw[u][i]);
      s = row16_sum(s);  // the 16 lanes of this key
      if (j0 + KS * u >= jend) continue;
      const float mn = fmaxf(mx, s);
      const float corr = exp2f(mx - mn);
      const float pj = exp2f(s - mn);
      l = l * corr + pj;
#pragma unroll
      for (int i = 0; i < DPL / 2; ++i) {
        o[2 * i] = o[2 * i] * corr + pj * bflo(vw[u][i]);
        o[2 * i + 1] = o[2 * i + 1] * corr + pj * bfhi(vw[u][i]);
      }
      mx = mn;
    }
  }
  LLJ_STAMP(3);
  // combine the key groups: the four 16-lane groups of a wave with lane swaps (rows 0+1 and
  // 2+3, then the two halves; every lane of a group holds the group's max and sum and its
  // DPL output dims), then the NWV wave partials through LDS in wave order
  {
    float mlo, mhi, llo, lhi, olo[DPL], ohi[DPL];
    lane_halves<false>(mx, mlo, mhi);
    lane_halves<false>(l, llo, lhi);
#pragma unroll
    for (int i = 0; i < DPL; ++i) lane_halves<false>(o[i], olo[i], ohi[i]);
    softmax_merge<DPL>(mx, l, o, mlo, mhi, llo, lhi, olo, ohi);
    lane_halves<true>(mx, mlo, mhi);
    lane_halves<true>(l, llo, lhi);
#pragma unroll
    for (int i = 0; i < DPL; ++i) lane_halves<true>(o[i], olo[i], ohi[i]);
    softmax_merge<DPL>(mx, l, o, mlo, mhi, llo, lhi, olo, ohi);
  }
  const int wv = threadIdx.x >> 6;
  if (kg % 4 == 0) {  // the first 16 lanes of each wave
#pragma unroll
    for (int i = 0; i < DPL; ++i) s_o[wv * HS + sub * DPL + i] = o[i];
    if (sub == 0) {
      s_m[wv] = mx;
      s_l[wv] = l;
    }
  }
  __syncthreads();
  LLJ_STAMP(4);
  if (threadIdx.x < HS) {  // waves 0 (and 1): adjacent dims leave as one 4-byte store
    const int d = threadIdx.x;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NWV; ++w) M = fmaxf(M, s_m[w]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
      const float f = s_m[w] == -INFINITY ? 0.f : exp2f(s_m[w] - M);
      L += s_l[w] * f;
      O += s_o[w * HS + d] * f;
    }
    if constexpr (PART) {  // unnormalized partial: outputs, then (max, sum)
      float* dst = part + ((size_t)(m * nh + h) * nsplit + split) * kAttPart<HS>;
      dst[d] = O;
      if (d == 0) {
        dst[HS] = M;
        dst[HS + 1] = L;
      }
      LLJ_STAMP(5);
      return;
    }
    const uint32_t ob = (uint32_t)f2bf(O / L);
    const uint32_t pr = lane_xor1(ob);
    if (!(d & 1)) {
      const size_t eo = (size_t)m * C + h * HS + d;
      st_out32(y + eo, ob | (pr << 16));
    }
    if (st) i8_emit_stats64(st, thr, m, h * HS + (d & ~63), ob, h);  // uniform; one SCA slot per head
  }
  LLJ_STAMP(5);
}

// Merge the nsplit partials of one (head, row) in split order: y = sum_s O_s f_s / sum_s L_s f_s
// with f_s = exp2(M_s - max_s M_s) (empty ranges have M = -inf and contribute nothing).
template <int HS>
__global__ __launch_bounds__(HS) void attention_combine_kernel(const float* __restrict__ part, bf16_t* __restrict__ y,
                                                               int nh, int nsplit, uint32_t* __restrict__ st = nullptr,
                                                               float thr = 0.f, uint32_t* __restrict__ clr = nullptr,
                                                               int clr_words = 0) {
  const int h = blockIdx.x, m = blockIdx.y, d = threadIdx.x;
  const float* src = part + (size_t)(m * nh + h) * nsplit * kAttPart<HS>;
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, src[(size_t)s * kAttPart<HS> + HS]);
  float L = 0.f, O = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const float* ps = src + (size_t)s * kAttPart<HS>;
    const float f = ps[HS] == -INFINITY ? 0.f : exp2f(ps[HS] - M);
    L += ps[HS + 1] * f;
    O += ps[d] * f;
  }
  const uint32_t ob = (uint32_t)f2bf(O / L);
  const uint32_t pr = lane_xor1(ob);
  if (!(d & 1)) *reinterpret_cast<uint32_t*>(y + (size_t)m * nh * HS + h * HS + d) = ob | (pr << 16);
  if (st) i8_emit_stats64(st, thr, m, h * HS + (d & ~63), ob, h);
  if (clr && h == 0 && m == 0)
    for (int i = d; i < clr_words; i += HS) clr[i] = 0u;
}

}  // namespace llj

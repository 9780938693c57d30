// Decode attention over the KV cache (device code shared by the standalone launch in ops.hip
// and the chained decode-layer launch in gemv.hip).
//
// Query rows m = b*T + t against cache slots of sequence b. Reference semantics
// (model.py:101-104, 218-237): the query at absolute position p attends the slots holding
// tokens <= p; once p >= S (sliding window after the roll) it attends all S slots. Slots are a
// ring (token p lives at p % S): the same key set as the reference's roll-by-one, so the
// softmax is identical up to summation order.
// 16 lanes per key (HS/16 dims each); NG = NTH/16 key groups, U keys per group per pass, so one
// pass has NG*U keys in flight, all loads of a pass issued before any use. Per-group online
// softmax, combined through LDS.
#pragma once
#include "chain.h"
#include "common.h"

namespace llj {

template <int HS, int NTH>
constexpr int attention_lds_floats() {
  constexpr int NG = NTH / 16, PARTS = NTH / HS;
  return 2 * NG + NG * (HS + 1) + PARTS * HS + PARTS;
}

// CH: chained launch — wait for the QKV op, then read q and the cache with sc1 loads and
// store y with sc1 stores (chain.h protocol).
// SIG: signal a consumer op of the same launch (sc1 y stores, drain, count done); CH implies it.
template <int HS, int U, int NTH, bool CH, bool SIG = CH>
__device__ __forceinline__ void attention_body(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc,
                                               const bf16_t* __restrict__ vc, bf16_t* __restrict__ y,
                                               const int* __restrict__ pos, int T, int S, int nh, float scale_log2,
                                               int h, int m, float* lds, const ChainCtl& cc) {
  constexpr int DPL = HS / 16;
  constexpr int NG = NTH / 16;
  constexpr int PARTS = NTH / HS;
  float* s_m = lds;
  float* s_l = s_m + NG;
  float* s_o = s_l + NG;                // [NG][HS + 1]
  float* s_po = s_o + NG * (HS + 1);    // [PARTS][HS]
  float* s_pl = s_po + PARTS * HS;      // [PARTS]
  LLJ_STAMP(0);
  if constexpr (CH) chain_wait(cc);
  LLJ_STAMP(1);
  const int b = m / T, t = m % T;
  const int ps = pos[t];
  const int nvalid = ps < S ? ps + 1 : S;
  const int sub = threadIdx.x & 15, kg = threadIdx.x >> 4;
  const int C = nh * HS;
  const size_t base = ((size_t)(b * nh + h) * S) * HS + sub * DPL;  // elements
  float qf[DPL];
  {
    const size_t qo = (size_t)m * C + h * HS + sub * DPL;
    if constexpr (DPL == 8) {
      uint4 a;
      if constexpr (CH) a = __builtin_bit_cast(uint4, ld16_sc1(q, (unsigned)(qo * 2)));
      else a = *reinterpret_cast<const uint4*>(q + qo);
      const uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        qf[2 * i] = bflo(w[i]) * scale_log2;
        qf[2 * i + 1] = bfhi(w[i]) * scale_log2;
      }
    } else {
      uint2 a;
      if constexpr (CH) a = ld8_sc1(q, (unsigned)(qo * 2));
      else a = *reinterpret_cast<const uint2*>(q + qo);
      qf[0] = bflo(a.x) * scale_log2;
      qf[1] = bfhi(a.x) * scale_log2;
      qf[2] = bflo(a.y) * scale_log2;
      qf[3] = bfhi(a.y) * scale_log2;
    }
  }
  float mx = -INFINITY, l = 0.f, o[DPL];
#pragma unroll
  for (int i = 0; i < DPL; ++i) o[i] = 0.f;

  for (int j0 = kg; j0 < nvalid; j0 += NG * U) {
    uint32_t kw[U][DPL / 2], vw[U][DPL / 2];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // every load of the pass first (clamped: always valid rows)
      const int j = j0 + NG * u < nvalid ? j0 + NG * u : j0;
      const size_t eo = base + (size_t)j * HS;
      if constexpr (DPL == 8) {
        uint4 a, c;
        if constexpr (CH) {
          a = __builtin_bit_cast(uint4, ld16_sc1(kc, (unsigned)(eo * 2)));
          c = __builtin_bit_cast(uint4, ld16_sc1(vc, (unsigned)(eo * 2)));
        } else {
          a = *reinterpret_cast<const uint4*>(kc + eo);
          c = *reinterpret_cast<const uint4*>(vc + eo);
        }
        kw[u][0] = a.x; kw[u][1] = a.y; kw[u][2] = a.z; kw[u][3] = a.w;
        vw[u][0] = c.x; vw[u][1] = c.y; vw[u][2] = c.z; vw[u][3] = c.w;
      } else {
        uint2 a, c;
        if constexpr (CH) {
          a = ld8_sc1(kc, (unsigned)(eo * 2));
          c = ld8_sc1(vc, (unsigned)(eo * 2));
        } else {
          a = *reinterpret_cast<const uint2*>(kc + eo);
          c = *reinterpret_cast<const uint2*>(vc + eo);
        }
        kw[u][0] = a.x; kw[u][1] = a.y;
        vw[u][0] = c.x; vw[u][1] = c.y;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < DPL / 2; ++i) s += qf[2 * i] * bflo(kw[u][i]) + qf[2 * i + 1] * bfhi(kw[u][i]);
      s = row16_sum(s);  // the 16 lanes of this key
      if (j0 + NG * u >= nvalid) continue;
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
  if (sub == 0) {
    s_m[kg] = mx;
    s_l[kg] = l;
  }
#pragma unroll
  for (int i = 0; i < DPL; ++i) s_o[kg * (HS + 1) + sub * DPL + i] = o[i];
  __syncthreads();
  // combine the NG groups: HS output dims x PARTS partial sums over the groups
  {
    const int d = threadIdx.x % HS, part = threadIdx.x / HS;
    float M = -INFINITY;
#pragma unroll 8
    for (int g = 0; g < NG; ++g) M = fmaxf(M, s_m[g]);
    float L = 0.f, O = 0.f;
    for (int g = part; g < NG; g += PARTS) {
      const float f = s_m[g] == -INFINITY ? 0.f : exp2f(s_m[g] - M);
      L += s_l[g] * f;
      O += s_o[g * (HS + 1) + d] * f;
    }
    s_po[part * HS + d] = O;
    if (d == 0) s_pl[part] = L;
  }
  __syncthreads();
  if (threadIdx.x < HS) {  // waves 0 (and 1): adjacent dims leave as one 4-byte store
    const int d = threadIdx.x;
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int pp = 0; pp < PARTS; ++pp) {
      L += s_pl[pp];
      O += s_po[pp * HS + d];
    }
    const uint32_t ob = (uint32_t)f2bf(O / L);
    const uint32_t pr = lane_xor1(ob);
    if (!(d & 1)) {
      const size_t eo = (size_t)m * C + h * HS + d;
      if constexpr (SIG) st4_sc1(y, (unsigned)(eo * 2), ob | (pr << 16));
      else *reinterpret_cast<uint32_t*>(y + eo) = ob | (pr << 16);
    }
  }
  if constexpr (SIG) {
    // every storing wave drains; the workgroup counts done once all have (LDS barrier)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) chain_count_done(cc);
  }
  LLJ_STAMP(5);
}

}  // namespace llj

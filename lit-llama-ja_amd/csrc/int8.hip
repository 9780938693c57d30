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
#include "lit_llama_amd.h"

namespace llj {

__device__ __forceinline__ float to_f16f(float x) { return (float)(_Float16)x; }

// Pass 1, one block per k-range: outlier columns (any row |A16| >= thr) as flags and an
// ascending list, and per-row absmax of the other elements.
__global__ __launch_bounds__(256) void i8_stats_kernel(const bf16_t* __restrict__ A, int lda, int M, int K,
                                                       float thr, char* __restrict__ ws, int kb) {
  __shared__ int flag[1024];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const I8Layout L = i8_layout(ws, M, K);
  if (b == 0 && tid == 0) *reinterpret_cast<I8WsHeader*>(ws) = I8WsHeader{M, K, kNSB, kb}, L.avh[0] = 0;  // no aval
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

// Pass 1 for many rows (prompt windows, M >= kRowsStatsMin): block (k-block b, 32-row group);
// wave w takes rows r0 + w, r0 + w + 4, ... (8 rows, loaded together), its lanes the k-block's
// vectors of 8 columns (kb <= 512). Per-(k-block, row) maxima of the elements below the threshold
// into part; outlier columns OR-ed into the flag bytes (zeroed before the launch) by 32-bit atomics.
// The list / counts follow from the complete flags in pass 2 (i8_quant_act_kernel, `list`). Same
// workspace bytes as i8_stats_kernel (max and OR do not depend on the order).
constexpr int kRowsStatsMin = 32;
__global__ __launch_bounds__(256) void i8_stats_rows_kernel(const bf16_t* __restrict__ A, int lda, int M, int K,
                                                            float thr, char* __restrict__ ws, int kb) {
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const I8Layout L = i8_layout(ws, M, K);
  if (b == 0 && blockIdx.y == 0 && tid == 0) *reinterpret_cast<I8WsHeader*>(ws) = I8WsHeader{M, K, kNSB, kb}, L.avh[0] = 0;  // no aval
  const int k0 = b * kb, k1 = min(K, k0 + kb);
  const int nv = k1 > k0 ? (k1 - k0) >> 3 : 0;
  const bool act = lane < nv;
  const int kk = k0 + 8 * (act ? lane : 0);
  const int r0 = blockIdx.y * 32 + wave;
  uint4 xa[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = r0 + 4 * i < M ? r0 + 4 * i : M - 1;
    xa[i] = *reinterpret_cast<const uint4*>(A + (size_t)m * lda + (kk < K ? kk : 0));
  }
  unsigned fl = 0;  // bit e: column kk + e is an outlier in one of this wave's rows
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = r0 + 4 * i;  // uniform per wave
    if (m >= M) break;
    float mx = 0.f;
    if (act) {
      const uint32_t aw[4] = {xa[i].x, xa[i].y, xa[i].z, xa[i].w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float av = fabsf(to_f16f((e & 1) ? bfhi(aw[e >> 1]) : bflo(aw[e >> 1])));
        if (av >= thr) fl |= 1u << e;
        else mx = fmaxf(mx, av);
      }
    }
    mx = wave_max(mx);
    if (lane == 0) L.part[(size_t)b * M + m] = mx;
  }
  if (act && fl) {
    auto bytes = [](unsigned f4) {
      return (f4 & 1u) | ((f4 & 2u) << 7) | ((f4 & 4u) << 14) | ((f4 & 8u) << 21);
    };
    unsigned* fw = reinterpret_cast<unsigned*>(L.flag + kk);
    if (fl & 0xFu) atomicOr(fw, bytes(fl & 0xFu));
    if (fl >> 4) atomicOr(fw + 1, bytes(fl >> 4));
  }
}

// Pass 1 fused with the RMSNorm before it (decode rows, M <= MR): every block reduces the
// sums of squares of all M rows itself -- the rmsnorm_kernel's summation order exactly (thread t:
// vectors t, t + 256, ... in order; wave sums; the 4 wave partials in order), so r is bit-identical
// to llj_rmsnorm's --, writes the normalized rows of its own k-range (xn) and takes the outlier
// flags / row maxima of those values (the i8_stats_kernel rule). One launch instead of two.
template <int MR, int VPT>
__global__ __launch_bounds__(256) void i8_norm_stats_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                            float eps, bf16_t* __restrict__ xn, int M, int K, float thr,
                                                            char* __restrict__ ws, int kb) {
  constexpr int RG = 4;  // rows whose vectors are in flight together
  __shared__ int flag[1024];
  __shared__ float red[4][MR];
  __shared__ float rr[MR];
  __shared__ int rmax[MR];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const I8Layout L = i8_layout(ws, M, K);
  if (b == 0 && tid == 0) *reinterpret_cast<I8WsHeader*>(ws) = I8WsHeader{M, K, kNSB, kb}, L.avh[0] = 0;  // no aval
  const int k0 = b * kb;
  const int k1 = min(K, k0 + kb);
  const int nvec = K >> 3;
  const int vpr = k1 > k0 ? (k1 - k0) >> 3 : 0;  // vectors of 8 per row in this block's range
  // this thread's (row, vector) of the own range (M * vpr <= 256 on this path), loaded first
  const bool own = tid < M * vpr;
  const int om = own ? tid / vpr : 0, ov = own ? (k0 >> 3) + tid % vpr : 0;
  const uint4 oa = reinterpret_cast<const uint4*>(x + (size_t)om * K)[ov];
  const uint4 og = reinterpret_cast<const uint4*>(w)[ov];
  for (int i = tid; i < kb; i += 256) flag[i] = 0;
  if (tid < MR) rmax[tid] = 0;
  float ss[MR];
#pragma unroll
  for (int m0 = 0; m0 < MR; m0 += RG) {
    uint4 xa[RG][VPT];
#pragma unroll
    for (int r = 0; r < RG; ++r)
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const int m = m0 + r < M ? m0 + r : M - 1, v = tid + 256 * j < nvec ? tid + 256 * j : nvec - 1;
        xa[r][j] = reinterpret_cast<const uint4*>(x + (size_t)m * K)[v];
      }
#pragma unroll
    for (int r = 0; r < RG; ++r) {
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        if (tid + 256 * j < nvec) {
          const uint32_t aw[4] = {xa[r][j].x, xa[r][j].y, xa[r][j].z, xa[r][j].w};
#pragma unroll
          for (int i = 0; i < 4; ++i) a += round_bf(bflo(aw[i]) * bflo(aw[i])) + round_bf(bfhi(aw[i]) * bfhi(aw[i]));
        }
      }
      ss[m0 + r] = a;
    }
  }
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    const float t = wave_sum(ss[m]);
    if (lane == 0) red[wave][m] = t;
  }
  __syncthreads();
  if (tid < MR) {
    const float tot = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
    rr[tid] = round_bf(rsqrtf(round_bf(round_bf(tot / (float)K) + eps)));
  }
  __syncthreads();
  if (own) {  // normalize, store, statistics of the own (row, vector)
    const float r = rr[om];
    const uint4 o = make_uint4(norm_pair(oa.x, og.x, r), norm_pair(oa.y, og.y, r), norm_pair(oa.z, og.z, r),
                               norm_pair(oa.w, og.w, r));
    reinterpret_cast<uint4*>(xn + (size_t)om * K)[ov] = o;
    const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float av = fabsf(to_f16f((i & 1) ? bfhi(ow[i >> 1]) : bflo(ow[i >> 1])));
      if (av >= thr) flag[8 * ov + i - k0] = 1;
      else mx = fmaxf(mx, av);
    }
    atomicMax(&rmax[om], __float_as_int(mx));  // non-negative floats order as their bits
  }
  __syncthreads();
  if (tid < M && tid < MR) L.part[(size_t)b * M + tid] = __int_as_float(rmax[tid]);
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

// The whole activation preparation in ONE launch for decode batches (M <= 8 rows): one 1024-thread
// block per k-block (kNSB blocks). Every block reads all M rows (four 256-thread groups, group g
// taking rows g and g + 4 with llj_rmsnorm's thread-to-vector map, so with norm_w the sums of
// squares -- and xn -- are bit-identical to llj_rmsnorm's) and reduces each row's SCA = max of the
// elements below the threshold itself (redundant across blocks, no grid-wide dependency); then it
// finishes its own k-block: outlier flags, the list, part, the normalized rows (xn) and the
// quantized rows (aq). Block 0 writes the header and SCA.
#ifndef LLJ_PREP_ABL
#define LLJ_PREP_ABL 0  // timing ablations only (results wrong): 1 no sums of squares, 2 no row maxima, 4 no row loads, 8 no list
#endif
template <bool NORM, int VPT>
__global__ __launch_bounds__(1024) void i8_prep_one_kernel(const bf16_t* __restrict__ x, int lda,
                                                           const bf16_t* __restrict__ w, float eps,
                                                           bf16_t* __restrict__ xn, int M, int K, float thr,
                                                           char* __restrict__ ws, int kb,
                                                           uint32_t* __restrict__ st = nullptr) {
  constexpr int MR = 8;
  __shared__ int flag[1024];
  __shared__ float red[MR][4];
  __shared__ float rr[MR];
  __shared__ float mred[16][MR];
  __shared__ int pmax[MR];
  __shared__ uint4 vals[MR][1024 / 8];  // the own k-block's (normalized) rows, for aval
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int grp = tid >> 8, lt = tid & 255, gw = lt >> 6;  // row group, thread / wave within it
  const I8Layout L = i8_layout(ws, M, K);
  const int nvec = K >> 3;
  const int k0 = b * kb, k1 = min(K, k0 + kb);
  const int vpr = k1 > k0 ? (k1 - k0) >> 3 : 0;
  // own k-block item (row, vector), loaded first (M * vpr <= 1024 on this path)
  const bool own = tid < M * vpr;
  const int om = own ? tid / vpr : 0, ov = own ? (k0 >> 3) + tid % vpr : 0;
  const uint4 oa = reinterpret_cast<const uint4*>(x + (size_t)om * lda)[ov];
  uint4 og = oa;
  if (NORM) og = reinterpret_cast<const uint4*>(w)[ov];
  // rows grp and grp + 4, vectors lt + 256 j (past the row: zeros, which add nothing to either pass)
  uint4 xa[2][VPT], ga[VPT];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const bool ok = lt + 256 * j < nvec;
      const int m = grp + 4 * r < M ? grp + 4 * r : M - 1, v = ok ? lt + 256 * j : nvec - 1;
      const uint4 t = (LLJ_PREP_ABL & 4) ? oa : reinterpret_cast<const uint4*>(x + (size_t)m * lda)[v];
      xa[r][j] = ok ? t : make_uint4(0u, 0u, 0u, 0u);
    }
  if (NORM) {
#pragma unroll
    for (int j = 0; j < VPT; ++j) ga[j] = reinterpret_cast<const uint4*>(w)[lt + 256 * j < nvec ? lt + 256 * j : nvec - 1];
  }
  for (int i = tid; i < kb; i += 1024) flag[i] = 0;
  if (tid < MR) pmax[tid] = 0;
  if (NORM && !(LLJ_PREP_ABL & 1)) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const uint32_t aw[4] = {xa[r][j].x, xa[r][j].y, xa[r][j].z, xa[r][j].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // a += bf16(lo * lo) + bf16(hi * hi), llj_rmsnorm's order
          const f32x2 q = unpk(cvt_pk(unpk(aw[i]) * unpk(aw[i])));
          a += q.x + q.y;
        }
      }
      a = wave_sum(a);
      if (lane == 0) red[grp + 4 * r][gw] = a;
    }
    __syncthreads();
    if (tid < MR) rr[tid] = round_bf(rsqrtf(round_bf(round_bf((red[tid][0] + red[tid][1] + red[tid][2] + red[tid][3]) / (float)K) + eps)));
    __syncthreads();
  }
  if ((LLJ_PREP_ABL & 1) && tid < MR) rr[tid] = 1.f;
  if (LLJ_PREP_ABL & 1) __syncthreads();
  // each row's maximum of the (normalized) elements below the threshold. The elements are bf16
  // values, exact in fp16 wherever |v| >= 2^-14, and fp16 rounding is monotonic: for a threshold
  // >= 2^-14, max f16(|v|) over f16(|v|) < thr is f16(max |v| over |v| < thr) -- no per-element
  // conversion (the i8_stats_kernel rule, bit for bit)
#pragma unroll
  for (int r = 0; r < ((LLJ_PREP_ABL & 2) ? 0 : 2); ++r) {
    const float rn = NORM ? rr[grp + 4 * r < M ? grp + 4 * r : M - 1] : 1.f;
    const f32x2 rn2 = {rn, rn};
    float mx = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const uint32_t aw[4] = {xa[r][j].x, xa[r][j].y, xa[r][j].z, xa[r][j].w};
      const uint32_t gw4[4] = {ga[j].x, ga[j].y, ga[j].z, ga[j].w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f32x2 v = unpk(aw[i]);
        if (NORM) v = unpk(cvt_pk(unpk(gw4[i]) * unpk(cvt_pk(v * rn2))));  // g * bf16(x * r), rounded
        const float a0 = fabsf(v.x), a1 = fabsf(v.y);
        mx = fmaxf(mx, a0 < thr ? a0 : 0.f);
        mx = fmaxf(mx, a1 < thr ? a1 : 0.f);
      }
    }
    mx = to_f16f(wave_max(mx));
    if (lane == 0) mred[tid >> 6][r] = mx;  // wave (grp, gw): slot r <-> row grp + 4 r
  }
  if (!NORM) __syncthreads();  // flag / pmax zeroed before any thread sets them (NORM: synced above)
  // own k-block: normalize, flags, per-row maximum
  uint4 on = oa;
  if (NORM && own) {
    const float rn = rr[om];
    on = make_uint4(norm_pair(oa.x, og.x, rn), norm_pair(oa.y, og.y, rn), norm_pair(oa.z, og.z, rn),
                    norm_pair(oa.w, og.w, rn));
  }
  if (own) {
    if (NORM) reinterpret_cast<uint4*>(xn + (size_t)om * K)[ov] = on;
    vals[om][ov - (k0 >> 3)] = on;
    const uint32_t ow[4] = {on.x, on.y, on.z, on.w};
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float av = fabsf(to_f16f((i & 1) ? bfhi(ow[i >> 1]) : bflo(ow[i >> 1])));
      if (av >= thr) flag[8 * ov + i - k0] = 1;
      else mx = fmaxf(mx, av);
    }
    atomicMax(&pmax[om], __float_as_int(mx));  // non-negative floats order as their bits
  }
  __syncthreads();
  // SCA of row m: max over the 4 waves of its group (slot m >> 2)
  if (own) {
    const int g = om & 3, r = om >> 2;
    const float sca = fmaxf(fmaxf(mred[4 * g][r], mred[4 * g + 1][r]), fmaxf(mred[4 * g + 2][r], mred[4 * g + 3][r]));
    const float inv = sca > 0.f ? 127.f / sca : 0.f;
    const int c = 8 * ov - k0;
    const uint2 fb = make_uint2(flag[c] | (flag[c + 1] << 8) | (flag[c + 2] << 16) | (flag[c + 3] << 24),
                                flag[c + 4] | (flag[c + 5] << 8) | (flag[c + 6] << 16) | (flag[c + 7] << 24));
    reinterpret_cast<uint2*>(L.aq + (size_t)om * K)[ov] = quant8(on, fb, inv);
    if (om == 0) reinterpret_cast<uint2*>(L.flag)[ov] = fb;
    if (b == 0 && ov == (k0 >> 3)) L.sca[om] = sca;
  }
  if (tid < M) L.part[(size_t)b * M + tid] = __int_as_float(pmax[tid]);
  if (b == 0 && tid == 0) *reinterpret_cast<I8WsHeader*>(ws) = I8WsHeader{M, K, kNSB, kb}, L.avh[0] = 1;  // aval written
  if (st) {  // uniform: the decode hand-off block (i8ws.h) for the streamed int8 GEMVs (AM_I8Q)
    if (b == 0 && tid < 8 * kI8StSlots) {  // SCA in slot 0, the other slots 0
      const int m = tid;
      float sca = 0.f;
      if (m < M) {
        const int g = m & 3, r = m >> 2;
        sca = fmaxf(fmaxf(mred[4 * g][r], mred[4 * g + 1][r]), fmaxf(mred[4 * g + 2][r], mred[4 * g + 3][r]));
      }
      st[kI8StSca + tid] = __float_as_uint(sca);
    }
    for (int wd = tid; 32 * wd < k1 - k0; wd += 1024) {  // this k-block's flag words (kb % 32 == 0)
      uint32_t bits = 0;
      for (int j = 0; j < 32 && 32 * wd + j < k1 - k0; ++j) bits |= (uint32_t)(flag[32 * wd + j] != 0) << j;
      st[kI8StFlags + (k0 >> 5) + wd] = bits;
    }
  }
  if ((LLJ_PREP_ABL & 8) && tid == 0) L.cnt[b] = 0;  // the ablation skips the list, never the count a consumer reads
  if (tid < 64 && !(LLJ_PREP_ABL & 8)) {  // compact the flags into the list, 64 columns per ballot
    int c = 0;
    for (int i0 = 0; i0 < k1 - k0; i0 += 64) {
      const bool f = i0 + lane < k1 - k0 && flag[i0 + lane];
      const unsigned long long bal = __ballot(f);
      if (f) {
        const int e = b * kb + c + __popcll(bal & ((1ull << lane) - 1ull)), kc = i0 + lane;
        L.list[e] = k0 + kc;
        uint32_t h[4] = {0u, 0u, 0u, 0u};  // f16(A) of rows 0..7 (rows >= M: 0)
#pragma unroll
        for (int m = 0; m < MR; ++m) {
          if (m < M) {
            const uint4 v = vals[m][kc >> 3];
            const uint32_t wv = (kc & 7) < 4 ? ((kc & 7) < 2 ? v.x : v.y) : ((kc & 7) < 6 ? v.z : v.w);
            const float a = (kc & 1) ? bfhi(wv) : bflo(wv);
            h[m >> 1] |= (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a) << (16 * (m & 1));
          }
        }
        L.aval[e] = make_uint4(h[0], h[1], h[2], h[3]);
      }
      c += __popcll(bal);
    }
    if (lane == 0) L.cnt[b] = c;
  }
}

// Pass 2, one block per row: SCA = max over the k-blocks, then the row quantized once (outlier
// columns 0: their contribution is the fp16 side product). The row and its flags (up to QV
// vectors of 8 per thread, K <= 8 * 256 * QV) are loaded BEFORE the k-block maxima are reduced, so
// both reads share one memory latency.
constexpr int QV = 8;
// list: also compact the flags of k-blocks m, m + M, ... into the list / counts (after
// i8_stats_rows_kernel, whose flags are complete only at this launch).
__global__ __launch_bounds__(256) void i8_quant_act_kernel(const bf16_t* __restrict__ A, int lda, int M, int K,
                                                           char* __restrict__ ws, bool list = false) {
  __shared__ float s_sca;
  const int m = blockIdx.x, tid = threadIdx.x;
  const I8Layout L = i8_layout(ws, M, K);
  if (list && tid < 64) {
    const int kb = i8_kb(K), lane = tid;
    for (int b = m; b < kNSB; b += M) {
      const int k0 = b * kb, k1 = min(K, k0 + kb);
      int c = 0;
      for (int i0 = 0; i0 < k1 - k0; i0 += 64) {
        const bool f = i0 + lane < k1 - k0 && L.flag[k0 + i0 + lane];
        const unsigned long long bal = __ballot(f);
        if (f) L.list[b * kb + c + __popcll(bal & ((1ull << lane) - 1ull))] = k0 + i0 + lane;
        c += __popcll(bal);
      }
      if (lane == 0) L.cnt[b] = c;
    }
  }
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


// ---- outlier gathers for the LLM.int8 prefill GEMM's side product (llj_gemm_i8_*): the outlier
// columns (ascending, from the per-k-block lists) of the activation as f16 rows ao16[M][kpad] and of
// the weight as f16(CB * SCB / 127) rows w16[N][kpad]; entries past the outlier count up to the next
// multiple of 64 are zero, so the GEMM reads whole 64-deep chunks with 16-byte loads.
// The flat list is rebuilt in LDS by every block (counts prefix + the per-block lists), its first
// `cap` entries only: kpad is a fixed capacity (the host cannot know the count without a sync);
// when the count exceeds it nothing is gathered and the GEMM runs its per-tile side product.
__device__ __forceinline__ int i8_flat_list(const I8Layout& L, const I8WsHeader& h, int* s_pre, int* s_list, int cap) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int nsb = i8_nsb_clamp(h.nsb);
  if (tid < 64) {
    const int c = tid < nsb ? i8_cnt_clamp(L.cnt[tid], h.kb) : 0;
    int x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    s_pre[tid + 1] = x;
    if (tid == 0) s_pre[0] = 0;
  }
  __syncthreads();
  if (s_pre[nsb] > cap) return s_pre[nsb];  // over capacity: the caller gathers nothing
  for (int b = 0; b < nsb; ++b)
    for (int j = tid; j < s_pre[b + 1] - s_pre[b]; j += blockDim.x)
      s_list[s_pre[b] + j] = i8_col_clamp(L.list[b * h.kb + j], h.K);
  __syncthreads();
  return s_pre[nsb];
}

__global__ __launch_bounds__(256) void i8_gather_act_kernel(const bf16_t* __restrict__ A, int lda, const char* __restrict__ ws,
                                                            _Float16* __restrict__ ao16, int kpad) {
  extern __shared__ int g_lds[];
  const I8WsHeader h = *reinterpret_cast<const I8WsHeader*>(ws);
  const I8Layout L = i8_layout(ws, h.mtot, h.K);
  const int total = i8_flat_list(L, h, g_lds, g_lds + 80, kpad);
  if (total > kpad) return;  // the GEMM sees the same count and takes its per-tile side product
  const int* s_list = g_lds + 80;
  const int m = blockIdx.x, nop = (total + 63) & ~63;
  for (int j0 = threadIdx.x; j0 < nop; j0 += 256 * 8) {  // 8 loads in flight per thread
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + 256 * u;
      v[u] = j < total ? bf2f(A[(size_t)m * lda + s_list[j]]) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (j0 + 256 * u < nop) ao16[(size_t)m * kpad + j0 + 256 * u] = (_Float16)v[u];
  }
}

// block: 16 weight rows (one I8P tile) x the outlier columns; thread: row tid >> 4, columns
// (tid & 15) + 16 i (16 consecutive halves per row and step: coalesced stores)
__global__ __launch_bounds__(256) void i8_gather_weight_kernel(const int8_t* __restrict__ CB, const float* __restrict__ SCB,
                                                               int K, const char* __restrict__ ws,
                                                               _Float16* __restrict__ w16, int kpad) {
  extern __shared__ int g_lds[];
  const I8WsHeader h = *reinterpret_cast<const I8WsHeader*>(ws);
  const I8Layout L = i8_layout(ws, h.mtot, h.K);
  const int total = i8_flat_list(L, h, g_lds, g_lds + 80, kpad);
  if (total > kpad) return;
  const int* s_list = g_lds + 80;
  const int nt = blockIdx.x, r = threadIdx.x >> 4, n = nt * 16 + r, nop = (total + 63) & ~63;
  const float scb = SCB[n] / 127.f;
  for (int j0 = threadIdx.x & 15; j0 < nop; j0 += 16 * 8) {  // 8 byte loads in flight per thread
    int q[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + 16 * u;
      const int k = j < total ? i8_col_clamp(s_list[j], K) : 0, kk = k & 127;
      q[u] = CB[(((size_t)nt * (K >> 7) + (k >> 7)) * 2 + (kk >> 6)) * 1024 + (16 * ((kk >> 4) & 3) + r) * 16 + (kk & 15)];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + 16 * u;
      if (j < nop) w16[(size_t)n * kpad + j] = j < total ? (_Float16)((float)q[u] * scb) : (_Float16)0.f;
    }
  }
}

// i8_prep_one_kernel for M <= 8, K <= 6 * 2048 (with the norm 4 * 2048), M * (k-block width / 8) <= 1024: returns 0 after the
// launch (or -hipError), 1 when the shape is outside that envelope (nothing launched)
static int i8_prep_one(bool norm, const bf16_t* x, int lda, const bf16_t* w, float eps, bf16_t* xn, int M, int K,
                       float thr, void* ws, void* stream, uint32_t* st = nullptr) {
  const int kb = i8_kb(K), vpt = (K / 8 + 255) / 256;
  if (M > 8 || vpt > (norm ? 4 : 6) || M * (kb / 8) > 1024 || lda % 8) return 1;
  // its row maximum compares bf16 values with thr and rounds the maximum to fp16 once, which is the
  // per-element fp16 rule only for 2^-14 <= thr <= 65504 (fp16's normal range): else the two passes
  if (!(thr >= 0x1p-14f && thr <= 65504.f)) return 1;
  hipStream_t s = (hipStream_t)stream;
#define LLJ_P1(N, V) \
  hipLaunchKernelGGL((i8_prep_one_kernel<N, V>), dim3(kNSB), dim3(1024), 0, s, x, lda, w, eps, xn, M, K, thr, (char*)ws, kb, st)
  if (norm) {
    if (vpt <= 2) LLJ_P1(true, 2); else LLJ_P1(true, 4);
  } else {
    if (vpt <= 2) LLJ_P1(false, 2); else if (vpt <= 4) LLJ_P1(false, 4); else LLJ_P1(false, 6);
  }
#undef LLJ_P1
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : -(int)e;
}

}  // namespace llj

using namespace llj;

extern "C" {

// Bytes of the statistics workspace for an (M, K) activation.
size_t llj_i8_ws_bytes(int M, int K) { return i8_offsets(M, K).total; }

int llj_i8_stats(const void* A, int lda, int M, int K, float threshold, void* ws, void* stream) {
  LLJ_REQUIRE(M > 0 && K > 0 && K % 16 == 0 && lda % 8 == 0 && i8_kb(K) <= 1024);
  if (int e = i8_prep_one(false, (const bf16_t*)A, lda, nullptr, 0.f, nullptr, M, K, threshold, ws, stream); e <= 0)
    return -e;  // one launch (decode batches), or past its envelope (> 0): the two passes
  hipStream_t s = (hipStream_t)stream;
  if (M >= kRowsStatsMin && i8_kb(K) <= 512 && lda % 8 == 0) {  // many rows: a 2-D pass 1
    const I8Offsets o = i8_offsets(M, K);
    if (hipError_t e = hipMemsetAsync((char*)ws + o.flag, 0, (size_t)K, s)) return (int)e;
    hipLaunchKernelGGL(i8_stats_rows_kernel, dim3(kNSB, (M + 31) / 32), dim3(256), 0, s, (const bf16_t*)A, lda, M, K,
                       threshold, (char*)ws, i8_kb(K));
    LLJ_CHECK_LAUNCH();
    hipLaunchKernelGGL(i8_quant_act_kernel, dim3(M), dim3(256), 0, s, (const bf16_t*)A, lda, M, K, (char*)ws, true);
    LLJ_CHECK_LAUNCH();
    return 0;
  }
  hipLaunchKernelGGL(i8_stats_kernel, dim3(kNSB), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)A, lda, M, K,
                     threshold, (char*)ws, i8_kb(K));
  LLJ_CHECK_LAUNCH();
  hipLaunchKernelGGL(i8_quant_act_kernel, dim3(M), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)A, lda, M, K,
                     (char*)ws);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_i8_norm_stats(const void* x, const void* norm_w, float eps, void* xn, int M, int K, float threshold, void* ws,
                      void* stream) {
  const int kb = i8_kb(K), nvec = K / 8, vpt = (nvec + 255) / 256;
  LLJ_REQUIRE(M > 0 && K > 0 && K % 16 == 0 && kb <= 1024);
  if (M > 16 || vpt > 4 || M * (kb / 8) > 256) {  // outside the one-launch form: the two ops
    if (int e = llj_rmsnorm(x, norm_w, eps, xn, M, K, stream)) return e;
    return llj_i8_stats(xn, K, M, K, threshold, ws, stream);
  }
  hipStream_t s = (hipStream_t)stream;
  const bf16_t *xb = (const bf16_t*)x, *wb = (const bf16_t*)norm_w;
  if (int e = i8_prep_one(true, xb, K, wb, eps, (bf16_t*)xn, M, K, threshold, ws, stream); e <= 0) return -e;
#define LLJ_NS(MR, VPT) \
  hipLaunchKernelGGL((i8_norm_stats_kernel<MR, VPT>), dim3(kNSB), dim3(256), 0, s, xb, wb, eps, (bf16_t*)xn, M, K, \
                     threshold, (char*)ws, kb)
  if (M <= 8) {
    if (vpt <= 2) LLJ_NS(8, 2); else LLJ_NS(8, 4);
  } else {
    if (vpt <= 2) LLJ_NS(16, 2); else LLJ_NS(16, 4);
  }
#undef LLJ_NS
  LLJ_CHECK_LAUNCH();
  hipLaunchKernelGGL(i8_quant_act_kernel, dim3(M), dim3(256), 0, s, (const bf16_t*)xn, K, M, K, (char*)ws);
  LLJ_CHECK_LAUNCH();
  return 0;
}

// llj_i8_norm_stats for decode rows (M <= 8, one launch) that also writes the decode hand-off block
// `st` (i8ws.h: SCA in slot 0, the outlier bits) read by the streamed int8 GEMVs (wfmt 2 |
// LLJ_WF_I8_ROWSTATS). norm_w NULL: statistics of x itself (no norm, xn unused).
int llj_i8_norm_rowstats(const void* x, const void* norm_w, float eps, void* xn, int M, int K, float threshold, void* ws,
                         void* st, void* stream) {
  LLJ_REQUIRE(st && M > 0 && M <= 8 && K > 0 && K % 16 == 0 && i8_kb(K) <= 1024 && (!norm_w || xn));
  const int e = i8_prep_one(norm_w != nullptr, (const bf16_t*)x, K, (const bf16_t*)norm_w, eps, (bf16_t*)xn, M, K,
                            threshold, ws, stream, (uint32_t*)st);
  return e > 0 ? LLJ_EINVAL : -e;  // > 0: outside the one-launch envelope
}

int llj_i8_gather_act(const void* A, int lda, int M, int K, const void* ws, void* ao16, int kpad, void* stream) {
  LLJ_REQUIRE(M > 0 && K > 0 && kpad >= 64 && kpad % 64 == 0 && ws && ao16);
  const size_t lds = (80 + (size_t)kpad) * sizeof(int);
  LLJ_REQUIRE(lds <= 65536);
  hipLaunchKernelGGL(i8_gather_act_kernel, dim3(M), dim3(256), lds, (hipStream_t)stream, (const bf16_t*)A, lda,
                     (const char*)ws, (_Float16*)ao16, kpad);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_i8_gather_weight(const void* CB, const void* SCB, int N, int K, const void* ws, void* w16, int kpad,
                         void* stream) {
  LLJ_REQUIRE(N > 0 && N % 16 == 0 && K % 128 == 0 && kpad >= 64 && kpad % 64 == 0 && ws && w16);
  const size_t lds = (80 + (size_t)kpad) * sizeof(int);
  LLJ_REQUIRE(lds <= 65536);
  hipLaunchKernelGGL(i8_gather_weight_kernel, dim3(N / 16), dim3(256), lds, (hipStream_t)stream, (const int8_t*)CB,
                     (const float*)SCB, K, (const char*)ws, (_Float16*)w16, kpad);
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

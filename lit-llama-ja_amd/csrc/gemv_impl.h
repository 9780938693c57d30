// Weight-streaming skinny GEMM ("GEMV", M <= 16 rows per pass) for the LLaMA decode step on
// gfx950, with the reference's per-layer elementwise work fused into prologue/epilogue.
//
// Replaces, for the decode path:
//   reference lit_llama/quantization.py:282-331 (qlinear_4bit_weight / Triton
//   linear_kernel_4bit_weight 80-280) and :411-421 (ColBlockQuantizedLinear.forward),
//   :36-75 (Linear8bitLt = bitsandbytes LLM.int8() matmul), plus torch.nn.Linear (F.linear)
//   for the bf16 model; fused with model.py:276-283 (RMSNorm), :204-228 (c_attn split,
//   apply_rope, KV-cache write), :172-173 (residual adds) and :258 (silu(c_fc1) * c_fc2).
//
// Work decomposition: one workgroup (NW waves) owns one 16-column n-tile over the whole K;
// its waves split K into 128-deep chunks round-robin and the partial sums are reduced in
// LDS, so no cross-workgroup reduction exists. A chunk is 4 MFMA 16x16x32 bf16 steps (or 2
// MFMA 16x16x64 i8 steps). The weight stream uses non-temporal loads, D chunks in flight.
//
// Weight formats (WF):
//  * WF_W4 — int4 repacked "W4P" layout (w4pack.hip): per (n-tile, k-chunk) one contiguous
//    1 KiB block; lane l's 16 bytes are the 32 codes of column 16*nt + (l&15) for
//    k = 128*kc + 32*(l>>4) + [0,32), so one global_load_dwordx4 per wave fetches a fully
//    coalesced 1 KiB and needs no LDS. Codes become bf16 (128 + q) with one v_and_or_b32
//    (magic exponent) per pair; the 128 + zero offset is removed in the epilogue with the
//    row sums of A, computed by an extra MFMA against a ones fragment:
//      y[m,n] = s[n] * (sum_k A[m,k] (128 + q[k,n]) - (128 + z[n]) * sum_k A[m,k])
//             = sum_k A[m,k] * (q[k,n] - z[n]) * s[n]          (get_weight semantics)
//  * WF_W8 — gptq.int8 (ColBlock bits=8): the 8-bit codes as two int4 planes in the W4P
//    layout, per (n-tile, k-chunk) 2 KiB = [low nibbles 1 KiB][high nibbles 1 KiB]. The low
//    nibble dequantizes to bf16 128 + lo (exponent 0x43), the high one to 2048 + 16 hi
//    (exponent 0x45, same v_and_or_b32), both into ONE accumulator:
//      sum_k A (128 + lo) + A (2048 + 16 hi) = sum_k A q + 2176 sum_k A,
//    so y = s * (acc - (2176 + z) * sum_k A), the W4 epilogue with offset 2176.
//  * WF_BF16 — torch.nn.Linear weight (N, K) row-major bf16, read in place.
//  * WF_I8 — LLM.int8(): CB (N, K) int8 row-quantized weight in the I8P tiling (per (tile,
//    chunk) 2 KiB, one contiguous KiB per MFMA step: llj_i8_repack) + SCB (N) fp32. A is quantized
//    per row in the prologue (absmax over non-outlier elements, outlier columns zeroed,
//    statistics from llj_i8_stats in int8.hip), int32 MFMA accumulation, dequant by
//    SCA*SCB/127^2, plus the fp16 side product over the outlier columns.
//  * WF_W4G — grouped int4 (ColBlock bits=4, tile_cols = g, g % 128 == 0; reference
//    quantization.py:338-409 with scales (N, ceil(K / g))): the W4P tiles of WF_W4 plus one
//    (scale, 128 + zero) pair per (group, column), group-major (G, N). Each 128-deep chunk lies in
//    one group, so a wave accumulates the chunk into a fresh accumulator (and its A row sums
//    through a ones fragment) and adds s_g * (acc_c - (128 + z_g) * sum_c A) to the running sum.
#pragma once
#include <algorithm>

#include "common.h"
#include "i8ws.h"
#include "attention.h"
#include "lit_llama_amd.h"

namespace llj {

enum : int { WF_W4 = 0, WF_BF16 = 1, WF_I8 = 2, WF_W8 = 3, WF_W4G = 4 };
// A operand modes: AM_GLOBAL fragments straight from global memory; AM_LDS / AM_NORM one LDS
// image of all M rows staged (and RMS-normalised) before the weight stream is consumed;
// AM_STREAM / AM_SNORM (batched rows, 2 <= M <= 8): each wave loads the M rows of ITS OWN
// 128-deep chunks together with the chunk's weights (16 B per lane per row group: only real
// rows travel), normalises them in registers with the row statistics handed over by the
// producer (nstat, AM_SNORM) and passes them through a 2-slot per-wave LDS ring into the MFMA
// fragments -- no workgroup-wide A image, no prologue barrier, no separate RMSNorm launch.
// AM_I8Q (LLM.int8, batched decode rows): the bf16 activation rows are streamed like AM_STREAM and
// quantized per chunk with the row statistics its producer handed over (i8st: SCA per row, outlier
// column bits), and the fp16 outlier side product is taken from the chunk's weight registers as the
// chunk streams -- no statistics launch, no int8 A image, no side-product pass after the stream.
// AM_I8S (LLM.int8, batched decode rows with a statistics workspace): the rows quantized once by the
// statistics launch (ws aq) are streamed per chunk into the same per-wave ring as AM_I8Q's -- no
// workgroup-wide int8 A image, no prologue barrier.
// AM_MERGE (one row, the attn.c_proj residual op): the LDS image of AM_LDS built from the decode
// attention's unnormalized per-split partials (apart: llj_attention_part) -- the split merge of
// attention_combine_kernel, in its order, in the prologue instead of a combine launch
enum : int { AM_GLOBAL = 0, AM_LDS = 1, AM_NORM = 2, AM_STREAM = 3, AM_SNORM = 4, AM_I8Q = 5, AM_I8S = 6, AM_MERGE = 7 };
constexpr int kMergeMax = 4;  // AM_MERGE: at most this many key splits per head
// streamed A: elements per staged row (128 + 8 pad: rows land on distinct bank groups) and per slot
constexpr int kSRow = 136;
constexpr int kSSlot = 8 * kSRow;
__host__ __device__ constexpr bool am_stream(int am) { return am == AM_STREAM || am == AM_SNORM; }
// AM_I8Q per-wave ring slot: the quantized rows (8 x 144 B) then, for chunks with outlier columns,
// those columns' f16(A) of the 8 rows, column-major (128 x 16 B; only outlier columns written / read)
#ifndef LLJ_I8Q_FAST
#define LLJ_I8Q_FAST 1  // AM_I8Q: 1 quant8_fast for rows with SCA >= 1/64, 0 quant8f always
#endif
constexpr int kQRow = 144;
constexpr int kQSlotBytes = 8 * kQRow + 128 * 32;  // AM_I8Q: + the outlier columns' f16(A) as fp32 (32 B per column)
constexpr int kQSlotBytesS = 8 * kQRow;            // AM_I8S: the int8 rows only
enum : int { EP_STORE = 0, EP_RESID = 1, EP_QKV = 2, EP_SWIGLU = 3 };

// int8 activation workspace written by llj_i8_stats (int8.hip): i8ws.h

struct GemvParams {
  const bf16_t* A;  // (M, K), row stride lda elements
  int lda;
  const bf16_t* norm_w;  // AM_NORM: RMSNorm scale (K)
  float eps;
  int M, N, K;
  const void* W;   // WF_W4: W4P tiles; WF_W8: W8P tiles; WF_BF16: (N, K) bf16; WF_I8: (N, K) int8
  const void* W2;  // EP_SWIGLU: c_fc2
  const float2* sz;   // WF_W4 / WF_W8: per column (scale, 128 / 2176 + zero); WF_I8: (const float*) SCB
  const float2* sz2;
  const bf16_t* bias;  // optional (N)
  bf16_t* C;  // EP_STORE / EP_SWIGLU: out (M, ldc); EP_RESID: residual stream updated in place
  int ldc;
  // EP_QKV
  bf16_t* q_out;   // (B*T, n_embd)
  bf16_t* kcache;  // (B, n_head, S, hs)
  bf16_t* vcache;
  const float* rope;  // (block_size, hs/2, 2)
  const int* pos;     // (T) absolute positions of the T rows of each sequence
  int n_head, head_size, S, T;
  int m0;  // global row index of local row 0 (QKV row chunks; int8 statistics rows)
  const void* i8ws;
  // int4: sum_k A[m,k] of this call's rows as the MFMA sees them (pre-normalized rows,
  // llj_rmsnorm_rows); nullptr = computed in the prologue
  const float* rowsum;
  // RMSNorm statistics hand-off (M <= kNstRows): nstat[q * kNstRows + m], q < npart, partial sums
  // of the bf16-rounded squares of row m (consumer, norm-fused forms); nstat_out: the same,
  // written per 16-column tile by a residual op (producer)
  const float* nstat;
  int npart;
  float* nstat_out;
  int gch;  // WF_W4G: group size in 128-deep chunks (tile_cols / 128)
  // LLM.int8() decode statistics (i8ws.h kI8StFlags): i8st = the consumer's row statistics (AM_I8Q:
  // A is the bf16 activation, quantized per chunk in the GEMV); i8st_out = the statistics of this
  // op's output (EP_SWIGLU producer); clr / clr_words = a statistics block zeroed by workgroup 0
  const uint32_t* i8st;
  uint32_t* i8st_out;
  uint32_t* clr;
  int clr_words;
  float thr;
  // AM_MERGE: attention partials [(n_head)][asplit][head_size + 4] floats (attention.h kAttPart) of row 0
  const float* apart;
  int asplit;
};
constexpr int kNstRows = 16;
#ifndef LLJ_SACC_NORM
#define LLJ_SACC_NORM 0  // 7B bs=8 hand-off: 1.877 -> 1.800 ms, bs=2: 1.339 -> 1.353 (the hand-off runs at bs=2 only)
#endif

// ------------------------------------------------------------------------------------
// Stage A rows [0, M) into LDS (row stride K + 8 elements; MFMA lanes of rows >= M read row 0
// and their output rows are discarded). With NORM, rows are RMS-normalised with the reference's bf16
// rounding points (model.py:281-283 evaluated on bf16 tensors).
__device__ __forceinline__ float rms_rstd(float sumsq_over_k, float eps) {
  // bf16: mean(x*x) -> +eps -> rsqrt, each rounded (torch bf16 ops, model.py:281-282)
  return round_bf(rsqrtf(round_bf(round_bf(sumsq_over_k) + eps)));
}

// g * bf16(x * r), rounded to bf16, two elements per packed op (model.py:283 in bf16)
__device__ __forceinline__ uint4 norm8(uint4 x, uint4 g, float r) {
  uint32_t xw[4] = {x.x, x.y, x.z, x.w}, gw[4] = {g.x, g.y, g.z, g.w}, o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = cvt_pk(unpk(gw[i]) * unpk(cvt_pk(unpk(xw[i]) * r)));
  return make_uint4(o[0], o[1], o[2], o[3]);
}
// sum of the bf16-rounded squares of the 8 elements (model.py:281: x * x in bf16)
__device__ __forceinline__ f32x2 sumsq8(const u32x4 x, f32x2 acc) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x2 v = unpk(x[i]);
    acc += unpk(cvt_pk(v * v));
  }
  return acc;
}

template <int NW, bool NORM>
__device__ void stage_a(const GemvParams& p, bf16_t* As, int a_stride, float* red) {
  const int tid = threadIdx.x;
  constexpr int NT = NW * 64;
  const int K = p.K, M = p.M;
  const int nvec = K >> 3;
  float ss[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) ss[m] = 0.f;
  const bool from_stat = NORM && p.nstat;  // sums of squares handed over by the producer
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    if (m < M) {
      const uint4* src = reinterpret_cast<const uint4*>(p.A + (size_t)m * p.lda);
      uint4* dst = reinterpret_cast<uint4*>(As + (size_t)m * a_stride);
      f32x2 acc = {0.f, 0.f};
      for (int v = tid; v < nvec; v += NT) {
        uint4 x = src[v];
        dst[v] = x;
        if (NORM && !from_stat) acc = sumsq8(__builtin_bit_cast(u32x4, x), acc);
      }
      if (from_stat)
        for (int q = tid; q < p.npart; q += NT) acc.x += p.nstat[(size_t)q * kNstRows + m];
      ss[m] = acc.x + acc.y;
    }
  }
  if (!NORM) return;
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    float s = wave_sum(ss[m]);
    if (lane == 0) red[wave * 8 + m] = s;
  }
  __syncthreads();
  if (tid < 8) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[w * 8 + tid];
    red[NW * 8 + tid] = rms_rstd(s / (float)K, p.eps);
  }
  __syncthreads();
  const uint4* g4 = reinterpret_cast<const uint4*>(p.norm_w);
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    if (m < M) {
      const float r = red[NW * 8 + m];
      uint4* row = reinterpret_cast<uint4*>(As + (size_t)m * a_stride);
      for (int v = tid; v < nvec; v += NT) row[v] = norm8(row[v], g4[v], r);
    }
  }
}

// int8: copy rows [0, M) of the activation quantized once by llj_i8_stats (outlier columns
// already 0) into LDS int8 rows (stride K + 16 bytes); sca[] receives SCA per local row.
template <int NW>
__device__ void stage_i8(const GemvParams& p, int8_t* Aq, int q_stride, float* sca) {
  const int tid = threadIdx.x;
  constexpr int NT = NW * 64;
  const int K = p.K, M = p.M;
  const I8WsHeader h = *reinterpret_cast<const I8WsHeader*>(p.i8ws);
  const I8Layout L = i8_layout(p.i8ws, h.mtot, h.K);
  if (tid < M) sca[tid] = L.sca[p.m0 + tid];
  const int nv = K >> 4;
  for (int m = 0; m < M; ++m) {
    const uint4* src = reinterpret_cast<const uint4*>(L.aq + (size_t)(p.m0 + m) * K);
    uint4* dst = reinterpret_cast<uint4*>(Aq + (size_t)m * q_stride);
    for (int v = tid; v < nv; v += NT) dst[v] = src[v];
  }
}

__device__ __forceinline__ bf16x8 dequant_w4(uint32_t w, uint32_t msk, uint32_t mag) {
  uint4 b = make_uint4(and_or(w, msk, mag), and_or(w >> 4, msk, mag), and_or(w >> 8, msk, mag),
                       and_or(w >> 12, msk, mag));
  return __builtin_bit_cast(bf16x8, b);
}

template <int WF>
__device__ __forceinline__ int kofs(int t, int grp) {
  // k offset inside a 128-deep chunk of the elements lane-group `grp` feeds at MFMA step t
  return (WF == WF_W4 || WF == WF_W8 || WF == WF_W4G) ? 32 * grp + 8 * t : WF == WF_BF16 ? 32 * t + 8 * grp : 64 * t + 16 * grp;
}

// fp16 side product of LLM.int8() over the outlier columns, for this workgroup's 16 columns
// and M <= 8 rows: side[m][n] = sum_k f16(A[m,k]) * f16(CB[n,k] * SCB[n] / 127). The outlier
// columns are taken in chunks of kSideChunk: their indices and f16(A) values are staged in LDS
// (`stage`, free A-image space) once per workgroup, then thread t (column t % 16, every
// (NW*4)-th outlier of the chunk) accumulates; the four lanes of a wave sharing a column are
// combined by shuffles and the per-wave partials land in part[NW][8][16]. Ends with a barrier.
// Fast path (every k-block has <= SPC = kSpE * NT / kNSB outlier columns): the list entries were
// loaded speculatively in the prologue (`spk[e]`: entry q % SPC of k-block q / SPC, q = tid + NT e),
// so after the stream the chain is prefix (LDS) -> the f16(A) values and the tile's 16
// CB bytes of each column in ONE memory latency -> accumulate from LDS, instead of list -> A ->
// CB (three). Same per-thread accumulation order: bit-identical to the general path.
constexpr int kSideChunk = 256;
// speculative list entries per thread: 8 (4 waves) / 32 (8 waves) per k-block, so ~300 random
// outlier columns of the down projection's input (9.4 per k-block on average) stay on the fast path
#ifndef LLJ_I8_SPE
#define LLJ_I8_SPE 0  // 0: 1 (4 waves, K = 4096) / 2 (8 waves, K = 11008); else that many per thread (A/B)
#endif
// (A/B on one box, profiles/r03_c3_side_fastpath.json: each extra entry costs ~0.6 us per call at few
// outliers; at ~300 columns two entries save 6.5 us on the 8-wave down projection)
template <int NW>
constexpr int kSpE = LLJ_I8_SPE ? LLJ_I8_SPE : (NW == 4 ? 1 : 2);
template <int NW>
__device__ void i8_side_tile(const GemvParams& p, const int8_t* CB, const float* SCB, int n0, float* part,
                             unsigned char* stage, int cnt_lane, const int (&spk)[kSpE<NW>]) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nl = tid & 15, g = tid >> 4;
  constexpr int NG = NW * 4, NT = NW * 64;
  I8WsHeader h = *reinterpret_cast<const I8WsHeader*>(p.i8ws);
  const I8Layout L = i8_layout(p.i8ws, h.mtot, h.K);
  h.nsb = i8_nsb_clamp(h.nsb);  // counts and list entries bounded by what they index (i8ws.h)
  int* s_pre = reinterpret_cast<int*>(stage);           // [kNSB + 1] prefix of the block counts
  int* s_k = s_pre + 64;                                // [kSideChunk] column indices
  float* s_a = reinterpret_cast<float*>(s_k + kSideChunk);  // [8][kSideChunk] f16(A) values
  const int n = n0 + nl, M = p.M;
  const float scb = SCB[n] / 127.f;
  if (tid < 64) {  // prefix sum of the per-block outlier counts (kNSB <= 64; cnt_lane = cnt[lane], loaded early)
    int c = tid < h.nsb ? i8_cnt_clamp(cnt_lane, h.kb) : 0;
    int x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    s_pre[tid + 1] = x;
    if (tid == 0) s_pre[0] = 0;
    const unsigned long long ov = __ballot(tid < h.nsb && c > kSpE<NW> * NT / kNSB);
    if (tid == 0) s_pre[63] = ov != 0ull;  // a k-block past the speculative entries
  }
  __syncthreads();
  const int total = s_pre[h.nsb];
  const bool general = s_pre[63];
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (!general) {  // every entry is one thread's speculative list load: one memory latency in all
    constexpr int E = kSpE<NW>, SPC = E * NT / kNSB;
    _Float16* s_a16 = reinterpret_cast<_Float16*>(s_k);                      // [8][kSideChunk]
    uint32_t* s_cb = reinterpret_cast<uint32_t*>(s_a16 + 8 * kSideChunk);  // [kSideChunk][16 bytes]
    int ie[E];
    float av[E][8];
    uint32_t cw[E][4];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int q = tid + NT * e, b = q / SPC, j = q % SPC;
      const bool mine = b < h.nsb && j < s_pre[b + 1] - s_pre[b];
      ie[e] = mine ? s_pre[b] + j : -1;
      const int k = mine ? i8_col_clamp(spk[e], p.K) : 0, kk = k & 127;  // (k = 0: a valid address, never stored)
#pragma unroll
      for (int m = 0; m < 8; ++m) av[e][m] = bf2f(p.A[(size_t)(m < M ? m : 0) * p.lda + k]);
      const int8_t* cbp = CB + (((size_t)(n0 >> 4) * (p.K >> 7) + (k >> 7)) * 2 + (kk >> 6)) * 1024 +
                          (16 * ((kk >> 4) & 3)) * 16 + (kk & 15);
#pragma unroll
      for (int w = 0; w < 4; ++w) cw[e][w] = 0;
#pragma unroll
      for (int c = 0; c < 16; ++c) cw[e][c >> 2] |= (uint32_t)(uint8_t)cbp[c * 16] << (8 * (c & 3));
    }
    for (int c0 = 0; c0 < total; c0 += kSideChunk) {  // rounds of kSideChunk entries (LDS)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int i = ie[e];
        if (i >= c0 && i < c0 + kSideChunk) {
#pragma unroll
          for (int m = 0; m < 8; ++m) s_a16[m * kSideChunk + i - c0] = m < M ? (_Float16)av[e][m] : (_Float16)0.f;
          *reinterpret_cast<uint4*>(s_cb + 4 * (i - c0)) = make_uint4(cw[e][0], cw[e][1], cw[e][2], cw[e][3]);
        }
      }
      __syncthreads();
      const int8_t* cb8 = reinterpret_cast<const int8_t*>(s_cb);
      const int len = min(kSideChunk, total - c0);
      for (int ii = g; ii < len; ii += NG) {  // NG divides kSideChunk: the general path's order
        const float w = (float)(_Float16)((float)cb8[ii * 16 + nl] * scb);
#pragma unroll
        for (int m = 0; m < 8; ++m) acc[m] += (float)s_a16[m * kSideChunk + ii] * w;
      }
      __syncthreads();
    }
  }
  for (int c0 = 0; c0 < (general ? total : 0); c0 += kSideChunk) {
    const int len = min(kSideChunk, total - c0);
    for (int i = tid; i < len; i += NT) {
      const int fi = c0 + i;
      int b = 0;
      while (b + 1 < h.nsb && s_pre[b + 1] <= fi) ++b;  // blocks are few (kNSB)
      const int k = i8_col_clamp(L.list[b * h.kb + (fi - s_pre[b])], p.K);
      s_k[i] = k;
#pragma unroll
      for (int m = 0; m < 8; ++m)
        s_a[m * kSideChunk + i] = m < M ? (float)(_Float16)bf2f(p.A[(size_t)m * p.lda + k]) : 0.f;
    }
    __syncthreads();
    // the CB bytes of SB outlier columns are loaded together (independent loads, one latency),
    // then accumulated in the same column order as one at a time
    constexpr int SB = 8;
    for (int i0 = g; i0 < len; i0 += NG * SB) {
      int cbv[SB];
#pragma unroll
      for (int u = 0; u < SB; ++u) {
        const int i = i0 + NG * u < len ? i0 + NG * u : i0;
        const int k = s_k[i], kk = k & 127;  // byte of (n, k) in the I8P tiling
        const size_t off = (((size_t)(n >> 4) * (p.K >> 7) + (k >> 7)) * 2 + (kk >> 6)) * 1024 +
                           (16 * ((kk >> 4) & 3) + (n & 15)) * 16 + (kk & 15);
        cbv[u] = CB[off];
      }
#pragma unroll
      for (int u = 0; u < SB; ++u) {
        const int i = i0 + NG * u;
        if (i < len) {
          const float w = (float)(_Float16)((float)cbv[u] * scb);
#pragma unroll
          for (int m = 0; m < 8; ++m) acc[m] += s_a[m * kSideChunk + i] * w;
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    acc[m] += __shfl_xor(acc[m], 16, 64);
    acc[m] += __shfl_xor(acc[m], 32, 64);
    if (lane < 16) part[(wave * 8 + m) * 16 + nl] = acc[m];
  }
  __syncthreads();
}

// Output value of one element for the plain / SwiGLU epilogues (SwiGLU: model.py:258 in bf16).
template <int EP>
__device__ __forceinline__ float out_value(float y, float y2) {
  if (EP == EP_SWIGLU) {
    const float a1 = round_bf(y), a2 = round_bf(y2);
    const float sl = round_bf(a1 / (1.f + __expf(-a1)));  // F.silu in bf16
    return sl * a2;
  }
  return y;
}


// LLM.int8() row quantization of 8 bf16 elements (packed in a u32x4): q = clamp(rint(f16(a) * inv))
// with inv = 127 / SCA, outlier columns (bit e of fb) 0 -- the prep pass's quant8 (int8.hip)
__device__ __forceinline__ uint2 quant8f(const u32x4 x, uint32_t fb, float inv) {
  uint32_t o[2] = {0, 0};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int qa = (int)fminf(fmaxf(rintf(f16r(bflo(x[i])) * inv), -127.f), 127.f);
    int qb = (int)fminf(fmaxf(rintf(f16r(bfhi(x[i])) * inv), -127.f), 127.f);
    if ((fb >> (2 * i)) & 1u) qa = 0;
    if ((fb >> (2 * i + 1)) & 1u) qb = 0;
    o[i >> 1] |= ((uint32_t)(qa & 0xFF) | ((uint32_t)(qb & 0xFF) << 8)) << (16 * (i & 1));
  }
  return make_uint2(o[0], o[1]);
}

// quant8f without the per-element fp16 round trip, clamp and convert, for rows with SCA >= 1/64:
// bf16 values are exact in fp16 above 2^-14 (below it, |a| * 127 / SCA < 0.5 either way: code 0),
// |f16(a)| <= SCA bounds |a * inv| by 127, and rint comes from adding 1.5 * 2^23 (round to nearest
// even, the code in the low byte, two's complement). Bitwise quant8f's codes for finite rows.
__device__ __forceinline__ uint2 quant8_fast(const u32x4 x, uint32_t fb, float inv) {
  uint32_t b[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    // fl(fl(a * inv) + 1.5 * 2^23): the product is pinned (empty asm) so that it is not contracted
    // into one fma (a single rounding would differ at ties); scalar: the packed-vector form of this
    // loop was miscompiled (ROCm 7.2: the odd elements dropped)
    float p = ((e & 1) ? bfhi(x[e >> 1]) : bflo(x[e >> 1])) * inv;
    asm volatile("" : "+v"(p));
    b[e] = __builtin_bit_cast(uint32_t, p + 12582912.f);
  }
  auto pack4 = [](uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3, uint32_t nib) {
    const uint32_t w = (b0 & 0xFFu) | ((b1 & 0xFFu) << 8) | ((b2 & 0xFFu) << 16) | (b3 << 24);  // low bytes
    const uint32_t m1 = (nib * 0x00204081u) & 0x01010101u;  // bit e of nib -> byte e = 1
    const uint32_t m = (m1 << 8) - m1;                       // ... = 0xFF (borrow-free), the outlier bytes
    return w & ~m;
  };
  return make_uint2(pack4(b[0], b[1], b[2], b[3], fb & 0xFu), pack4(b[4], b[5], b[6], b[7], (fb >> 4) & 0xFu));
}

template <int V>
struct IC {
  static constexpr int value = V;
};

// Register-staged A prologue. Loads return to VGPRs in issue order, so the A-side loads
// (RMSNorm partial statistics, activation rows, norm weights) and the epilogue operands are
// issued BEFORE the weight prefetch: waiting for them then does not also wait for the
// weight chunks' HBM latency, and the LDS image is written while the weights are in flight.
// MB = row class of the instantiation (1: M == 1; 8: M <= 8); register budget per lane:
//   XR 16-byte activation registers (MB 1: one row of K <= 8*XR*NT; MB 8: RS = 2 per row for
//   M <= 8, K <= 16*NT, or RS = 4 for M <= 4), GR norm-weight registers.
template <int MB, bool NORM>
struct APre {
  static constexpr int XR = MB == 1 ? (NORM ? 4 : 8) : 16;
  static constexpr int GR = NORM ? 4 : 1;
  static constexpr int SR = NORM ? (MB == 1 ? 1 : 8) : 1;  // handed-over partials: rows per partial
  u32x4 x[XR];
  u32x4 g[GR];
  float ns[2][SR];  // 2 partials per thread (scalar loads: a vector-element read of these miscompiled)
};

#ifndef LLJ_ABAR
#define LLJ_ABAR 0
#endif
#ifndef LLJ_ABL
#define LLJ_ABL 0  // ablation switches for profiling only (1 no A prologue, 2 no compute, 4 no epilogue, 8 no AM_I8Q side loop, 16 no streamed-A loads, 32 no epilogue stores)
#endif
#ifndef LLJ_I8_SIS
#define LLJ_I8_SIS 1  // int8 A image: in-stream fp16 side product from the prep's aval table (0: after the stream)
#endif
#ifndef LLJ_I8_SIS_E
#define LLJ_I8_SIS_E 2  // outlier entries per chunk loaded with its weights (a k-block with more: side product after the stream)
#endif
#ifndef LLJ_I8S
#define LLJ_I8S 1  // int8 GEMVs with a statistics workspace: stream its quantized rows (AM_I8S) for 2..8 rows
#endif
#ifndef LLJ_LOADFENCE
#define LLJ_LOADFENCE 0  // 1: the weight refills stay where the loop issues them (see the main loop)
#endif
#ifndef LLJ_AFRAG
#define LLJ_AFRAG 1  // 1: a chunk's NSTEP A fragments read together before its MFMAs (0: one read per step)
#endif
#ifndef LLJ_PF
#define LLJ_PF 0  // L2 prefetch distance of the weight stream in chunks (0 off; A/B)
#endif
#ifndef LLJ_FLAT_EPI
#define LLJ_FLAT_EPI 1  // 1: batched-row epilogues spread over every thread of the workgroup (0: per owner lane)
#endif
#ifndef LLJ_ROT
#define LLJ_ROT 0  // 1: each workgroup starts its chunk walk at a rotation (A/B of HBM access spread)
#endif

// LDS tail (floats) behind the A image / reduction scratch: [0, 8) per-row RMSNorm rstd (int8:
// SCA), [8, 8 + 16 NW) the norm's per-wave fp64 / fp32 row partials, then [TL_RS, TL_RS + 8 NW)
// the per-wave row sums of the staged A (int4 / int8-GPTQ offset removal).
__host__ __device__ constexpr int tail_floats(int nw) { return 8 + 24 * nw; }

// One workgroup computes TPW consecutive 16-column tiles nt0 .. nt0 + TPW - 1 (tiles past the
// last one are loaded as a copy of it and never stored): every wave streams its K-chunks of
// all TPW tiles behind ONE staged A image, so the prologue (activation rows, RMSNorm) runs
// once per workgroup instead of once per tile. TPW > 1 only for the standalone LDS-A forms.
template <int WF, int AM, int EP, int NW, int D, int MB, int TPW = 1>
__device__ __forceinline__ void gemv_body(const GemvParams& p, const int nt0, unsigned char* smem) {
  static_assert(TPW == 1 || (WF != WF_I8 && AM != AM_GLOBAL), "multi-tile: LDS-A forms");
  constexpr int TL_RS = 8 + 16 * NW;
  constexpr bool DUAL = (EP == EP_SWIGLU);
  constexpr bool I8 = (WF == WF_I8);
  constexpr bool W4L = (WF == WF_W4 || WF == WF_W8);  // nibble-coded: offset removed with row sums
  constexpr bool GRP = (WF == WF_W4G);  // grouped int4: offset and scale removed per chunk
  constexpr bool STRM = am_stream(AM);  // A rows streamed per chunk (see AM_STREAM)
  constexpr bool SNRM = (AM == AM_SNORM);
  static_assert(!STRM || (MB == 8 && !I8), "streamed A: batched rows, non-int8 formats");
  constexpr bool I8Q = (AM == AM_I8Q);  // int8 rows quantized per chunk from handed-over statistics
  static_assert(!I8Q || (I8 && MB == 8 && TPW == 1), "AM_I8Q: int8, batched rows, one tile per workgroup");
  constexpr bool I8S = (AM == AM_I8S);  // int8 rows of the statistics workspace streamed per chunk
  static_assert(!I8S || (I8 && MB == 8 && TPW == 1), "AM_I8S: int8, batched rows, one tile per workgroup");
  constexpr bool ASTR = STRM || I8Q;  // bf16 A rows streamed per chunk
  constexpr bool QRING = I8Q || I8S;  // int8 rows through the per-wave ring
  constexpr int QSB = I8Q ? kQSlotBytes : kQSlotBytesS;  // its slot bytes
  constexpr bool ALDS = (I8 && !QRING) || (AM != AM_GLOBAL && !STRM && !QRING);
  // row sums of A for the nibble offset: an extra MFMA against a ones fragment for the global-A
  // form and for batched norm-fused rows (LLJ_SACC_NORM; the VALU sums + 8 wave reductions of the
  // prologue sit on its critical path), else summed while the LDS image is written
  constexpr bool SACC = W4L && (!ALDS || (LLJ_SACC_NORM && AM == AM_NORM && MB > 1));
  constexpr int WV = (WF == WF_W4 || GRP) ? 1 : (WF == WF_BF16 ? 4 : 2);  // 16-B loads per lane per chunk per matrix
  constexpr int NSTEP = I8 ? 2 : 4;
  const int lane = threadIdx.x & 63;
  const int wave = uniform(threadIdx.x >> 6);
  const int K = p.K, M = p.M, KC = K >> 7;
  const int ntiles = p.N >> 4;
  if (p.clr && blockIdx.x == 0)  // a statistics block to be zeroed before its producer runs (uniform)
    for (int i = threadIdx.x; i < p.clr_words; i += NW * 64) p.clr[i] = 0u;
  int ntj[TPW];  // tile of slot j (clamped copy of the last tile past the end)
  bool tvalid[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    tvalid[j] = nt0 + j < ntiles;
    ntj[j] = tvalid[j] ? nt0 + j : ntiles - 1;
  }
  const int row = lane & 15, grp = lane >> 4;
  // LDS carve: [A image, aliased after the main loop by the NW x 64 x 12-word reduction
  // scratch] [tail: 128 words for staging scratch / int8 SCA]
  const int a_stride = I8 ? K + 16 : K + 8;  // elements (bytes for int8)
  const size_t a_bytes = ALDS ? (((size_t)M * a_stride * (I8 ? 1 : 2) + 15) & ~(size_t)15)
                              : STRM ? (size_t)NW * 2 * kSSlot * 2 : QRING ? (size_t)NW * 2 * QSB : 0;
  constexpr int NV = 8 * TPW + 4;  // reduction words per lane: acc, acc2 of every tile, sacc
  constexpr size_t kRedBytes = (size_t)NW * 64 * NV * 4;
  constexpr size_t kScratch = kRedBytes + (I8 ? (size_t)2 * NW * 8 * 16 * 4 : 0);  // + int8 side partials
  float* red = reinterpret_cast<float*>(smem);
  float* tail = reinterpret_cast<float*>(smem + (a_bytes > kScratch ? a_bytes : kScratch));
  float* sca = tail;

  const bool arow = row < M;
  const unsigned char* abase;  // byte address of this lane's A row
  if (ALDS) {
    abase = smem + (size_t)(arow ? row : 0) * a_stride * (I8 ? 1 : 2);  // rows >= M read row 0 (outputs discarded)
  } else {
    abase = reinterpret_cast<const unsigned char*>(p.A + (size_t)(arow ? row : 0) * p.lda);
  }
  constexpr int EB = I8 ? 1 : 2;  // A element bytes

  // mask in an SGPR and magic in a VGPR, hidden from constant folding (empty asm, no
  // instruction) so that (w & msk) | mag selects one v_and_or_b32 (no literal in VOP3 on gfx9)
  uint32_t msk = 0x000F000Fu, mag = 0x43004300u, mag_hi = 0x45004500u;  // mag_hi: WF_W8 high nibbles, 2048 + 16 hi
  asm volatile("" : "+s"(msk));
  asm volatile("" : "+v"(mag));
  if constexpr (WF == WF_W8) asm volatile("" : "+v"(mag_hi));
  const bf16x8 ones = __builtin_bit_cast(bf16x8, make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u));
  const u32x4 zero4 = {0, 0, 0, 0};

  // weight stream pointers (lane-resolved), in 16-byte units
  const u32x4* w1[TPW];
  const u32x4* w2[TPW];
  size_t wstep;  // 16-B units between consecutive chunks of this lane
  int vstride;   // 16-B units between the WV loads of one chunk
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int nt = ntj[j], n0 = nt * 16;
    w2[j] = nullptr;
    if (WF == WF_W4 || GRP) {
      w1[j] = reinterpret_cast<const u32x4*>(p.W) + (size_t)nt * KC * 64 + lane;
      if (DUAL) w2[j] = reinterpret_cast<const u32x4*>(p.W2) + (size_t)nt * KC * 64 + lane;
      wstep = 64; vstride = 0;
    } else if (WF == WF_W8) {  // 2 KiB per (tile, chunk): low plane, then high plane
      w1[j] = reinterpret_cast<const u32x4*>(p.W) + (size_t)nt * KC * 128 + lane;
      if (DUAL) w2[j] = reinterpret_cast<const u32x4*>(p.W2) + (size_t)nt * KC * 128 + lane;
      wstep = 128; vstride = 64;
    } else if (WF == WF_BF16) {
      const size_t off = (size_t)(n0 + row) * K + 8 * grp;  // elements
      w1[j] = reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(p.W) + off);
      if (DUAL) w2[j] = reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(p.W2) + off);
      wstep = 16; vstride = 4;  // chunk = 256 B of a row; step t at +64 B
    } else {  // I8P tiles (llj_i8_repack): per (tile, chunk) 2 KiB, step t at +1 KiB
      w1[j] = reinterpret_cast<const u32x4*>(p.W) + (size_t)nt * KC * 128 + lane;
      if (DUAL) w2[j] = reinterpret_cast<const u32x4*>(p.W2) + (size_t)nt * KC * 128 + lane;
      wstep = 128; vstride = 64;
    }
  }

  f32x4 acc[TPW], acc2[TPW], sacc = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < TPW; ++j) acc[j] = acc2[j] = sacc;
  i32x4 iacc = {0, 0, 0, 0}, iacc2 = {0, 0, 0, 0};
  const int nmy = uniform((KC - wave + NW - 1) / NW);

  u32x4 r1[D][TPW][WV], r2[D][TPW][WV];
  u32x4 ra[D][4];
  float2 rg[D][TPW], rg2[D][TPW];  // WF_W4G: (scale, 128 + zero) of the chunk's group, this lane's column
  // streamed A: lane l carries 16-B segment (l & 15) of rows (l >> 4) and (l >> 4) + 4 of each of
  // its chunks (rows past M: clamped copies of row M - 1, never stored), plus the norm weights'
  // segment (AM_SNORM); rn0 / rn1 = the RMSNorm rstd of those two rows
  u32x4 sa[ASTR ? D : 1][2], sg[SNRM ? D : 1];
  u32x4 sfl[I8Q ? D : 1];  // AM_I8Q: the chunk's 128 outlier-column bits (the same in every lane)
  float qi0 = 0.f, qi1 = 0.f, i8scb = 0.f, i8scb2 = 0.f;  // AM_I8Q: 127 / SCA of the lane's two rows; SCB[n] / 127
  bool qfast = false;  // AM_I8Q: every row's SCA >= 1/64 (quant8_fast's exactness condition)
  // AM_I8Q: this lane's fp16 side-product partials of rows 0..7 (its column, its k group; sd2: c_fc2)
  float sd[I8 ? 8 : 1], sd2[I8 && DUAL ? 8 : 1];
#pragma unroll
  for (int m = 0; m < (I8 ? 8 : 1); ++m) sd[m] = 0.f;
#pragma unroll
  for (int m = 0; m < (I8 && DUAL ? 8 : 1); ++m) sd2[m] = 0.f;
  // int8 A image (SIS): the chunk's outlier count and its first LLJ_I8_SIS_E (column, f16(A) rows)
  // entries of the prep's list / aval table, loaded with the chunk's weights (the workspace layout
  // from this launch's M and K: valid addresses whatever the header says; used only when `sis`)
  constexpr bool SIS = I8 && !I8Q && LLJ_I8_SIS && D <= 4;  // (the depth-8 forms: registers)
  constexpr int SE = SIS ? LLJ_I8_SIS_E : 1;
  int scn[SIS ? D : 1], sk[SIS ? D : 1][SE];
  u32x4 sav[SIS ? D : 1][SE];
  bool sis = false;  // uniform: the workspace carries aval and its k-blocks are the chunks
  const I8Layout Lp = i8_layout(p.i8ws, SIS ? p.M : 1, SIS ? p.K : 128);
  // AM_I8S: lane l carries 16-B segment (l & 7) of quantized row (l >> 3) of each of its chunks (rows
  // past M: clamped copies of row M - 1, never stored); the workspace holds exactly these M rows
  u32x4 s8[I8S ? D : 1];
  const int8_t* s8ptr = I8S ? reinterpret_cast<const int8_t*>(p.i8ws) + i8_offsets(1, p.K).aq +
                                  (size_t)(p.m0 + ((lane >> 3) < M ? (lane >> 3) : M - 1)) * p.K + 16 * (lane & 7)
                            : nullptr;  // (aq first in the workspace: row r at a fixed offset, i8ws.h)
  const bf16_t* aptr[2];
  const bf16_t* gptr = p.norm_w + 8 * (lane & 15);
  float rn0 = 1.f, rn1 = 1.f;
  if constexpr (ASTR) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int rr = (lane >> 4) + 4 * h;
      aptr[h] = p.A + (size_t)(rr < M ? rr : M - 1) * p.lda + 8 * (lane & 15);
    }
  }
  // chunk of the wave's i-th step: its chunks wave, wave + NW, ... in order, or (LLJ_ROT) started at a
  // per-workgroup rotation so that the workgroups do not all stream the same chunk offsets together
  const int rot = LLJ_ROT && nmy > 0 ? uniform((int)(blockIdx.x % (unsigned)nmy)) : 0;
  auto chunk_of = [&](int i) {
    int ii = i < nmy ? i : nmy - 1;
    if (LLJ_ROT) ii = ii + rot >= nmy ? ii + rot - nmy : ii + rot;
    return wave + NW * ii;
  };
  const int vz = (I8Q || SIS) ? vzero() : 0;  // uniform side data stays in VGPRs (common.h vzero)
  // L2 prefetch (LLJ_PF > 0): with chunk i's loads, one dword per lane of chunk i + LLJ_PF's weight
  // blocks (a wave's 64 lanes touch the whole 1 KiB block, so its lines are in L2 when the real
  // 16-byte loads come): in-flight bytes past the register ring at 1 VGPR per block. The dword is
  // "used" (an empty asm) when its slot is reloaded, so the compiler counts it in its waits.
  constexpr int PF = LLJ_PF;
  uint32_t pfv[PF > 0 ? D : 1][TPW][WV][2];
#pragma unroll
  for (int d = 0; d < (PF > 0 ? D : 1); ++d)
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
      for (int v = 0; v < WV; ++v) pfv[d][j][v][0] = pfv[d][j][v][1] = 0u;
  auto load = [&](int d, int i) {
    int c = chunk_of(i);
    c = c < 0 ? 0 : (c >= KC ? KC - 1 : c);  // always a valid chunk (loads past the end are unused)
    if constexpr (ASTR) {  // the chunk's activation rows first: they arrive before its weights
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if constexpr ((LLJ_ABL & 16) != 0)  // ablation: no activation traffic (constant rows)
          sa[d][h] = u32x4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u};
        else
          sa[d][h] = *reinterpret_cast<const u32x4*>(aptr[h] + 128 * c);
      }
      if constexpr (SNRM) sg[d] = *reinterpret_cast<const u32x4*>(gptr + 128 * c);
      if constexpr (I8Q) sfl[d] = *reinterpret_cast<const u32x4*>(p.i8st + kI8StFlags + 4 * c + vz);
    }
    if constexpr (I8S) s8[d] = *reinterpret_cast<const u32x4*>(s8ptr + 128 * c);
    if constexpr (SIS) {
      scn[d] = Lp.cnt[(c < kNSB ? c : kNSB - 1) + vz];
#pragma unroll
      for (int e = 0; e < SE; ++e) {
        sk[d][e] = Lp.list[128 * c + e + vz];
        sav[d][e] = __builtin_bit_cast(u32x4, Lp.aval[128 * c + e + vz]);
      }
    }
    if constexpr (GRP) {
      const size_t go = (size_t)(c / p.gch) * p.N + row;
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        rg[d][j] = p.sz[go + ntj[j] * 16];
        if (DUAL) rg2[d][j] = p.sz2[go + ntj[j] * 16];
      }
    }
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
      for (int v = 0; v < WV; ++v) {
        r1[d][j][v] = __builtin_nontemporal_load(w1[j] + (size_t)c * wstep + vstride * v);
        if (DUAL) r2[d][j][v] = __builtin_nontemporal_load(w2[j] + (size_t)c * wstep + vstride * v);
      }
    if constexpr (PF > 0) {
      int cp = i + PF < nmy ? chunk_of(i + PF) : -1;
      const bool pf_on = cp >= 0;  // (past the wave's last chunk: a re-read of chunk c, an L2 hit)
      cp = pf_on ? cp : c;
#pragma unroll
      for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int v = 0; v < WV; ++v) {
          asm volatile("" ::"v"(pfv[d][j][v][0]), "v"(pfv[d][j][v][1]));  // the slot's previous prefetch
          pfv[d][j][v][0] = *reinterpret_cast<const uint32_t*>(w1[j] + (size_t)cp * wstep + vstride * v);
          if (DUAL) pfv[d][j][v][1] = *reinterpret_cast<const uint32_t*>(w2[j] + (size_t)cp * wstep + vstride * v);
        }
    }
    if (!ALDS) {
#pragma unroll
      for (int t = 0; t < NSTEP; ++t)
        ra[d][t] = *reinterpret_cast<const u32x4*>(abase + EB * (128 * c + kofs<WF>(t, grp)));  // rows >= M: row 0
    }
  };
  auto compute = [&](int d, int i) {
    const int c = chunk_of(i);
    if constexpr ((LLJ_ABL & 2) != 0) {  // ablation: loads only
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        acc[j][0] += __builtin_bit_cast(float, (r1[d][j][0].x ^ r1[d][j][0].w) & 0x3FFu);
        if (DUAL) acc2[j][0] += __builtin_bit_cast(float, (r2[d][j][0].x ^ r2[d][j][0].w) & 0x3FFu);
      }
      return;
    }
    f32x4 gt[TPW], gt2[TPW], gs = {0, 0, 0, 0};  // WF_W4G: this chunk's sums
#pragma unroll
    for (int j = 0; j < TPW; ++j) gt[j] = gt2[j] = gs;
    // streamed A: this chunk's rows (normalised: g * bf16(x * r), model.py:283 in bf16) into the
    // wave's ring slot d % 2, read back as MFMA fragments (one wave writes and reads its own slot:
    // LDS keeps a wave's accesses in order, no barrier)
    bf16_t* slot = reinterpret_cast<bf16_t*>(smem) + (size_t)(wave * 2 + (d & 1)) * kSSlot;
    unsigned char* qslot = smem + (size_t)(wave * 2 + (d & 1)) * QSB;
    if constexpr (I8S) *reinterpret_cast<u32x4*>(qslot + (lane >> 3) * kQRow + 16 * (lane & 7)) = s8[d];
    if constexpr (I8Q) {
      // quantize the lane's two row segments (LLM.int8 rows with the producer's SCA and outlier bits)
      const u32x4 fw = sfl[d];
      const int seg = lane & 15;
      auto pick = [&](int i) {  // fw[i] for a lane-varying i (selects: no dynamic register index)
        return i == 0 ? fw[0] : i == 1 ? fw[1] : i == 2 ? fw[2] : fw[3];
      };
      const uint32_t fb = (pick(seg >> 2) >> (8 * (seg & 3))) & 0xFFu;
      if (qfast) {  // uniform: every row's SCA >= 1/64 (the prologue)
        *reinterpret_cast<uint2*>(qslot + (lane >> 4) * kQRow + 8 * seg) = quant8_fast(sa[d][0], fb, qi0);
        *reinterpret_cast<uint2*>(qslot + ((lane >> 4) + 4) * kQRow + 8 * seg) = quant8_fast(sa[d][1], fb, qi1);
      } else {
        *reinterpret_cast<uint2*>(qslot + (lane >> 4) * kQRow + 8 * seg) = quant8f(sa[d][0], fb, qi0);
        *reinterpret_cast<uint2*>(qslot + ((lane >> 4) + 4) * kQRow + 8 * seg) = quant8f(sa[d][1], fb, qi1);
      }
      bool continue_side = true;  // (LLJ_ABL & 8: timing ablation without the side loop)
      if ((fw[0] | fw[1] | fw[2] | fw[3]) != 0u) {  // uniform: the chunk has outlier columns
        // fp16 side product from the weight registers: lane (column n, k group g) holds CB[n, k] of
        // k = 64 t + 16 g + j (t = 0, 1; j < 16) of the chunk. The outlier columns' f16(A) of all 8
        // rows go to a column-major table in the slot (16 B per column: one read per column), each
        // lane writing the outlier columns of its own two row segments
        float* ocol = reinterpret_cast<float*>(qslot + 8 * kQRow);  // f16(A) values held as fp32: no convert per read
        // Registers a loop reads are pinned first (an empty asm that "writes" them): a loop reading
        // a register its load is still filling gets a vmcnt(0) inside it -- which also waits for
        // the weight prefetch of the next chunks (measured: the down projection's side product
        // cost 7 us of 24 with it)
        u32x4 p0 = sa[d][0], p1 = sa[d][1];
        asm volatile("" : "+v"(p0), "+v"(p1));
        for (uint32_t rb = fb; rb; rb &= rb - 1u) {  // divergent, usually no or one column
          const int e = __builtin_ctz(rb), kc = 8 * seg + e;
          const uint32_t w0 = p0[e >> 1], w1 = p1[e >> 1];
          ocol[8 * kc + (lane >> 4)] = f16r((e & 1) ? bfhi(w0) : bflo(w0));
          ocol[8 * kc + (lane >> 4) + 4] = f16r((e & 1) ? bfhi(w1) : bflo(w1));
        }
        const uint32_t m32 = ((pick(grp >> 1) >> (16 * (grp & 1))) & 0xFFFFu) |
                             (((pick(2 + (grp >> 1)) >> (16 * (grp & 1))) & 0xFFFFu) << 16);
        if constexpr ((LLJ_ABL & 8) != 0) continue_side = false;
        // each k group walks its own outlier columns (ascending j: the per-lane order of a walk over
        // the union), two columns per trip so that their table reads share one LDS latency; the walk
        // ends when no lane has a column left (a ballot per trip, no per-chunk trip count)
        u32x4 c0 = r1[d][0][0], c1 = r1[d][0][1];
        u32x4 e0 = DUAL ? r2[d][0][0] : c0, e1 = DUAL ? r2[d][0][1] : c1;
        asm volatile("" : "+v"(c0), "+v"(c1));  // pinned before the loop (see above)
        if constexpr (DUAL) asm volatile("" : "+v"(e0), "+v"(e1));
        auto cbyte = [](const u32x4 lo, const u32x4 hi, int j) {  // int8 code j (0..31, per lane) as float
          const bool h = (j & 16) != 0;  // the 16-byte half, then the word in it (selects, no indexing)
          const int wi = (j >> 2) & 3;
          const uint32_t a = h ? hi[0] : lo[0], b = h ? hi[1] : lo[1], c = h ? hi[2] : lo[2], e = h ? hi[3] : lo[3];
          const uint32_t wd = wi == 0 ? a : wi == 1 ? b : wi == 2 ? c : e;
          return (float)(int)(int8_t)((wd >> (8 * (j & 3))) & 0xFFu);
        };
        auto kk_of = [&](int jb) { return 64 * (jb >> 4) + 16 * grp + (jb & 15); };
        uint32_t rem = continue_side ? m32 : 0u;
        while (__ballot(rem != 0u) != 0ull) {
          const bool v0 = rem != 0u;
          const int j0 = v0 ? __builtin_ctz(rem) : 0;
          rem &= rem - 1u;
          const bool v1 = rem != 0u;
          const int j1 = v1 ? __builtin_ctz(rem) : 0;
          rem &= rem - 1u;
          // f16(A) of rows 0..7 of both columns (a lane without a column reads a valid slot, unused)
          const float4 oa0 = *reinterpret_cast<const float4*>(ocol + 8 * kk_of(j0));
          const float4 ob0 = *reinterpret_cast<const float4*>(ocol + 8 * kk_of(j0) + 4);
          const float4 oa1 = *reinterpret_cast<const float4*>(ocol + 8 * kk_of(j1));
          const float4 ob1 = *reinterpret_cast<const float4*>(ocol + 8 * kk_of(j1) + 4);
          auto acc_col = [&](int jb, const float4 oa, const float4 ob) {
            const float w = f16r(cbyte(c0, c1, jb) * i8scb);
            const float a16[8] = {oa.x, oa.y, oa.z, oa.w, ob.x, ob.y, ob.z, ob.w};
#pragma unroll
            for (int m = 0; m < 8; ++m) sd[m] += a16[m] * w;
            if constexpr (DUAL) {
              const float w2 = f16r(cbyte(e0, e1, jb) * i8scb2);
#pragma unroll
              for (int m = 0; m < 8; ++m) sd2[m] += a16[m] * w2;
            }
          };
          if (v0) acc_col(j0, oa0, ob0);
          if (v1) acc_col(j1, oa1, ob1);
        }
      }
    }
    if constexpr (SIS) {
      if (sis) {  // uniform
        const int n = uniform(scn[d]);
        u32x4 c0 = r1[d][0][0], c1 = r1[d][0][1];
        u32x4 e0 = DUAL ? r2[d][0][0] : c0, e1 = DUAL ? r2[d][0][1] : c1;
        if (n > 0) {  // pinned before the loops (see the AM_I8Q side product)
          asm volatile("" : "+v"(c0), "+v"(c1));
          if constexpr (DUAL) asm volatile("" : "+v"(e0), "+v"(e1));
        }
        auto side_col = [&](int k, const u32x4 ov) {  // one outlier column k of this chunk (uniform)
          const int kk = k - 128 * c, t = kk >> 6;
          if (((kk >> 4) & 3) == grp) {  // the lanes holding CB[n, k]
            const int jj = kk & 15, wi = jj >> 2;
            const u32x4 cv = t ? c1 : c0;
            const uint32_t wd = wi == 0 ? cv[0] : wi == 1 ? cv[1] : wi == 2 ? cv[2] : cv[3];
            const float w = f16r((float)(int)(int8_t)((wd >> (8 * (jj & 3))) & 0xFFu) * i8scb);
            float a16[8];
#pragma unroll
            for (int m = 0; m < 8; ++m) {
              a16[m] = (float)__builtin_bit_cast(_Float16, (uint16_t)((ov[m >> 1] >> (16 * (m & 1))) & 0xFFFFu));
              sd[m] += a16[m] * w;
            }
            if constexpr (DUAL) {
              const u32x4 cv2 = t ? e1 : e0;
              const uint32_t wd2 = wi == 0 ? cv2[0] : wi == 1 ? cv2[1] : wi == 2 ? cv2[2] : cv2[3];
              const float w2 = f16r((float)(int)(int8_t)((wd2 >> (8 * (jj & 3))) & 0xFFu) * i8scb2);
#pragma unroll
              for (int m = 0; m < 8; ++m) sd2[m] += a16[m] * w2;
            }
          }
        };
#pragma unroll
        for (int e = 0; e < SE; ++e)  // every chunk has at most SE (the prologue's condition for sis)
          if (e < n) side_col(uniform(sk[d][e]), sav[d][e]);
      }
    }
    if constexpr (STRM) {
      u32x4 x0 = sa[d][0], x1 = sa[d][1];
      if constexpr (SNRM) {
        x0 = __builtin_bit_cast(u32x4, norm8(__builtin_bit_cast(uint4, x0), __builtin_bit_cast(uint4, sg[d]), rn0));
        x1 = __builtin_bit_cast(u32x4, norm8(__builtin_bit_cast(uint4, x1), __builtin_bit_cast(uint4, sg[d]), rn1));
      }
      *reinterpret_cast<u32x4*>(slot + (lane >> 4) * kSRow + 8 * (lane & 15)) = x0;
      *reinterpret_cast<u32x4*>(slot + ((lane >> 4) + 4) * kSRow + 8 * (lane & 15)) = x1;
    }
    // the chunk's A fragments, all read before the first MFMA: one LDS latency per chunk (LLJ_AFRAG;
    // read per step, a uniform branch between the steps kept every step's read behind a full
    // lgkmcnt(0) wait -- exposed at one wave per SIMD, the batched forms)
    u32x4 avs[NSTEP];
#pragma unroll
    for (int t = 0; t < NSTEP; ++t) {
      // LDS lanes of rows >= M read row 0 (abase clamped): their output rows are never stored, and
      // an unconditional read keeps the hot loop free of divergent LDS accesses
      avs[t] = STRM ? *reinterpret_cast<const u32x4*>(slot + (row & 7) * kSRow + kofs<WF>(t, grp))
               : QRING ? *reinterpret_cast<const u32x4*>(qslot + (row & 7) * kQRow + kofs<WF>(t, grp))
               : ALDS ? *reinterpret_cast<const u32x4*>(abase + EB * (128 * c + kofs<WF>(t, grp))) : ra[d][t];
    }
#pragma unroll
    for (int t = 0; t < NSTEP; ++t) {
      const u32x4 av = avs[t];
      if constexpr (WF == WF_W4) {
        const bf16x8 a = __builtin_bit_cast(bf16x8, av);
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          acc[j] = mfma_bf16(a, dequant_w4(r1[d][j][0][t], msk, mag), acc[j]);
          if (DUAL) acc2[j] = mfma_bf16(a, dequant_w4(r2[d][j][0][t], msk, mag), acc2[j]);
        }
        // (a uniform branch; the unconditional form with a zero fragment measured slower: without
        // the block boundaries the compiler sank the refills to the loop end, 5,243 -> 4,821
        // tokens/s at bs=8, profiles/r05_ab_bs8.jsonl). LLJ_AFRAG: one branch per chunk, after the steps
        if (!LLJ_AFRAG && SACC && !p.rowsum) sacc = mfma_bf16(a, ones, sacc);  // else: row sums from the prologue / caller
      } else if constexpr (GRP) {
        const bf16x8 a = __builtin_bit_cast(bf16x8, av);
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          gt[j] = mfma_bf16(a, dequant_w4(r1[d][j][0][t], msk, mag), gt[j]);
          if (DUAL) gt2[j] = mfma_bf16(a, dequant_w4(r2[d][j][0][t], msk, mag), gt2[j]);
        }
        gs = mfma_bf16(a, ones, gs);
      } else if constexpr (WF == WF_W8) {
        const bf16x8 a = __builtin_bit_cast(bf16x8, av);
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          acc[j] = mfma_bf16(a, dequant_w4(r1[d][j][0][t], msk, mag), acc[j]);
          acc[j] = mfma_bf16(a, dequant_w4(r1[d][j][1][t], msk, mag_hi), acc[j]);
          if (DUAL) {
            acc2[j] = mfma_bf16(a, dequant_w4(r2[d][j][0][t], msk, mag), acc2[j]);
            acc2[j] = mfma_bf16(a, dequant_w4(r2[d][j][1][t], msk, mag_hi), acc2[j]);
          }
        }
        if (!LLJ_AFRAG && SACC && !p.rowsum) sacc = mfma_bf16(a, ones, sacc);
      } else if constexpr (WF == WF_BF16) {
        const bf16x8 a = __builtin_bit_cast(bf16x8, av);
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          acc[j] = mfma_bf16(a, __builtin_bit_cast(bf16x8, r1[d][j][t]), acc[j]);
          if (DUAL) acc2[j] = mfma_bf16(a, __builtin_bit_cast(bf16x8, r2[d][j][t]), acc2[j]);
        }
      } else {
        const i32x4 a = __builtin_bit_cast(i32x4, av);
        iacc = mfma_i8(a, __builtin_bit_cast(i32x4, r1[d][0][t]), iacc);
        if (DUAL) iacc2 = mfma_i8(a, __builtin_bit_cast(i32x4, r2[d][0][t]), iacc2);
      }
    }
    if constexpr (LLJ_AFRAG && W4L && SACC) {  // the chunk's A row sums (nibble offset), one uniform branch
      if (!p.rowsum) {
#pragma unroll
        for (int t = 0; t < NSTEP; ++t) sacc = mfma_bf16(__builtin_bit_cast(bf16x8, avs[t]), ones, sacc);
      }
    }
    if constexpr (GRP) {  // s_g * (sum_c A (128 + q) - (128 + z_g) * sum_c A)
#pragma unroll
      for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          acc[j][r] += rg[d][j].x * (gt[j][r] - rg[d][j].y * gs[r]);
          if (DUAL) acc2[j][r] += rg2[d][j].x * (gt2[j][r] - rg2[d][j].y * gs[r]);
        }
    }
  };

  LLJ_STAMP(0);
  // ---- epilogue operands, loaded first. Every prologue load is branch-free with a clamped
  // (always valid) address and its validity applied where the value is used: a load under
  // divergent control flow makes the compiler's wait before the first use a vmcnt(0), which
  // would also wait for the weight prefetch issued after it.
  int nj[TPW];  // output column of this lane in tile slot j
#pragma unroll
  for (int j = 0; j < TPW; ++j) nj[j] = ntj[j] * 16 + row;
  // accumulator rows a lane can hold a live output for: 4 (rows 4*grp + r), or 1 when the
  // instantiation is for M == 1 (MB == 1), so per-row operands load once instead of 4 times
  constexpr int RR = MB == 1 ? 1 : 4;
  int e_ps[4] = {0, 0, 0, 0};
  auto issue_pos = [&]() {
    if constexpr (EP == EP_QKV && !(MB > 1 && LLJ_FLAT_EPI != 0)) {
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        const int mm = 4 * grp + r < M ? 4 * grp + r : M - 1;
        e_ps[r] = p.pos[(p.m0 + mm) % p.T];
      }
    }
  };
  float2 e_a[TPW], e_b[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    e_a[j] = e_b[j] = make_float2(1.f, 0.f);
  }
  float e_rs[4] = {0.f, 0.f, 0.f, 0.f};  // caller's row sums (p.rowsum) of rows 4*grp + r
  auto issue_const = [&]() {  // weights-side epilogue operands (never written in a launch)
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int n = nj[j];
      if constexpr (W4L) {
        e_a[j] = p.sz[n];
        if (DUAL) e_b[j] = p.sz2[n];
      } else if constexpr (I8) {
        e_a[j].x = reinterpret_cast<const float*>(p.sz)[n];
        if (DUAL) e_b[j].x = reinterpret_cast<const float*>(p.sz2)[n];
      }
    }
    // an epilogue load under divergent control flow would put a vmcnt(0) between the
    // row stores (stores count in vmcnt): read the row sums here (the branch is uniform)
    if (W4L && p.rowsum && !(MB > 1 && LLJ_FLAT_EPI != 0)) {
#pragma unroll
      for (int r = 0; r < RR; ++r) e_rs[r] = p.rowsum[4 * grp + r < M ? 4 * grp + r : M - 1];
    }
  };
  // flat epilogue (batched rows, LLJ_FLAT_EPI): after the reduction every thread of the workgroup
  // finishes whole output elements -- element e = tid + NT q of the (tile slot j, row m, column c)
  // space, c fastest, so c = tid & 15 = this lane's column `row` in every slot (e_a / e_b
  // apply as loaded) and (j, m) follow from rm = (tid >> 4) + 4 NW q. The per-lane form runs 4 rows
  // per lane on the TPW owner waves and idles the lanes of MFMA rows >= M (half of them at M = 8)
  constexpr bool FLAT = MB > 1 && LLJ_FLAT_EPI != 0;
  constexpr int FQ = FLAT ? (TPW * 16 * 16 + NW * 64 - 1) / (NW * 64) : 1;  // passes for M <= 16
  int f_j[FQ], f_m[FQ], f_ps[FQ];
  bool f_v[FQ];
  float f_rs[FQ];
  bf16_t f_xr[FQ];
  float2 f_cs[FQ];
#pragma unroll
  for (int q = 0; q < FQ; ++q) {
    f_j[q] = f_m[q] = f_ps[q] = 0;
    f_v[q] = false;
    f_rs[q] = 0.f;
    f_xr[q] = 0;
    f_cs[q] = make_float2(1.f, 0.f);
  }
  auto issue_flat = [&]() {  // the flat elements' row operands (branch-free, clamped addresses)
    if constexpr (FLAT) {
#pragma unroll
      for (int q = 0; q < FQ; ++q) {
        const int rm = (int)(threadIdx.x >> 4) + 4 * NW * q;
        const int jj = rm / M, mm = rm - jj * M;
        const bool v = jj < TPW && nt0 + jj < ntiles;
        f_v[q] = v;
        f_j[q] = v ? jj : 0;
        f_m[q] = v ? mm : 0;
        const int nt = nt0 + f_j[q] < ntiles ? nt0 + f_j[q] : ntiles - 1;
        if constexpr (EP == EP_QKV) f_ps[q] = p.pos[p.T == 1 ? 0 : (p.m0 + f_m[q]) % p.T];  // (T rows per sequence)
        if constexpr (EP == EP_RESID) f_xr[q] = p.C[(size_t)f_m[q] * p.ldc + nt * 16 + row];
        if (W4L && p.rowsum) f_rs[q] = p.rowsum[f_m[q]];
      }
    }
  };
  bf16_t e_xr[TPW][4];
  auto issue_xr = [&]() {  // residual stream values this workgroup updates
    if constexpr (EP == EP_RESID && !FLAT) {
#pragma unroll
      for (int j = 0; j < TPW; ++j)
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        const int mm = 4 * grp + r < M ? 4 * grp + r : M - 1;
        const int n = nj[j];
        e_xr[j][r] = p.C[(size_t)mm * p.ldc + n];
      }
    }
  };

  // ---- A prologue, register form (see APre) or LDS-staged after the prefetch (rs == 0)
  constexpr bool NORM = (AM == AM_NORM);
  constexpr int NT = NW * 64;
  using AP = APre<MB, NORM>;
  const int tid = threadIdx.x;
  const int nvec = K >> 3;
  const int JA = (nvec + NT - 1) / NT;
  int rs = 0;
  if (ALDS && !I8 && (LLJ_ABL & 1) == 0 && M <= MB) {
    const bool g_ok = !NORM || JA <= AP::GR;
    if (g_ok) {
      if (MB == 1) rs = JA <= 1 ? 1 : JA <= 2 ? 2 : JA <= 4 ? 4 : JA <= AP::XR ? AP::XR : 0;
      else if (JA <= 2) rs = 2;
      else if (JA <= 4 && M <= 4) rs = 4;
    }
  }
  rs = uniform(rs);
  AP ap;
  const u32x4* g4 = reinterpret_cast<const u32x4*>(p.norm_w);
  // rows held in registers: MB == 1 -> 1; else the smallest of 2 / 4 / 8 covering M (rows past M
  // are clamped duplicates of row M-1: loaded, never used)
  const int mr = MB == 1 ? 1 : uniform(M <= 2 ? 2 : M <= 4 ? 4 : 8);
  // AM_MERGE: per A vector (8 dims of one head) and split, the partial's 8 outputs and (max, sum)
  constexpr bool MERGE = (AM == AM_MERGE);
  // (plain floats: a u32x4 element read with a computed index returned element 0 for every index, §8)
  float mo[MERGE ? APre<MB, NORM>::XR : 1][MERGE ? kMergeMax : 1][8];
  float2 mml[MERGE ? APre<MB, NORM>::XR : 1][MERGE ? kMergeMax : 1];
  auto a_issue = [&](auto rsc, auto mrc) {
    constexpr int RS = decltype(rsc)::value;
    constexpr int MR = decltype(mrc)::value;
    static_assert(MR * RS <= AP::XR, "A registers");
    if constexpr (MERGE && RS > 4) {  // (K < 8192 on this path: never more than 4 vectors per thread)
      return;
    } else if constexpr (MERGE) {  // one row: the partials of this thread's vectors (clamped: always valid)
      const int hs = p.head_size, hsh = 31 - __builtin_clz(hs);
#pragma unroll
      for (int j = 0; j < RS; ++j) {
        const int v = tid + NT * j, vv = v < nvec ? v : nvec - 1;
        const int hh = (8 * vv) >> hsh, d0 = (8 * vv) & (hs - 1);
#pragma unroll
        for (int sp = 0; sp < kMergeMax; ++sp) {
          const int sc = sp < p.asplit ? sp : p.asplit - 1;
          const float* rec = p.apart + ((size_t)hh * p.asplit + sc) * (hs + 4);
          const float4 o0 = *reinterpret_cast<const float4*>(rec + d0);
          const float4 o1 = *reinterpret_cast<const float4*>(rec + d0 + 4);
          mo[j][sp][0] = o0.x; mo[j][sp][1] = o0.y; mo[j][sp][2] = o0.z; mo[j][sp][3] = o0.w;
          mo[j][sp][4] = o1.x; mo[j][sp][5] = o1.y; mo[j][sp][6] = o1.z; mo[j][sp][7] = o1.w;
          mml[j][sp] = *reinterpret_cast<const float2*>(rec + hs);
        }
      }
      return;
    }
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
      for (int j = 0; j < RS; ++j) {
        const int v = tid + NT * j;
        const int mm = m < M ? m : M - 1, vv = v < nvec ? v : nvec - 1;
        const size_t eo = (size_t)mm * p.lda + 8 * vv;
        ap.x[m * RS + j] = *reinterpret_cast<const u32x4*>(p.A + eo);
      }
    if (NORM) {
      constexpr int GJ = RS < AP::GR ? RS : AP::GR;
#pragma unroll
      for (int j = 0; j < GJ; ++j) {
        const int v = tid + NT * j;
        ap.g[j] = g4[v < nvec ? v : nvec - 1];
      }
      // the producer's partial sums of squares (thread: partials tid and tid + NT), branch-free:
      // without a hand-off the loads read the norm weights and are never used
      const bool st = p.nstat != nullptr;
      const int np = st ? p.npart : 1;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int qi = tid + NT * q < np ? tid + NT * q : np - 1;
        const float* src = st ? p.nstat + (size_t)qi * kNstRows : reinterpret_cast<const float*>(g4);
#pragma unroll
        for (int m = 0; m < (MR < AP::SR ? MR : AP::SR); ++m) ap.ns[q][m] = src[m];
      }
    }
  };
  auto a_finish = [&](auto rsc, auto mrc) {
    constexpr int RS = decltype(rsc)::value;
    constexpr int MR = decltype(mrc)::value;
    if constexpr (MERGE && RS <= 4) {  // y = sum_s O_s f_s / sum_s L_s f_s, f_s = exp2(M_s - max M): attention_combine_kernel's order
#pragma unroll
      for (int j = 0; j < RS; ++j) {
        float Mx = -INFINITY;
#pragma unroll
        for (int sp = 0; sp < kMergeMax; ++sp)
          if (sp < p.asplit) Mx = fmaxf(Mx, mml[j][sp].x);
        float L = 0.f, O[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int sp = 0; sp < kMergeMax; ++sp) {
          if (sp >= p.asplit) break;
          const float f = mml[j][sp].x == -INFINITY ? 0.f : exp2f(mml[j][sp].x - Mx);
          L += mml[j][sp].y * f;
#pragma unroll
          for (int i = 0; i < 8; ++i) O[i] += mo[j][sp][i] * f;
        }
        u32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (uint32_t)f2bf(O[2 * i] / L) | ((uint32_t)f2bf(O[2 * i + 1] / L) << 16);
        ap.x[j] = o;
      }
    }
    if (NORM) {
      float* redf = tail + 8;  // [wave][8] fp32
      {
#pragma unroll
        for (int m = 0; m < MR; ++m) {
          float ss = 0.f;
          if (p.nstat) {  // uniform: the producer's partials (rows >= M: unused)
#pragma unroll
            for (int q = 0; q < 2; ++q)
              if (tid + NT * q < p.npart) ss += ap.ns[q][m < AP::SR ? m : 0];
          } else {
            f32x2 acc = {0.f, 0.f};
#pragma unroll
            for (int j = 0; j < RS; ++j) {
              const u32x4 xv = (m < M && tid + NT * j < nvec) ? ap.x[m * RS + j] : zero4;
              acc = sumsq8(xv, acc);
            }
            ss = acc.x + acc.y;
          }
          ss = wave_sum(ss);
          if (lane == 0) redf[wave * 8 + m] = ss;
        }
        __syncthreads();
        if (tid < M) {
          float sf = 0.f;
#pragma unroll
          for (int w = 0; w < NW; ++w) sf += redf[w * 8 + tid];
          tail[tid] = rms_rstd(sf / (float)K, p.eps);
        }
      }
      __syncthreads();
    }
    bf16_t* As = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      float rsum = 0.f;
      if (m < M) {
        const float r = NORM ? tail[m] : 1.f;
#pragma unroll
        for (int j = 0; j < RS; ++j) {
          const int v = tid + NT * j;
          if (v < nvec) {
            u32x4 o = ap.x[m * RS + j];
            if (NORM) {
              const uint4 nv = norm8(__builtin_bit_cast(uint4, o), __builtin_bit_cast(uint4, ap.g[j < AP::GR ? j : 0]), r);
              o = __builtin_bit_cast(u32x4, nv);
            }
            *reinterpret_cast<u32x4*>(As + (size_t)m * a_stride + 8 * v) = o;
            if (W4L && !SACC && !p.rowsum) {
              f32x2 rp = unpk(o[0]) + unpk(o[1]);
              rp += unpk(o[2]) + unpk(o[3]);
              rsum += rp.x + rp.y;
            }
          }
        }
      }
      if (W4L && !SACC && m < M && !p.rowsum) {
        rsum = wave_sum(rsum);
        if (lane == 0) tail[TL_RS + wave * 8 + m] = rsum;
      }
    }
    __syncthreads();
  };
  // one (RS, MR) instantiation per register layout, chosen uniformly (a macro, not a lambda
  // taking the lambda: passing it through a call put the A registers in scratch)
#define LLJ_A_DISPATCH(F)                              \
  do {                                                 \
    if constexpr (MB == 1) {                           \
      if (rs == 1) F(IC<1>{}, IC<1>{});                \
      else if (rs == 2) F(IC<2>{}, IC<1>{});           \
      else if (rs == 4) F(IC<4>{}, IC<1>{});           \
      else if (rs == AP::XR) F(IC<AP::XR>{}, IC<1>{}); \
    } else {                                           \
      if (rs == 2) {                                   \
        if (mr == 2) F(IC<2>{}, IC<2>{});              \
        else if (mr == 4) F(IC<2>{}, IC<4>{});         \
        else F(IC<2>{}, IC<AP::XR / 2>{});             \
      } else if (rs == 4) {                            \
        if (mr == 2) F(IC<4>{}, IC<2>{});              \
        else F(IC<4>{}, IC<AP::XR / 4>{});             \
      }                                                \
    }                                                  \
  } while (0)
  auto a_issue_any = [&]() { LLJ_A_DISPATCH(a_issue); };

  // every input is final when the launch starts, so the A-side loads go first (a wait for
  // them then never waits for the weight chunks issued after them)
  issue_pos();
  issue_const();
  issue_xr();
  issue_flat();
  a_issue_any();
#if LLJ_ABAR
  __builtin_amdgcn_s_barrier();  // experiment: every wave's A loads ahead of any weight load
#endif
  // AM_SNORM: the producer's partial sums of squares, partials q = lane + 64 i (i < kSnQ) of rows
  // 0..7 (two 16-B loads per partial), issued before the weight stream
  // AM_I8Q: the producer's SCA partials of rows 0..7, slot = lane (bits of non-negative floats),
  // before the weight stream
  float4 isc[I8Q ? 2 : 1];
  if constexpr (I8Q) {
    static_assert(kI8StSlots == 64, "one SCA slot per lane");
    isc[0] = *reinterpret_cast<const float4*>(p.i8st + kI8StSca + 8 * lane);
    isc[1] = *reinterpret_cast<const float4*>(p.i8st + kI8StSca + 8 * lane + 4);
  }
  constexpr int kSnQ = 4;
  float4 snv[SNRM ? kSnQ : 1][2];
  if constexpr (SNRM) {
#pragma unroll
    for (int i = 0; i < kSnQ; ++i) {
      const int q = lane + 64 * i < p.npart ? lane + 64 * i : p.npart - 1;
      snv[i][0] = *reinterpret_cast<const float4*>(p.nstat + (size_t)q * kNstRows);
      snv[i][1] = *reinterpret_cast<const float4*>(p.nstat + (size_t)q * kNstRows + 4);
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d) load(d, d);  // the weight stream starts before any A wait
  if constexpr (SNRM) {  // every wave reduces the partials itself (same order everywhere: one rstd per row)
    float ss[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) ss[m] = 0.f;
#pragma unroll
    for (int i = 0; i < kSnQ; ++i) {
      if (lane + 64 * i < p.npart) {
        ss[0] += snv[i][0].x; ss[1] += snv[i][0].y; ss[2] += snv[i][0].z; ss[3] += snv[i][0].w;
        ss[4] += snv[i][1].x; ss[5] += snv[i][1].y; ss[6] += snv[i][1].z; ss[7] += snv[i][1].w;
      }
    }
    for (int q = lane + 64 * kSnQ; q < p.npart; q += 64) {  // n_embd > 4096 (rare: one more latency)
#pragma unroll
      for (int m = 0; m < 8; ++m) ss[m] += p.nstat[(size_t)q * kNstRows + m];
    }
    const int r0 = lane >> 4, r1i = (lane >> 4) + 4;
    const int m0c = r0 < M ? r0 : M - 1, m1c = r1i < M ? r1i : M - 1;  // clamped rows: copies of row M - 1
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const float r = rms_rstd(wave_sum(ss[m]) / (float)K, p.eps);
      if (m == m0c) rn0 = r;
      if (m == m1c) rn1 = r;
    }
  }
  if constexpr (I8Q) {
    const float sv[8] = {wave_max(isc[0].x), wave_max(isc[0].y), wave_max(isc[0].z), wave_max(isc[0].w),
                         wave_max(isc[1].x), wave_max(isc[1].y), wave_max(isc[1].z), wave_max(isc[1].w)};
    const int r0 = lane >> 4, r1i = (lane >> 4) + 4;
    const int m0c = r0 < M ? r0 : M - 1, m1c = r1i < M ? r1i : M - 1;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const float inv = sv[m] > 0.f ? 127.f / sv[m] : 0.f;
      if (m == m0c) qi0 = inv;
      if (m == m1c) qi1 = inv;
    }
    qfast = LLJ_I8Q_FAST != 0;
#pragma unroll
    for (int m = 0; m < 8; ++m) qfast = qfast && (m >= M || sv[m] >= 0.015625f);
    float mine = sv[0];  // the epilogue's SCA (tail; rows >= M unused); selects, not a dynamic index
#pragma unroll
    for (int m = 1; m < 8; ++m) mine = tid == m ? sv[m] : mine;
    if (tid < 8) sca[tid] = mine;
    i8scb = e_a[0].x / 127.f;
    if constexpr (DUAL) i8scb2 = e_b[0].x / 127.f;
  }
  // int8: the per-k-block outlier counts the side product starts from, loaded now (one memory
  // latency less in the tail; needed once the stream is done)
  int i8cnt = 0, i8spk[kSpE<NW>] = {};
  if constexpr (I8 && !I8Q) {  // + the speculative outlier-list entries of the side product's fast path
    const I8WsHeader h = *reinterpret_cast<const I8WsHeader*>(p.i8ws);
    const I8Layout L8 = i8_layout(p.i8ws, h.mtot, h.K);
    i8cnt = L8.cnt[lane < kNSB ? lane : 0];
    if constexpr (SIS) {
      // in-stream only when every chunk's outlier columns are among its prefetched entries (no
      // load inside a loop in the stream: that would wait for the weight prefetch); else after it
      const float most = wave_max((float)(lane < h.nsb ? i8cnt : 0));
      sis = h.kb == 128 && h.mtot == M && h.K == p.K && p.m0 == 0 && M <= 8 && L8.avh[0] == 1 && most <= (float)SE;
      i8scb = e_a[0].x / 127.f;
      if constexpr (DUAL) i8scb2 = e_b[0].x / 127.f;
    }
    constexpr int SPC = kSpE<NW> * NT / kNSB;
#pragma unroll
    for (int e = 0; e < kSpE<NW>; ++e) {
      const int q = tid + NT * e, sb = q / SPC < kNSB ? q / SPC : 0;
      i8spk[e] = L8.list[sb * h.kb + q % SPC];
    }
  }
  LLJ_STAMP(1);
  float2 e_cs[TPW][4];
  if constexpr (EP == EP_QKV && FLAT) {  // the flat elements' RoPE (cos, sin) (needs f_ps: waits for it only)
    const int Cd = p.n_head * p.head_size;
#pragma unroll
    for (int q = 0; q < FQ; ++q) {
      const int nt = nt0 + f_j[q] < ntiles ? nt0 + f_j[q] : ntiles - 1;
      const int n0 = nt * 16, region = n0 >= 2 * Cd ? 2 : (n0 >= Cd ? 1 : 0);
      const int dd = (n0 + row - region * Cd) & (p.head_size - 1);
      f_cs[q] = *reinterpret_cast<const float2*>(p.rope + ((size_t)f_ps[q] * (p.head_size >> 1) + (dd >> 1)) * 2);
    }
  } else if constexpr (EP == EP_QKV) {  // RoPE rows of the rows' positions (needs e_ps: waits for it only)
    const int Cd = p.n_head * p.head_size;
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int dd = (nj[j] - (ntj[j] * 16 / Cd) * Cd) % p.head_size;
#pragma unroll
      for (int r = 0; r < RR; ++r)
        e_cs[j][r] =
            *reinterpret_cast<const float2*>(p.rope + ((size_t)e_ps[r] * (p.head_size >> 1) + (dd >> 1)) * 2);
    }
  }
  if constexpr ((LLJ_ABL & 1) != 0) {  // ablation: no A prologue (garbage A)
  } else if constexpr (I8Q) {
  } else if constexpr (I8S) {  // the epilogue's SCA only (read after the reduction barrier)
    const I8WsHeader h = *reinterpret_cast<const I8WsHeader*>(p.i8ws);
    if (tid < M) sca[tid] = i8_layout(p.i8ws, h.mtot, h.K).sca[p.m0 + tid];
  } else if constexpr (I8) {
    stage_i8<NW>(p, reinterpret_cast<int8_t*>(smem), a_stride, sca);
    __syncthreads();
  } else if constexpr (ALDS) {
    if (rs == 0) {
      stage_a<NW, AM == AM_NORM>(p, reinterpret_cast<bf16_t*>(smem), a_stride, tail);
      __syncthreads();
      if (W4L && !SACC && !p.rowsum) {  // row sums of the staged rows (offset removal, see header)
        const bf16_t* As = reinterpret_cast<const bf16_t*>(smem);
        for (int m = 0; m < M; ++m) {
          float rsum = 0.f;
          for (int v = tid; v < nvec; v += NT) {
            const u32x4 o = *reinterpret_cast<const u32x4*>(As + (size_t)m * a_stride + 8 * v);
#pragma unroll
            for (int i = 0; i < 4; ++i) rsum += bflo(o[i]) + bfhi(o[i]);
          }
          rsum = wave_sum(rsum);
          if (lane == 0) tail[TL_RS + wave * 8 + m] = rsum;
        }
      }
    } else {
      LLJ_A_DISPATCH(a_finish);
    }
#undef LLJ_A_DISPATCH
  }
  LLJ_STAMP(2);
  // chunk i lives in buffer i % D; after computing it the buffer is refilled with chunk i + D.
  // The steady loop runs while every refill is a real chunk; the peeled tail (< 2D chunks)
  // issues no loads past the last chunk, so nothing is in flight when the epilogue waits.
  // LLJ_LOADFENCE: an empty asm with a memory clobber after each refill keeps the compiler from
  // sinking the refills to the end of the unrolled loop body (it did, for register pressure: then
  // every D-chunk round started with a full memory latency exposed)
  int i0 = 0;
  for (; i0 + 2 * D <= nmy; i0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      compute(d, i0 + d);
      load(d, i0 + d + D);
      if constexpr (LLJ_LOADFENCE != 0) asm volatile("" ::: "memory");
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d) {
    if (i0 + d < nmy) compute(d, i0 + d);
    if (i0 + d + D < nmy) load(d, i0 + d + D);
    if constexpr (LLJ_LOADFENCE != 0) asm volatile("" ::: "memory");
  }
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (i0 + D + d < nmy) compute(d, i0 + D + d);
  LLJ_STAMP(3);
  // ---- reduce the NW partial tiles in LDS (each wave: 64 lanes x NV words; int8 sums stay
  // int32 — they exceed 2^24 at K = 11008, so they must not round-trip through fp32). Tile slot
  // j is finished by wave j % NW, which sums the NW partials in wave order (the same order for
  // every TPW, so results do not depend on the tiling).
  // int8 side products in the LDS beyond the reduction scratch (the A image is no longer read)
  float* side = reinterpret_cast<float*>(smem + kRedBytes);
  if (NW > 1) {
    if (ALDS || ASTR || QRING) __syncthreads();  // every wave is done reading the A image / ring it aliases
    auto side_partials = [&]() {  // the in-stream side partials: sum the 4 k groups, one per (wave, row, column)
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        float v = sd[m];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if (lane < 16) side[(wave * 8 + m) * 16 + lane] = v;
        if constexpr (DUAL) {
          float v2 = sd2[m];
          v2 += __shfl_xor(v2, 16, 64);
          v2 += __shfl_xor(v2, 32, 64);
          if (lane < 16) side[NW * 8 * 16 + (wave * 8 + m) * 16 + lane] = v2;
        }
      }
    };
    if constexpr (I8Q) {
      side_partials();
    } else if constexpr (I8) {
      if (sis) {  // uniform (SIS)
        side_partials();
      } else {
        i8_side_tile<NW>(p, reinterpret_cast<const int8_t*>(p.W), reinterpret_cast<const float*>(p.sz), ntj[0] * 16,
                         side, smem, i8cnt, i8spk);
        if (DUAL)
          i8_side_tile<NW>(p, reinterpret_cast<const int8_t*>(p.W2), reinterpret_cast<const float*>(p.sz2),
                           ntj[0] * 16, side + NW * 8 * 16, smem, i8cnt, i8spk);
      }
    }
    if constexpr (I8) {
      int* mine = reinterpret_cast<int*>(red) + (size_t)(wave * 64 + lane) * NV;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        mine[r] = iacc[r];
        mine[4 + r] = iacc2[r];
      }
    } else {
      float* mine = red + (size_t)(wave * 64 + lane) * NV;
#pragma unroll
      for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          mine[8 * j + r] = acc[j][r];
          mine[8 * j + 4 + r] = acc2[j][r];
        }
#pragma unroll
      for (int r = 0; r < 4; ++r) mine[8 * TPW + r] = sacc[r];
    }
    __syncthreads();
    if (!FLAT && wave >= TPW) return;  // owns no tile slot (the flat epilogue uses every wave)
  }
  LLJ_STAMP(4);

  // ---- epilogue: output element (tile slot j, local row m, this lane's column `row`) from its reduced
  // accumulators. Every lane of a 16-lane column group calls it together (the RoPE partner and the
  // 16-column row sums / maxima are DPP exchanges inside the group); act: the element exists (the
  // row is < M and the tile slot is a real tile). Returns the int8 SwiGLU statistics' outlier flag.
  // (LLJ_ABL & 32: timing ablation, every output computed, no store issued -- ldc is never negative)
  auto epi_store = [&](void* dst, uint32_t v) {
    if ((LLJ_ABL & 32) == 0 || p.ldc < 0) st_out32(dst, v);
  };
  auto sel = [](auto const& arr, int j) {  // arr[j] for a runtime j < TPW (selects, no dynamic register index)
    auto v = arr[0];
#pragma unroll
    for (int i = 1; i < TPW; ++i) v = j == i ? arr[i] : v;
    return v;
  };
  auto elem = [&](const int j, const int m, const bool act, const float ya, const float yb, const float ys,
                  const int yi, const int yi2, const int ps, const float2 cs, const float rsv,
                  const bf16_t xr) -> bool {
    const int nt = nt0 + j < ntiles ? nt0 + j : ntiles - 1;
    const int n = nt * 16 + row, n0 = nt * 16;
    const float2 ea = sel(e_a, j), eb = sel(e_b, j);
    const float s1 = ea.x, o1 = ea.y, s2 = eb.x, o2 = eb.y;
    // (no Linear of the LLaMA path has a bias: the read stays in the epilogue, behind a uniform branch)
    const float bias = p.bias ? bf2f(p.bias[n]) : 0.f;
    float y, y2 = 0.f;
    if (W4L) {
      float sa = ys;
      if (p.rowsum) {
        sa = rsv;  // rows >= M hold a clamped copy; their outputs are not stored
      } else if constexpr (ALDS && !SACC) {
        sa = 0.f;
        if (act) {
#pragma unroll
          for (int w = 0; w < NW; ++w) sa += tail[TL_RS + w * 8 + m];
        }
      }
      y = s1 * (ya - o1 * sa);
      if (DUAL) y2 = s2 * (yb - o2 * sa);
    } else if (WF == WF_BF16 || GRP) {
      y = ya;
      y2 = yb;
    } else {
      // mm_dequant (fp16 out) + fp16 outlier product, then cast back (bnb MatMul8bitLt)
      const float sa = act ? sca[m] : 0.f;
      const float kq = 1.f / (127.f * 127.f);
      y = (float)yi * (sa * s1 * kq);
      if (DUAL) y2 = (float)yi2 * (sa * s2 * kq);
      if (act) {
        float sd = 0.f, sd2 = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          sd += side[(w * 8 + m) * 16 + row];
          if (DUAL) sd2 += side[NW * 128 + (w * 8 + m) * 16 + row];
        }
        y = (float)(_Float16)((float)(_Float16)y + sd);
        if (DUAL) y2 = (float)(_Float16)((float)(_Float16)y2 + sd2);
      }
    }
    y += bias;
    bool big = false;
    if (EP == EP_QKV) {
      // c_attn output rounded to bf16 (model.py:204), then RoPE in fp32 (model.py:318-329)
      const float v = round_bf(y);
      const float partner = lane_xor1(v);
      if (act) {
        // head_size is a power of two (64 / 128, checked on the host): shifts, no divisions
        const int Cd = p.n_head * p.head_size;
        const int hs_sh = uniform(31 - __builtin_clz(p.head_size));
        const int region = n0 >= 2 * Cd ? 2 : (n0 >= Cd ? 1 : 0);  // 0 q, 1 k, 2 v (per tile)
        const int nc = n - region * Cd;
        const int h = nc >> hs_sh, dd = nc & (p.head_size - 1);
        const int mg = p.m0 + m;
        const int b = p.T == 1 ? mg : mg / p.T;
        float out = v;
        if (region < 2) out = (dd & 1) ? (v * cs.x + partner * cs.y) : (v * cs.x - partner * cs.y);
        const uint32_t ob = (uint32_t)f2bf(out);
        const uint32_t pr = lane_xor1(ob);  // columns (dd, dd + 1) leave as one 4-byte store
        if (!(dd & 1)) {
          bf16_t* dst;
          size_t ei;
          if (region == 0) {
            dst = p.q_out;
            ei = (size_t)mg * Cd + nc;
          } else {
            int slot = ps;
            if (slot >= p.S) slot %= p.S;  // ring wrap only (no division on the common path)
            dst = region == 1 ? p.kcache : p.vcache;
            ei = (((size_t)b * p.n_head + h) * p.S + slot) * p.head_size + dd;
          }
          epi_store(dst + ei, ob | (pr << 16));
        }
      }
    } else if (EP == EP_RESID) {
      // x = x + h in bf16 (model.py:172-173)
      const float xn = round_bf(bf2f(xr) + round_bf(y));
      const uint32_t xb = (uint32_t)f2bf(xn);
      const uint32_t pr = lane_xor1(xb);
      if (act && !(row & 1)) epi_store(p.C + (size_t)m * p.ldc + n, xb | (pr << 16));
      if (p.nstat_out) {  // uniform: the next RMSNorm's sum of squares over this tile's 16 columns
        const float sq = row16_sum(act ? round_bf(xn * xn) : 0.f);
        if (row == 0 && act) epi_store(p.nstat_out + (size_t)nt * kNstRows + m, __builtin_bit_cast(uint32_t, sq));
      }
    } else {
      const uint32_t ob = (uint32_t)f2bf(out_value<EP>(y, y2));
      const uint32_t pr = lane_xor1(ob);
      if (act && !(row & 1)) epi_store(p.C + (size_t)m * p.ldc + n, ob | (pr << 16));
      if constexpr (EP == EP_SWIGLU && I8) {
        if (p.i8st_out) {  // uniform: LLM.int8 statistics of h for the int8 mlp.c_proj (AM_I8Q)
          const float a16 = fabsf(f16r(bflo(ob)));
          big = act && a16 >= p.thr;
          const float mx = row16_max(act && !big ? a16 : 0.f);
          if (row == 0 && act) atomicMax(p.i8st_out + kI8StSca + 8 * (nt % kI8StSlots) + m, __float_as_uint(mx));
        }
      }
    }
    return big;
  };

  if constexpr ((LLJ_ABL & 4) != 0) {  // ablation: minimal epilogue
    if (wave == 0 && acc[0][0] == 1234.5f && row < M) p.C[nj[0]] = f2bf(acc[0][1] + acc2[0][2]);
  } else if constexpr (FLAT) {
    // every thread finishes the elements e = tid + NT q of the (tile slot, row, column) space (f_j /
    // f_m / f_v from the prologue); the element's NW wave partials are summed in wave order, as below
#pragma unroll
    for (int q = 0; q < FQ; ++q) {
      const int j = f_j[q], m = f_m[q];
      const int src = ((m >> 2) << 4) | row, r = m & 3;  // the lane holding (m, row) in the MFMA layout
      float ya = 0.f, yb = 0.f, ys = 0.f;
      int yi = 0, yi2 = 0;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const float* o = red + (size_t)(w * 64 + src) * NV;
        if constexpr (I8) {
          const int* oi = reinterpret_cast<const int*>(o);
          yi = w == 0 ? oi[r] : yi + oi[r];
          yi2 = w == 0 ? oi[4 + r] : yi2 + oi[4 + r];
        } else {
          ya = w == 0 ? o[8 * j + r] : ya + o[8 * j + r];
          if (DUAL) yb = w == 0 ? o[8 * j + 4 + r] : yb + o[8 * j + 4 + r];
          if (SACC) ys = w == 0 ? o[8 * TPW + r] : ys + o[8 * TPW + r];
        }
      }
      const bool big = elem(j, m, f_v[q], ya, yb, ys, yi, yi2, f_ps[q], f_cs[q], f_rs[q], f_xr[q]);
      if constexpr (EP == EP_SWIGLU && I8) {
        if (p.i8st_out) {  // each 16-lane group's outlier columns: 16 bits of its tile's flag word
          const unsigned long long bal = __ballot(big);
          const uint32_t bits = (uint32_t)(bal >> (lane & 48)) & 0xFFFFu;
          const int nt = nt0 + j < ntiles ? nt0 + j : ntiles - 1;
          if (row == 0 && bits) atomicOr(p.i8st_out + kI8StFlags + (nt >> 1), bits << (16 * (nt & 1)));
        }
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      if (j % NW != wave || !tvalid[j]) continue;  // uniform
      f32x4 ya = acc[j], yb = acc2[j], ys = sacc;
      i32x4 yi = iacc, yi2 = iacc2;
      if (NW > 1) {
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          if constexpr (I8) {
            const int* o = reinterpret_cast<const int*>(red) + (size_t)(w * 64 + lane) * NV;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              yi[r] = w == 0 ? o[r] : yi[r] + o[r];
              yi2[r] = w == 0 ? o[4 + r] : yi2[r] + o[4 + r];
            }
          } else {
            const float* o = red + (size_t)(w * 64 + lane) * NV;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              ya[r] = w == 0 ? o[8 * j + r] : ya[r] + o[8 * j + r];
              yb[r] = w == 0 ? o[8 * j + 4 + r] : yb[r] + o[8 * j + 4 + r];
              ys[r] = w == 0 ? o[8 * TPW + r] : ys[r] + o[8 * TPW + r];
            }
          }
        }
      }
      bool i8col = false;  // EP_SWIGLU int8 statistics: this lane's column has an outlier
#pragma unroll
      for (int r = 0; r < RR; ++r) {
        if (r >= M) break;  // m = 4 grp + r >= r: no lane of the wave has a row left (uniform)
        const int m = 4 * grp + r;
        i8col |= elem(j, m, m < M, ya[r], yb[r], ys[r], yi[r], yi2[r], e_ps[r], e_cs[j][r], e_rs[r], e_xr[j][r]);
      }
      if constexpr (EP == EP_SWIGLU && I8) {
        if (p.i8st_out) {  // the tile's outlier columns (any row), 16 bits of one flag word
          const int n0 = ntj[j] * 16;
          uint32_t f = i8col ? 1u : 0u;
          f |= (uint32_t)__shfl_xor((int)f, 16, 64);
          f |= (uint32_t)__shfl_xor((int)f, 32, 64);
          const uint32_t bits = (uint32_t)(__ballot(f != 0u) & 0xFFFFull);
          if (lane == 0 && bits) atomicOr(p.i8st_out + kI8StFlags + (n0 >> 5), bits << (n0 & 31));
        }
      }
    }
  }
  LLJ_STAMP(5);
}

template <int WF, int AM, int EP, int NW, int D, int MB, int TPW>
__global__ __launch_bounds__(NW * 64) void gemv_kernel(GemvParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  gemv_body<WF, AM, EP, NW, D, MB, TPW>(p, blockIdx.x * TPW, smem);
}

// ------------------------------------------------------------------------------------
#ifndef LLJ_NW
#define LLJ_NW 4  // waves per workgroup (K split across them)
#endif
// weight chunks in flight per wave of the one-row SwiGLU (two matrices, so 2 D chunks): 2 vs 4,
// 7B gptq.int4 bs=1 decode-only 866 -> 892 tokens/s (dominant launch 11.3 -> 10.3 us), 13B 488 ->
// 514, gptq.int8 575 -> 590, bf16 321 -> 323 (profiles/r04_swiglu_depth_ab.json; 3: 871, 1: 885)
#ifndef LLJ_D
#define LLJ_D 2
#endif
#ifndef LLJ_D1
#define LLJ_D1 4  // chunks in flight per wave for the single-matrix ops (QKV, c_proj, down, head)
#endif
// The residual ops have only N / 16 = C / 16 workgroups (256 at 7B, one per CU); with a long K
// (mlp.c_proj, K = n_hidden) twice the waves keep twice the weight chunks in flight per CU
// (measured 7B bs=1: 8.8 -> 8.2 us; c_proj with K = C gains nothing and keeps 4 waves).
#ifndef LLJ_NWR
#define LLJ_NWR 8  // waves per workgroup of a residual op with K >= LLJ_NWR_KMIN
#endif
#ifndef LLJ_NWR_KMIN
#define LLJ_NWR_KMIN 8192
#endif
constexpr int kNW = LLJ_NW;
constexpr int kD = LLJ_D;

static inline size_t a_image_bytes(int wf, int am, int M, int K, int nw = kNW) {
  if (am == AM_I8Q) return (size_t)nw * 2 * kQSlotBytes;  // per-wave 2-slot rings
  if (am == AM_I8S) return (size_t)nw * 2 * kQSlotBytesS;
  if (wf == WF_I8) return (((size_t)M * (K + 16)) + 15) & ~(size_t)15;
  if (am == AM_GLOBAL) return 0;
  if (am_stream(am)) return (size_t)nw * 2 * kSSlot * 2;  // per-wave 2-slot rings
  return (((size_t)M * (K + 8) * 2) + 15) & ~(size_t)15;
}
static inline size_t gemv_smem(int wf, int am, int M, int K, int nw = kNW, int tpw = 1) {
  const size_t a = a_image_bytes(wf, am, M, K, nw);
  // reduction scratch (8 words per tile slot + 4 per lane); int8: the side-product partials
  // (2 matrices x NW x 8 rows x 16 columns) follow it
  const size_t red = (size_t)nw * 64 * (8 * tpw + 4) * 4 + (wf == WF_I8 ? (size_t)2 * nw * 8 * 16 * 4 : 0);
  return (a > red ? a : red) + (((size_t)tail_floats(nw) * 4 + 15) & ~(size_t)15);
}

#ifndef LLJ_TPW_MAX
#define LLJ_TPW_MAX 4  // tiles per workgroup at most (1 = one tile per workgroup)
#endif
// run-time cap on tiles per workgroup (llj_set_tpw_max, gemv.hip; A/B and equality tests)
extern int g_tpw_max;
// Compute units of the current device (cached per device; the query is not a stream
// operation, so it is legal while a graph is being captured).
static inline int device_cus() {
  static int cus[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 256;
  if (!cus[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}
// tiles per workgroup: ceil(tiles / CUs), i.e. about one workgroup per CU with every CU's
// share of tiles minimal, capped at LLJ_TPW_MAX and the run-time cap. Batched rows only
// (M >= 2: one staged A image of M rows per CU instead of per tile, 1.966 -> 1.865 ms at 7B
// bs=8); a single row keeps one tile per workgroup, where several workgroups per CU interleave
// on each SIMD (measured 7B bs=1: 1.205 ms with one tile, 1.305 ms with three per workgroup).
// Below LLJ_TPW_MIN_M rows the staged image is small and one tile per workgroup wins (7B
// decode ms/token, tiles per workgroup 1 vs ceil(tiles / CUs): bs=2 1.427 vs 1.509, bs=4 1.574
// vs 1.646, bs=6 1.683 vs 1.722, bs=8 1.889 vs 1.793).
#ifndef LLJ_TPW_MIN_M
#define LLJ_TPW_MIN_M 7
#endif
static inline int pick_tpw(int ntiles, int M) {
  if (M < LLJ_TPW_MIN_M) return 1;
  const int cu = device_cus();
  const int cap = g_tpw_max < LLJ_TPW_MAX ? g_tpw_max : LLJ_TPW_MAX;
  const int t = (ntiles + cu - 1) / cu;
  return t < 1 ? 1 : (t > cap ? cap : t);
}
// multi-tile instantiations: nibble-coded weights with the LDS A image or streamed A
template <int WF, int AM>
constexpr bool tpw_ok() { return (WF == WF_W4 || WF == WF_W8) && AM != AM_GLOBAL && LLJ_TPW_MAX > 1; }
// run-time switch of the streamed-A forms (llj_set_stream_a, gemv.hip; A/B and equality tests):
// 0 off, 1 = rows 2..8 (default), 2 = rows 1..8
extern int g_stream_a;

// the LDS A image must leave room for the reduction scratch: <= 96 KiB, M <= 8 rows
#ifndef LLJ_GEMV_LDS_A_MAX
#define LLJ_GEMV_LDS_A_MAX (96 * 1024)  // profiling variant: 56 KiB keeps every non-int8 launch under 64 KiB
#endif
static inline size_t lds_a_max() {  // option LLJ_OPT_GEMV_LDS_A_KB (56..96 KiB): A/B of the A-image cap
  const int kb = opt(LLJ_OPT_GEMV_LDS_A_KB);
  return kb > 0 ? (size_t)kb * 1024 : (size_t)(LLJ_GEMV_LDS_A_MAX);
}
static inline bool lds_fits(int wf, int M, int K) {
  return M <= 8 && a_image_bytes(wf, AM_LDS, M, K) <= (wf == WF_I8 ? 96 * 1024 : lds_a_max());
}

// waves per workgroup: the global-A form (rows whose A image does not fit the LDS) keeps twice
// as many waves, each with fewer chunks, for more A-fragment loads in flight
template <int AM>
constexpr int nw_of() { return AM == AM_GLOBAL ? 2 * kNW : kNW; }
#ifndef LLJ_DR
#define LLJ_DR 8  // chunks in flight per wave for the residual ops (attn / mlp c_proj; 8 vs 4: bs=1 1.167 -> 1.157 ms, bs=8 1.819 -> 1.803)
#endif
// batched rows (MB > 1, multi-tile workgroups): chunks in flight per wave (r1[D][TPW] registers
// scale with the tiles per workgroup) and waves per workgroup, tunable apart from the M == 1 forms
#ifndef LLJ_DM
#define LLJ_DM 2  // single-matrix ops (QKV, lm_head): streamed-A 7B bs=8 2 vs 4: 5,047 -> 5,116 tokens/s (6: 4,913)
#endif
#ifndef LLJ_DMS
#define LLJ_DMS 2  // SwiGLU (two matrices): 2 vs 4 at 7B gptq.int4 bs=8 4,341 -> 4,423 tokens/s (3: 4,362)
#endif
#ifndef LLJ_NWM
#define LLJ_NWM LLJ_NW
#endif
#ifndef LLJ_NWS
#define LLJ_NWS LLJ_NWM  // waves per workgroup of the batched-row SwiGLU (A/B)
#endif
#ifndef LLJ_DRM
#define LLJ_DRM 4  // residual ops of batched rows: streamed-A 7B bs=8 4 vs 8: 5,047 -> 5,207 tokens/s
#endif
template <int EP, int MB = 1>
constexpr int d_of() {
  return MB > 1 ? (EP == EP_SWIGLU ? LLJ_DMS : EP == EP_RESID ? LLJ_DRM : LLJ_DM)
                : (EP == EP_SWIGLU ? kD : EP == EP_RESID ? LLJ_DR : LLJ_D1);
}

#ifndef LLJ_DI8Q
#define LLJ_DI8Q 4  // AM_I8Q: chunks (2 KiB of int8 weights each) in flight per wave (8 spills)
#endif
template <int WF, int AM, int EP, int MB, int NW, int TPW>
static int launch_t(const GemvParams& p, hipStream_t s) {
  const size_t sm = gemv_smem(WF, AM, p.M, p.K, NW, TPW);
  auto kern = gemv_kernel<WF, AM, EP, NW, AM == AM_I8Q ? (EP == EP_SWIGLU ? LLJ_DMS : LLJ_DI8Q) : d_of<EP, MB>(), MB, TPW>;
  static bool attr_set[16] = {};  // per instantiation and device; set before any graph capture
  if (sm > 64 * 1024) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
    if (dev >= 16 || !attr_set[dev]) {
      hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (e != hipSuccess) return (int)e;
      if (dev < 16) attr_set[dev] = true;
    }
  }
  const int ntiles = p.N / 16;
  hipLaunchKernelGGL(kern, dim3((ntiles + TPW - 1) / TPW), dim3(NW * 64), sm, s, p);
  LLJ_CHECK_LAUNCH();
  return 0;
}

template <int WF, int AM, int EP, int MB, int NW = nw_of<AM>()>
static int launch_mb(const GemvParams& p, hipStream_t s) {
  if constexpr (tpw_ok<WF, AM>() && MB > 1) {  // M == 1 (MB 1) always one tile: pick_tpw
    // the residual ops (8 chunks in flight) take at most 2 tiles per workgroup (3 and 4 spill;
    // C / 16 tiles need 2 only past 256 CUs' worth: 13B / 30B / 65B)
    const int t = pick_tpw(p.N / 16, p.M);
    switch (EP == EP_RESID && t > 2 ? 2 : t) {
      case 2: return launch_t<WF, AM, EP, MB, NW, 2>(p, s);
      case 3: if constexpr (EP != EP_RESID) return launch_t<WF, AM, EP, MB, NW, 3>(p, s); break;
      case 4: if constexpr (EP != EP_RESID) return launch_t<WF, AM, EP, MB, NW, 4>(p, s); break;
      default: break;
    }
  }
  return launch_t<WF, AM, EP, MB, NW, 1>(p, s);
}

template <int WF, int AM, int EP>
static int launch(const GemvParams& p, hipStream_t s) {
  if constexpr (am_stream(AM) || AM == AM_I8Q || AM == AM_I8S) {  // batched rows only (M <= 8)
    if constexpr (EP == EP_RESID && LLJ_NWR != kNW)
      if (p.K >= LLJ_NWR_KMIN) return launch_mb<WF, AM, EP, 8, LLJ_NWR>(p, s);
    if constexpr (EP == EP_SWIGLU && LLJ_NWS != LLJ_NWM) return launch_mb<WF, AM, EP, 8, LLJ_NWS>(p, s);
    return launch_mb<WF, AM, EP, 8, LLJ_NWM>(p, s);
  } else {
  // the register-staged prologue has an M == 1 class (bs = 1 decode) and an M <= 8 class
  if constexpr (EP == EP_RESID && AM != AM_GLOBAL && LLJ_NWR != kNW) {
    if (p.K >= LLJ_NWR_KMIN) {  // residual ops: 256 workgroups, more waves each
      if (WF != WF_I8 && p.M == 1) return launch_mb<WF, AM, EP, 1, LLJ_NWR>(p, s);
      // one tile per workgroup: an 8-row image of K >= 8192 exceeds the LDS cap, so the multi-tile
      // forms (M >= 7) were unreachable here (and spilled: 256 VGPRs + scratch)
      return launch_t<WF, AM, EP, 8, LLJ_NWR, 1>(p, s);
    }
  }
  if (WF != WF_I8 && AM != AM_GLOBAL && p.M == 1) return launch_mb<WF, AM, EP, 1>(p, s);
  if constexpr (AM != AM_GLOBAL && WF != WF_I8) return launch_mb<WF, AM, EP, 8, LLJ_NWM>(p, s);
  return launch_mb<WF, AM, EP, 8>(p, s);
  }
}

// A mode for a call: batched rows (2..8) stream A per chunk (the fused RMSNorm then takes the
// producer's statistics, nstat); otherwise the fused RMSNorm needs the LDS image, and plain rows
// are staged when they fit.
static int pick_am(int wf, const GemvParams& p) {
  if (p.apart) return (p.M == 1 && !p.norm_w && lds_fits(wf, 1, p.K)) ? AM_MERGE : -1;
  if (wf == WF_I8 && p.i8st) return (p.norm_w || p.M > 8) ? -1 : AM_I8Q;  // handed-over row statistics
  if (wf == WF_I8) {
    if (p.norm_w || !p.i8ws) return -1;
    if (LLJ_I8S && g_stream_a && p.M >= 2 && p.M <= 8) return AM_I8S;
    return lds_fits(wf, p.M, p.K) ? AM_LDS : -1;
  }
  if (g_stream_a && p.M >= (g_stream_a >= 2 ? 1 : 2) && p.M <= 8) {
    if (!p.norm_w) return AM_STREAM;
    if (p.nstat && (reinterpret_cast<uintptr_t>(p.nstat) & 15) == 0) return AM_SNORM;
  }
  if (p.norm_w) return lds_fits(wf, p.M, p.K) ? AM_NORM : -1;
  return lds_fits(wf, p.M, p.K) ? AM_LDS : AM_GLOBAL;
}

static int check_shape(int wf, const GemvParams& p) {
  if (p.M < 1 || p.M > 16 || p.N % 16 || p.K % 128 || p.K < 128) return LLJ_EINVAL;
  if (wf != WF_W4 && wf != WF_BF16 && wf != WF_I8 && wf != WF_W8 && wf != WF_W4G) return LLJ_EINVAL;
  if (wf == WF_W4G && p.gch < 1) return LLJ_EINVAL;
  if (wf != WF_BF16 && !p.sz) return LLJ_EINVAL;
  if (p.C && (p.ldc & 1)) return LLJ_EINVAL;  // epilogues store column pairs as 4-byte words
  return 0;
}

// Per-weight-format launchers, one translation unit each (gemv_w4.hip, gemv_bf16.hip,
// gemv_w8.hip, gemv_i8.hip) so the instantiations compile in parallel.
int gemv_launch_w4(int am, int ep, const GemvParams& p, hipStream_t s);
int gemv_launch_bf16(int am, int ep, const GemvParams& p, hipStream_t s);
int gemv_launch_w8(int am, int ep, const GemvParams& p, hipStream_t s);
int gemv_launch_i8(int am, int ep, const GemvParams& p, hipStream_t s);
int gemv_launch_w4g(int am, int ep, const GemvParams& p, hipStream_t s);

template <int WF, int AM>
static int launch_ep(int ep, const GemvParams& p, hipStream_t s) {
  switch (ep) {
    case EP_STORE: return launch<WF, AM, EP_STORE>(p, s);
    case EP_RESID: return launch<WF, AM, EP_RESID>(p, s);
    case EP_QKV: return launch<WF, AM, EP_QKV>(p, s);
    case EP_SWIGLU: return launch<WF, AM, EP_SWIGLU>(p, s);
  }
  return LLJ_EINVAL;
}
template <int WF>
static int launch_fmt(int am, int ep, const GemvParams& p, hipStream_t s) {
  if (am == AM_MERGE) {  // the attn.c_proj residual op of one row (llj_linear_resid_attn)
    if constexpr (WF == WF_W4 || WF == WF_BF16 || WF == WF_W8) {
      if (ep == EP_RESID && p.M == 1 && p.K < LLJ_NWR_KMIN) return launch_mb<WF, AM_MERGE, EP_RESID, 1>(p, s);
    }
    return LLJ_EINVAL;
  }
  if constexpr (WF == WF_I8) {
    if (am == AM_I8Q) return launch_ep<WF_I8, AM_I8Q>(ep, p, s);
    if (am == AM_I8S) return launch_ep<WF_I8, AM_I8S>(ep, p, s);
    return launch_ep<WF_I8, AM_LDS>(ep, p, s);
  } else {
    if (am == AM_SNORM) return launch_ep<WF, AM_SNORM>(ep, p, s);
    if (am == AM_STREAM) return launch_ep<WF, AM_STREAM>(ep, p, s);
    if (am == AM_NORM) return launch_ep<WF, AM_NORM>(ep, p, s);
    if (am == AM_LDS) return launch_ep<WF, AM_LDS>(ep, p, s);
    return launch_ep<WF, AM_GLOBAL>(ep, p, s);
  }
}

}  // namespace llj

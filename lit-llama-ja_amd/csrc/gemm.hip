// Prefill GEMM (many rows: a prompt / a perplexity window) for gfx950, the compute-bound
// regime of the same Linear layers the decode GEMVs stream (gemv_impl.h).
//
// Replaces, for M >> 16 rows: reference lit_llama/quantization.py:282-331
// (qlinear_4bit_weight / Triton linear_kernel_4bit_weight, which pads M to 256 and runs an
// autotuned tl.dot GEMM) and torch.nn.Linear (F.linear) of the bf16 model, with the block's
// elementwise work in the epilogue: model.py:204-228 (c_attn split, RoPE, KV-cache write),
// :172-173 (residual adds), :258 (silu(c_fc1) * c_fc2).
//
// Tiling: a 256-thread workgroup owns a 128 x 128 output tile and walks K in 64-deep chunks;
// the chunk's A tile (128 rows x 64 k bf16) and B tile (W4P: the half of each of the eight 1 KiB
// W4P tiles of its 128 columns that holds these 64 k; bf16: 128 rows x 64 k) are staged through
// double-buffered LDS (one barrier per chunk: the loads of chunk c + 1 are in flight while chunk
// c is multiplied). 22.5 KiB (W4) / 36 KiB (bf16) per stage, so 3 / 2 workgroups share a CU and
// one's barrier or load wait is covered by another's MFMAs (128-deep chunks with 86 / 139 KiB of
// LDS held one workgroup per CU and left the chunk loads exposed: 0.17 of the MFMA peak). The 4
// waves form a 2 x 2 grid of 64 x 64 sub-tiles = 4 x 4 MFMA 16x16x32 bf16 accumulators each.
// MFMA step s of a chunk: lane group g supplies k = 32 s + 8 g + [0, 8) (A from LDS rows); for W4
// those 8 codes are word g of the W4P lane (16 (2 h + s) + column) of the chunk's half h, so a B
// fragment is one 4-byte LDS read + the GEMV's v_and_or_b32 dequant into bf16 (128 + q); the
// 128 + zero offset is removed in the epilogue with the row sums of A, accumulated while the A
// tile is staged:
//   y[m,n] = s[n] * (sum_k A[m,k] (128 + q[k,n]) - (128 + z[n]) * sum_k A[m,k]).
// gptq.int8 (W8P: per 16 columns x 128 k the W4P tile of the low nibbles, then that of the high
// nibbles) stages both planes' halves (8 KiB per chunk) and feeds both to the same accumulator,
// the high plane dequantized to bf16 2048 + 16 hi (exponent 0x45): the epilogue is the int4 one
// with the offset 2176 + zero (llj_w8_scale_zero).
// Grouped int4 (ColBlock tile_cols = g, g % 128 == 0) stages the W4P tiles like int4 and
// dequantizes each B fragment to bf16((q - z_g) * s_g) with its chunk's group pair -- exactly the
// weights of the reference's grouped forward, F.linear over get_weight(bf16)
// (quantization.py:390-421) -- so its epilogue takes the accumulator as is.
// LLM.int8() (Linear8bitLt, reference quantization.py:36-75 over bitsandbytes' MatMul8bitLt):
// the activation quantized once by llj_i8_stats (aq rows, outlier columns 0, SCA per row) and CB
// in the I8P tiling (per 16 columns x 128 k: 2 KiB = the two 64-deep MFMA steps, a lane's 16 B
// being its B fragment) are staged per 128-deep chunk (16 KiB each) and multiplied with MFMA
// 16x16x64 i8 into int32; after the K loop the fp16 outlier side product runs on the same tile:
// the outlier columns 32 at a time, f16(A) (from the bf16 rows) and f16(CB * SCB / 127) gathered
// into LDS, MFMA 16x16x32 f16 into fp32 (products exact, fp32 sums); the epilogue forms the GEMV's
// y = f16(f16(acc * SCA * SCB / 127^2) + side) (bnb's mm_dequant in fp16 + the fp16 outlier matmul).
// Tile order is XCD-aware: the 8 XCDs take contiguous ranges of tiles; inside a range bf16 weights
// go m fastest (the row tiles of one weight panel run together on one XCD and share it through its
// L2), int4 weights n fastest (one 128-row A panel shared while the XCD sweeps the columns).
#include <cstdlib>

#include "common.h"
#include "i8ws.h"
#include "lit_llama_amd.h"

namespace llj {

// GWF_W4Z: int4 W4P with integral zeros (LLJ_WF_ZINT) in the convert-once LDS-DMA GEMM (internal)
enum : int { GWF_W4 = 0, GWF_BF16 = 1, GWF_I8 = 2, GWF_W8 = 3, GWF_W4G = 4, GWF_W4Z = 5 };
// GEP_SWIGLU: h = bf16(silu(bf16(A . W1^T))) * bf16(A . W2^T) in one pass (convert-once int4: both weights'
// codes staged per chunk, one A tile feeding both; W2 / sz2)
// GEP_PARTIAL: split-K slice of a residual GEMM -- fp32 partials y (scale applied) of K range slice
// blockIdx.x % nsplit into ws[slice][M][N]; llj_gemm_resid_ws's reduce adds them and the residual
// GEP_SWIGLU_PART: split-K slice of the dual SwiGLU pass (its last partial wave of tiles) -- fp32 partials of
// c_fc1 and c_fc2 (scales applied) into ws[slice][2][M][N]; llj_gemm_swiglu_ws's reduce finishes h
enum : int { GEP_STORE = 0, GEP_RESID = 1, GEP_QKV = 2, GEP_SILU_MUL = 3, GEP_SWIGLU = 4, GEP_PARTIAL = 5, GEP_SWIGLU_PART = 6 };

struct GemmParams {
  const bf16_t* A;  // (M, K) rows with stride lda
  int lda;
  int M, N, K;
  const void* W;      // GWF_W4: W4P tiles; GWF_W8: W8P tiles; GWF_BF16: (N, K) bf16 row-major
  const float2* sz;   // GWF_W4 / GWF_W8: per column (scale, 128 / 2176 + zero)
  bf16_t* C;          // STORE: out; RESID: residual (updated); SILU_MUL: h (holds bf16 fc1 output)
  int ldc;
  // GEP_QKV
  bf16_t* q_out;
  bf16_t* kcache;
  bf16_t* vcache;
  const float* rope;
  const int* pos;
  int n_head, head_size, S, T;
  int gch;  // GWF_W4G: group size in 128-deep chunks; sz = (scale, 128 + zero) per (group, column), (G, N)
  const char* i8ws;  // GWF_I8: llj_i8_stats workspace of A (aq, SCA, outlier list); sz = (const float*) SCB
  // GWF_I8 (optional): the outlier columns pre-gathered by llj_i8_gather_act / _weight, f16 rows of
  // stride kpad (a fixed capacity, multiple of 64), zero past the outlier count up to a multiple of
  // 64: the side product then runs as a dense f16 GEMM over them (coalesced 64-deep chunks) instead
  // of per-tile gathers; a count above kpad (nothing gathered) takes the per-tile side product
  const _Float16* ao16;
  const _Float16* w16;
  int kpad;
  // GEP_SWIGLU: the second weight (c_fc2) and its (scale, 128 + zero) pairs
  const void* W2;
  const float2* sz2;
  // GEP_PARTIAL: nsplit K slices of kcs 64-deep chunks each (kcs even), fp32 partials [nsplit][M][N]
  float* ws;
  int nsplit, kcs;
};

// Tile epilogues run in two phases per 16-column block: every element's operand is loaded first
// (gemm_operand: the residual / fc1 value, or the RoPE pair of the row's position), then each
// element is computed and stored (gemm_store_elem) -- one load latency per block instead of a
// load -> store dependence per element (7B 2048-token window: the QKV and silu * mul GEMMs ran
// 20-26 % slower than the plain store GEMM of the same shape with per-element loads).
#ifndef LLJ_QKV_LDS
#define LLJ_QKV_LDS 1  // LDS-DMA GEMM at 256 x 128 (bf16, convert-once int4): QKV epilogue through LDS, 16-byte row stores
#endif
#ifndef LLJ_GLDS_LDS_EPI
#define LLJ_GLDS_LDS_EPI 1  // LDS-DMA GEMM at 256 x 128: store / residual / SwiGLU epilogues through LDS, 16-byte rows
#endif
#ifndef LLJ_QKV_GI
#define LLJ_QKV_GI 4  // LDS-DMA GEMM QKV epilogue: 16-row blocks whose RoPE operands are loaded together (A/B)
#endif
#ifndef LLJ_QKV_ABL
#define LLJ_QKV_ABL 0  // prompt QKV epilogue timing ablations (profiling only): 1 no RoPE operand loads, 2 no stores
#endif
// QKV rows: sequence b, position ps and KV-cache ring slot of (clamped) row m, computed once per row
// and tile (the divisions by T and S stay out of the per-element path)
struct QkvRow {
  int ps;    // position (RoPE row)
  int kvrow; // element offset of (sequence b, head 0, ring slot) in the K / V caches
};
__device__ __forceinline__ QkvRow qkv_row(const GemmParams& p, int m) {
  const int mm = m < p.M ? m : p.M - 1;
  const int ps = p.pos[mm % p.T];
  const int slot = ps < p.S ? ps : ps % p.S;
  return QkvRow{ps, ((mm / p.T) * p.n_head * p.S + slot) * p.head_size};
}
// QKV columns: region (0 q, 1 k, 2 v; uniform per 16-column block), column within the region, head
// offset in the caches and dimension, computed once per 16-column block and lane
struct QkvCol {
  int region, nc, hoff, dd;
};
__device__ __forceinline__ QkvCol qkv_col(const GemmParams& p, int nblk, int n, int Cd) {
  QkvCol c;
  c.region = nblk / Cd;
  c.nc = n - c.region * Cd;
  const int h = c.nc / p.head_size;
  c.dd = c.nc - h * p.head_size;
  c.hoff = h * p.S * p.head_size;
  return c;
}
template <int EP>
__device__ __forceinline__ float2 gemm_operand(const GemmParams& p, int m, int n, const QkvRow& qr, const QkvCol& qc) {
  if constexpr (EP == GEP_RESID || EP == GEP_SILU_MUL) {
    const int mm = m < p.M ? m : p.M - 1;  // rows past M: a clamped copy, never stored
    return make_float2(bf2f(p.C[(size_t)mm * p.ldc + n]), 0.f);
  } else if constexpr (EP == GEP_QKV) {
    if (LLJ_QKV_ABL & 1) return make_float2(1.f, 0.f);  // timing ablation: no RoPE operand loads (results wrong)
    if (qc.region < 2) return *reinterpret_cast<const float2*>(p.rope + ((size_t)qr.ps * (p.head_size >> 1) + (qc.dd >> 1)) * 2);
    return make_float2(1.f, 0.f);
  } else {
    return make_float2(0.f, 0.f);
  }
}

// One output element of a tile epilogue: y (the dequantized accumulator, fp32) at row m (live: m < M;
// rows past M are computed on a clamped copy and never stored), column n; row = lane & 15 (the column
// within the block); op = gemm_operand's value, qr / qc = qkv_row's / qkv_col's. Every lane of the
// wave calls it (lane_xor1 pairs neighbouring columns into one 4-byte store).
template <int EP>
__device__ __forceinline__ void gemm_store_elem(const GemmParams& p, float y, int m, int n, bool live, int row,
                                                int Cd, float2 op, const QkvRow& qr, const QkvCol& qc) {
  const int M = p.M;
  if constexpr (EP == GEP_QKV) {
    const float v = round_bf(y);  // c_attn output in bf16 (model.py:204), RoPE in fp32
    const float partner = lane_xor1(v);
    const int dd = qc.dd;
    const int mm = live ? m : M - 1;
    float out = v;
    if (qc.region < 2) out = (dd & 1) ? (v * op.x + partner * op.y) : (v * op.x - partner * op.y);
    const uint32_t ob = (uint32_t)f2bf(out);
    const uint32_t pr = lane_xor1(ob);
    if (live && !(dd & 1) && !(LLJ_QKV_ABL & 2)) {  // (LLJ_QKV_ABL & 2: timing ablation, no q / k / v stores)
      bf16_t* dst;
      size_t ei;
      if (qc.region == 0) {
        dst = p.q_out;
        ei = (size_t)mm * Cd + qc.nc;
      } else {
        dst = qc.region == 1 ? p.kcache : p.vcache;
        ei = (size_t)qr.kvrow + qc.hoff + dd;
      }
      *reinterpret_cast<uint32_t*>(dst + ei) = ob | (pr << 16);
    }
  } else {
    bf16_t* cp = p.C + (size_t)(live ? m : M - 1) * p.ldc + n;
    float o;
    if constexpr (EP == GEP_RESID) {
      o = round_bf(op.x + round_bf(y));  // x + y in bf16 (model.py:172-173)
    } else if constexpr (EP == GEP_SILU_MUL) {
      const float a1 = op.x;  // bf16(c_fc1 x), stored by the first pass
      const float sl = round_bf(a1 / (1.f + __expf(-a1)));  // F.silu in bf16
      o = sl * round_bf(y);
    } else {
      o = y;
    }
    const uint32_t ob = (uint32_t)f2bf(o);
    const uint32_t pr = lane_xor1(ob);
    if (live && !(row & 1)) *reinterpret_cast<uint32_t*>(cp) = ob | (pr << 16);
  }
}

constexpr int kGBM = 128, kGBN = 128, kGBK = 64, kGNT = 256;
#ifndef LLJ_GEMM_PRIO
#define LLJ_GEMM_PRIO 0
#endif
#ifndef LLJ_GEMM_MFAST
#define LLJ_GEMM_MFAST 1
#endif
#ifndef LLJ_GDEPTH
#define LLJ_GDEPTH 2  // W4: chunks in flight per thread (register ring); bf16 keeps 1 (registers)
#endif
// 256 x 128 tiles with 8 waves (4 row groups x 2 column groups of 64 x 64) for M >= 256: a weight
// panel's 128-deep chunk feeds twice the rows (A + B bytes per MFMA 0.75x), one workgroup per CU
#ifndef LLJ_GEMM_BM256
#define LLJ_GEMM_BM256 1  // bf16 (7B 2048-token window 70.5 -> 42.6 ms with 2 chunks in flight)
#endif
#ifndef LLJ_GEMM_BM256_I8
#define LLJ_GEMM_BM256_I8 1  // LLM.int8
#endif
#ifndef LLJ_GEMM_BM256_W4
#define LLJ_GEMM_BM256_W4 1  // int4 W4P (39.6 -> 38.4 ms; 256 VGPRs + 64-72 B of scratch per lane)
#endif
#ifndef LLJ_GEMM_W4_WIDE
#define LLJ_GEMM_W4_WIDE 0  // int4 256-row tiles as 2 x 4 waves of 128 x 32 (A/B)
#endif
#ifndef LLJ_GEMM_MFAST_W4
#define LLJ_GEMM_MFAST_W4 0  // int4: m-fastest tile order too (A/B)
#endif
#ifndef LLJ_GDEPTH_W4_256
#define LLJ_GDEPTH_W4_256 LLJ_GDEPTH  // int4 256-row tiles (188 VGPRs at 2 chunks in flight)
#endif
#ifndef LLJ_GDEPTH_DENSE
#define LLJ_GDEPTH_DENSE 1  // bf16 / int8 in 128-row tiles (32 VGPRs of A + B per chunk in flight)
#endif
#ifndef LLJ_GDEPTH_DENSE256
#define LLJ_GDEPTH_DENSE256 2  // bf16 / int8 in 256-row tiles (7B bf16 window 59.6 ms at 1, 42.6 at 2)
#endif
constexpr int kAP = kGBK + 8;  // A / bf16-B LDS row pitch (elements): 144 B

template <int WF>
constexpr size_t gemm_b_bytes() {
  return (WF == GWF_W4 || WF == GWF_W4G) ? (size_t)kGBN * kGBK / 2
         : WF == GWF_W8                  ? (size_t)kGBN * kGBK
         : WF == GWF_I8                  ? (size_t)kGBN * 128  // 8 I8P tile blocks of 2 KiB
                                         : (size_t)kGBN * kAP * 2;
}
// GWF_I8 side product staging (in the A / B buffers after the K loop): 32 outlier columns per
// round, f16 rows of 64 B at a pitch of 80 B
constexpr int kSideK = 32, kSideP = 40;  // pitch in halves
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
template <int WF, int BM = kGBM>
constexpr size_t gemm_lds_bytes() {
  // GWF_I8: also the dense side loop's two (A, B) f16 chunk buffers at the bf16 pitch
  const size_t main = 2 * ((size_t)BM * kAP * 2 + gemm_b_bytes<WF>()) + BM * sizeof(float);
  const size_t side = 2 * ((size_t)BM * kAP * 2 + (size_t)kGBN * kAP * 2);
  return WF == GWF_I8 && side > main ? side : main;
}

// BM: rows per tile (128, or 256 for bf16 with 8 waves: 4 row groups x 2 column groups of 64 x 64)
template <int WF, int EP, int BM = kGBM>
__global__ __launch_bounds__(2 * BM) void gemm_kernel(GemmParams p) {
  static_assert(BM == kGBM || WF == GWF_BF16 || WF == GWF_I8 || WF == GWF_W4, "256-row tiles: bf16, int8, int4");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr bool NIB = WF == GWF_W4 || WF == GWF_W8;  // nibble-coded: offset removed with the A row sums
  constexpr bool GRP = WF == GWF_W4G;                  // grouped int4: dequantized to the weight values
  constexpr bool I8 = WF == GWF_I8;                    // LLM.int8(): int8 MFMA + fp16 outlier side product
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // wave grid: WRN row groups x WCN column groups of (16 MI) x (16 NJ) outputs; int4 256-row tiles
  // optionally 2 x 4 waves of 128 x 32 (LLJ_GEMM_W4_WIDE: each B fragment dequantized by 2 waves, not 4)
  constexpr bool WIDE = WF == GWF_W4 && BM == 256 && LLJ_GEMM_W4_WIDE;
  constexpr int WRN = WIDE ? 2 : BM / 64;  // row groups of waves
  constexpr int WCN = 2 * BM / 64 / WRN;   // column groups (2 * BM threads = 2 * BM / 64 waves)
  constexpr int MI = BM / WRN / 16, NJ = kGBN / WCN / 16;
  const int wr = wave % WRN, wc = wave / WRN;
  const int row = lane & 15, g = lane >> 4;
  const int M = p.M, K = p.K, KC = I8 ? K / 128 : K / kGBK, KC128 = K / 128;
  const int mtiles = (M + BM - 1) / BM, ntiles = p.N / kGBN;
  const int total = mtiles * ntiles;
  int t = blockIdx.x;
  if (total % 8 == 0) t = (t % 8) * (total / 8) + t / 8;  // contiguous tile range per XCD
  // m fastest (LLJ_GEMM_MFAST): the workgroups resident on one XCD cover a few weight column
  // panels x every row panel, so a weight panel is fetched once and shared through L2 by all
  // its row tiles (n fastest re-streamed every weight panel once per 128-row panel)
  // (bf16 weights: 7B T = 2048 window 86.3 -> 71.9 ms; int4 weights, 4x smaller: 40.0 vs 40.6 ms, kept n fastest)
  constexpr bool MF = (WF == GWF_BF16 || I8 || (WF == GWF_W4 && LLJ_GEMM_MFAST_W4)) && LLJ_GEMM_MFAST;
  const int nb = MF ? t / mtiles : t % ntiles, mb = MF ? t % mtiles : t / ntiles;
  const int m0 = mb * BM, n0 = nb * kGBN;

  // LDS: [A buf 0][A buf 1][B buf 0][B buf 1][row sums]
  constexpr size_t kAB = (size_t)BM * kAP * 2, kBB = gemm_b_bytes<WF>();
  auto As = [&](int b) { return reinterpret_cast<bf16_t*>(smem + b * kAB); };
  auto Bs = [&](int b) { return smem + 2 * kAB + b * kBB; };
  float* rs_lds = reinterpret_cast<float*>(smem + 2 * (kAB + kBB));

  // ---- staging: thread -> (A row, half of the 128-B chunk row) = 4 x 16 B; B: W4 1 x 16 B
  // (tile tid / 32, W4P lane 32 h + tid % 32), bf16 4 x 16 B (row, half) like A
  const int ar = tid >> 1, ah = tid & 1;
  const int agm = m0 + ar < M ? m0 + ar : M - 1;  // rows past M: a clamped copy, never stored
  const bf16_t* asrc = p.A + (size_t)agm * p.lda + ah * 32;
  I8Layout L8{};
  if constexpr (I8) {
    const I8WsHeader h8 = *reinterpret_cast<const I8WsHeader*>(p.i8ws);
    L8 = i8_layout(p.i8ws, h8.mtot, h8.K);
  }
  // GWF_I8: the thread's half of its row of the quantized activation (128 B per 128-deep chunk)
  const int8_t* aqsrc = I8 ? L8.aq + (size_t)agm * K + ah * 64 : nullptr;
  // register ring of GDEPTH chunks in flight (chunk c lives in slot c % GDEPTH)
  constexpr int GDEPTH = (WF == GWF_W4 && BM == 256) ? LLJ_GDEPTH_W4_256
                         : (NIB || GRP) ? LLJ_GDEPTH : BM == 256 ? LLJ_GDEPTH_DENSE256 : LLJ_GDEPTH_DENSE;
  constexpr int BV = (WF == GWF_W4 || GRP) ? 1 : WF == GWF_W8 ? 2 : BM == 256 ? 2 : 4;  // GWF_I8: 4 (64 B of its tile block)
  // bf16 B with 256-row tiles: 512 threads over the 128 weight rows, a quarter row (32 B) each
  const int br = BM == 256 ? tid >> 2 : ar, bq = BM == 256 ? tid & 3 : ah;
  // int8 B: the 8 tile blocks of 128 x 16 B over TPB threads each; int4 B: the first 256 threads
  constexpr int TPB = BM / 4;
  const int bt = tid & 255;
  u32x4 areg[GDEPTH][4], breg[GDEPTH][BV];
  float2 szr[GDEPTH][4];  // GWF_W4G: (scale, 128 + zero) of the chunk's group for the lane's column of tile j
  auto load_chunk = [&](int slot, int c) {
    c = c < KC ? c : KC - 1;  // past the end: a valid duplicate, never stored
    if constexpr (I8) {
#pragma unroll
      for (int v = 0; v < 4; ++v) areg[slot][v] = *reinterpret_cast<const u32x4*>(aqsrc + (size_t)c * 128 + 16 * v);
      const u32x4* w = reinterpret_cast<const u32x4*>(p.W);  // I8P: (tile, chunk) block of 128 x 16 B
      const size_t o = ((size_t)(n0 / 16 + tid / TPB) * KC128 + c) * 128 + tid % TPB;
#pragma unroll
      for (int v = 0; v < BV; ++v) breg[slot][v] = __builtin_nontemporal_load(w + o + TPB * v);
      return;
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) areg[slot][v] = *reinterpret_cast<const u32x4*>(asrc + (size_t)c * kGBK + 8 * v);
    if constexpr (WF == GWF_W4 || GRP) {
      const u32x4* w = reinterpret_cast<const u32x4*>(p.W);
      const size_t nt = (size_t)(n0 / 16 + (bt >> 5));  // (256-row tiles: threads 256.. load a copy, never stored)
      breg[slot][0] = __builtin_nontemporal_load(w + (nt * KC128 + (c >> 1)) * 64 + 32 * (c & 1) + (bt & 31));
      if constexpr (GRP) {
        const size_t go = (size_t)((c >> 1) / p.gch) * p.N + n0 + wc * 16 * NJ + row;
#pragma unroll
        for (int j = 0; j < NJ; ++j) szr[slot][j] = p.sz[go + 16 * j];
      }
    } else if constexpr (WF == GWF_W8) {  // the same W4P lane of the low plane and of the high plane
      const u32x4* w = reinterpret_cast<const u32x4*>(p.W);
      const size_t nt = (size_t)(n0 / 16 + (tid >> 5));
      const size_t o = (nt * KC128 + (c >> 1)) * 128 + 32 * (c & 1) + (tid & 31);
      breg[slot][0] = __builtin_nontemporal_load(w + o);
      breg[slot][1] = __builtin_nontemporal_load(w + o + 64);
    } else {
      const bf16_t* w = reinterpret_cast<const bf16_t*>(p.W) + (size_t)(n0 + br) * K + (size_t)c * kGBK + bq * 8 * BV;
#pragma unroll
      for (int v = 0; v < BV; ++v) breg[slot][v] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(w + 8 * v));
    }
  };
  f32x2 rsum2 = {0.f, 0.f};  // this thread's share of sum_k A[ar, k]
  auto store_chunk = [&](int slot, int buf) {
    if constexpr (I8) {  // A rows of 128 B at the bf16 pitch (144 B); B: the 8 tile blocks as stored
      unsigned char* a8 = reinterpret_cast<unsigned char*>(As(buf)) + ar * (kAP * 2) + ah * 64;
#pragma unroll
      for (int v = 0; v < 4; ++v) *reinterpret_cast<u32x4*>(a8 + 16 * v) = areg[slot][v];
#pragma unroll
      for (int v = 0; v < BV; ++v) reinterpret_cast<u32x4*>(Bs(buf))[(tid / TPB) * 128 + tid % TPB + TPB * v] = breg[slot][v];
      return;
    }
    bf16_t* a = As(buf) + ar * kAP + ah * 32;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      *reinterpret_cast<u32x4*>(a + 8 * v) = areg[slot][v];
      if constexpr (NIB) {
        rsum2 += unpk(areg[slot][v][0]) + unpk(areg[slot][v][1]);
        rsum2 += unpk(areg[slot][v][2]) + unpk(areg[slot][v][3]);
      }
    }
    if constexpr (WF == GWF_W4 || GRP) {
      if (BM == 128 || tid < 256) reinterpret_cast<u32x4*>(Bs(buf))[tid] = breg[slot][0];
    } else if constexpr (WF == GWF_W8) {  // [low plane halves 4 KiB][high plane halves 4 KiB]
      reinterpret_cast<u32x4*>(Bs(buf))[tid] = breg[slot][0];
      reinterpret_cast<u32x4*>(Bs(buf))[kGNT + tid] = breg[slot][1];
    } else {
      bf16_t* b = reinterpret_cast<bf16_t*>(Bs(buf)) + br * kAP + bq * 8 * BV;
#pragma unroll
      for (int v = 0; v < BV; ++v) *reinterpret_cast<u32x4*>(b + 8 * v) = breg[slot][v];
    }
  };

  uint32_t msk = 0x000F000Fu, mag = 0x43004300u, mag_hi = 0x45004500u;  // mag_hi: W8 high nibbles, 2048 + 16 hi
  asm volatile("" : "+s"(msk));
  asm volatile("" : "+v"(mag));
  if constexpr (WF == GWF_W8) asm volatile("" : "+v"(mag_hi));
  f32x4 acc[MI][NJ];
  i32x4 iacc[MI][NJ];  // GWF_I8
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      iacc[i][j] = i32x4{0, 0, 0, 0};
    }

  auto step = [&](int slot, int c) {  // chunk c: stage it, refill its slot with c + GDEPTH, multiply
    const int buf = c & 1;
    float2 gsz[4];  // GWF_W4G: this chunk's group pairs (the slot is refilled below)
#pragma unroll
    for (int j = 0; j < 4; ++j) gsz[j] = szr[slot][j];
    store_chunk(slot, buf);
    __syncthreads();  // chunk c staged; every wave is done with chunk c - 1's buffer
    load_chunk(slot, c + GDEPTH);
    if constexpr (I8) {  // two 64-deep MFMA steps; lane group g: k = 64 s + 16 g + [0, 16)
      const unsigned char* a8 = reinterpret_cast<const unsigned char*>(As(buf));
      const u32x4* b8 = reinterpret_cast<const u32x4*>(Bs(buf));
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        i32x4 af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[i] = __builtin_bit_cast(i32x4, *reinterpret_cast<const u32x4*>(a8 + (wr * 64 + 16 * i + row) * (kAP * 2) +
                                                                            64 * s + 16 * g));
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = __builtin_bit_cast(i32x4, b8[(wc * 4 + j) * 128 + 64 * s + lane]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) iacc[i][j] = mfma_i8(af[i], bfr[j], iacc[i][j]);
      }
      return;
    }
    const bf16_t* a = As(buf);
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // MFMA k-steps of the chunk: k = 32 s + 8 g + [0, 8)
      bf16x8 af[MI], bfr[NJ], bhi[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int r = wr * 16 * MI + 16 * i + row;
        af[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(a + r * kAP + 32 * s + 8 * g));
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if constexpr (WF == GWF_W4) {
          // word g of W4P lane 16 (2h + s) + column of tile wc * NJ + j (the chunk's half)
          const uint32_t w = reinterpret_cast<const uint32_t*>(Bs(buf))[((wc * NJ + j) * 32 + 16 * s + row) * 4 + g];
          const uint4 d = make_uint4(and_or(w, msk, mag), and_or(w >> 4, msk, mag), and_or(w >> 8, msk, mag),
                                     and_or(w >> 12, msk, mag));
          bfr[j] = __builtin_bit_cast(bf16x8, d);
        } else if constexpr (GRP) {
          // bf16(fp32(q - z) * s), the reference's get_weight(bf16) (quantization.py:402-408: the bf16
          // weight times the scale in the scale's precision, then stored to bf16): (128 + q) - (128 + z)
          // is an exact small integer, its product with s rounds once to fp32 (exact for bf16 / fp16
          // scales, the reference's fp32 product for fp32 scales), the conversion once to bf16
          const uint32_t w = reinterpret_cast<const uint32_t*>(Bs(buf))[((wc * NJ + j) * 32 + 16 * s + row) * 4 + g];
          const f32x2 sc = {gsz[j].x, gsz[j].x}, zz = {gsz[j].y, gsz[j].y};
          uint32_t o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = cvt_pk((unpk(and_or(w >> (4 * e), msk, mag)) - zz) * sc);
          bfr[j] = __builtin_bit_cast(bf16x8, make_uint4(o[0], o[1], o[2], o[3]));
        } else if constexpr (WF == GWF_W8) {
          const uint32_t* b32 = reinterpret_cast<const uint32_t*>(Bs(buf));
          const int wi = ((wc * NJ + j) * 32 + 16 * s + row) * 4 + g;
          const uint32_t wl = b32[wi], wh = b32[kGNT * 4 + wi];
          bfr[j] = __builtin_bit_cast(bf16x8, make_uint4(and_or(wl, msk, mag), and_or(wl >> 4, msk, mag),
                                                         and_or(wl >> 8, msk, mag), and_or(wl >> 12, msk, mag)));
          bhi[j] = __builtin_bit_cast(bf16x8, make_uint4(and_or(wh, msk, mag_hi), and_or(wh >> 4, msk, mag_hi),
                                                         and_or(wh >> 8, msk, mag_hi), and_or(wh >> 12, msk, mag_hi)));
        } else {
          const int n = wc * 16 * NJ + 16 * j + row;
          bfr[j] = __builtin_bit_cast(
              bf16x8, *reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(Bs(buf)) + n * kAP + 32 * s + 8 * g));
        }
      }
      if (LLJ_GEMM_PRIO) __builtin_amdgcn_s_setprio(1);  // the MFMA cluster ahead of the other waves' staging
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          acc[i][j] = mfma_bf16(af[i], bfr[j], acc[i][j]);
          if constexpr (WF == GWF_W8) acc[i][j] = mfma_bf16(af[i], bhi[j], acc[i][j]);
        }
      if (LLJ_GEMM_PRIO) __builtin_amdgcn_s_setprio(0);
    }
  };
#pragma unroll
  for (int d = 0; d < GDEPTH; ++d) load_chunk(d, d);
  int c = 0;  // KC is a multiple of 2 (K % 128 == 0); the ring slots are static inside the unrolled body
  // 64-deep chunks (all but LLM.int8): KC = K / 64 is even and >= 2, so with GDEPTH <= 2 the loop
  // runs at least once and no tail step is left (without this the compiler keeps the prologue's
  // chunk live across the loop for the tail and spills it at 256 VGPRs)
  if constexpr ((WF == GWF_W4 || WF == GWF_BF16) && GDEPTH <= 2) __builtin_assume(KC >= 2 && KC % 2 == 0);
  for (; c + GDEPTH <= KC; c += GDEPTH) {
#pragma unroll
    for (int d = 0; d < GDEPTH; ++d) step(d, c + d);
  }
#pragma unroll
  for (int d = 0; d < GDEPTH; ++d)
    if (c + d < KC) step(d, c + d);
  float rsum = rsum2.x + rsum2.y;
  // row sums of A (both halves of a row are adjacent lanes)
  rsum += lane_xor1(rsum);
  if (!ah) rs_lds[ar] = rsum;
  __syncthreads();

  // ---- GWF_I8: fp16 outlier side product into sacc (the K loop's LDS is free now)
  f32x4 sacc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) sacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (I8) {
    int* s_pre = reinterpret_cast<int*>(smem);  // [kNSB + 1] prefix of the per-block outlier counts
    int* s_k = s_pre + 64;                      // [kSideK] this round's columns
    _Float16* sa16 = reinterpret_cast<_Float16*>(smem + 512);          // [128 rows][kSideP]
    _Float16* sb16 = sa16 + BM * kSideP;                               // [128 columns][kSideP]
    I8WsHeader h8 = *reinterpret_cast<const I8WsHeader*>(p.i8ws);
    h8.nsb = i8_nsb_clamp(h8.nsb);
    if (tid < 64) {
      const int cn = tid < h8.nsb ? i8_cnt_clamp(L8.cnt[tid], h8.kb) : 0;
      int x = cn;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      s_pre[tid + 1] = x;
      if (tid == 0) s_pre[0] = 0;
    }
    __syncthreads();
    const int total = s_pre[h8.nsb];
    const int sn = n0 + (bt >> 1);  // staging: W column (B) bt >> 1 / A row (A) ar, outliers 16 ah + [0, 16)
    const float scb = reinterpret_cast<const float*>(p.sz)[sn] / 127.f;
    const bool gathered = p.ao16 && total <= p.kpad;  // else: more outliers than the gathers' capacity
    if (gathered) {  // dense f16 GEMM over the pre-gathered outlier columns, 64-deep chunks
      __syncthreads();  // every thread has read `total` before the chunk buffers overwrite s_pre
      const int SKC = (total + 63) >> 6;
      constexpr int BVD = BM == 256 ? 2 : 4;
      _Float16* SA = reinterpret_cast<_Float16*>(smem);  // [2][BM][kAP]
      _Float16* SB = SA + 2 * BM * kAP;                  // [2][128][kAP]
      u32x4 ra[4], rb[BVD];
      auto sload = [&](int c) {
        const _Float16* a = p.ao16 + (size_t)agm * p.kpad + c * 64 + ah * 32;
#pragma unroll
        for (int v = 0; v < 4; ++v) ra[v] = *reinterpret_cast<const u32x4*>(a + 8 * v);
        const _Float16* b = p.w16 + (size_t)(n0 + br) * p.kpad + c * 64 + bq * 8 * BVD;
#pragma unroll
        for (int v = 0; v < BVD; ++v) rb[v] = *reinterpret_cast<const u32x4*>(b + 8 * v);
      };
      if (SKC > 0) sload(0);
      for (int c = 0; c < SKC; ++c) {
        const int buf = c & 1;
        _Float16* sa = SA + (size_t)buf * BM * kAP;
        _Float16* sb = SB + (size_t)buf * kGBN * kAP;
#pragma unroll
        for (int v = 0; v < 4; ++v) *reinterpret_cast<u32x4*>(sa + ar * kAP + ah * 32 + 8 * v) = ra[v];
#pragma unroll
        for (int v = 0; v < BVD; ++v) *reinterpret_cast<u32x4*>(sb + br * kAP + bq * 8 * BVD + 8 * v) = rb[v];
        __syncthreads();  // chunk c staged; every wave is done with chunk c - 1's buffer
        if (c + 1 < SKC) sload(c + 1);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          f16x8 af[4], bfr[4];
#pragma unroll
          for (int i = 0; i < 4; ++i)
            af[i] = *reinterpret_cast<const f16x8*>(sa + (wr * 64 + 16 * i + row) * kAP + 32 * s2 + 8 * g);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            bfr[j] = *reinterpret_cast<const f16x8*>(sb + (wc * 64 + 16 * j + row) * kAP + 32 * s2 + 8 * g);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              sacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bfr[j], sacc[i][j], 0, 0, 0);
        }
      }
    }
    for (int c0 = 0; c0 < (gathered ? 0 : total); c0 += kSideK) {
      if (tid < kSideK) {
        const int fi = c0 + tid;
        int k = -1;
        if (fi < total) {
          int b = 0;
          while (b + 1 < h8.nsb && s_pre[b + 1] <= fi) ++b;
          k = i8_col_clamp(L8.list[b * h8.kb + (fi - s_pre[b])], p.K);
        }
        s_k[tid] = k;
      }
      __syncthreads();
      {
        _Float16 av[16], wv[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int k = s_k[16 * ah + e];
          const int kk = k < 0 ? 0 : k;
          const float a = bf2f(p.A[(size_t)agm * p.lda + kk]);
          const int q = reinterpret_cast<const int8_t*>(p.W)[  // byte (sn, kk) of the I8P tiling
              (((size_t)(sn >> 4) * KC128 + (kk >> 7)) * 2 + ((kk & 127) >> 6)) * 1024 +
              (16 * ((kk >> 4) & 3) + (sn & 15)) * 16 + (kk & 15)];
          av[e] = k < 0 ? (_Float16)0.f : (_Float16)a;
          wv[e] = k < 0 ? (_Float16)0.f : (_Float16)((float)q * scb);
        }
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          *reinterpret_cast<f16x8*>(sa16 + ar * kSideP + 16 * ah + 8 * v) =
              f16x8{av[8 * v], av[8 * v + 1], av[8 * v + 2], av[8 * v + 3], av[8 * v + 4], av[8 * v + 5], av[8 * v + 6], av[8 * v + 7]};
          if (BM == 128 || tid < 256)
            *reinterpret_cast<f16x8*>(sb16 + (bt >> 1) * kSideP + 16 * ah + 8 * v) =
              f16x8{wv[8 * v], wv[8 * v + 1], wv[8 * v + 2], wv[8 * v + 3], wv[8 * v + 4], wv[8 * v + 5], wv[8 * v + 6], wv[8 * v + 7]};
        }
      }
      __syncthreads();
      f16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const f16x8*>(sa16 + (wr * 64 + 16 * i + row) * kSideP + 8 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = *reinterpret_cast<const f16x8*>(sb16 + (wc * 64 + 16 * j + row) * kSideP + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) sacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bfr[j], sacc[i][j], 0, 0, 0);
      __syncthreads();
    }
  }

  // ---- epilogue: lane holds rows m0 + wr*64 + 16i + 4g + r, column n0 + wc*64 + 16j + row
  const int Cd = p.n_head * p.head_size;
  QkvRow qrow[EP == GEP_QKV ? MI : 1][4] = {};  // QKV: per row, once per tile
  if constexpr (EP == GEP_QKV) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) qrow[i][r] = qkv_row(p, m0 + wr * 16 * MI + 16 * i + 4 * g + r);
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = n0 + wc * 16 * NJ + 16 * j + row;
    float2 szn = make_float2(1.f, 0.f);
    if constexpr (NIB) szn = p.sz[n];
    if constexpr (I8) szn.x = reinterpret_cast<const float*>(p.sz)[n];  // SCB
    const int nblk = n0 + wc * 16 * NJ + 16 * j;  // first column of this 16-column block
    const QkvCol qc = EP == GEP_QKV ? qkv_col(p, nblk, n, Cd) : QkvCol{};
    constexpr int GI = I8 ? (EP == GEP_QKV ? 1 : 2) : 4;  // row blocks whose operands are in flight together (LLM.int8: 3 accumulator sets live)
#pragma unroll
    for (int i0 = 0; i0 < MI; i0 += GI) {
      float2 opv[GI][4];
#pragma unroll
      for (int i = 0; i < GI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wr * 16 * MI + 16 * (i0 + i) + 4 * g + r;
          opv[i][r] = gemm_operand<EP>(p, m, n, qrow[EP == GEP_QKV ? i0 + i : 0][r], qc);
        }
#pragma unroll
      for (int i = 0; i < GI; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ml = wr * 16 * MI + 16 * (i0 + i) + 4 * g + r;
          const int m = m0 + ml;
          float y = acc[i0 + i][j][r];
          if constexpr (NIB) y = szn.x * (y - szn.y * rs_lds[ml]);
          const bool live = m < M;
          if constexpr (I8) {  // mm_dequant in fp16, + the fp16 outlier product, in fp16 (the GEMV's epilogue)
            const float sa = L8.sca[live ? m : M - 1];
            y = (float)iacc[i0 + i][j][r] * (sa * szn.x * (1.f / (127.f * 127.f)));
            y = (float)(_Float16)((float)(_Float16)y + sacc[i0 + i][j][r]);
          }
          gemm_store_elem<EP>(p, y, m, n, live, row, Cd, opv[i][r], qrow[EP == GEP_QKV ? i0 + i : 0][r], qc);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the next group's operand loads out of this one's live range
    }
  }
}

template <int WF, int EP, int BM = kGBM>
static int gemm_launch(const GemmParams& p, hipStream_t s) {
  auto kern = gemm_kernel<WF, EP, BM>;
  static bool attr_set = false;  // per instantiation, before any graph capture
  const size_t lds = gemm_lds_bytes<WF, BM>();
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  const int tiles = ((p.M + BM - 1) / BM) * (p.N / kGBN);
  hipLaunchKernelGGL(kern, dim3(tiles), dim3(2 * BM), lds, s, p);
  LLJ_CHECK_LAUNCH();
  return 0;
}


// ---------------------------------------------------------------------------------------------
// 256-row LDS-DMA GEMM (bf16 and int4 W4P weights, M >= 256): a 512-thread workgroup (8 waves, one
// per CU) owns a 256 x BN output tile (BN 256: waves 2 x 4 of 128 x 64; BN 128: 4 x 2 of 64 x 64)
// and walks K in 64-deep chunks. A chunk's A tile (256 rows x 128 B) and B tile (bf16: BN rows x
// 128 B; W4P: the 512-B half of each of its BN / 16 tiles that holds the chunk) go global -> LDS
// by global_load_lds_dwordx4 (no VGPR staging, no ds_write), NST stages deep: the loads of chunks
// t + 1 .. t + NST - 1 stay in flight across the barrier while chunk t is multiplied; the wait for
// chunk t is a counted vmcnt (never 0 while a later chunk is outstanding) and the barrier a raw
// s_barrier (a __syncthreads() would drain every DMA in flight). The LDS image is lane-linear (the
// DMA writes base + 16 * lane) with the 16-B segments of a 128-B row permuted by
// seg ^ ((row >> 1) & 7) on the SOURCE side, so a fragment read (16 rows x 16 B per lane group)
// hits 16 distinct bank slots. int4: the 128 + zero offset is removed with the row sums of A,
// which the waves form from the A fragments they already hold (v_dot2 with (1, 1); wave column wc
// sums the 16-row blocks i = wc mod WN) and combine through LDS after the loop.
#ifndef LLJ_GEMM_GLDS_BF16
#define LLJ_GEMM_GLDS_BF16 1  // 7B 2048-token bf16 window 43.1 -> 36.5 ms (profiles/r04_prefill_ab.json)
#endif
#ifndef LLJ_GEMM_GLDS_W4
#define LLJ_GEMM_GLDS_W4 0  // int4: 42.5 ms vs 37.6 with the register-staged 256-row kernel
#endif
#ifndef LLJ_GLDS_W4_WN
#define LLJ_GLDS_W4_WN 4
#endif
#ifndef LLJ_GLDS_PRE
#define LLJ_GLDS_PRE 1  // 256 x 128 tiles: read both MFMA steps' fragments of a chunk before its MFMAs (bf16 window 35.9 -> 35.4 ms)
#endif
#ifndef LLJ_GLDS_GROUPM
#define LLJ_GLDS_GROUPM 0  // A/B only: grouped tile order (row tiles per group); 0 = the m- / n-fastest orders below
#endif
#ifndef LLJ_GLDS_NFAST_W4Z
#define LLJ_GLDS_NFAST_W4Z 1  // convert-once int4 LDS-DMA GEMM: n-fastest tile order (A/B)
#endif
#ifndef LLJ_GLDS_NFAST_BF16
#define LLJ_GLDS_NFAST_BF16 0  // bf16 LDS-DMA GEMM: n-fastest tile order (A/B)
#endif
#ifndef LLJ_GLDS_FDB
#define LLJ_GLDS_FDB 1  // LDS-DMA GEMM at 256 x 128: chunk t + 1's fragments read during chunk t's MFMAs (A/B)
#endif
#ifndef LLJ_FDB_DSPM
#define LLJ_FDB_DSPM 0  // fragment double buffering: LDS fragment reads per MFMA in the sched_group pattern (0: the scheduler's)
#endif
#ifndef LLJ_W4Z_PRIO
#define LLJ_W4Z_PRIO 0  // convert-once int4: s_setprio around the MFMA clusters (1; 0: none, so the conversion interleaves with them)
#endif
#ifndef LLJ_W4Z_WAVES
#define LLJ_W4Z_WAVES 8  // convert-once int4: waves converting a chunk's codes (8 or 4)
#endif
#ifndef LLJ_W4Z_SPLIT
#define LLJ_W4Z_SPLIT 1  // convert-once int4, 8 converting waves: codes read before the fragment reads (A/B)
#endif
#ifndef LLJ_W4Z_IGLP
#define LLJ_W4Z_IGLP 1  // convert-once int4: sched_group_barrier interleave of the conversion with the MFMAs
#endif
#ifndef LLJ_W4Z_VPM
#define LLJ_W4Z_VPM 1  // VALU instructions per MFMA in that interleave (with fragment double buffering: 1 vs 2 vs 3 = 29.4-29.5 vs 29.9-30.0 vs 31.1 ms per 7B window)
#endif
#ifndef LLJ_W4Z_AFTER
#define LLJ_W4Z_AFTER 0  // convert-once int4: the converting waves convert after their MFMAs (A/B)
#endif
#ifndef LLJ_GLDS_COST128
#define LLJ_GLDS_COST128 55  // time of a 256 x 128 tile in % of a 256 x 256 one (tile-shape choice)
#endif
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

template <int WF, int BN>
struct GldsGeo {
  // waves along N: 4 at BN 256; at BN 128, 2 for bf16 and the convert-once int4 (64 x 64 per wave:
  // fewer A fragment reads) and LLJ_GLDS_W4_WN for the per-fragment int4 (4: 128 x 32 per wave, each B
  // fragment dequantized by 2 waves instead of 4)
  static constexpr bool CVT = WF == GWF_W4Z;
  static constexpr int WN = BN == 256 ? 4 : WF == GWF_W4 ? LLJ_GLDS_W4_WN : 2, WM = 8 / WN;
  static constexpr int MI = 256 / WM / 16, NJ = BN / WN / 16;
  static constexpr size_t SA = 256 * 128;
  // int4 (both forms) at BN 128: the chunk's 4 KiB of W4P codes, waves 4-7 staging a copy (equal DMA
  // counts per wave)
  static constexpr size_t SB = (WF == GWF_W4 || CVT) ? 8192 : (size_t)BN * 128;
  static constexpr size_t STAGE = SA + SB;
  // convert-once int4: two bf16 (q - z) B tiles (BN rows x 128 B, the bf16 image) after the stages
  static constexpr size_t BF = CVT ? 2 * (size_t)BN * 128 : 0;
  static constexpr int NST = 3 * STAGE + BF + 1024 <= 160 * 1024 ? 3 : 2;
  static constexpr size_t LDS = NST * STAGE + BF + 1024;  // + the row sums (per-fragment int4)
  static constexpr int NG = 4 + ((WF == GWF_W4 || CVT) ? 1 : BN / 64);  // glds per thread per chunk
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int WF, int EP, int BN>
__global__ __launch_bounds__(512, 1) void gemm_glds_kernel(GemmParams p) {
  static_assert(WF == GWF_BF16 || WF == GWF_W4 || WF == GWF_W4Z, "LDS-DMA GEMM: bf16 and int4 W4P");
  static_assert(WF != GWF_W4Z || BN == 128, "convert-once int4: 256 x 128 tiles");
  // the dual SwiGLU form: 64 output columns per tile, B rows 0-63 from W1 and 64-127 from W2 (the same
  // columns), wave column group wc holding output columns 32 wc .. + 31 of BOTH (fragments j < NJ / 2
  // from W1, j >= NJ / 2 from W2), so each lane has fc1 and fc2 of the same element
  constexpr bool DUAL = EP == GEP_SWIGLU || EP == GEP_SWIGLU_PART;
  static_assert(!DUAL || WF == GWF_W4Z, "dual SwiGLU GEMM: convert-once int4");
  static_assert(EP != GEP_PARTIAL || ((WF == GWF_W4Z || WF == GWF_BF16) && BN == 128), "split-K slices: 256 x 128");
  constexpr int NOUT = DUAL ? BN / 2 : BN;  // output columns per tile
  using G = GldsGeo<WF, BN>;
  constexpr int MI = G::MI, NJ = G::NJ, WN = G::WN, NST = G::NST;
  constexpr bool NIB = WF == GWF_W4;  // per-fragment dequant (bf16 128 + q) + row sums
  constexpr bool CVT = G::CVT;        // W4P codes converted once per chunk into a bf16 (q - z) tile
  constexpr bool FDB = LLJ_GLDS_FDB && BN == 128 && G::NST == 3 && (WF == GWF_BF16 || (CVT && LLJ_W4Z_WAVES == 8));
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w / WN, wc = w % WN;
  const int row = lane & 15, g = lane >> 4;
  constexpr bool PART = EP == GEP_PARTIAL || EP == GEP_SWIGLU_PART;  // split-K slice (kc0 .. kc0 + KC of the K chunks)
  const int M = p.M, K = p.K, KC128 = K / 128;
  const int split = PART ? (int)blockIdx.x % p.nsplit : 0;
  const int kc0 = PART ? split * p.kcs : 0;  // even: the W4P chunk pairs stay aligned
  const int KC = PART ? min(p.kcs, K / 64 - kc0) : K / 64;
  const int mtiles = (M + 255) / 256, ntiles = p.N / NOUT, total = mtiles * ntiles;
  int t = PART ? (int)blockIdx.x / p.nsplit : (int)blockIdx.x;
  {  // contiguous tile ranges per XCD (bijective for any total)
    const int q = total / 8, r = total % 8, x = t % 8;
    t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + t / 8;
  }
  // tile order inside an XCD's contiguous range: m fastest (a weight panel's row tiles run together and
  // share it through the XCD's L2) or n fastest (an A row panel stays in L2 while the XCD sweeps the
  // weight columns: the A re-reads go from one per column tile to one per XCD -- the int4 weights are a
  // quarter of the bf16 bytes, so re-reading them per row panel is the cheaper side)
  constexpr bool NFAST = CVT ? LLJ_GLDS_NFAST_W4Z != 0 : LLJ_GLDS_NFAST_BF16 != 0;
  // (LLJ_GLDS_GROUPM > 0, A/B: groups of that many row tiles sweep the columns together, m fastest inside)
  int nb = NFAST ? t % ntiles : t / mtiles, mb = NFAST ? t / ntiles : t % mtiles;
  if constexpr (LLJ_GLDS_GROUPM > 0) {
    const int gm = LLJ_GLDS_GROUPM, grp = t / (gm * ntiles), first = grp * gm;
    const int rows = mtiles - first < gm ? mtiles - first : gm;
    const int in = t - grp * gm * ntiles;
    mb = first + in % rows;
    nb = in / rows;
  }
  const int m0 = mb * 256, n0 = nb * NOUT;
  float* rs_lds = reinterpret_cast<float*>(smem + NST * G::STAGE);

  // ---- DMA sources: A rows q * 64 + 8 w + lane / 8 (q < 4), physical segment lane % 8 holds the
  // logical segment (lane % 8) ^ ((row >> 1) & 7); bf16 B the same over BN rows
  const int drow = 8 * w + (lane >> 3), dseg = (lane & 7) ^ ((drow >> 1) & 7);  // (row >> 1) & 7 same for +64 q
  const bf16_t* asrc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int m = m0 + 64 * q + drow;
    asrc[q] = p.A + (size_t)(m < M ? m : M - 1) * p.lda + 8 * dseg + (size_t)kc0 * 64;
  }
  const char* bsrc;
  if constexpr (NIB || CVT) {  // W4P: wave w stages tiles 2 w, 2 w + 1 (BN 128: waves 4-7 a copy of 0-3's)
    const int tl = (2 * w + (lane >> 5)) % (BN / 16);
    if (DUAL)  // B tiles 0-3: W1's columns n0 .. + 63, tiles 4-7: W2's
      bsrc = reinterpret_cast<const char*>(tl < 4 ? p.W : p.W2) + (size_t)(n0 / 16 + (tl & 3)) * KC128 * 1024 + 16 * (lane & 31) +
             (size_t)(kc0 >> 1) * 1024;
    else
      bsrc = reinterpret_cast<const char*>(p.W) + (size_t)(n0 / 16 + tl) * KC128 * 1024 + 16 * (lane & 31) +
             (size_t)(kc0 >> 1) * 1024;
  } else {
    bsrc = reinterpret_cast<const char*>(reinterpret_cast<const bf16_t*>(p.W) + (size_t)(n0 + drow) * K + 8 * dseg +
                                         (size_t)kc0 * 64);
  }
  // convert-once int4: the codes run one chunk ahead of A (DMA group c = A(c) + the codes of chunk
  // c + 1, into the stage buffer of chunk c + 1), so a chunk's codes have landed one iteration before
  // its MFMAs and are converted into its bf16 tile in between
  auto stage_codes = [&](int buf, int c) {
    __builtin_amdgcn_global_load_lds(bsrc + (size_t)(c >> 1) * 1024 + 512 * (c & 1),
                                     (lds_void_t*)(smem + (size_t)buf * G::STAGE + G::SA + 1024 * w), 16, 0, 0);
  };
  auto stage = [&](int buf, int c) {
    unsigned char* base = smem + (size_t)buf * G::STAGE;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds(asrc[q] + (size_t)c * 64, (lds_void_t*)(base + (64 * q + 8 * w) * 128), 16, 0, 0);
    if constexpr (CVT) {
      stage_codes(buf + 1 == NST ? 0 : buf + 1, c + 1 < KC ? c + 1 : KC - 1);
    } else if constexpr (NIB) {
      __builtin_amdgcn_global_load_lds(bsrc + (size_t)(c >> 1) * 1024 + 512 * (c & 1),
                                       (lds_void_t*)(base + G::SA + 1024 * w), 16, 0, 0);
    } else {
#pragma unroll
      for (int q = 0; q < BN / 64; ++q)
        __builtin_amdgcn_global_load_lds(bsrc + ((size_t)64 * q * K + (size_t)c * 64) * 2,
                                         (lds_void_t*)(base + G::SA + (64 * q + 8 * w) * 128), 16, 0, 0);
    }
  };

  // ---- fragment reads: A row wr * 16 MI + 16 i + row, B row (column) wc * 16 NJ + 16 j + row; MFMA
  // step s reads logical segment 4 s + g at physical (4 s + g) ^ sw
  const int sw = (row >> 1) & 7;
  const int aoff0 = (wr * 16 * MI + row) * 128, boff0 = (wc * 16 * NJ + row) * 128;
  // B row (tile column) of fragment j: DUAL -> W1 rows 32 wc + 16 j (j < NJ / 2), W2 rows 64 + 32 wc + 16 (j - NJ / 2)
  auto brow_off = [&](int j) {
    return DUAL ? ((j >= NJ / 2 ? 64 : 0) + wc * 16 * (NJ / 2) + 16 * (j % (NJ / 2)) + row) * 128 : boff0 + 16 * j * 128;
  };
  uint32_t msk = 0x000F000Fu, mag = 0x43004300u;
  asm volatile("" : "+s"(msk));
  asm volatile("" : "+v"(mag));
  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // W4: partial row sums of A. The WN waves of a row group split the chunk's (block, k) pairs: WN 4
  // -> wave wc sums the blocks of parity wc >> 1 in MFMA step wc & 1; WN 2 -> every block in step wc
  float rsp[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) rsp[i] = 0.f;
  if constexpr (NIB) {
    if (tid < 256) rs_lds[tid] = 0.f;  // ordered before the adds by the K loop's barriers
  }

  auto frags = [&](const unsigned char* Ab, const unsigned char* Bb, int s, bf16x8 (&af)[MI], bf16x8 (&bfr)[NJ]) {
    const int so = ((4 * s + g) ^ sw) * 16;
#pragma unroll
    for (int i = 0; i < MI; ++i) af[i] = *reinterpret_cast<const bf16x8*>(Ab + aoff0 + 16 * i * 128 + so);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if constexpr (NIB) {  // word g of W4P lane 16 s + column of tile wc * NJ + j (the chunk's half)
        const uint32_t wv = reinterpret_cast<const uint32_t*>(Bb)[((wc * NJ + j) * 32 + 16 * s + row) * 4 + g];
        bfr[j] = __builtin_bit_cast(bf16x8, make_uint4(and_or(wv, msk, mag), and_or(wv >> 4, msk, mag),
                                                       and_or(wv >> 8, msk, mag), and_or(wv >> 12, msk, mag)));
      } else {
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bb + brow_off(j) + so);
      }
    }
  };
  auto mma = [&](int s, const bf16x8 (&af)[MI], const bf16x8 (&bfr)[NJ]) {
    if constexpr (NIB) {  // (not v_dot2c_f32_bf16: ROCm 7.2 clang feeds element 0 of a bit-cast vector to every call)
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const bool mine = WN == 4 ? ((i & 1) == (wc >> 1) && s == (wc & 1)) : s == wc;
        if (mine) {
          const u32x4 a = __builtin_bit_cast(u32x4, af[i]);
          const f32x2 p2 = (unpk(a[0]) + unpk(a[1])) + (unpk(a[2]) + unpk(a[3]));
          rsp[i] += p2.x + p2.y;
        }
      }
    }
    if (!CVT || LLJ_W4Z_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = mfma_bf16(af[i], bfr[j], acc[i][j]);
    if (!CVT || LLJ_W4Z_PRIO) __builtin_amdgcn_s_setprio(0);
  };
  // convert-once int4: the chunk's codes are converted into 16-B segments 4 s + g of B row
  // 16 tile + column (W4P lane L = 16 s + column of the tile), in the bf16 image's swizzle:
  // bf16(128 + q) - (128 + z) in fp32 is q - z exactly (integral zeros), so the tile holds exact
  // integers and the scale is applied in the epilogue. LLJ_W4Z_WAVES 8: every wave converts its
  // own tile w, word pair (lane & 1) of W4P lane lane >> 1, branch-free after its MFMAs (the
  // scheduler may interleave the VALU with them); 4: waves 0-3 convert tiles 2 w, 2 w + 1 (all four
  // words of lane L = lane & 31 of tile 2 w + (lane >> 5)), before (LLJ_W4Z_AFTER 0) or after their MFMAs
  constexpr int CW = LLJ_W4Z_WAVES;
  const unsigned char* bf_lds = smem + NST * G::STAGE;
  const int ctile = CW == 8 ? w : 2 * w + (lane >> 5), cl = CW == 8 ? lane >> 1 : lane & 31, ccol = cl & 15,
            cs = cl >> 4, cg = CW == 8 ? 2 * (lane & 1) : 0;
  float zoff = 0.f;  // 128 + zero of this lane's column
  if constexpr (CVT) {
    if (CW == 8 || w < 4) zoff = DUAL ? (ctile < 4 ? p.sz : p.sz2)[n0 + 16 * (ctile & 3) + ccol].y : p.sz[n0 + 16 * ctile + ccol].y;
  }
  // CW 8, split: the codes read issued before the chunk's fragment reads (asm, no wait; LDS reads
  // complete in order, so the compiler's own lgkmcnt waits for the later fragment reads cover it, and
  // the explicit wait below ties the value to it), the conversion after them, in the MFMAs' block
  auto cread = [&](int buf) {
    const uint32_t ra = (uint32_t)(uintptr_t)(lds_void_t*)(smem + (size_t)buf * G::STAGE + G::SA + 512 * ctile + 16 * cl +
                                                           4 * cg);
    uint2 t;
    // (s_nop: the destination may be a register an MFMA of the previous chunk read as an operand)
    asm volatile("s_nop 4\n\tds_read_b64 %0, %1" : "=v"(t) : "v"(ra) : "memory");
    return t;
  };
  auto cfinish = [&](uint2 t, int slot) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(t));
    const uint32_t da = (uint32_t)(uintptr_t)(lds_void_t*)(bf_lds + (size_t)slot * BN * 128 + (16 * ctile + ccol) * 128);
#pragma unroll
    for (int g4 = 0; g4 < 2; ++g4) {
      const uint32_t wv = g4 ? t.y : t.x;
      uint32_t o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t d = and_or(wv >> (4 * e), msk, mag);  // bf16 pair (128 + q_lo, 128 + q_hi)
        // as fp32 (exact), minus 128 + z in one packed add, back to a bf16 pair in one convert (exact)
        const f32x2 v = f32x2{__uint_as_float(d << 16), __uint_as_float(d & 0xFFFF0000u)} - f32x2{zoff, zoff};
        o[e] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
      }
      const u32x4 ov = {o[0], o[1], o[2], o[3]};
      asm volatile("ds_write_b128 %0, %1" ::"v"(da + (((4 * cs + cg + g4) ^ ((ccol >> 1) & 7)) * 16)), "v"(ov) : "memory");
    }
  };
  auto convert = [&](int buf, int slot) {
    // the read in asm, with its own wait: read as a plain LDS load, hipcc waits vmcnt(0) for every
    // LDS-DMA in flight first (the next chunks' too), de-pipelining the loop
    const uint32_t ra = (uint32_t)(uintptr_t)(lds_void_t*)(smem + (size_t)buf * G::STAGE + G::SA + 512 * ctile + 16 * cl +
                                                           4 * cg);
    constexpr int NWD = CW == 8 ? 2 : 4;  // words per lane
    uint32_t wv4[NWD];
    if constexpr (CW == 8) {
      uint2 t;
      asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(t) : "v"(ra) : "memory");
      wv4[0] = t.x;
      wv4[1] = t.y;
    } else {
      u32x4 t;
      asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(t) : "v"(ra) : "memory");
      wv4[0] = t[0]; wv4[1] = t[1]; wv4[2] = t[2]; wv4[3] = t[3];
    }
    const uint32_t da = (uint32_t)(uintptr_t)(lds_void_t*)(bf_lds + (size_t)slot * BN * 128 + (16 * ctile + ccol) * 128);
#pragma unroll
    for (int g4 = 0; g4 < NWD; ++g4) {
      const uint32_t wv = wv4[g4];
      uint32_t o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t d = and_or(wv >> (4 * e), msk, mag);  // bf16 pair (128 + q_lo, 128 + q_hi)
        const float lo = __uint_as_float(d << 16) - zoff, hi = __uint_as_float(d & 0xFFFF0000u) - zoff;
        o[e] = (__float_as_uint(lo) >> 16) | (__float_as_uint(hi) & 0xFFFF0000u);  // exact: small integers
      }
      // (asm too: hipcc also waits vmcnt(0) before a plain LDS store while LDS-DMAs are in flight; the
      // loop's lgkmcnt(0) before its barrier retires it)
      const u32x4 ov = {o[0], o[1], o[2], o[3]};
      asm volatile("ds_write_b128 %0, %1" ::"v"(da + (((4 * cs + cg + g4) ^ ((ccol >> 1) & 7)) * 16)), "v"(ov) : "memory");
    }
  };
  auto compute = [&](int buf, int slot) {
    const unsigned char* Ab = smem + (size_t)buf * G::STAGE;
    const unsigned char* Bb = CVT ? bf_lds + (size_t)slot * BN * 128 : Ab + G::SA;
    if constexpr (LLJ_GLDS_PRE && BN == 128) {  // both MFMA steps' fragments read before either's MFMAs
      bf16x8 af0[MI], bf0[NJ], af1[MI], bf1[NJ];
      frags(Ab, Bb, 0, af0, bf0);
      frags(Ab, Bb, 1, af1, bf1);
      mma(0, af0, bf0);
      mma(1, af1, bf1);
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 af[MI], bfr[NJ];
        frags(Ab, Bb, s, af, bfr);
        mma(s, af, bfr);
      }
    }
  };

  // ---- K loop, fragment double buffering (LLJ_GLDS_FDB, bf16 and convert-once int4 at 256 x 128): the
  // fragments of chunk t + 1 are read from LDS while chunk t's MFMAs run (two register sets), so the DMA
  // runs three chunks ahead (every stage issued, past the end with a clamped chunk index: equal DMA
  // counts per wave in every iteration) and each iteration waits for chunk t + 1 instead of t
  if constexpr (FDB) {
    struct Fr {
      bf16x8 a0[MI], b0[NJ], a1[MI], b1[NJ];
    };
    auto rd = [&](int buf, int slot, Fr& f) {
      const unsigned char* Ab = smem + (size_t)buf * G::STAGE;
      const unsigned char* Bb = CVT ? bf_lds + (size_t)slot * BN * 128 : Ab + G::SA;
      frags(Ab, Bb, 0, f.a0, f.b0);
      frags(Ab, Bb, 1, f.a1, f.b1);
    };
    auto step = [&](int t, Fr& cur, Fr& nxt) {
      wait_vm<G::NG>();  // chunk t + 1 (and the codes of t + 2) landed; t + 2 in flight
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of chunk t's fragments (and codes) are done
      __builtin_amdgcn_s_barrier();
      const int b0 = t % 3;
      stage(b0, t + 3 < KC ? t + 3 : KC - 1);
      uint2 ct = {0u, 0u};
      if constexpr (CVT) ct = cread(b0 + 2 >= 3 ? b0 - 1 : b0 + 2);  // codes of chunk t + 2
      if (t + 1 < KC) rd(b0 + 1 == 3 ? 0 : b0 + 1, (t + 1) & 1, nxt);
      mma(0, cur.a0, cur.b0);
      mma(1, cur.a1, cur.b1);
      if constexpr (CVT) cfinish(ct, t & 1);  // chunk t + 2's tile into chunk t's slot (read in the previous iteration)
      // the MFMAs interleaved with the next chunk's fragment reads (LLJ_FDB_DSPM per MFMA) and the
      // conversion's VALU (LLJ_W4Z_VPM per MFMA)
      if constexpr ((CVT && LLJ_W4Z_IGLP) || LLJ_FDB_DSPM > 0) {
#pragma unroll
        for (int q = 0; q < 2 * MI * NJ; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if constexpr (LLJ_FDB_DSPM > 0) __builtin_amdgcn_sched_group_barrier(0x100, LLJ_FDB_DSPM, 0);
          if constexpr (CVT && LLJ_W4Z_IGLP) __builtin_amdgcn_sched_group_barrier(0x002, LLJ_W4Z_VPM, 0);
        }
      }
    };
    // prologue: chunks 0 and 1 (CVT: and chunk 0's codes, then both tiles converted) before chunk 2 is
    // staged -- chunk 2's group carries chunk 3's codes into stage buffer 0, over chunk 0's
    if constexpr (CVT) stage_codes(0, 0);
    stage(0, 0);
    stage(1, 1 < KC ? 1 : KC - 1);
    wait_vm<G::NG>();  // chunk 0 (CVT: the codes of chunks 0 and 1)
    __builtin_amdgcn_s_barrier();
    if constexpr (CVT) {
      convert(0, 0);
      convert(1, 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave's code reads done, both tiles written
    }
    stage(2, 2 < KC ? 2 : KC - 1);
    Fr F0, F1;
    rd(0, 0, F0);
    for (int t = 0; t < KC; t += 2) {
      step(t, F0, F1);
      if (t + 1 < KC) step(t + 1, F1, F0);
    }
    wait_vm<0>();  // the clamped stages past the end land before the workgroup's LDS is released
  } else {
  // ---- K loop: NST - 1 chunks staged ahead
  if constexpr (CVT) {  // chunk 0's codes first, converted before the loop
    static_assert(NST == 3, "convert-once int4: three stages");
    stage_codes(0, 0);
  }
#pragma unroll
  for (int c = 0; c < NST - 1; ++c)
    if (c < KC) stage(c, c);
  if constexpr (CVT) {
    wait_vm<2 * G::NG>();  // chunk 0's codes (KC >= 2: both groups were issued)
    __builtin_amdgcn_s_barrier();
    if (CW == 8 || w < 4) convert(0, 0);
  }
  int cb = 0;  // buffer of chunk t
  for (int tc = 0; tc < KC; ++tc) {
    if constexpr (NST == 3) {
      if (tc + 1 < KC) wait_vm<G::NG>(); else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads (and tile writes) of chunk t - 1 are done
    __builtin_amdgcn_s_barrier();  // chunk t landed for every wave (CVT: and chunk t + 1's codes); t - 1's buffers are free
    if (tc + NST - 1 < KC) stage(cb == 0 ? NST - 1 : cb - 1, tc + NST - 1);
    if constexpr (CVT && CW == 4 && !LLJ_W4Z_AFTER) {
      if (tc + 1 < KC && w < 4) convert(cb + 1 == NST ? 0 : cb + 1, (tc + 1) & 1);
    }
    if constexpr (CVT && CW == 8 && LLJ_W4Z_SPLIT) {
      const uint2 ct = cread(cb + 1 == NST ? 0 : cb + 1);
      compute(cb, tc & 1);
      cfinish(ct, (tc + 1) & 1);
      if constexpr (LLJ_W4Z_IGLP) {  // the conversion's VALU between the MFMAs: 1 MFMA, LLJ_W4Z_VPM VALU, ...
#pragma unroll
        for (int q = 0; q < 2 * MI * NJ; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, LLJ_W4Z_VPM, 0);
        }
      }
    } else {
      compute(cb, tc & 1);
    }
    if constexpr (CVT && CW == 4 && LLJ_W4Z_AFTER) {
      if (tc + 1 < KC && w < 4) convert(cb + 1 == NST ? 0 : cb + 1, (tc + 1) & 1);
    }
    // branch-free: past the last chunk it converts the clamped codes into the unused slot
    if constexpr (CVT && CW == 8 && !LLJ_W4Z_SPLIT) convert(cb + 1 == NST ? 0 : cb + 1, (tc + 1) & 1);
    cb = cb + 1 == NST ? 0 : cb + 1;
  }
  }

  // ---- epilogue: lane holds rows m0 + wr * 16 MI + 16 i + 4 g + r, column n0 + wc * 16 NJ + 16 j + row
  if constexpr (EP == GEP_QKV && LLJ_QKV_LDS && !NIB && BN == 128 && MI <= 4) if ((p.head_size & 7) == 0) {
    // QKV through LDS: the tile's bf16 c_attn outputs (model.py:204) go to LDS in the accumulator layout,
    // then every thread takes 8 consecutive columns (4 RoPE pairs: no lane exchange) of one row and
    // stores them as one 16-byte vector -- a tile row is 256 contiguous bytes of q, or of one K / V cache
    // row (the head dimension), instead of 4-byte pairs from every other lane
    constexpr int TP = BN + 8;  // row pitch (elements): 16-B aligned rows on shifted banks
    bf16_t* Ts = reinterpret_cast<bf16_t*>(smem);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();  // every wave is past its last fragment read of the K loop
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int nl = wc * 16 * NJ + 16 * j + row;
      const float sc = CVT ? p.sz[n0 + nl].x : 1.f;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) Ts[(wr * 16 * MI + 16 * i + 4 * g + r) * TP + nl] = f2bf(sc * acc[i][j][r]);
    }
    __syncthreads();
    const int Cd = p.n_head * p.head_size, seg = tid & 15;
    const int nc0 = n0 + 8 * seg, region = nc0 / Cd, nc = nc0 - region * Cd;
    const int h = nc / p.head_size, dd = nc - h * p.head_size;  // 8 | head_size: the 8 columns share a head
#pragma unroll 2
    for (int k = 0; k < 8; ++k) {
      const int rl = (tid >> 4) + 32 * k, m = m0 + rl;
      if (m >= M) continue;
      const uint4 v = *reinterpret_cast<const uint4*>(Ts + rl * TP + 8 * seg);
      const QkvRow qr = qkv_row(p, m);
      uint4 o = v;
      if (region < 2) {
        const float4* rp = reinterpret_cast<const float4*>(p.rope + ((size_t)qr.ps * (p.head_size >> 1) + (dd >> 1)) * 2);
        const float4 c01 = rp[0], c23 = rp[1];  // (cos, sin) of pairs dd / 2 .. + 3
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        const float cs[8] = {c01.x, c01.y, c01.z, c01.w, c23.x, c23.y, c23.z, c23.w};
        uint32_t ow[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float e0 = bflo(w[q]), e1 = bfhi(w[q]), c = cs[2 * q], sn = cs[2 * q + 1];
          ow[q] = pack2bf(e0 * c - e1 * sn, e1 * c + e0 * sn);
        }
        o = make_uint4(ow[0], ow[1], ow[2], ow[3]);
      }
      bf16_t* dst = region == 0 ? p.q_out + (size_t)m * Cd + nc
                                : (region == 1 ? p.kcache : p.vcache) + (size_t)qr.kvrow + (size_t)h * p.S * p.head_size + dd;
      *reinterpret_cast<uint4*>(dst) = o;
    }
    return;
  }
  if constexpr (LLJ_GLDS_LDS_EPI && !NIB && !PART && BN == 128 && MI <= 4 &&
                (EP == GEP_STORE || EP == GEP_RESID || EP == GEP_SILU_MUL || EP == GEP_SWIGLU))
    if ((p.ldc & 7) == 0 && (reinterpret_cast<uintptr_t>(p.C) & 15) == 0) {
      // the other bf16 epilogues through LDS as well: the tile's bf16 values (y, or the whole SwiGLU product) to
      // LDS in the accumulator layout, then 16-byte row segments (8 columns) per thread, the residual / c_fc1
      // operand read the same way -- rows of 256 (SwiGLU: 128) contiguous bytes instead of 4-byte pairs
      constexpr int TW = DUAL ? BN / 2 : BN, TP = TW + 8, SEGS = TW / 8, RPP = 512 / SEGS;
      bf16_t* Ts = reinterpret_cast<bf16_t*>(smem);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __syncthreads();  // every wave is past its last fragment read of the K loop
#pragma unroll
      for (int j = 0; j < (DUAL ? NJ / 2 : NJ); ++j) {
        const int nl = wc * 16 * (DUAL ? NJ / 2 : NJ) + 16 * j + row;
        const float s1 = CVT ? p.sz[n0 + nl].x : 1.f;
        float s2 = 1.f;
        if constexpr (DUAL) s2 = p.sz2[n0 + nl].x;
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float o;
            if constexpr (DUAL) {  // h = bf16(silu(bf16(fc1))) * bf16(fc2)
              const float a1 = round_bf(s1 * acc[i][j][r]);
              const float sl = round_bf(a1 / (1.f + __expf(-a1)));
              o = sl * round_bf(s2 * acc[i][j + NJ / 2][r]);
            } else {
              o = s1 * acc[i][j][r];
            }
            Ts[(wr * 16 * MI + 16 * i + 4 * g + r) * TP + nl] = f2bf(o);
          }
      }
      __syncthreads();
      const int seg = tid % SEGS;
#pragma unroll 2
      for (int k = 0; k < 256 / RPP; ++k) {
        const int rl = tid / SEGS + RPP * k, m = m0 + rl;
        if (m >= M) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(Ts + rl * TP + 8 * seg);
        uint4* cp = reinterpret_cast<uint4*>(p.C + (size_t)m * p.ldc + n0 + 8 * seg);
        uint4 o = v;
        if constexpr (EP == GEP_RESID || EP == GEP_SILU_MUL) {
          const uint4 c = *cp;
          const uint32_t vw[4] = {v.x, v.y, v.z, v.w}, cw[4] = {c.x, c.y, c.z, c.w};
          uint32_t ow[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float y0 = bflo(vw[q]), y1 = bfhi(vw[q]), c0 = bflo(cw[q]), c1 = bfhi(cw[q]);
            if constexpr (EP == GEP_RESID) {
              ow[q] = pack2bf(c0 + y0, c1 + y1);  // x + y in bf16 (model.py:172-173)
            } else {
              const float l0 = round_bf(c0 / (1.f + __expf(-c0))), l1 = round_bf(c1 / (1.f + __expf(-c1)));
              ow[q] = pack2bf(l0 * y0, l1 * y1);  // silu(bf16(c_fc1 x)) * bf16(c_fc2 x)
            }
          }
          o = make_uint4(ow[0], ow[1], ow[2], ow[3]);
        }
        *cp = o;
      }
      return;
    }
  if constexpr (PART && DUAL) {  // the slice's c_fc1 / c_fc2 fp32 partials, scales applied, two planes
    float* wsl = p.ws + (size_t)split * 2 * M * p.N;
#pragma unroll
    for (int j = 0; j < NJ / 2; ++j) {
      const int n = n0 + wc * 16 * (NJ / 2) + 16 * j + row;
      const float s1 = p.sz[n].x, s2 = p.sz2[n].x;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wr * 16 * MI + 16 * i + 4 * g + r;
          if (m < M) {
            wsl[(size_t)m * p.N + n] = s1 * acc[i][j][r];
            wsl[(size_t)(M + m) * p.N + n] = s2 * acc[i][j + NJ / 2][r];
          }
        }
    }
    return;
  }
  if constexpr (PART) {  // the slice's fp32 partials, scale applied (summed over the slices by the reduce)
    float* wsl = p.ws + (size_t)split * M * p.N;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wc * 16 * NJ + 16 * j + row;
      const float sc = CVT ? p.sz[n].x : 1.f;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wr * 16 * MI + 16 * i + 4 * g + r;
          if (m < M) wsl[(size_t)m * p.N + n] = sc * acc[i][j][r];
        }
    }
    return;
  }
  if constexpr (DUAL) {  // h = bf16(silu(bf16(fc1))) * bf16(fc2), fc1 in fragments j < NJ / 2, fc2 at j + NJ / 2
#pragma unroll
    for (int j = 0; j < NJ / 2; ++j) {
      const int n = n0 + wc * 16 * (NJ / 2) + 16 * j + row;
      const float s1 = p.sz[n].x, s2 = p.sz2[n].x;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wr * 16 * MI + 16 * i + 4 * g + r;
          const float a1 = round_bf(s1 * acc[i][j][r]);  // bf16(c_fc1 x)
          const float sl = round_bf(a1 / (1.f + __expf(-a1)));  // F.silu in bf16
          const uint32_t ob = (uint32_t)f2bf(sl * round_bf(s2 * acc[i][j + NJ / 2][r]));
          const uint32_t pr = lane_xor1(ob);
          if (m < M && !(row & 1)) *reinterpret_cast<uint32_t*>(p.C + (size_t)m * p.ldc + n) = ob | (pr << 16);
        }
    }
    return;
  }
  if constexpr (NIB) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {  // two waves hold parts of each row: 0 + a + b is order-free
      if (WN == 4 && (i & 1) != (wc >> 1)) continue;
      float v = rsp[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (g == 0) atomicAdd(rs_lds + wr * 16 * MI + 16 * i + row, v);
    }
    __syncthreads();
  }
  const int Cd = p.n_head * p.head_size;
  // QKV rows' (position, cache offset) once per tile where registers allow (MI <= 4; the 256 x 256
  // tile recomputes them per row group)
  constexpr bool QH = EP == GEP_QKV && MI <= 4;
  QkvRow qrow[QH ? MI : 1][4] = {};
  if constexpr (QH) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) qrow[i][r] = qkv_row(p, m0 + wr * 16 * MI + 16 * i + 4 * g + r);
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int nblk = n0 + wc * 16 * NJ + 16 * j;
    const int n = nblk + row;
    float2 szn = make_float2(1.f, 0.f);
    if constexpr (NIB || CVT) szn = p.sz[n];
    const QkvCol qc = EP == GEP_QKV ? qkv_col(p, nblk, n, Cd) : QkvCol{};
    constexpr int GI = EP == GEP_QKV ? (MI > 4 ? 1 : LLJ_QKV_GI) : 4;  // row blocks whose operands are in flight together
#pragma unroll
    for (int i0 = 0; i0 < MI; i0 += GI) {
      float2 opv[GI][4];
      QkvRow qg[GI][4] = {};
#pragma unroll
      for (int i = 0; i < GI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wr * 16 * MI + 16 * (i0 + i) + 4 * g + r;
          if constexpr (QH) qg[i][r] = qrow[i0 + i][r];
          else if constexpr (EP == GEP_QKV) qg[i][r] = qkv_row(p, m);
          opv[i][r] = gemm_operand<EP>(p, m, n, qg[i][r], qc);
        }
#pragma unroll
      for (int i = 0; i < GI; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ml = wr * 16 * MI + 16 * (i0 + i) + 4 * g + r;
          const int m = m0 + ml;
          float y = acc[i0 + i][j][r];
          if constexpr (NIB) y = szn.x * (y - szn.y * rs_lds[ml]);
          if constexpr (CVT) y = szn.x * y;
          gemm_store_elem<EP>(p, y, m, n, m < M, row, Cd, opv[i][r], qg[i][r], qc);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the next group's operand loads out of this one's live range
    }
  }
}

template <int WF, int EP, int BN>
static int gemm_glds_launch(const GemmParams& p, hipStream_t s) {
  auto kern = gemm_glds_kernel<WF, EP, BN>;
  static bool attr_set = false;  // per instantiation, before any graph capture
  const size_t lds = GldsGeo<WF, BN>::LDS;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  constexpr bool DUAL = EP == GEP_SWIGLU || EP == GEP_SWIGLU_PART;
  const int tiles = ((p.M + 255) / 256) * (p.N / (DUAL ? BN / 2 : BN)) *
                    (EP == GEP_PARTIAL || EP == GEP_SWIGLU_PART ? p.nsplit : 1);
  hipLaunchKernelGGL(kern, dim3(tiles), dim3(512), lds, s, p);
  LLJ_CHECK_LAUNCH();
  return 0;
}

// option LLJ_OPT_GEMM_GLDS (llj_set_option / LLJ_GEMM_GLDS) 1 / 0: the LDS-DMA / the register-staged
// kernels for every format (A/B in one process); unset: the per-format default
static bool glds_enabled(int wf) {
  const int o = opt(LLJ_OPT_GEMM_GLDS);
  if (o >= 0) return o != 0;
  return wf == GWF_BF16 ? LLJ_GEMM_GLDS_BF16 != 0 : LLJ_GEMM_GLDS_W4 != 0;
}

// 256 x 256 or 256 x 128 tiles: the shape with the fewer tile-time units over the CUs (waves of
// tiles rounded up, a 256 x 128 tile costing LLJ_GLDS_COST128 % of a 256 x 256 one)
template <int WF, int EP>
static int gemm_glds_run(const GemmParams& p, hipStream_t s) {
  int cus = 256;
  {
    static int cached = 0;
    if (!cached) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cached, hipDeviceAttributeMultiprocessorCount, dev);
      if (cached <= 0) cached = 256;
    }
    cus = cached;
  }
  const long mt = (p.M + 255) / 256;
  const long w256 = p.N % 256 == 0 ? (mt * (p.N / 256) + cus - 1) / cus : -1;
  const long w128 = (mt * (p.N / 128) + cus - 1) / cus;
  const int oc = opt(LLJ_OPT_GLDS_COST128);  // A/B and tests: 0 forces 256 x 128, >= 100 prefers 256 x 256
  const long cost = oc >= 0 ? oc : LLJ_GLDS_COST128;
  if (w256 > 0 && 100 * w256 <= cost * w128) return gemm_glds_launch<WF, EP, 256>(p, s);
  return gemm_glds_launch<WF, EP, 128>(p, s);
}

// split-K residual GEMM (few row tiles: a prompt of 256..1024 rows leaves the 4096-column GEMMs at
// 64..128 workgroups): x = bf16(x + bf16(sum over the slices of their fp32 partials)), slices in order
__global__ __launch_bounds__(256) void gemm_splitk_reduce_kernel(const float* __restrict__ ws, int nsplit, int M, int N,
                                                                 bf16_t* __restrict__ x, int ldx) {
  const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4;  // 4 consecutive columns (N % 4 == 0)
  if (i >= (size_t)M * N) return;
  const int m = (int)(i / N), n = (int)(i % N);
  float4 y = *reinterpret_cast<const float4*>(ws + i);
  for (int sp = 1; sp < nsplit; ++sp) {
    const float4 v = *reinterpret_cast<const float4*>(ws + (size_t)sp * M * N + i);
    y.x += v.x; y.y += v.y; y.z += v.z; y.w += v.w;
  }
  uint2* xp = reinterpret_cast<uint2*>(x + (size_t)m * ldx + n);
  const uint2 xv = *xp;
  const uint32_t lo = pack2bf(round_bf(bflo(xv.x) + round_bf(y.x)), round_bf(bfhi(xv.x) + round_bf(y.y)));
  const uint32_t hi = pack2bf(round_bf(bflo(xv.y) + round_bf(y.z)), round_bf(bfhi(xv.y) + round_bf(y.w)));
  *xp = make_uint2(lo, hi);
}

// K slices for a residual GEMM on the LDS-DMA kernels (0: none): when the row tiles x 128-column tiles
// fill at most half the CUs, up to 8 slices of >= 8 64-deep chunks (an even count each)
static int splitk_plan(int wfmt, int M, int N, int K, int* kcs_out);

// option LLJ_OPT_GEMM_W4Z (LLJ_GEMM_W4Z) 1 / 0: int4 with integral zeros (LLJ_WF_ZINT) in the
// convert-once LDS-DMA kernel / in the int4 default kernel
#ifndef LLJ_GEMM_W4Z
#define LLJ_GEMM_W4Z 1
#endif
#ifndef LLJ_GEMM_SPLITK
#define LLJ_GEMM_SPLITK 1  // split-K residual GEMMs for few row tiles (llj_gemm_resid_ws)
#endif
static bool w4z_enabled() {
  const int o = opt(LLJ_OPT_GEMM_W4Z);
  return o >= 0 ? o != 0 : LLJ_GEMM_W4Z != 0;
}

static int splitk_plan(int wfmt, int M, int N, int K, int* kcs_out) {
  const bool w4z = wfmt == (GWF_W4 | LLJ_WF_ZINT) && w4z_enabled();
  const bool bf = wfmt == GWF_BF16 && glds_enabled(GWF_BF16);
  if ((!w4z && !bf) || M < 256 || N % 128 || K % 128 || K < 1024 || !LLJ_GEMM_SPLITK) return 0;
  int cus = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const long tiles = (long)((M + 255) / 256) * (N / 128);
  if (2 * tiles > cus) return 0;
  const int KC = K / 64;
  int ns = (int)(cus / tiles);
  ns = ns > 8 ? 8 : ns;
  ns = ns > KC / 8 ? KC / 8 : ns;
  if (ns < 2) return 0;
  int kcs = (KC + ns - 1) / ns;
  kcs += kcs & 1;
  ns = (KC + kcs - 1) / kcs;
  if (kcs_out) *kcs_out = kcs;
  return ns < 2 ? 0 : ns;
}

template <int EP>
static int gemm_run(int wfmt, GemmParams& p, void* stream) {
  const bool zint = (wfmt & LLJ_WF_ZINT) != 0;  // int4 only: every zero is an integer
  wfmt &= ~LLJ_WF_ZINT;
  if (zint && wfmt != GWF_W4) return LLJ_EINVAL;
  if (p.M < 1 || p.N % kGBN || p.K % kGBK || p.K < kGBK || (p.lda & 7)) return LLJ_EINVAL;
  if (EP != GEP_QKV && (!p.C || (p.ldc & 1))) return LLJ_EINVAL;
  // the int4 / bf16 kernels assume an even count of 64-deep chunks (gemm_body's __builtin_assume)
  if ((wfmt == GWF_W4 || wfmt == GWF_BF16) && p.K % 128) return LLJ_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (wfmt == GWF_W4) {
    if (!p.sz) return LLJ_EINVAL;
    if (zint && p.M >= 256 && w4z_enabled()) return gemm_glds_launch<GWF_W4Z, EP, 128>(p, s);
    if (p.M >= 256 && p.K % 128 == 0 && glds_enabled(GWF_W4)) return gemm_glds_run<GWF_W4, EP>(p, s);
    if (LLJ_GEMM_BM256_W4 && p.M >= 256) return gemm_launch<GWF_W4, EP, 256>(p, s);
    return gemm_launch<GWF_W4, EP>(p, s);
  }
  if (wfmt == GWF_W8) return p.sz ? gemm_launch<GWF_W8, EP>(p, s) : LLJ_EINVAL;
  if ((wfmt & 0xff) == GWF_W4G) {  // grouped int4: group size (128-deep chunks) in the bits above
    p.gch = wfmt >> 8;
    return (p.sz && p.gch >= 1 && p.K % 128 == 0) ? gemm_launch<GWF_W4G, EP>(p, s) : LLJ_EINVAL;
  }
  if (wfmt == GWF_BF16) {
    if (p.M >= 256 && glds_enabled(GWF_BF16)) return gemm_glds_run<GWF_BF16, EP>(p, s);
    if (LLJ_GEMM_BM256 && p.M >= 256) return gemm_launch<GWF_BF16, EP, 256>(p, s);
    return gemm_launch<GWF_BF16, EP>(p, s);
  }
  if (wfmt == GWF_I8) {
    if (!p.sz || !p.i8ws || p.K % 128) return LLJ_EINVAL;
    if (!p.ao16 != !p.w16 || (p.ao16 && (p.kpad < 64 || p.kpad % 64))) return LLJ_EINVAL;
    if (LLJ_GEMM_BM256_I8 && p.M >= 256) return gemm_launch<GWF_I8, EP, 256>(p, s);
    return gemm_launch<GWF_I8, EP>(p, s);
  }
  return LLJ_EINVAL;
}

}  // namespace llj

using namespace llj;

extern "C" {

int llj_gemm_linear(int wfmt, const void* A, int lda, const void* W, const void* sz, void* C, int ldc, int M, int N,
                    int K, void* stream) {
  GemmParams p{};
  p.A = (const bf16_t*)A; p.lda = lda; p.M = M; p.N = N; p.K = K; p.W = W; p.sz = (const float2*)sz;
  p.C = (bf16_t*)C; p.ldc = ldc;
  return gemm_run<GEP_STORE>(wfmt, p, stream);
}

int llj_gemm_resid(int wfmt, const void* A, int lda, const void* W, const void* sz, void* x, int ldx, int M, int N,
                   int K, void* stream) {
  GemmParams p{};
  p.A = (const bf16_t*)A; p.lda = lda; p.M = M; p.N = N; p.K = K; p.W = W; p.sz = (const float2*)sz;
  p.C = (bf16_t*)x; p.ldc = ldx;
  return gemm_run<GEP_RESID>(wfmt, p, stream);
}

int llj_gemm_silu_mul(int wfmt, const void* A, int lda, const void* W, const void* sz, void* h, int ldh, int M, int N,
                      int K, void* stream) {
  GemmParams p{};
  p.A = (const bf16_t*)A; p.lda = lda; p.M = M; p.N = N; p.K = K; p.W = W; p.sz = (const float2*)sz;
  p.C = (bf16_t*)h; p.ldc = ldh;
  return gemm_run<GEP_SILU_MUL>(wfmt, p, stream);
}

// Workspace bytes llj_gemm_resid_ws needs for this residual GEMM (0: it would not split K -- call
// llj_gemm_resid).
size_t llj_gemm_resid_ws_bytes(int wfmt, int M, int N, int K) {
  int kcs = 0;
  const int ns = splitk_plan(wfmt, M, N, K, &kcs);
  return ns ? (size_t)ns * M * N * sizeof(float) : 0;
}

// llj_gemm_resid with the K range split over workgroups (few row tiles): fp32 partials into ws
// (llj_gemm_resid_ws_bytes), then one reduce launch adds them in slice order and the residual.
int llj_gemm_resid_ws(int wfmt, const void* A, int lda, const void* W, const void* sz, void* x, int ldx, int M, int N,
                      int K, void* ws, size_t ws_bytes, void* stream) {
  int kcs = 0;
  const int ns = splitk_plan(wfmt, M, N, K, &kcs);
  if (!ns) return llj_gemm_resid(wfmt, A, lda, W, sz, x, ldx, M, N, K, stream);
  if (!ws || ws_bytes < (size_t)ns * M * N * sizeof(float) || (lda & 7) || (ldx & 3) || !A || !W || !x) return LLJ_EINVAL;
  if ((wfmt & ~LLJ_WF_ZINT) == GWF_W4 && !sz) return LLJ_EINVAL;
  GemmParams p{};
  p.A = (const bf16_t*)A; p.lda = lda; p.M = M; p.N = N; p.K = K; p.W = W; p.sz = (const float2*)sz;
  p.ws = (float*)ws; p.nsplit = ns; p.kcs = kcs;
  hipStream_t s = (hipStream_t)stream;
  const int rc = wfmt == GWF_BF16 ? gemm_glds_launch<GWF_BF16, GEP_PARTIAL, 128>(p, s)
                                  : gemm_glds_launch<GWF_W4Z, GEP_PARTIAL, 128>(p, s);
  if (rc) return rc;
  const size_t n4 = (size_t)M * N / 4;
  hipLaunchKernelGGL(gemm_splitk_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, (const float*)ws, ns,
                     M, N, (bf16_t*)x, ldx);
  LLJ_CHECK_LAUNCH();
  return 0;
}

// the dual SwiGLU pass's tail: h[m, n] = bf16(silu(bf16(a))) * bf16(b), a / b the c_fc1 / c_fc2 partials of the
// slices summed in slice order (4 consecutive columns per thread, N % 4 == 0)
__global__ __launch_bounds__(256) void gemm_swiglu_reduce_kernel(const float* __restrict__ ws, int nsplit, int M, int N,
                                                                 bf16_t* __restrict__ h, int ldh) {
  const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const size_t MN = (size_t)M * N;
  if (i >= MN) return;
  const int m = (int)(i / N), n = (int)(i % N);
  float4 a = *reinterpret_cast<const float4*>(ws + i), b = *reinterpret_cast<const float4*>(ws + MN + i);
  for (int sp = 1; sp < nsplit; ++sp) {
    const float4 u = *reinterpret_cast<const float4*>(ws + 2 * sp * MN + i);
    const float4 v = *reinterpret_cast<const float4*>(ws + (2 * sp + 1) * MN + i);
    a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
    b.x += v.x; b.y += v.y; b.z += v.z; b.w += v.w;
  }
  const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
  float o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float a1 = round_bf(av[q]);
    const float sl = round_bf(a1 / (1.f + __expf(-a1)));  // F.silu in bf16
    o[q] = sl * round_bf(bv[q]);
  }
  *reinterpret_cast<uint2*>(h + (size_t)m * ldh + n) = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
}

#ifndef LLJ_GEMM_SWIGLU_TAIL
#define LLJ_GEMM_SWIGLU_TAIL 1  // the dual SwiGLU pass's partial last wave of tiles as split-K halves
#endif
// The dual SwiGLU pass over (row tiles) x (H / 64 column tiles): when the tiles leave a partial last wave
// over the CUs, its column tiles (tc of them, at the right end) run as two K halves -- twice the
// workgroups at half the length, fitting one wave -- and the full-K launch keeps only whole waves.
// Returns the tail's column tiles (0: no split), kcs = its 64-deep chunks per half.
static int swiglu_tail_plan(int M, int H, int K, int* kcs_out) {
  if (!LLJ_GEMM_SWIGLU_TAIL || M < 256 || H % 64 || K % 128 || K / 64 < 16) return 0;
  int cus = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const long mt = (M + 255) / 256, ntn = H / 64, tiles = mt * ntn;
  const long full = tiles / cus * cus;
  if (full == tiles || full == 0) return 0;
  const long tc = ntn - full / mt;  // the full-K launch keeps (ntn - tc) column tiles: at most the whole waves
  if (tc <= 0 || tc >= ntn || 2 * mt * tc > cus) return 0;
  int kcs = (K / 64 + 1) / 2;
  kcs += kcs & 1;
  if (kcs_out) *kcs_out = kcs;
  return (int)tc;
}

// h[M, H] = bf16(silu(bf16(A . W1^T))) * bf16(A . W2^T) in one pass: int4 W4P with integral zeros
// (wfmt 0 | LLJ_WF_ZINT), M >= 256, H % 64 == 0 (the convert-once kernel with both weights' codes per chunk)
int llj_gemm_swiglu(int wfmt, const void* A, int lda, const void* W1, const void* sz1, const void* W2, const void* sz2,
                    void* h, int ldh, int M, int H, int K, void* stream) {
  if (wfmt != (GWF_W4 | LLJ_WF_ZINT) || M < 256 || H % 64 || K % 128 || K < 128 || (lda & 7) || (ldh & 1) || !A ||
      !W1 || !W2 || !sz1 || !sz2 || !h)
    return LLJ_EINVAL;
  GemmParams p{};
  p.A = (const bf16_t*)A; p.lda = lda; p.M = M; p.N = H; p.K = K; p.W = W1; p.sz = (const float2*)sz1;
  p.W2 = W2; p.sz2 = (const float2*)sz2; p.C = (bf16_t*)h; p.ldc = ldh;
  return gemm_glds_launch<GWF_W4Z, GEP_SWIGLU, 128>(p, (hipStream_t)stream);
}

// Workspace bytes llj_gemm_swiglu_ws needs (0: no partial last wave to split -- call llj_gemm_swiglu).
size_t llj_gemm_swiglu_ws_bytes(int wfmt, int M, int H, int K) {
  if (wfmt != (GWF_W4 | LLJ_WF_ZINT) || !w4z_enabled()) return 0;
  int kcs = 0;
  const int tc = swiglu_tail_plan(M, H, K, &kcs);
  return tc ? (size_t)2 * 2 * M * (64 * tc) * sizeof(float) : 0;
}

// llj_gemm_swiglu with the partial last wave of column tiles split into two K halves (fp32 partials of both
// weights into ws, llj_gemm_swiglu_ws_bytes), one reduce launch finishing those columns of h
int llj_gemm_swiglu_ws(int wfmt, const void* A, int lda, const void* W1, const void* sz1, const void* W2, const void* sz2,
                       void* h, int ldh, int M, int H, int K, void* ws, size_t ws_bytes, void* stream) {
  int kcs = 0;
  const int tc = (wfmt == (GWF_W4 | LLJ_WF_ZINT) && w4z_enabled()) ? swiglu_tail_plan(M, H, K, &kcs) : 0;
  if (!tc) return llj_gemm_swiglu(wfmt, A, lda, W1, sz1, W2, sz2, h, ldh, M, H, K, stream);
  const int Ht = 64 * tc, Hc = H - Ht;
  if ((lda & 7) || (ldh & 3) || !A || !W1 || !W2 || !sz1 || !sz2 || !h || !ws ||
      ws_bytes < (size_t)2 * 2 * M * Ht * sizeof(float))
    return LLJ_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  int rc = llj_gemm_swiglu(wfmt, A, lda, W1, sz1, W2, sz2, h, ldh, M, Hc, K, stream);  // whole waves, full K
  if (rc) return rc;
  GemmParams p{};  // the tail's columns Hc .. H - 1: W4P column tiles are K-contiguous, so pointer offsets
  const size_t woff = (size_t)Hc * K / 2;
  p.A = (const bf16_t*)A; p.lda = lda; p.M = M; p.N = Ht; p.K = K;
  p.W = (const char*)W1 + woff; p.sz = (const float2*)sz1 + Hc;
  p.W2 = (const char*)W2 + woff; p.sz2 = (const float2*)sz2 + Hc;
  p.ws = (float*)ws; p.nsplit = 2; p.kcs = kcs;
  rc = gemm_glds_launch<GWF_W4Z, GEP_SWIGLU_PART, 128>(p, s);
  if (rc) return rc;
  const size_t n4 = (size_t)M * Ht / 4;
  hipLaunchKernelGGL(gemm_swiglu_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, (const float*)ws, 2, M,
                     Ht, (bf16_t*)h + Hc, ldh);
  LLJ_CHECK_LAUNCH();
  return 0;
}

// LLM.int8() forms (wfmt 2): W = CB in the I8P tiling, sz = SCB (fp32), i8ws = llj_i8_stats of A
int llj_gemm_i8_linear(const void* A, int lda, const void* CB, const void* SCB, const void* i8ws, const void* ao16,
                       const void* w16, int kpad, void* C, int ldc, int M, int N, int K, void* stream) {
  GemmParams p{};
  p.ao16 = (const _Float16*)ao16; p.w16 = (const _Float16*)w16; p.kpad = kpad;
  p.A = (const bf16_t*)A; p.lda = lda; p.M = M; p.N = N; p.K = K; p.W = CB; p.sz = (const float2*)SCB;
  p.C = (bf16_t*)C; p.ldc = ldc; p.i8ws = (const char*)i8ws;
  return gemm_run<GEP_STORE>(GWF_I8, p, stream);
}

int llj_gemm_i8_resid(const void* A, int lda, const void* CB, const void* SCB, const void* i8ws, const void* ao16,
                      const void* w16, int kpad, void* x, int ldx, int M, int N, int K, void* stream) {
  GemmParams p{};
  p.ao16 = (const _Float16*)ao16; p.w16 = (const _Float16*)w16; p.kpad = kpad;
  p.A = (const bf16_t*)A; p.lda = lda; p.M = M; p.N = N; p.K = K; p.W = CB; p.sz = (const float2*)SCB;
  p.C = (bf16_t*)x; p.ldc = ldx; p.i8ws = (const char*)i8ws;
  return gemm_run<GEP_RESID>(GWF_I8, p, stream);
}

int llj_gemm_i8_silu_mul(const void* A, int lda, const void* CB, const void* SCB, const void* i8ws, const void* ao16,
                         const void* w16, int kpad, void* h, int ldh, int M, int N, int K, void* stream) {
  GemmParams p{};
  p.ao16 = (const _Float16*)ao16; p.w16 = (const _Float16*)w16; p.kpad = kpad;
  p.A = (const bf16_t*)A; p.lda = lda; p.M = M; p.N = N; p.K = K; p.W = CB; p.sz = (const float2*)SCB;
  p.C = (bf16_t*)h; p.ldc = ldh; p.i8ws = (const char*)i8ws;
  return gemm_run<GEP_SILU_MUL>(GWF_I8, p, stream);
}

int llj_gemm_i8_qkv_rope(const void* x, const void* CB, const void* SCB, const void* i8ws, const void* ao16,
                         const void* w16, int kpad, void* q_out, void* kcache, void* vcache, const float* rope,
                         const int* pos, int B, int T, int C, int n_head, int S, void* stream) {
  if (B < 1 || T < 1 || n_head < 1 || C % n_head || S < 1 || !pos || !rope) return LLJ_EINVAL;
  GemmParams p{};
  p.ao16 = (const _Float16*)ao16; p.w16 = (const _Float16*)w16; p.kpad = kpad;
  p.A = (const bf16_t*)x; p.lda = C; p.M = B * T; p.N = 3 * C; p.K = C; p.W = CB; p.sz = (const float2*)SCB;
  p.q_out = (bf16_t*)q_out; p.kcache = (bf16_t*)kcache; p.vcache = (bf16_t*)vcache; p.rope = rope; p.pos = pos;
  p.n_head = n_head; p.head_size = C / n_head; p.S = S; p.T = T; p.i8ws = (const char*)i8ws;
  if (p.head_size & 1 || C % 16) return LLJ_EINVAL;
  return gemm_run<GEP_QKV>(GWF_I8, p, stream);
}

int llj_gemm_qkv_rope(int wfmt, const void* x, const void* W, const void* sz, void* q_out, void* kcache, void* vcache,
                      const float* rope, const int* pos, int B, int T, int C, int n_head, int S, void* stream) {
  if (B < 1 || T < 1 || n_head < 1 || C % n_head || S < 1 || !pos || !rope) return LLJ_EINVAL;
  GemmParams p{};
  p.A = (const bf16_t*)x; p.lda = C; p.M = B * T; p.N = 3 * C; p.K = C; p.W = W; p.sz = (const float2*)sz;
  p.q_out = (bf16_t*)q_out; p.kcache = (bf16_t*)kcache; p.vcache = (bf16_t*)vcache; p.rope = rope; p.pos = pos;
  p.n_head = n_head; p.head_size = C / n_head; p.S = S; p.T = T;
  if (p.head_size & 1 || C % 16) return LLJ_EINVAL;
  return gemm_run<GEP_QKV>(wfmt, p, stream);
}

}  // extern "C"

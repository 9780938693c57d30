// Causal attention of a whole prompt / perplexity window (T query rows per sequence) on the
// MFMA units: the prefill / no-cache path of reference model.py:237 (F.scaled_dot_product_attention
// with the tril mask rows of positions p0 .. p0 + T - 1, model.py:101-104), flash-style (online
// softmax over 64-key tiles, nothing of size T x T is materialized).
//
// One 256-thread workgroup per (64-query block, head, sequence); wave w owns queries
// 16w .. 16w + 15 of the block. Everything is computed transposed so that no operand needs a
// register transpose: S^T = K . Q^T (MFMA 16x16x32 bf16; A = K rows from LDS, B = the wave's Q
// fragments held in registers for the whole walk), so a lane's accumulator column is its query
// and the softmax statistics are per-lane; P^T goes straight from the S^T accumulators into the
// B operand of O^T = V^T . P^T (the 32-key MFMA step's k order is chosen as
// key = 4 g + (j & 3) + 16 (j >> 2) in each of its two 16-key halves, which is exactly what lane
// group g holds). V is staged row-major like K (16-B stores) and its V^T fragments are read with
// gfx950's transposing LDS read (ds_read_b64_tr_b16: 4 keys x 16 head dims per 16-lane group,
// delivered column-major); staging V^T with 2-byte scattered stores cost 8-way bank conflicts
// and 32 LDS writes per thread per tile (7B T = 2048: 357 us per layer). Keys are the cache slots
// 0 .. p of a query at position p (no ring wrap: p0 + T <= S, checked by the caller), masked on
// the diagonal tile.
#include <cstdlib>

#include "common.h"
#include "lit_llama_amd.h"

namespace llj {

constexpr int kFK = 64;   // keys per tile
typedef short s16x4 __attribute__((ext_vector_type(4)));

#ifndef LLJ_FLASH_OCC
#define LLJ_FLASH_OCC 3  // workgroups per CU the QB = 1 register budget is sized for (152 VGPRs, no spill; 2: 7B T=2048 window 40.0 vs 39.5 ms)
#endif
#ifndef LLJ_FLASH_PAIR
#define LLJ_FLASH_PAIR 1  // causal balance: one workgroup per (long, short) pair of query blocks (7B window -1.0 ms)
#endif
#ifndef LLJ_FLASH_FAST
#define LLJ_FLASH_FAST 1  // softmax: mask only the diagonal tiles, raw-score max, v_exp_f32, rescale only when a max moved
#endif
#ifndef LLJ_FLASH_NWQ
#define LLJ_FLASH_NWQ 4  // waves per workgroup (16 queries each) of the head-size-128 one-block form (8: 128 queries share a K / V tile)
#endif
#ifndef LLJ_FLASH_PF
#define LLJ_FLASH_PF 1  // K / V tiles in flight in registers (2: two register sets; 7B window 32.03-32.06 ms at 1 vs 32.13-32.31 at 2)
#endif
#ifndef LLJ_FLASH_QB2_MIN_T
#define LLJ_FLASH_QB2_MIN_T 2048
#endif
#ifndef LLJ_FLASH_QB
#define LLJ_FLASH_QB 1  // 16-query blocks per wave (2: every K / V fragment read feeds two MFMAs; with the pairing 1 is faster)
#endif
// QB 16-query blocks per wave: 64 QB queries per workgroup; a K fragment (S^T) and a V^T fragment
// (O^T) read from LDS feed QB MFMAs, and the tile's staging and barriers are shared by 4 x 16 QB queries
template <int HS, int QB, bool PAIR, int NWQ = 4>
__global__ __launch_bounds__(64 * NWQ, NWQ == 8 ? 1 : QB == 1 && LLJ_FLASH_PF == 1 ? LLJ_FLASH_OCC : 2) void flash_prefill_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc,
                                                            const bf16_t* __restrict__ vc, bf16_t* __restrict__ y,
                                                            const int* __restrict__ pos, int T, int S, int nh,
                                                            float sl2) {
  constexpr int KP = HS + 8;   // K tile pitch (elements): 16-B row reads
  constexpr int VP = HS + 16;  // V tile pitch: 8 rows x 4 lanes x 8 B of a transposed read on distinct banks
  constexpr int KS = HS / 32;  // MFMA k-steps over the head dim
  constexpr int DB = HS / 16;  // 16-row output blocks of O^T
  __shared__ __attribute__((aligned(16))) bf16_t Ks[kFK * KP];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[kFK * VP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, g = lane >> 4;
  constexpr int NT = 64 * NWQ;       // threads per workgroup
  constexpr int kFQ = 16 * NWQ * QB;  // queries per workgroup
  auto run = [&](const int qb) {
    const int h = blockIdx.y, b = blockIdx.z;
    const int C = nh * HS;
    const int p0 = pos[0];
    int t[QB], qpos[QB];  // this lane's query rows (rows past T are computed on a copy, never stored)
    // Q^T fragments: lane holds Q[t][32 kk + 8 g .. + 8]
    u32x4 qf[QB][KS];
  #pragma unroll
    for (int qi = 0; qi < QB; ++qi) {
      t[qi] = qb * kFQ + wave * 16 * QB + 16 * qi + col;
      qpos[qi] = p0 + t[qi];
      const int tq = t[qi] < T ? t[qi] : T - 1;
      const bf16_t* qrow = q + ((size_t)b * T + tq) * C + h * HS;
  #pragma unroll
      for (int kk = 0; kk < KS; ++kk) qf[qi][kk] = *reinterpret_cast<const u32x4*>(qrow + 32 * kk + 8 * g);
    }
    const int tlast = min(T, qb * kFQ + kFQ) - 1;
    const int kmax = p0 + tlast;  // last key any query of the block attends
    const int ntile = kmax / kFK + 1;
    const bf16_t* kbase = kc + ((size_t)(b * nh + h) * S) * HS;
    const bf16_t* vbase = vc + ((size_t)(b * nh + h) * S) * HS;
    // staging map: 64 keys x HS/8 vectors = 64 * HS / 8 16-B pieces over NT threads
    constexpr int PV = kFK * HS / 8 / NT;
    // two register sets (LLJ_FLASH_PF 2): tile kt + 2's loads are issued while tile kt is multiplied,
    // so each tile's K / V loads have two tiles of MFMA work to land in (one with LLJ_FLASH_PF 1)
    u32x4 kA[PV], vA[PV], kB[PV], vB[PV];
    auto load_into = [&](int kt, u32x4 (&kr)[PV], u32x4 (&vr)[PV]) {
  #pragma unroll
      for (int i = 0; i < PV; ++i) {
        const int piece = tid + NT * i;
        const int key = piece / (HS / 8), v8 = piece % (HS / 8);
        int slot = kt * kFK + key;
        slot = slot <= kmax ? slot : kmax;  // clamped: masked below
        kr[i] = *reinterpret_cast<const u32x4*>(kbase + (size_t)slot * HS + 8 * v8);
        vr[i] = *reinterpret_cast<const u32x4*>(vbase + (size_t)slot * HS + 8 * v8);
      }
    };
    float m_run[QB], l_run[QB];
    f32x4 acc_o[QB][DB];
  #pragma unroll
    for (int qi = 0; qi < QB; ++qi) {
      m_run[qi] = -INFINITY;
      l_run[qi] = 0.f;
  #pragma unroll
      for (int d = 0; d < DB; ++d) acc_o[qi][d] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    auto step = [&](int kt, u32x4 (&kr)[PV], u32x4 (&vr)[PV], u32x4 (&kn)[PV], u32x4 (&vn)[PV]) {
      __syncthreads();  // the previous tile's readers are done with Ks / Vt
  #pragma unroll
      for (int i = 0; i < PV; ++i) {
        const int piece = tid + NT * i;
        const int key = piece / (HS / 8), v8 = piece % (HS / 8);
        *reinterpret_cast<u32x4*>(Ks + key * KP + 8 * v8) = kr[i];
        *reinterpret_cast<u32x4*>(Vs + key * VP + 8 * v8) = vr[i];
      }
      __syncthreads();
      if (LLJ_FLASH_PF == 2) {
        if (kt + 2 < ntile) load_into(kt + 2, kr, vr);  // the set just staged is free
      } else {
        if (kt + 1 < ntile) load_into(kt + 1, kn, vn);  // in flight during this tile's MFMAs
      }
      // S^T = K . Q^T for the tile's four 16-key blocks
      f32x4 s[QB][4];
  #pragma unroll
      for (int j = 0; j < 4; ++j) {
  #pragma unroll
        for (int qi = 0; qi < QB; ++qi) s[qi][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  #pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          const bf16x8 a = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(Ks + (16 * j + col) * KP + 32 * kk + 8 * g));
  #pragma unroll
          for (int qi = 0; qi < QB; ++qi) s[qi][j] = mfma_bf16(a, __builtin_bit_cast(bf16x8, qf[qi][kk]), s[qi][j]);
        }
      }
      uint32_t pb[QB][4][2];  // bf16 P^T pairs per key block: (r0, r1), (r2, r3)
      // only the tiles that reach past the wave's first query need the causal mask (wave-uniform)
      const bool masked = kt * kFK + kFK - 1 > p0 + qb * kFQ + wave * 16 * QB;
  #pragma unroll
      for (int qi = 0; qi < QB; ++qi) {
        // mask (key slot > query position); per-query max of the raw scores (the scale sl2 > 0
        // commutes with the max and is applied in the exponent's fma)
        if (LLJ_FLASH_FAST == 0 || masked) {
  #pragma unroll
          for (int j = 0; j < 4; ++j)
  #pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int key = kt * kFK + 16 * j + 4 * g + r;
              s[qi][j][r] = key <= qpos[qi] ? s[qi][j][r] : -INFINITY;
            }
        }
        float mx = -INFINITY;
  #pragma unroll
        for (int j = 0; j < 4; ++j)
  #pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[qi][j][r]);
        {  // max over the 4 lane groups holding this query's keys (lanes col, col+16, col+32, col+48)
          float lo, hi;
          lane_halves<false>(mx, lo, hi);
          mx = fmaxf(lo, hi);
          lane_halves<true>(mx, lo, hi);
          mx = fmaxf(lo, hi);
        }
        // finite: key 0 of tile 0 is visible to every query, so no tile leaves m_new at -inf and
        // exp2(-inf - m_new) = 0 needs no select
        const float m_new = fmaxf(m_run[qi], mx * sl2);
        const float corr = m_run[qi] == -INFINITY ? 0.f : exp2f(m_run[qi] - m_new);
        float psum = 0.f;
  #pragma unroll
        for (int j = 0; j < 4; ++j) {
          float pr[4];
  #pragma unroll
          for (int r = 0; r < 4; ++r) {
  #pragma clang fp contract(off)
            // the scaled score rounded before the subtraction (no fma contraction): the same p as the
            // scale-first form; v_exp_f32 directly (exp2f's denormal-range path only moves p < 2^-126)
            const float sc = s[qi][j][r] * sl2;
            pr[r] = LLJ_FLASH_FAST ? __builtin_amdgcn_exp2f(sc - m_new) : (s[qi][j][r] == -INFINITY ? 0.f : exp2f(sc - m_new));
            psum += pr[r];
          }
          pb[qi][j][0] = pack2bf(pr[0], pr[1]);
          pb[qi][j][1] = pack2bf(pr[2], pr[3]);
        }
        {
          float lo, hi;
          lane_halves<false>(psum, lo, hi);
          psum = lo + hi;
          lane_halves<true>(psum, lo, hi);
          psum = lo + hi;
        }
        l_run[qi] = l_run[qi] * corr + psum;
        m_run[qi] = m_new;
        if (LLJ_FLASH_FAST == 0 || __any(corr != 1.f)) {  // the running max moved for some query of the wave
  #pragma unroll
          for (int d = 0; d < DB; ++d)
  #pragma unroll
            for (int r = 0; r < 4; ++r) acc_o[qi][d][r] *= corr;
        }
      }
      // O^T += V^T . P^T, two 32-key steps
  #pragma unroll
      for (int u = 0; u < 2; ++u) {
        bf16x8 bfrag[QB];
  #pragma unroll
        for (int qi = 0; qi < QB; ++qi) {
          const u32x4 bw = {pb[qi][2 * u][0], pb[qi][2 * u][1], pb[qi][2 * u + 1][0], pb[qi][2 * u + 1][1]};
          bfrag[qi] = __builtin_bit_cast(bf16x8, bw);
        }
  #pragma unroll
        for (int d = 0; d < DB; ++d) {
          // lane 4q + p of group g addresses keys 32u + 4g + q (+16), dims 16d + 4p .. +3; lane col
          // receives dim 16d + col of those 4 keys
          const bf16_t* vr = Vs + (32 * u + 4 * g + ((lane >> 2) & 3)) * VP + 16 * d + 4 * (lane & 3);
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)vr);
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(vr + 16 * VP));
          const uint2 l2 = __builtin_bit_cast(uint2, lo), h2 = __builtin_bit_cast(uint2, hi);
          const u32x4 aw = {l2.x, l2.y, h2.x, h2.y};
  #pragma unroll
          for (int qi = 0; qi < QB; ++qi) acc_o[qi][d] = mfma_bf16(__builtin_bit_cast(bf16x8, aw), bfrag[qi], acc_o[qi][d]);
        }
      }
    };
    load_into(0, kA, vA);
    if (LLJ_FLASH_PF == 2) {
      if (ntile > 1) load_into(1, kB, vB);
      for (int kt = 0; kt < ntile; kt += 2) {
        step(kt, kA, vA, kB, vB);
        if (kt + 1 < ntile) step(kt + 1, kB, vB, kA, vA);
      }
    } else {
      for (int kt = 0; kt < ntile; kt += 2) {
        step(kt, kA, vA, kB, vB);
        if (kt + 1 < ntile) step(kt + 1, kB, vB, kA, vA);
      }
    }
    // y[b*T + t][h*HS + d] = O / l; lane holds d = 16 db + 4 g + r of its query
  #pragma unroll
    for (int qi = 0; qi < QB; ++qi) {
      if (t[qi] < T) {
        const float inv = 1.f / l_run[qi];
        bf16_t* yrow = y + ((size_t)b * T + t[qi]) * C + h * HS;
  #pragma unroll
        for (int d = 0; d < DB; ++d) {
          const uint2 o = make_uint2(pack2bf(acc_o[qi][d][0] * inv, acc_o[qi][d][1] * inv),
                                     pack2bf(acc_o[qi][d][2] * inv, acc_o[qi][d][3] * inv));
          *reinterpret_cast<uint2*>(yrow + 16 * d + 4 * g) = o;
        }
      }
    }
  };
  const int nqb = (T + kFQ - 1) / kFQ;
  if constexpr (PAIR) {  // block x takes query blocks nqb - 1 - x (long) and x (short): equal work per workgroup
    const int qz = nqb - 1 - (int)blockIdx.x, qa = blockIdx.x;
    run(qz);
    if (qa < qz) {
      __syncthreads();  // the first block's last readers are done with Ks / Vs
      run(qa);
    }
  } else {
    run(gridDim.x - 1 - blockIdx.x);  // long (late) query blocks first
  }
}

template <int HS, int QB, int NWQ = 4>
static void flash_launch(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T,
                         int n_head, int S, float sl2, bool pair, hipStream_t st) {
  const int nqb = (T + 16 * NWQ * QB - 1) / (16 * NWQ * QB);
  if (pair) {
    hipLaunchKernelGGL((flash_prefill_kernel<HS, QB, true, NWQ>), dim3((nqb + 1) / 2, n_head, B), dim3(64 * NWQ), 0, st,
                       (const bf16_t*)q, (const bf16_t*)kcache, (const bf16_t*)vcache, (bf16_t*)y, pos, T, S, n_head, sl2);
  } else {
    hipLaunchKernelGGL((flash_prefill_kernel<HS, QB, false, NWQ>), dim3(nqb, n_head, B), dim3(64 * NWQ), 0, st,
                       (const bf16_t*)q, (const bf16_t*)kcache, (const bf16_t*)vcache, (bf16_t*)y, pos, T, S, n_head, sl2);
  }
}

}  // namespace llj

using namespace llj;

extern "C" {

int llj_attention_prefill(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T,
                          int n_head, int head_size, int S, void* stream) {
  LLJ_REQUIRE(B > 0 && T > 0 && n_head > 0 && S > 0 && pos);
  const float sl2 = 1.4426950408889634f / sqrtf((float)head_size);
  hipStream_t st = (hipStream_t)stream;
  const int oq = opt(LLJ_OPT_FLASH_QB), op = opt(LLJ_OPT_FLASH_PAIR);  // A/B options (llj_set_option)
  // 1 or 2 query blocks per wave: 2 from LLJ_FLASH_QB2_MIN_T queries on (7B T = 2048: 29.28 / 29.43 vs
  // 29.45 / 29.67 ms per window, profiles/r06aa_flash_qb.jsonl), where the grid still fills the CUs
  const int qbw = oq > 0 ? oq : (T >= LLJ_FLASH_QB2_MIN_T ? 2 : LLJ_FLASH_QB);
  const bool pair = op >= 0 ? op != 0 : LLJ_FLASH_PAIR != 0;  // a long and a short query block per workgroup
  if (head_size == 128) {
    if (qbw == 2) flash_launch<128, 2>(q, kcache, vcache, y, pos, B, T, n_head, S, sl2, pair, st);
    else if (LLJ_FLASH_NWQ == 8) flash_launch<128, 1, 8>(q, kcache, vcache, y, pos, B, T, n_head, S, sl2, pair, st);
    else flash_launch<128, 1>(q, kcache, vcache, y, pos, B, T, n_head, S, sl2, pair, st);
  } else if (head_size == 64) {
    if (qbw == 2) flash_launch<64, 2>(q, kcache, vcache, y, pos, B, T, n_head, S, sl2, pair, st);
    else flash_launch<64, 1>(q, kcache, vcache, y, pos, B, T, n_head, S, sl2, pair, st);
  } else {
    return LLJ_EINVAL;
  }
  LLJ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

// Persistent decode engine: ONE launch per decode token for batch 1 with int4 (W4P) weights.
//
// Replaces, for a whole decode step, the launch chain of LLaMA.forward (reference
// lit_llama/model.py:84-128: embedding, n_layer x Block.forward 162-175 = rms_1 + c_attn + RoPE +
// KV write + SDPA + c_proj + residual, rms_2 + c_fc1/c_fc2 + silu*mul + c_proj + residual, then
// ln_f + lm_head) and the greedy next-token choice of generate.py:66-74 (top_k = 1).
//
// Why: a launch boundary costs 1.2-1.9 us and every launch re-ramps its weight stream behind the
// activation it waits for. Here the weight stream never stops at an op edge
// (MI355X_MICROARCH.md price list: ldsdma-fill, prefetch-credit, allgather, engine-vs-launches):
//  * grid = one 512-thread workgroup per CU, resident for the whole step (LDS > half a CU).
//  * the last wave of every workgroup is a LOADER: it streams this CU's weight blocks (1 KiB W4P
//    tiles = 16 columns x 128 k) into an LDS ring by LDS-DMA (global_load_lds_dwordx4 ... nt) in
//    the order the CU consumes them, across op and layer boundaries -- weights do not depend on
//    activations, so the next op's blocks land while the consumers wait for that op's input. It
//    publishes `landed` (blocks in LDS) and waits on the consumers' progress words before reusing a
//    slot. Its DMAs never sit in a consumer's vmcnt queue.
//  * the other NC waves CONSUME: chunk c of a tile goes to wave c % NC (bf16 MFMA 16x16x32 on the
//    dequantized codes, as the GEMVs) in a software pipeline -- the ring read of a wave's next block
//    is in flight while it dequantizes and multiplies the current one, landing checks are scalar and
//    re-read the loader's word only when the cached count is behind; partial sums meet in LDS, one
//    wave runs each tile's epilogue. They synchronise through an LDS counter barrier.
//  * op outputs travel between CUs as 8-byte {tag, payload} granules written by one agent-scope
//    (sc1) store each and read by sc1 polling loads: the data is its own flag, no fence, no grid
//    barrier. tag = epoch * 128 + layer + 1 (epoch advanced on the device once per step), never 0.
//  * QKV is dealt per (head h, 16-dim slice j) unit: the CU of unit (h, j) computes the q, k and v
//    columns h * hs + 16 j + [0, 16), so attention needs no q/k/v hand-off: it computes the partial
//    scores of its 16 dims for every key, the J = hs / 16 CUs of a head exchange them as granules
//    (one hop), each sums the J partials in the same order (bitwise-equal scores on every CU of the
//    head), runs the softmax and P.V over its own 16 value dims, and publishes its slice of y. With
//    U = n_head * J = CUs (7B: 256) the J CUs of a head share an XCD (block b on XCD b % 8: speed
//    only, never correctness). Every other op's tile t runs on CU t % G.
// Per layer: gather x -> rms_1 -> QKV tiles (RoPE, KV-cache write, q/k/v slices into LDS) ->
// partial scores -> score exchange -> softmax, P.V -> publish y slice -> gather y -> c_proj tile +
// residual (publish x_mid) -> gather x_mid -> rms_2 -> SwiGLU tiles (publish h) -> gather h -> down
// tile + residual (publish x). After the last layer: ln_f + lm_head tiles (logits to HBM, per-CU
// argmax publish); the last CU to arrive picks the token, writes it and advances the device position
// and the epoch.
// Numerics follow the GEMV path (gemv_impl.h): bf16 rounding points of the reference, int4 offset
// removed with the row sum of the normalized input, RoPE / softmax in fp32.
// Every spin is bounded (kSpinTicks from the step's start); a timeout sets ctl[2] and turns every
// later wait into a pass-through, so a faulty step still terminates (the host checks ctl[2]).
#include "common.h"
#include "lit_llama_amd.h"

namespace llj {
namespace eng {

#ifndef LLJ_ENG_NC
#define LLJ_ENG_NC 7       // consumer waves
#endif
constexpr int NWV = LLJ_ENG_NC + 1;  // waves per workgroup (two per SIMD at 8)
constexpr int NC = LLJ_ENG_NC;  // consumer waves (0 .. NC-1); wave NC is the loader
static_assert(NC >= 3 && NC <= 15, "consumer waves");
constexpr int NTH = 64 * NWV;
constexpr int TG = 4;      // tiles per partial-sum group (the red scratch holds TG tiles x 2 matrices)
#ifndef LLJ_ENG_D
#define LLJ_ENG_D 48       // DMAs the loader keeps in flight (vmcnt immediate)
#endif
constexpr int D = LLJ_ENG_D;
static_assert(D >= 1 && D <= 62, "vmcnt immediate");
constexpr int GK = 8;      // granules per lane per gather batch (x, y, x_mid: one batch at 7B; h: two)
constexpr int GN = 6;      // RMSNorm gain pairs per lane (C / 2 <= GN * 64 * NC: C <= 5376)
constexpr unsigned long long kSpinTicks = 5000000ull;  // 50 ms of s_memrealtime (100 MHz)
constexpr int kMaxCUs = LLJ_ENGINE_MAX_CUS;
constexpr int kMaxS = 512;  // cache slots (the score exchange arena holds kMaxS keys per unit)
constexpr int kKPT = (kMaxS + 64 * NC - 1) / (64 * NC);  // keys per consumer thread at most

enum : int { OP_QKV = 0, OP_O = 1, OP_SW = 2, OP_DOWN = 3, OP_HEAD = 4, OP_END = 5 };
enum : unsigned { ERR_TIMEOUT = 1u };

// granule arena (u64 units) and the control words behind it
struct Arena {
  unsigned long long *gx, *gy, *gxm, *gh, *garg, *gsc;
  unsigned* ctl;  // [0] epoch, [1] end-of-step arrivals, [2] error bits
};
__host__ __device__ inline size_t arena_granules(int C, int H) {
  // x, y, x_mid | h | argmax | partial scores: (C / 16 units) x kMaxS keys
  return (size_t)3 * (C / 2) + (size_t)H / 2 + (size_t)kMaxCUs + (size_t)(C / 16) * kMaxS;
}
__device__ inline Arena arena_of(const llj_engine_plan& P) {
  Arena a;
  unsigned long long* b = reinterpret_cast<unsigned long long*>(P.arena);
  const int C = P.C, H = P.H;
  a.gx = b;
  a.gy = a.gx + C / 2;
  a.gxm = a.gy + C / 2;
  a.gh = a.gxm + C / 2;
  a.garg = a.gh + H / 2;
  a.gsc = a.garg + kMaxCUs;
  a.ctl = reinterpret_cast<unsigned*>(a.gsc + (size_t)(C / 16) * kMaxS);
  return a;
}

__device__ __forceinline__ unsigned long long ld_gran(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_load_dwordx2 sc1
}
__device__ __forceinline__ void st_gran(unsigned long long* p, unsigned tag, uint32_t v) {
  __hip_atomic_store(p, ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ unsigned lds_ld(const unsigned* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_st(unsigned* p, unsigned v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void cbar() { asm volatile("" ::: "memory"); }  // compiler-only ordering point

typedef bf16x8 afrag_t;
constexpr uint32_t kDqMag = 0x43004300u;  // bf16 128
__device__ __forceinline__ bf16x8 dequant(uint32_t w, uint32_t msk, uint32_t mag) {
  uint4 b = make_uint4(and_or(w, msk, mag), and_or(w >> 4, msk, mag), and_or(w >> 8, msk, mag), and_or(w >> 12, msk, mag));
  return __builtin_bit_cast(bf16x8, b);
}
__device__ __forceinline__ f32x4 mfma_a(afrag_t a, bf16x8 b, f32x4 c) { return mfma_bf16(a, b, c); }
#define LLJ_DQ(w) dequant((w), msk, mag)
__device__ __forceinline__ float rstd_bf16(float ss_over_k, float eps) {
  return round_bf(rsqrtf(round_bf(round_bf(ss_over_k) + eps)));  // model.py:281-282 on bf16 tensors
}
__device__ __forceinline__ uint32_t bf_key(uint32_t b) { return (b & 0x8000u) ? (~b & 0xFFFFu) : (b | 0x8000u); }

// profiling stamps (plan.trace != NULL): [g][128]; consumers: 0 start, per layer l at 2 + 12 l:
// +0 x staged, +1 QKV done, +2 attention done, +3 y staged, +4 c_proj done, +5 x_mid staged,
// +6 SwiGLU done, +7 h staged, +8 down done, +9 scores published; the loader: 100 + op index of its
// last DMA of each op (per layer, layers 0..1 only: 100..107), 108..119 inside consume (QKV /
// SwiGLU of layers 0, 1: A in registers, blocks done, barrier passed), 120 stream end, 121 loader
// start; 126 head staged, 127 head done
__device__ __forceinline__ void stamp(const llj_engine_plan& P, int lane, int k) {
  if (P.trace && lane == 0 && k < 128) P.trace[(size_t)blockIdx.x * 128 + k] = __builtin_amdgcn_s_memrealtime();
}

// ------------------------------------------------------------------------------------ schedule
struct Shape {
  int C, H, V, nh, hs, S, L, G, g;
  int J;     // 16-dim slices per head (hs / 16)
  int unit;  // this CU's QKV unit u = h * J + j, or -1 (more CUs than units)
};
// QKV unit of CU g: with U = n_head * J == G (7B) and G % 8 == 0, J == 8, the J units of head h go to
// CUs g = h % 8 + 8 (J (h / 8) + j), which share g % 8 (one XCD under round-robin placement);
// otherwise unit g
__device__ __forceinline__ int unit_of_cu(int g, int G, int nh, int J) {
  const int U = nh * J;
  if (U == G && (G & 7) == 0 && J == 8 && (nh & 7) == 0) {
    const int x = g & 7, m = g >> 3;
    return (x + 8 * (m / J)) * J + (m % J);
  }
  return g < U ? g : -1;
}
__device__ __forceinline__ int op_ntiles(const Shape& s, int op) {
  return op == OP_QKV ? 3 * s.C / 16 : op == OP_SW ? s.H / 16 : op == OP_HEAD ? s.V / 16 : s.C / 16;
}
__device__ __forceinline__ int op_kc(const Shape& s, int op) { return (op == OP_DOWN ? s.H : s.C) >> 7; }
__device__ __forceinline__ int op_nmat(int op) { return op == OP_SW ? 2 : 1; }
__device__ __forceinline__ int tiles_of_cu(const Shape& s, int op) {
  if (op == OP_QKV) return s.unit >= 0 ? 3 : 0;
  const int n = op_ntiles(s, op);
  return s.g < n ? (n - s.g + s.G - 1) / s.G : 0;
}
// tile of slot j of this CU's share of op: QKV slots 0 / 1 / 2 = the q / k / v columns of its unit
__device__ __forceinline__ int tile_of(const Shape& s, int op, int j) {
  return op == OP_QKV ? j * (s.C / 16) + s.unit : s.g + j * s.G;
}
// Weight pointer of (layer, op, matrix) for the loader wave, read by a scalar load (the layer table
// is written by the host before the launch and only read here). A compiler-visible vector load
// would be followed by s_waitcnt vmcnt(0) at its use -- a wait that also drains every LDS-DMA the
// loader has in flight (the compiler does not see them), once per op edge.
__device__ __forceinline__ const char* op_weight(const llj_engine_plan& P, int l, int op, int m) {
  if (op == OP_HEAD) return reinterpret_cast<const char*>(P.w_head);
  const llj_engine_layer* Ly = P.layers + l;
  const void* const* f = op == OP_QKV ? &Ly->w_qkv : op == OP_O ? &Ly->w_o : op == OP_SW ? (m ? &Ly->w_fc2 : &Ly->w_fc1) : &Ly->w_down;
  uint64_t v;
  asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(f) : "memory");
  return reinterpret_cast<const char*>(v);
}

// ------------------------------------------------------------------------------------ LDS
// carve (bytes, 16-aligned): ctl words | A (max(C, H) bf16) | xown[2] (16 bf16) | red[2][NC][TG][2][16]
// f32 | eop[2] (epilogue operands) | misc[80] f32 ([0, NC) sums of squares, [16, 16 + NC) row sums,
// [32, 32 + NC) argmax, [48] last-arriver flag, [64, 64 + NC) f16 A' sums) | attention scratch | ring (nb x 1 KiB)
constexpr int kCtlWords = 32;  // [0] landed, [1 .. NC] next block per consumer, [16] consumer barrier, [17] max wanted block
// attention scratch (f32): q / k / v slices [3][16], per-wave max / sum [2][NC], per-wave P.V [NC][16]
constexpr int kAttFloats = 48 + 2 * NC + 16 * NC;
struct Lds {
  unsigned* ctl;
  unsigned char* ring;
  bf16_t* A;
  bf16_t* xown[2];  // the raw x / x_mid of this CU's c_proj / down tile columns (the residual inputs)
  float* red;
  float2* eop;  // [2][kEopTiles][2][16]
  float* misc;
  float* att;
  int nb;
  unsigned nb_magic;  // ceil(2^32 / nb): b % nb by one multiply-high
};
__host__ __device__ inline size_t al16(size_t b) { return (b + 15) & ~(size_t)15; }
// epilogue operands staged per op: (scale, 128 + zero) of both matrices for every tile of the CU
// (at most kEopTiles), or the RoPE (cos, sin) pairs of the QKV tiles
constexpr int kEopTiles = 8;
__host__ __device__ inline size_t lds_fixed(int C, int H) {
  const int K = C > H ? C : H;
  return (size_t)kCtlWords * 4 + al16((size_t)K * 2) + 2 * 32 + (size_t)2 * NC * TG * 2 * 16 * 4 +
         (size_t)2 * kEopTiles * 2 * 16 * 8 + 80 * 4 + al16((size_t)kAttFloats * 4);
}
// ring blocks that fit next to the fixed part in `budget` bytes
__host__ __device__ inline int ring_blocks(int C, int H, size_t budget) {
  const size_t f = lds_fixed(C, H);
  return f >= budget ? 0 : (int)((budget - f) / 1024) & ~7;  // whole runs of 8 slots (the loader's DMA runs)
}

// ------------------------------------------------------------------------------------ state
struct Ctx {
  Shape s;
  int wave, lane;
  unsigned* gctl;     // global control words
  unsigned long long t0;
  bool aborted;
  unsigned bar_gen;   // consumer barriers passed
  const llj_engine_plan* plan;
  int n_used;         // CU-stream index of the next block of this op (consumers)
  int landed;         // blocks published as landed, as last read (consumers; monotone)
  int stamp_base;     // profiling: stamp index base inside consume (-1 = none)
};

// bounded spin bookkeeping: true = give up (a timeout here or anywhere in the grid). Global polls
// sleep a little between passes; LDS spins only look at the clock every 256 passes.
__device__ __forceinline__ bool spin_timeout(unsigned* gctl, unsigned long long t0, int lane) {
  const unsigned long long now = __builtin_amdgcn_s_memrealtime();
  if (now - t0 > kSpinTicks || __hip_atomic_load(gctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
    if (lane == 0) __hip_atomic_fetch_or(gctl + 2, ERR_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  return false;
}
__device__ __forceinline__ bool spin_check(Ctx& X) {
  if (spin_timeout(X.gctl, X.t0, X.lane)) X.aborted = true;
  return X.aborted;
}
__device__ __forceinline__ bool spin_fail(Ctx& X, unsigned& it) {
  if (X.aborted) return true;
  __builtin_amdgcn_s_sleep(1);
  return (++it & 15u) == 0u && spin_check(X);
}
__device__ __forceinline__ bool spin_fail_lds(Ctx& X, unsigned& it) {
  if (X.aborted) return true;
  return (++it & 255u) == 0u && spin_check(X);
}
// the loader's spins: its own clock only -- a vector load of the global error word would come with
// a compiler s_waitcnt vmcnt(0) that drains the DMA window
__device__ __forceinline__ bool spin_fail_loader(Ctx& X, unsigned& it) {
  if (X.aborted) return true;
  if ((++it & 255u) == 0u && __builtin_amdgcn_s_memrealtime() - X.t0 > kSpinTicks) X.aborted = true;
  return X.aborted;
}

// barrier of the NC consumer waves (an LDS counter: the loader wave never takes part)
__device__ __forceinline__ void cbarrier(Ctx& X, const Lds& L) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS writes are done
  if (X.lane == 0) __hip_atomic_fetch_add(L.ctl + 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  const unsigned target = (X.bar_gen + 1) * NC;
  unsigned it = 0;
  while (lds_ld(L.ctl + 16) < target) {
    if (spin_fail_lds(X, it)) break;
  }
  ++X.bar_gen;
}

// Gather granules [0, n) of `g` tagged `tag`: consumer wave w takes indices lane + 64 (w + NC k);
// every load of a batch of GK per lane is in flight before any tag is checked; a batch is re-read
// until every tag matches. sink(idx, payload) for each.
template <int GK, typename F>
__device__ __forceinline__ void gather(Ctx& X, const unsigned long long* g, int n, unsigned tag, F&& sink) {
  const int first = X.lane + 64 * X.wave;
  constexpr int STEP = 64 * NC;
  for (int b0 = 0; b0 < n; b0 += STEP * GK) {
    unsigned long long v[GK];
    unsigned it = 0;
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int k = 0; k < GK; ++k) {
        const int idx = b0 + first + STEP * k;
        v[k] = ld_gran(g + (idx < n ? idx : 0));
      }
#pragma unroll
      for (int k = 0; k < GK; ++k) {
        const int idx = b0 + first + STEP * k;
        ok &= idx >= n || (unsigned)(v[k] >> 32) == tag;
      }
      if (__all(ok)) break;
      if (spin_fail(X, it)) break;
    }
#pragma unroll
    for (int k = 0; k < GK; ++k) {
      const int idx = b0 + first + STEP * k;
      if (idx < n) sink(idx, (uint32_t)v[k]);
    }
  }
}

// Stage the epilogue operands of op into eop (one of two LDS buffers, alternating per op: the
// previous op's epilogue may still read the other): per tile slot j (< kEopTiles) and matrix m, the
// (scale, 128 + zero) of column 16 tile + c at eop[(j * 2 + m) * 16 + c]. Loaded by the consumers
// ahead of the gather they are about to wait in, so the epilogue reads LDS only.
__device__ __forceinline__ void stage_sz(Ctx& X, float2* eop, const llj_engine_plan& P, int l, int op) {
  const Shape& s = X.s;
  const int nt = tiles_of_cu(s, op) < kEopTiles ? tiles_of_cu(s, op) : kEopTiles;
  const int nm = op_nmat(op);
  const llj_engine_layer* Ly = op == OP_HEAD ? nullptr : &P.layers[l];
  for (int i = X.lane + 64 * X.wave; i < nt * nm * 16; i += 64 * NC) {
    const int c = i & 15, m = (i >> 4) % nm, j = (i >> 4) / nm;
    const float2* sz = op == OP_HEAD ? reinterpret_cast<const float2*>(P.sz_head)
                       : op == OP_QKV ? reinterpret_cast<const float2*>(Ly->sz_qkv)
                       : op == OP_O   ? reinterpret_cast<const float2*>(Ly->sz_o)
                       : op == OP_SW  ? reinterpret_cast<const float2*>(m ? Ly->sz_fc2 : Ly->sz_fc1)
                                      : reinterpret_cast<const float2*>(Ly->sz_down);
    eop[(j * 2 + m) * 16 + c] = sz[16 * tile_of(s, op, j) + c];
  }
}

// Stage the input of an op into A (one call site for every op, so its code is in the kernel once):
// norm ops (QKV, SwiGLU, lm_head): x (gathered, or the embedding row at layer 0) -> A raw, then
// A = RMSNorm(x) * gain in place (model.py:276-283, bf16 rounding points) by the same threads that
// gathered each pair, and the raw pairs of this CU's residual tile columns -> xown[buf]; plain ops
// (c_proj, down): the gathered vector -> A. Returns sum_k A[k].
__device__ __forceinline__ float stage(Ctx& X, const Lds& L, bool norm, int buf, const unsigned long long* g, unsigned tag,
                                       const bf16_t* direct, const bf16_t* gain, float eps, int K) {
  uint32_t* xo2 = reinterpret_cast<uint32_t*>(L.xown[buf]);
  const int own0 = 8 * X.s.g;  // first pair of the CU's c_proj / down tile (tile g: n_embd / 16 <= CUs)
  uint32_t* a2 = reinterpret_cast<uint32_t*>(L.A);
  const uint32_t* g2 = reinterpret_cast<const uint32_t*>(gain);
  // this wave's gain pairs, loaded before the wait (K / 2 / (64 NC) <= GN per lane)
  uint32_t gv[GN];
  if (norm) {
#pragma unroll
    for (int k = 0; k < GN; ++k) {
      const int idx = X.lane + 64 * X.wave + 64 * NC * k;
      gv[k] = g2[idx < K / 2 ? idx : 0];
    }
  }
  // one accumulator: the sum of squares (norm) or of the values (plain) -- a select, not two
  // variables (which the compiler turns into a scratch array indexed by `norm`)
  float part = 0.f;
  auto sink = [&](int idx, uint32_t v) {
    a2[idx] = v;
    const f32x2 f = unpk(v);
    part += norm ? round_bf(f.x * f.x) + round_bf(f.y * f.y) : f.x + f.y;  // model.py:281: x * x in bf16
  };
  if (direct) {  // layer 0: the embedding row wte[cur] (model.py:110), read by every CU
    const uint32_t* d2 = reinterpret_cast<const uint32_t*>(direct);
    for (int idx = X.lane + 64 * X.wave; idx < K / 2; idx += 64 * NC) sink(idx, d2[idx]);
  } else {
    gather<GK>(X, g, K / 2, tag, sink);
  }
  float asum = norm ? 0.f : part;
  if (norm) {
    const float ss = wave_sum(part);
    if (X.lane == 0) L.misc[X.wave] = ss;
    cbarrier(X, L);
    float tot = 0.f;
#pragma unroll
    for (int w = 0; w < NC; ++w) tot += L.misc[w];
    const float r = rstd_bf16(tot / (float)K, eps);
#pragma unroll
    for (int k = 0; k < GN; ++k) {
      const int idx = X.lane + 64 * X.wave + 64 * NC * k;
      if (idx < K / 2) {  // the pair this thread gathered (gather's index map is this loop's for K / 2 <= 64 NC GK)
        const uint32_t raw = a2[idx];
        const uint32_t o = norm_pair(raw, gv[k], r);
        a2[idx] = o;
        asum += bflo(o) + bfhi(o);
        if (idx >= own0 && idx < own0 + 8) xo2[idx - own0] = raw;
      }
    }
  }
  asum = wave_sum(asum);
  if (X.lane == 0) L.misc[16 + X.wave] = asum;
  cbarrier(X, L);
  float a = 0.f;
#pragma unroll
  for (int w = 0; w < NC; ++w) a += L.misc[16 + w];
  return a;
}

// what the epilogue of each op needs (one epilogue function, switch on the op)
struct Epi {
  Arena ar;
  unsigned tag;
  int slot;            // cache slot of this step's position
  bf16_t *kcache, *vcache;
  const float2* rcs;   // RoPE (cos, sin) per QKV tile slot
  bf16_t* logits;
  uint32_t best;       // lm_head: (order key << 16) | (0xFFFF - column), max = argmax, lowest index on ties
};

// publish the bf16 pair (column n even: lanes 2i, 2i + 1 of a tile's 16) as one granule
__device__ __forceinline__ void publish_pair(unsigned long long* g, int n, unsigned tag, float v, int lane) {
  const uint32_t b = (uint32_t)f2bf(v);
  const uint32_t pr = lane_xor1(b);
  if (lane < 16 && !(lane & 1)) st_gran(g + n / 2, tag, b | (pr << 16));
}

// output column n (lanes 0..15 of the tile's 16) of tile slot sl of op: y1 (and y2 of SwiGLU's
// second matrix) in fp32 with the int4 offset removed
__device__ __forceinline__ void epilogue(Ctx& X, const Lds& L, int op, Epi& E, int sl, int tile, int n, float y1, float y2) {
  const Shape& s = X.s;
  const int lane = X.lane;
  switch (op) {
    case OP_QKV: {  // slot sl = 0 q, 1 k, 2 v of this CU's (head, 16-dim slice) unit
      const int C = s.C, hs = s.hs;
      const int nc = n - sl * C;
      const int hh = nc / hs, dd = nc % hs;
      const float v = round_bf(y1);  // c_attn output in bf16 (model.py:204)
      const float partner = lane_xor1(v);
      float out = v;
      if (sl < 2) {  // RoPE in fp32 (model.py:318-329)
        const float2 cs = E.rcs[sl * 8 + ((lane & 15) >> 1)];
        out = (dd & 1) ? (v * cs.x + partner * cs.y) : (v * cs.x - partner * cs.y);
      }
      const uint32_t ob = (uint32_t)f2bf(out);  // the bf16 q / k / v (type_as, model.py:329)
      const uint32_t pr = lane_xor1(ob);
      // the slice stays in this CU's LDS for the attention (q pre-scaled by log2(e) / sqrt(hs))
      if (lane < 16) L.att[sl * 16 + lane] = bf2f((bf16_t)ob) * (sl == 0 ? 1.4426950408889634f / sqrtf((float)hs) : 1.f);
      if (sl > 0 && lane < 16 && !(lane & 1)) {  // the cache row of this position, for later steps
        bf16_t* dst = (sl == 1 ? E.kcache : E.vcache) + ((size_t)hh * s.S + E.slot) * hs + dd;
        *reinterpret_cast<uint32_t*>(dst) = ob | (pr << 16);
      }
      break;
    }
    case OP_O:  // x + attn(x) in bf16 (model.py:172)
      publish_pair(E.ar.gxm, n, E.tag, round_bf(bf2f(L.xown[0][n & 15]) + round_bf(y1)), lane);
      break;
    case OP_SW: {
      const float a1 = round_bf(y1), a2 = round_bf(y2);
      const float sl2 = round_bf(a1 / (1.f + __expf(-a1)));  // F.silu in bf16 (model.py:258)
      publish_pair(E.ar.gh, n, E.tag, sl2 * a2, lane);
      break;
    }
    case OP_DOWN:  // model.py:173
      publish_pair(E.ar.gx, n, E.tag, round_bf(bf2f(L.xown[1][n & 15]) + round_bf(y1)), lane);
      break;
    default: {  // lm_head: bf16 logits + this wave's argmax key
      const uint32_t b = (uint32_t)f2bf(y1);
      const uint32_t pr = lane_xor1(b);
      if (lane < 16 && !(lane & 1)) *reinterpret_cast<uint32_t*>(E.logits + n) = b | (pr << 16);
      const uint32_t key = lane < 16 ? ((bf_key(b) << 16) | (0xFFFFu - (uint32_t)n)) : 0u;
      E.best = max(E.best, key);
    }
  }
}

// Consume this CU's blocks of `op`. Stream order (the loader's): tile groups of TG tiles, tile-major
// inside a group -- for tile slot jj: for chunk c: for matrix m (contiguous 1 KiB blocks of a tile
// for the DMA) -- and consumer w owns the chunks c = w (mod NC) of every tile. Per tile (per batch
// of 4 chunks for long K) a wave waits, by a scalar compare with its cached landed count, for its
// last block; issues every ring read of the tile (and, for long K, the A fragments) at once, branch
// free, so the compiler counts each chunk's wait (lgkmcnt(N)) instead of draining; publishes in
// ctl[1 + w] the stream index of its next block (its reads are ahead of that LDS write: one wave's
// LDS operations execute in order); then dequantizes and multiplies chunk by chunk. For K <=
// AREG_C * NC * 128 the A fragments of all a wave's chunks stay in registers for the whole op.
// Partial sums of output row 0 go to red per tile; after each group the epilogue of tile slot jj
// runs on consumer jj % NC, lanes 0..15 (column 16 tile + lane).
constexpr int AREG_C = 5;  // chunks per consumer whose A fragments stay in registers (K <= 4480 at NC 7)
constexpr int KB = 3;      // chunks per read batch of the long-K form (3 x 5 reads: lgkmcnt counts to 15)
template <int NM, bool AREG>
__device__ __forceinline__ void consume_t(Ctx& X, const Lds& L, const float2* eop, int op, float asum,
                                          int& red_par, Epi& E) {
  const Shape& s = X.s;
  const int nt = tiles_of_cu(s, op), kc = op_kc(s, op);
  const int lane = X.lane, grp = lane >> 4, w = X.wave;
  uint32_t msk = 0x000F000Fu, mag = kDqMag;  // 128 + q (bf16) via one v_and_or_b32 per pair
  asm volatile("" : "+s"(msk));
  asm volatile("" : "+v"(mag));
  const int nch = kc > w ? (kc - w + NC - 1) / NC : 0;  // chunks of every tile this wave takes
  afrag_t ar[AREG ? AREG_C : 1][4];
  if constexpr (AREG) {
#pragma unroll
    for (int ci = 0; ci < AREG_C; ++ci) {
      const int c = w + ci * NC < kc ? w + ci * NC : 0;
      const bf16_t* arow = L.A + 128 * c + 32 * grp;
#pragma unroll
      for (int t = 0; t < 4; ++t) ar[ci][t] = __builtin_bit_cast(afrag_t, *reinterpret_cast<const u32x4*>(arow + 8 * t));
    }
  }
  const int per_tile = kc * NM;
  const llj_engine_plan* SP = X.plan;
  if (X.stamp_base >= 0 && w == 0) stamp(*SP, lane, X.stamp_base + 0);  // A fragments in registers
  int gbase = X.n_used;  // CU-stream index of the current group's first block
  // block b landed (b wave-uniform): a scalar compare with the cached count; the loader's word is
  // re-read only when behind, and a consumer that has to wait records b in ctl[17] (LDS max) so the
  // loader, stalled on a full ring, knows to publish landings early
  auto wait_landed = [&](int b) {
    if (X.landed > b) return;
    X.landed = uniform((int)lds_ld(L.ctl + 0));
    if (X.landed > b) return;
    if (lane == 0) __hip_atomic_fetch_max(L.ctl + 17, (unsigned)b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    unsigned it = 0;
    for (;;) {
      X.landed = uniform((int)lds_ld(L.ctl + 0));
      if (X.landed > b || spin_fail_lds(X, it)) break;
    }
  };
  auto ring = [&](int b) -> u32x4 {
    const unsigned q = __umulhi((unsigned)b, L.nb_magic);
    return *reinterpret_cast<const u32x4*>(L.ring + (size_t)((unsigned)b - q * (unsigned)L.nb) * 1024 + 16 * lane);
  };
  auto progress = [&](int next) {
    cbar();
    if (lane == 0) lds_st(L.ctl + 1 + w, (unsigned)next);
  };
  for (int j0 = 0; j0 < nt; j0 += TG) {
    const int ng = nt - j0 < TG ? nt - j0 : TG;
    const int gend = gbase + ng * per_tile;
    float* red = L.red + (size_t)red_par * NC * TG * 2 * 16;
    for (int jj = 0; jj < ng; ++jj) {
      const int tb = gbase + jj * per_tile;                            // the tile's first block
      const int tnext = jj + 1 < ng ? tb + per_tile + w * NM : gend;  // this wave's first block after the tile
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
      if (nch == 0) {
        progress(tnext);
      } else if constexpr (AREG) {
        wait_landed(tb + (w + (nch - 1) * NC) * NM + NM - 1);
        u32x4 wt[AREG_C][NM];
#pragma unroll
        for (int ci = 0; ci < AREG_C; ++ci) {  // chunks past nch re-read chunk w (landed; unused)
          const int b = tb + (w + (ci < nch ? ci : 0) * NC) * NM;
#pragma unroll
          for (int m = 0; m < NM; ++m) wt[ci][m] = ring(b + m);
        }
        progress(tnext);
#pragma unroll
        for (int ci = 0; ci < AREG_C; ++ci) {
          if (ci < nch) {
            if constexpr (NM == 2) {
#pragma unroll
              for (int t = 0; t < 4; ++t) {
                a0 = mfma_a(ar[ci][t], LLJ_DQ(wt[ci][0][t]), a0);
                a1 = mfma_a(ar[ci][t], LLJ_DQ(wt[ci][1][t]), a1);
              }
            } else {  // two independent chains (odd fragments into a1): no MFMA waits on its predecessor
#pragma unroll
              for (int t = 0; t < 4; t += 2) {
                a0 = mfma_a(ar[ci][t], LLJ_DQ(wt[ci][0][t]), a0);
                a1 = mfma_a(ar[ci][t + 1], LLJ_DQ(wt[ci][0][t + 1]), a1);
              }
            }
          }
        }
      } else {  // long K (the down projection): batches of KB chunks, A fragments read with the weights
        for (int c0 = w; c0 < kc; c0 += KB * NC) {
          const int nbat = (kc - c0 + NC - 1) / NC < KB ? (kc - c0 + NC - 1) / NC : KB;
          wait_landed(tb + (c0 + (nbat - 1) * NC) * NM + NM - 1);
          u32x4 wt[KB][NM];
          afrag_t af[KB][4];
#pragma unroll
          for (int u = 0; u < KB; ++u) {
            const int c = u < nbat ? c0 + u * NC : c0;
#pragma unroll
            for (int m = 0; m < NM; ++m) wt[u][m] = ring(tb + c * NM + m);
            const bf16_t* arow = L.A + 128 * c + 32 * grp;
#pragma unroll
            for (int t = 0; t < 4; ++t) af[u][t] = __builtin_bit_cast(afrag_t, *reinterpret_cast<const u32x4*>(arow + 8 * t));
          }
          progress(c0 + KB * NC < kc ? tb + (c0 + KB * NC) * NM : tnext);
#pragma unroll
          for (int u = 0; u < KB; ++u) {
            if (u < nbat) {
              if constexpr (NM == 2) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                  a0 = mfma_a(af[u][t], LLJ_DQ(wt[u][0][t]), a0);
                  a1 = mfma_a(af[u][t], LLJ_DQ(wt[u][1][t]), a1);
                }
              } else {
#pragma unroll
                for (int t = 0; t < 4; t += 2) {
                  a0 = mfma_a(af[u][t], LLJ_DQ(wt[u][0][t]), a0);
                  a1 = mfma_a(af[u][t + 1], LLJ_DQ(wt[u][0][t + 1]), a1);
                }
              }
            }
          }
        }
      }
      if constexpr (NM == 1) a0 += a1;
      if (lane < 16) {  // partial sums of output row 0 (lanes 0..15, register 0)
        red[((w * TG + jj) * 2 + 0) * 16 + lane] = a0[0];
        red[((w * TG + jj) * 2 + 1) * 16 + lane] = a1[0];
      }
    }
    gbase = gend;
    if (X.stamp_base >= 0 && w == 0 && j0 == 0) stamp(*SP, lane, X.stamp_base + 1);  // group's blocks done
    cbarrier(X, L);
    if (X.stamp_base >= 0 && w == 0 && j0 == 0) stamp(*SP, lane, X.stamp_base + 2);  // barrier passed
    for (int jj = w; jj < ng; jj += NC) {
      const int slot = j0 + jj;
      const int tile = tile_of(s, op, slot);
      const int col = lane & 15;
      const int n = 16 * tile + col;
      float y1 = 0.f, y2 = 0.f;
#pragma unroll
      for (int v = 0; v < NC; ++v) {
        y1 += red[((v * TG + jj) * 2 + 0) * 16 + col];
        y2 += red[((v * TG + jj) * 2 + 1) * 16 + col];
      }
      const int es = slot < kEopTiles ? slot : kEopTiles - 1;
      const float2 e1 = eop[(es * 2 + 0) * 16 + col], e2 = eop[(es * 2 + 1) * 16 + col];
      y1 = e1.x * (y1 - e1.y * asum);  // s * (sum A (128 + q) - (128 + z) sum A)
      y2 = e2.x * (y2 - e2.y * asum);
      epilogue(X, L, op, E, slot, tile, n, y1, y2);
    }
    red_par ^= 1;
  }
  X.n_used = gbase;
}
// (C <= AREG_C * NC * 128 is required by llj_engine_step: only the down projection takes the long-K form)
__device__ __forceinline__ void consume(Ctx& X, const Lds& L, const float2* eop, int op, float asum, int& red_par,
                                        Epi& E) {
  if (op == OP_SW) consume_t<2, true>(X, L, eop, op, asum, red_par, E);
  else if (op == OP_DOWN) consume_t<1, false>(X, L, eop, op, asum, red_par, E);
  else consume_t<1, true>(X, L, eop, op, asum, red_par, E);
}

// Attention of this CU's unit (head h, dims 16 j + [0, 16)) for the token at position p
// (model.py:237, SDPA with scale 1 / sqrt(hs) over the valid keys): the q / k / v slices are in LDS
// from the QKV epilogue. 1) every consumer thread takes keys kk = t + 64 NC r: the partial score
// q . k over the 16 dims (cache rows of earlier positions; slot p % S is this step's and is
// skipped, the current key comes from LDS) -> one granule per (key, slice) in this head's score
// region; 2) the J partials of each key are read back from the head's J CUs and summed in slice
// order, so every CU of the head holds the bitwise-same scores; 3) softmax in fp32 (exp2 of
// log2(e)-scaled scores) and P.V over this CU's 16 value dims (kept in registers since step 1);
// 4) y slice -> bf16 -> 8 granules of y.
// The cache rows of this thread's first key (kk = t < 64 NC), loaded at the start of the layer's QKV
// op so their memory latency hides under the QKV tiles: [K lo, K hi, V lo, V hi]
__device__ __forceinline__ void kv_prefetch(const Ctx& X, const llj_engine_plan& P, int l, int p, u32x4 (&pre)[4]) {
  const Shape& s = X.s;
  const int J = s.J, h = s.unit / J, j = s.unit % J, hs = s.hs, Sc = s.S;
  const int nprev = p < Sc ? p : Sc - 1, cur_slot = p % Sc;
  const int t = X.wave * 64 + X.lane;
  const int ki = t < nprev ? t : 0;
  const int slot = p < Sc ? ki : (ki < cur_slot ? ki : ki + 1);
  const size_t off = ((size_t)h * Sc + slot) * hs + 16 * j;
  const u32x4* kp = reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(P.layers[l].kcache) + off);
  const u32x4* vp = reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(P.layers[l].vcache) + off);
  pre[0] = kp[0];
  pre[1] = kp[1];
  pre[2] = vp[0];
  pre[3] = vp[1];
}

template <int HS>
__device__ __forceinline__ void attention_dims(Ctx& X, const Lds& L, const llj_engine_plan& P, const Arena& ar, int l, int p,
                                            unsigned tag, const u32x4 (&pre)[4]) {
  const Shape& s = X.s;
  constexpr int J = HS / 16;
  const int u = s.unit, h = u / J, j = u % J;
  const int Sc = s.S;
  const int nprev = p < Sc ? p : Sc - 1;  // earlier positions still in the window
  const int NK = nprev + 1;
  const int cur_slot = p % Sc;
  const float* aq = L.att;
  const float* ak = aq + 16;
  const float* av = ak + 16;
  float* s_m = L.att + 48;
  float* s_l = s_m + NC;
  float* s_o = s_l + NC;  // [NC][16]
  const int t = X.wave * 64 + X.lane;
  const bf16_t* kc = reinterpret_cast<const bf16_t*>(P.layers[l].kcache) + (size_t)h * Sc * HS + 16 * j;
  const bf16_t* vc = reinterpret_cast<const bf16_t*>(P.layers[l].vcache) + (size_t)h * Sc * HS + 16 * j;
  unsigned long long* gs = ar.gsc + (size_t)h * J * kMaxS;  // [key][J]
  u32x4 kr[kKPT][2], vr[kKPT][2];
  kr[0][0] = pre[0];
  kr[0][1] = pre[1];
  vr[0][0] = pre[2];
  vr[0][1] = pre[3];
#pragma unroll
  for (int r = 1; r < kKPT; ++r) {  // cache rows (32 B of K and of V per key) past the prefetched one, branch-free
    const int kk = t + 64 * NC * r;
    const int ki = kk < nprev ? kk : 0;
    const int slot = p < Sc ? ki : (ki < cur_slot ? ki : ki + 1);
    const u32x4* kp = reinterpret_cast<const u32x4*>(kc + (size_t)slot * HS);
    const u32x4* vp = reinterpret_cast<const u32x4*>(vc + (size_t)slot * HS);
    kr[r][0] = kp[0];
    kr[r][1] = kp[1];
    vr[r][0] = vp[0];
    vr[r][1] = vp[1];
  }
  float q[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) q[d] = aq[d];
#pragma unroll
  for (int r = 0; r < kKPT; ++r) {
    const int kk = t + 64 * NC * r;
    float sc = 0.f;
    if (kk == nprev) {  // the current key (this step's k: not read back from the cache)
#pragma unroll
      for (int d = 0; d < 16; ++d) sc += q[d] * ak[d];
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t wv = kr[r][i >> 2][i & 3];
        sc += q[2 * i] * bflo(wv) + q[2 * i + 1] * bfhi(wv);
      }
    }
    if (kk < NK) st_gran(gs + (size_t)kk * J + j, tag, __float_as_uint(sc));
  }
  if (X.wave == 0 && l < 8) stamp(P, X.lane, 2 + 12 * l + 9);
  // the head's J partials of every key, summed in slice order
  float sfull[kKPT];
#pragma unroll
  for (int r = 0; r < kKPT; ++r) {
    const int kk = t + 64 * NC * r;
    const int ki = kk < NK ? kk : 0;
    unsigned long long v[J];
    unsigned it = 0;
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int jj = 0; jj < J; ++jj) v[jj] = ld_gran(gs + (size_t)ki * J + jj);
#pragma unroll
      for (int jj = 0; jj < J; ++jj) ok &= kk >= NK || (unsigned)(v[jj] >> 32) == tag;
      if (__all(ok)) break;
      if (spin_fail(X, it)) break;
    }
    float a = 0.f;
#pragma unroll
    for (int jj = 0; jj < J; ++jj) a += __uint_as_float((uint32_t)v[jj]);
    sfull[r] = kk < NK ? a : -INFINITY;
  }
  // softmax over the NK keys and P.V over this CU's 16 dims: every wave against its own running max
  // (flash-style partials (max, sum, o[16]) in LDS), merged by wave 0 in wave order -- one barrier
  float mx = -INFINITY;
#pragma unroll
  for (int r = 0; r < kKPT; ++r) mx = fmaxf(mx, sfull[r]);
  mx = wave_max(mx);
  float lsum = 0.f, o[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) o[d] = 0.f;
#pragma unroll
  for (int r = 0; r < kKPT; ++r) {
    const int kk = t + 64 * NC * r;
    const float e = kk < NK ? exp2f(sfull[r] - mx) : 0.f;
    lsum += e;
    if (kk == nprev) {
#pragma unroll
      for (int d = 0; d < 16; ++d) o[d] += e * av[d];
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t wv = vr[r][i >> 2][i & 3];
        o[2 * i] += e * bflo(wv);
        o[2 * i + 1] += e * bfhi(wv);
      }
    }
  }
  lsum = wave_sum(lsum);
#pragma unroll
  for (int d = 0; d < 16; ++d) o[d] = wave_sum(o[d]);
  if (X.lane == 0) {
    s_m[X.wave] = mx;
    s_l[X.wave] = lsum;
#pragma unroll
    for (int d = 0; d < 16; ++d) s_o[X.wave * 16 + d] = o[d];
  }
  cbarrier(X, L);
  if (X.wave == 0) {
    const int d = X.lane & 15;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NC; ++w) M = fmaxf(M, s_m[w]);
    float Ls = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < NC; ++w) {
      const float f = s_m[w] == -INFINITY ? 0.f : exp2f(s_m[w] - M);  // a wave without keys: -inf, weight 0
      Ls += s_l[w] * f;
      O += s_o[w * 16 + d] * f;
    }
    const uint32_t ob = (uint32_t)f2bf(O / Ls);
    const uint32_t pr = lane_xor1(ob);
    if (X.lane < 16 && !(X.lane & 1)) st_gran(ar.gy + (h * HS + 16 * j + d) / 2, tag, ob | (pr << 16));
  }
}

// ------------------------------------------------------------------------------------ loader
// Streams every block of this CU's step into the ring, in consumption order (tile-major: for each
// tile, its chunks, SwiGLU's two matrices interleaved per chunk). Slot b % nb is reused once every
// consumer's next block is past b - nb. One wave issues everything, so the issue sequence IS the
// stream rate: runs of 8 blocks go out as one asm block (saddr = matrix base, 32-bit VGPR offsets,
// M0 stepped in place: ~4.5 instructions per 1 KiB DMA); a general
// per-block sequence of ~25 dependent instructions held the wave to ~12 GB/s per CU where the
// memory system gives ~25 (tools/engine_trace.py probes, tools/micro/loader_probe.hip).
constexpr int LG = 8;
static_assert(D % LG == 0, "publish granularity");
// wait until at most (n rounded down to a multiple of 8) DMAs of this wave are in flight
__device__ __forceinline__ void wait_vm_le(int n) {
  switch (n >> 3) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<8>(); break;
    case 2: wait_vm<16>(); break;
    case 3: wait_vm<24>(); break;
    case 4: wait_vm<32>(); break;
    case 5: wait_vm<40>(); break;
    case 6: wait_vm<48>(); break;
    default: wait_vm<56>(); break;
  }
}
// one 1 KiB block: base + voff (per lane 16 B) -> LDS dst
__device__ __forceinline__ void dma1(const char* base, uint32_t voff, uint32_t dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(base), "s"(dst)
               : "memory");
}
#define LLJ_DMA_NEXT "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
// 8 consecutive blocks of one matrix into 8 consecutive slots. Per-DMA VGPR offsets, no immediate
// offsets: an LDS-DMA's immediate offset also moves its LDS destination (measured,
// tools/micro/glds_offset_probe.hip), so M0 alone steps the slots.
__device__ __forceinline__ void dma8_1(const char* base, uint32_t voff, uint32_t dst) {
  unsigned keep, t1, t2, t3, t4, t5, t6, t7;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %10\n\t"
               "v_add_u32 %1, 0x400, %8\n\tv_add_u32 %2, 0x800, %8\n\tv_add_u32 %3, 0xc00, %8\n\t"
               "v_add_u32 %4, 0x1000, %8\n\tv_add_u32 %5, 0x1400, %8\n\tv_add_u32 %6, 0x1800, %8\n\t"
               "v_add_u32 %7, 0x1c00, %8\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %8, %9 nt\n\t" LLJ_DMA_NEXT
               "global_load_lds_dwordx4 %1, %9 nt\n\t" LLJ_DMA_NEXT
               "global_load_lds_dwordx4 %2, %9 nt\n\t" LLJ_DMA_NEXT
               "global_load_lds_dwordx4 %3, %9 nt\n\t" LLJ_DMA_NEXT
               "global_load_lds_dwordx4 %4, %9 nt\n\t" LLJ_DMA_NEXT
               "global_load_lds_dwordx4 %5, %9 nt\n\t" LLJ_DMA_NEXT
               "global_load_lds_dwordx4 %6, %9 nt\n\t" LLJ_DMA_NEXT
               "global_load_lds_dwordx4 %7, %9 nt\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep), "=&v"(t1), "=&v"(t2), "=&v"(t3), "=&v"(t4), "=&v"(t5), "=&v"(t6), "=&v"(t7)
               : "v"(voff), "s"(base), "s"(dst)
               : "memory", "scc");
}
// 4 consecutive chunks of two matrices, interleaved per chunk, into 8 consecutive slots
__device__ __forceinline__ void dma8_2(const char* b0, const char* b1, uint32_t voff, uint32_t dst) {
  unsigned keep, t1, t2, t3;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %7\n\t"
               "v_add_u32 %1, 0x400, %4\n\tv_add_u32 %2, 0x800, %4\n\tv_add_u32 %3, 0xc00, %4\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %4, %5 nt\n\t" LLJ_DMA_NEXT
               "global_load_lds_dwordx4 %4, %6 nt\n\t" LLJ_DMA_NEXT
               "global_load_lds_dwordx4 %1, %5 nt\n\t" LLJ_DMA_NEXT
               "global_load_lds_dwordx4 %1, %6 nt\n\t" LLJ_DMA_NEXT
               "global_load_lds_dwordx4 %2, %5 nt\n\t" LLJ_DMA_NEXT
               "global_load_lds_dwordx4 %2, %6 nt\n\t" LLJ_DMA_NEXT
               "global_load_lds_dwordx4 %3, %5 nt\n\t" LLJ_DMA_NEXT
               "global_load_lds_dwordx4 %3, %6 nt\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep), "=&v"(t1), "=&v"(t2), "=&v"(t3)
               : "v"(voff), "s"(b0), "s"(b1), "s"(dst)
               : "memory", "scc");
}
#undef LLJ_DMA_NEXT

__device__ __forceinline__ void loader(Ctx& X, const Lds& L, const llj_engine_plan& P) {
  const Shape& s = X.s;
  const uint32_t ring = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)L.ring);
  const int nb = L.nb;  // a multiple of 8
  const bool free_run = (P.flags & 2) != 0;  // profiling: stream the step with no consumers
  const uint32_t lane16 = 16u * (uint32_t)X.lane;
  stamp(P, X.lane, 121);
  if (P.flags & 4) {  // profiling: consumers alone (every block "landed", nothing streamed; results invalid)
    if (X.lane == 0) lds_st(L.ctl + 0, 0x7fffffffu);
    return;
  }
  int b = 0, slot = 0;
  int pub = 0;    // blocks published as landed
  int limit = nb; // blocks that may be issued before the consumers' counts are read again
  int opi = 0;
  for (int l = 0; l <= s.L; ++l) {
    for (int op = (l == s.L ? OP_HEAD : OP_QKV); op <= (l == s.L ? OP_HEAD : OP_DOWN); ++op) {
      const int nt = tiles_of_cu(s, op), kc = op_kc(s, op), nm = op_nmat(op);
      const char* w0 = op_weight(P, l, op, 0);
      const char* w1 = op_weight(P, l, op, nm - 1);
      const int per_tile = kc * nm;
      for (int j = 0; j < nt; ++j) {
        const uint32_t toff = (uint32_t)tile_of(s, op, j) * (uint32_t)kc * 1024u;  // the tile's first chunk
        for (int r0 = 0; r0 < per_tile; r0 += LG) {
          const int n = per_tile - r0 < LG ? per_tile - r0 : LG;
          if (!free_run && b + n > limit) {
            // every block below F = min over consumers of their next block has been taken:
            // slots of blocks < F are free, so blocks < F + nb may be issued
            unsigned it = 0;
            for (;;) {
              int F = 0x7fffffff;
#pragma unroll
              for (int w = 0; w < NC; ++w) {
                const int f = (int)lds_ld(L.ctl + 1 + w);
                F = f < F ? f : F;
              }
              limit = F + nb;
              if (limit >= b + n) break;
              // ring full. A consumer waiting for an unpublished block (ctl[17]: the highest block
              // any consumer has waited for) gets the oldest group in flight published (a wait for
              // just those DMAs); draining the whole window here instead would make every
              // ring-bound phase stop-and-go at one DMA latency per group
              const int want = (int)lds_ld(L.ctl + 17);
              if (want >= pub && pub < b) {
                const int keep_n = b - pub > LG ? b - pub - LG : 0;
                const int kq = ((keep_n >> 3) << 3) < 56 ? ((keep_n >> 3) << 3) : 56;
                wait_vm_le(kq);
                pub = b - kq;
                if (X.lane == 0) lds_st(L.ctl + 0, (unsigned)pub);
              }
              if (spin_fail_loader(X, it)) { limit = b + nb; break; }
            }
          }
          if (n == LG && slot + LG <= nb) {
            const uint32_t dst = ring + (uint32_t)slot * 1024u;
            if (nm == 1) dma8_1(w0, toff + (uint32_t)r0 * 1024u + lane16, dst);
            else dma8_2(w0, w1, toff + (uint32_t)(r0 >> 1) * 1024u + lane16, dst);
            slot += LG;
            if (slot == nb) slot = 0;
          } else {
            for (int u = 0; u < n; ++u) {
              const int r = r0 + u;
              const int c = nm == 1 ? r : r >> 1;
              dma1((nm == 2 && (r & 1)) ? w1 : w0, toff + (uint32_t)c * 1024u + lane16, ring + (uint32_t)slot * 1024u);
              if (++slot == nb) slot = 0;
            }
          }
          b += n;
          if (b - pub >= D + LG) {  // publish: all but the newest D have landed
            wait_vm<D>();
            pub = b - D;
            if (X.lane == 0) lds_st(L.ctl + 0, (unsigned)pub);
          }
        }
      }
      if (opi < 8) stamp(P, X.lane, 100 + opi);
      ++opi;
    }
  }
  wait_vm<0>();
  if (X.lane == 0) lds_st(L.ctl + 0, (unsigned)b);
  stamp(P, X.lane, 120);
}

// ------------------------------------------------------------------------------------ kernel
__global__ __launch_bounds__(NTH, 1) void engine_step_kernel(llj_engine_plan P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  Ctx X;
  Shape& s = X.s;
  s.C = P.C; s.H = P.H; s.V = P.V; s.nh = P.n_head; s.hs = P.C / P.n_head; s.S = P.S; s.L = P.n_layer;
  s.G = gridDim.x; s.g = blockIdx.x;
  s.J = s.hs / 16;
  s.unit = unit_of_cu(s.g, s.G, s.nh, s.J);
  X.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  X.lane = threadIdx.x & 63;
  X.aborted = false;
  X.bar_gen = 0;
  X.n_used = 0;
  X.landed = 0;
  X.stamp_base = -1;
  X.plan = &P;
  X.t0 = __builtin_amdgcn_s_memrealtime();
  const int C = s.C, H = s.H;
  Lds L;
  {
    size_t o = 0;
    L.ctl = reinterpret_cast<unsigned*>(smem);
    o += kCtlWords * 4;
    L.A = reinterpret_cast<bf16_t*>(smem + o);
    o += al16((size_t)(C > H ? C : H) * 2);
    L.xown[0] = reinterpret_cast<bf16_t*>(smem + o);
    o += 32;
    L.xown[1] = reinterpret_cast<bf16_t*>(smem + o);
    o += 32;
    L.red = reinterpret_cast<float*>(smem + o);
    o += (size_t)2 * NC * TG * 2 * 16 * 4;
    L.eop = reinterpret_cast<float2*>(smem + o);
    o += (size_t)2 * kEopTiles * 2 * 16 * 8;
    L.misc = reinterpret_cast<float*>(smem + o);
    o += 80 * 4;
    L.att = reinterpret_cast<float*>(smem + o);
    o += al16((size_t)kAttFloats * 4);
    L.ring = smem + o;
    L.nb = P.ring_blocks;
    L.nb_magic = (unsigned)((0x100000000ull + (unsigned)L.nb - 1) / (unsigned)L.nb);
  }
  const Arena ar = arena_of(P);
  X.gctl = ar.ctl;
  if (threadIdx.x < kCtlWords) L.ctl[threadIdx.x] = 0u;
  __syncthreads();  // the only full-workgroup barrier: control words zeroed before any role starts
  if (X.wave == NC) {
    loader(X, L, P);
    return;
  }
  if (P.flags & 2) return;  // profiling (loader-only stream rate): no step state is touched
  // ---- consumers. Step state written by the previous step (an earlier launch).
  if (X.wave == 0) stamp(P, X.lane, 0);
  const unsigned epoch = ar.ctl[0];
  const int p = P.pos[0] + 1;  // position of the token this step processes
  const int tok = P.cur[0];
  int red_par = 0;
  const int hs = s.hs;
  Epi E;
  E.ar = ar;
  E.slot = p % s.S;
  E.logits = reinterpret_cast<bf16_t*>(P.logits);
  E.best = 0;
  // epilogue-operand buffers alternate per op (QKV 0, c_proj 1, SwiGLU 0, down 1, lm_head 0)
  float2* rcs = L.eop + kEopTiles * 2 * 16 - 8 * TG;  // RoPE (cos, sin) per QKV tile slot (<= TG per CU)
  E.rcs = rcs;
  u32x4 kvpre[4] = {};  // this thread's first key's cache rows (kv_prefetch at the QKV op)
  // One loop over (layer, op) -- every stage, consume and epilogue is in the code once (the
  // instruction cache holds the whole step's working set).
  for (int i = 0; i <= 4 * s.L; ++i) {
    const int l = i >> 2;
    const int op = i == 4 * s.L ? OP_HEAD : (i & 3);
    const llj_engine_layer* Ly = op == OP_HEAD ? nullptr : &P.layers[l];
    const unsigned tag = epoch * 128u + (unsigned)l + 1u;  // this layer's granules
    const unsigned tag_prev = epoch * 128u + (unsigned)l;  // x from the previous layer's down tiles
    const int sb = 2 + 12 * l;                             // this layer's stamps (profiling)
    E.tag = tag;
    float2* eop = L.eop + (op & 1) * kEopTiles * 2 * 16;
    if (op == OP_O) {
      if (X.wave == 0 && l < 8) stamp(P, X.lane, sb + 1);
      if (s.unit >= 0) {  // attention of this CU's (head, 16-dim slice) unit
        cbarrier(X, L);   // the QKV epilogue's q / k / v slices are in LDS
        if (hs == 128) attention_dims<128>(X, L, P, ar, l, p, tag, kvpre);
        else attention_dims<64>(X, L, P, ar, l, p, tag, kvpre);
      }
      if (X.wave == 0 && l < 8) stamp(P, X.lane, sb + 2);
    } else if (X.wave == 0 && l < 8 && op != OP_QKV) {
      stamp(P, X.lane, sb + (op == OP_SW ? 4 : 6));
    }
    stage_sz(X, eop, P, l, op);
    if (op == OP_QKV) {
      E.kcache = reinterpret_cast<bf16_t*>(Ly->kcache);
      E.vcache = reinterpret_cast<bf16_t*>(Ly->vcache);
      const int nt = tiles_of_cu(s, OP_QKV);
      for (int k = X.lane + 64 * X.wave; k < nt * 8 && k < 8 * TG; k += 64 * NC) {
        const int j = k >> 3, pr = k & 7;
        const int n = 16 * tile_of(s, OP_QKV, j) + 2 * pr;
        const int dd = (n % C) % hs;
        rcs[k] = *reinterpret_cast<const float2*>(P.rope + ((size_t)p * (hs >> 1) + (dd >> 1)) * 2);
      }
    }
    const bool norm = op == OP_QKV || op == OP_SW || op == OP_HEAD;
    const unsigned long long* g = op == OP_QKV || op == OP_HEAD ? ar.gx : op == OP_O ? ar.gy : op == OP_SW ? ar.gxm : ar.gh;
    const unsigned gtag = op == OP_QKV || op == OP_HEAD ? tag_prev : tag;
    const bf16_t* direct = op == OP_QKV && l == 0 ? reinterpret_cast<const bf16_t*>(P.wte) + (size_t)tok * C : nullptr;
    const void* gain = op == OP_QKV ? Ly->rms1 : op == OP_SW ? Ly->rms2 : P.ln_f;
    const float eps = op == OP_QKV ? Ly->eps1 : op == OP_SW ? Ly->eps2 : P.eps_f;
    const float asum = stage(X, L, norm, op == OP_SW ? 1 : 0, g, gtag, direct, reinterpret_cast<const bf16_t*>(gain), eps,
                             op == OP_DOWN ? H : C);
    if (X.wave == 0 && l < 8 && op != OP_HEAD) stamp(P, X.lane, sb + 2 * op + (op == OP_QKV ? 0 : 1));
    if (op == OP_HEAD && X.wave == 0) stamp(P, X.lane, 126);
    X.stamp_base = (l < 2 && (op == OP_SW || op == OP_QKV)) ? 108 + 3 * (2 * l + (op == OP_SW)) : -1;
    if (op == OP_QKV && s.unit >= 0) kv_prefetch(X, P, l, p, kvpre);  // lands while the QKV tiles run
    consume(X, L, eop, op, asum, red_par, E);
    if (X.wave == 0 && l < 8 && op == OP_DOWN) stamp(P, X.lane, sb + 8);
  }
  if (X.wave == 0) stamp(P, X.lane, 127);
  // CU best over its consumer waves -> one granule; the last CU to arrive picks the token
  const unsigned tag_head = epoch * 128u + 127u;
  uint32_t b = E.best;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) b = max(b, (uint32_t)__shfl_xor((int)b, o, 64));
  unsigned* mb = reinterpret_cast<unsigned*>(L.misc) + 32;
  if (X.lane == 0) mb[X.wave] = b;
  cbarrier(X, L);
  if (X.wave == 0 && X.lane == 0) {
    uint32_t cb = 0;
#pragma unroll
    for (int w = 0; w < NC; ++w) cb = max(cb, mb[w]);
    st_gran(ar.garg + s.g, tag_head, cb);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(ar.ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    mb[16] = (t + 1 == (unsigned)s.G) ? 1u : 0u;
  }
  if (X.wave != 0) return;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lds_ld(mb + 16) != 1u) return;
  uint32_t tb = 0;
  for (int b0 = 0; b0 < s.G; b0 += 64) {
    const int idx = b0 + X.lane;
    unsigned long long v;
    unsigned it = 0;
    for (;;) {
      v = ld_gran(ar.garg + (idx < s.G ? idx : 0));
      if (__all(idx >= s.G || (unsigned)(v >> 32) == tag_head)) break;
      if (spin_fail(X, it)) break;
    }
    if (idx < s.G) tb = max(tb, (uint32_t)v);
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) tb = max(tb, (uint32_t)__shfl_xor((int)tb, o, 64));
  if (X.lane == 0) {
    const int next = (int)(0xFFFFu - (tb & 0xFFFFu));
    if (P.flags & 1) {  // greedy (generate.py:66-74 with top_k = 1)
      P.cur[0] = next;
      if (P.tokens) P.tokens[p + 1] = next;
    }
    P.pos[0] = p;
    ar.ctl[1] = 0u;
    ar.ctl[0] = epoch + 1u;
  }
}

}  // namespace eng
}  // namespace llj

using namespace llj;

extern "C" {

size_t llj_engine_arena_bytes(int C, int H) { return eng::arena_granules(C, H) * 8 + 64; }

int llj_engine_ring_blocks(int C, int H, int n_head) {
  if (n_head < 1 || C % n_head) return 0;
  return eng::ring_blocks(C, H, 160 * 1024);
}

int llj_engine_step(const llj_engine_plan* plan, void* stream) {
  if (!plan) return LLJ_EINVAL;
  const llj_engine_plan& P = *plan;
  const int hs = P.n_head > 0 ? P.C / P.n_head : 0;
  LLJ_REQUIRE(P.layers && P.n_layer >= 1 && P.n_layer <= 126 && P.C % 128 == 0 && P.H % 128 == 0 && P.V % 16 == 0);
  LLJ_REQUIRE(P.V <= 65536 && (hs == 64 || hs == 128) && P.S >= 1 && P.S <= eng::kMaxS && P.arena && P.pos && P.cur &&
              P.logits);
  LLJ_REQUIRE(P.C / 2 <= eng::GN * 64 * eng::NC && P.C / 2 <= 64 * eng::NC * eng::GK);  // stage's gain registers, one gather batch
  LLJ_REQUIRE(P.C <= eng::AREG_C * eng::NC * 128 && P.H <= 32 * 64 * eng::NC);  // A of the K = C ops in registers; stage's map
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return LLJ_EINVAL;
  const int G = P.grid > 0 ? P.grid : cus;
  LLJ_REQUIRE(G >= 1 && G <= cus && G <= eng::kMaxCUs);
  // one QKV unit (head, 16-dim slice) per CU at most; kEopTiles tiles per op
  LLJ_REQUIRE(P.C / 16 <= G && (P.V / 16 + G - 1) / G <= eng::kEopTiles && (P.H / 16 + G - 1) / G <= eng::kEopTiles);
  const int nb = eng::ring_blocks(P.C, P.H, 160 * 1024);
  LLJ_REQUIRE(P.ring_blocks >= 2 * eng::D && P.ring_blocks <= nb && P.ring_blocks % eng::LG == 0);
  const size_t lds = eng::lds_fixed(P.C, P.H) + (size_t)P.ring_blocks * 1024;
  LLJ_REQUIRE(lds <= 160 * 1024 && lds > 80 * 1024);  // one workgroup per CU, every one resident
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)eng::engine_step_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  hipLaunchKernelGGL(eng::engine_step_kernel, dim3(G), dim3(eng::NTH), lds, (hipStream_t)stream, P);
  LLJ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

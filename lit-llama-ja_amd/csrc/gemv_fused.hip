// Multi-op launches of the decode layer (ops of one layer sharing a grid, chained through
// completion counters, chain.h): llj_attn_resid (attention + attn.c_proj) and
// llj_decode_layer (the whole layer; measured slower, off by default).
#include "gemv_impl.h"

namespace llj {

// ------------------------------------------------------------------------------------
// One decode layer as ONE launch (llj_decode_layer): the grid holds, in order,
//   [QKV 3C/16] [attention n_head*M] [c_proj C/16] [fc1/fc2 H/16] [mlp.c_proj C/16]
// workgroups. Each op's workgroups start their weight stream, then wait for the previous
// op's completion counter (chain.h); a workgroup only waits for lower-numbered ones, which
// the in-order dispatch has already placed, so the chain cannot deadlock.
struct LayerChain {
  GemvParams qkv, cproj, fc12, down;
  const bf16_t* q;
  const bf16_t* kc;
  const bf16_t* vc;
  bf16_t* y;
  const int* pos;
  int S, nh;
  float sl2;
  int b_att, b_cproj, b_fc12, b_down, n_qkv, n_att, n_cproj, n_fc12;
  int has_down;
  unsigned* ctr;  // [4 ops][kCtrWords] (chain.h)
  unsigned* err;
};

constexpr int kAttU = 8;  // attention keys per group per pass in the chained launch (256 threads)

template <int WF, int MB, int HS>
__global__ __launch_bounds__(256) void layer_chain_kernel(LayerChain c) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int bid = blockIdx.x;
  unsigned* const k0 = c.ctr;  // counter blocks: QKV, attention, c_proj, fc1/fc2
  unsigned* const k1 = c.ctr + kCtrWords;
  unsigned* const k2 = c.ctr + 2 * kCtrWords;
  unsigned* const k3 = c.ctr + 3 * kCtrWords;
  if (bid < c.b_att) {
    gemv_body<WF, AM_NORM, EP_QKV, kNW, kD, MB, true>(c.qkv, bid, smem,
                                                      ChainCtl{nullptr, 0, k0, c.n_qkv, c.err, bid});
  } else if (bid < c.b_cproj) {
    const int local = bid - c.b_att;
    attention_body<HS, kAttU, 256, true>(c.q, c.kc, c.vc, c.y, c.pos, 1, c.S, c.nh, c.sl2, local % c.nh, local / c.nh,
                                         reinterpret_cast<float*>(smem),
                                         ChainCtl{k0, c.n_qkv, k1, c.n_att, c.err, local});
  } else if (bid < c.b_fc12) {
    const int local = bid - c.b_cproj;
    gemv_body<WF, AM_LDS, EP_RESID, kNW, kD, MB, true>(c.cproj, local, smem,
                                                       ChainCtl{k1, c.n_att, k2, c.n_cproj, c.err, local});
  } else if (!c.has_down || bid < c.b_down) {
    const int local = bid - c.b_fc12;
    gemv_body<WF, AM_NORM, EP_SWIGLU, kNW, kD, MB, true>(c.fc12, local, smem,
                                                         ChainCtl{k2, c.n_cproj, c.has_down ? k3 : nullptr,
                                                                  c.n_fc12, c.err, local});
  } else {
    const int local = bid - c.b_down;
    gemv_body<WF, AM_LDS, EP_RESID, kNW, kD, MB, true>(c.down, local, smem,
                                                       ChainCtl{k3, c.n_fc12, nullptr, 0, c.err, local});
  }
}

// Does the register-staged prologue (the only one the chained path reads sc1) take this op?
static bool chain_prologue_ok(int am, int M, int K, int nst_parts) {
  const int MB = M == 1 ? 1 : 8;
  const bool norm = am == AM_NORM;
  const int NT = kNW * 64, JA = (K / 8 + NT - 1) / NT;
  const int XR = MB == 1 ? (norm ? 4 : 8) : 16, GR = norm ? 4 : 1, SM = MB == 1 ? 1 : 8, ST = MB == 1 ? 2 : 8;
  if (M > 8) return false;
  if (norm && nst_parts > 0 && nst_parts > ST * (NT / SM)) return false;
  if (norm && JA > GR) return false;
  if (MB == 1) return JA <= XR;
  return JA <= 2 || (JA <= 4 && M <= 4);
}

template <int WF, int MB, int HS>
static int launch_chain(const LayerChain& c, size_t lds, int grid, hipStream_t s) {
  auto kern = layer_chain_kernel<WF, MB, HS>;
  static bool attr_set = false;
  if (lds > 64 * 1024 && !attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, s, c);
  LLJ_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------
// attention + attn.c_proj (+ residual) as ONE launch (llj_attn_resid): the grid holds
//   [attention n_head*M workgroups] [c_proj C/16 workgroups].
// Attention reads a few KB per workgroup and leaves the rest of the chip (and HBM) idle for
// its whole duration; the c_proj workgroups use that window: each issues its ENTIRE weight
// slice (D = KC / NW chunks per wave, all in registers) before it waits for the attention
// completion counter (chain.h protocol), so the c_proj weight stream overlaps attention and
// the boundary between the two launches disappears. QKV (the attention's producer) is the
// previous launch: attention reads q / k / v with plain loads and only signals.
struct AttnResid {
  GemvParams proj;
  const bf16_t* q;
  const bf16_t* kc;
  const bf16_t* vc;
  bf16_t* y;
  const int* pos;
  int S, nh, n_att;
  float sl2;
  unsigned* ctr;  // kCtrWords, zeroed by the caller before the launch
  unsigned* err;
};

template <int WF, int MB, int HS, int DP>
__global__ __launch_bounds__(256) void attn_resid_kernel(AttnResid c) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int bid = blockIdx.x;
  if (bid < c.n_att) {
    attention_body<HS, kAttU, 256, false, true>(c.q, c.kc, c.vc, c.y, c.pos, 1, c.S, c.nh, c.sl2, bid % c.nh,
                                                 bid / c.nh, reinterpret_cast<float*>(smem),
                                                 ChainCtl{nullptr, 0, c.ctr, c.n_att, c.err, bid});
  } else {
    const int local = bid - c.n_att;
    gemv_body<WF, AM_LDS, EP_RESID, kNW, DP, MB, true>(c.proj, local, smem,
                                                       ChainCtl{c.ctr, c.n_att, nullptr, 0, c.err, local});
  }
}

template <int WF, int MB, int HS, int DP>
static int launch_attn_resid(const AttnResid& c, size_t lds, int grid, hipStream_t s) {
  auto kern = attn_resid_kernel<WF, MB, HS, DP>;
  static bool attr_set = false;
  if (lds > 64 * 1024 && !attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, s, c);
  LLJ_CHECK_LAUNCH();
  return 0;
}

}  // namespace llj

using namespace llj;

extern "C" {
LLJ_TRACE_EXPORT(fused)

// y = attention(q, caches) (llj_attention, T = 1 decode rows) and x[M, C] += y . W_proj^T
// (llj_linear_resid) in one launch; results bitwise equal to the two launches.
int llj_attn_resid(int wfmt, const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int M,
                   int n_head, int S, const void* W, const void* sz, void* x, int C, double* nstat_out,
                   unsigned* counters, unsigned* err, void* stream) {
  if (M < 1 || M > 8 || n_head < 1 || C % n_head || S < 1 || !counters || !err) return LLJ_EINVAL;
  if (wfmt != WF_W4 && wfmt != WF_BF16 && wfmt != WF_W8) return LLJ_EINVAL;
  const int hs = C / n_head;
  if (hs != 64 && hs != 128) return LLJ_EINVAL;
  AttnResid c{};
  GemvParams& pr = c.proj;
  pr.A = (const bf16_t*)y; pr.lda = C; pr.M = M; pr.N = C; pr.K = C; pr.W = W;
  pr.sz = (const float2*)sz; pr.C = (bf16_t*)x; pr.ldc = C; pr.nst_out = nstat_out;
  if (check_shape(wfmt, pr) || !chain_prologue_ok(AM_LDS, M, C, 0)) return LLJ_EINVAL;
  const int KC = C / 128;
  // every chunk of a wave in flight before the wait: D = ceil(KC / NW), instantiated for
  // 7B / 13B (K = 4096 / 5120: 8 / 10 chunks per wave) and smaller models (<= 4)
  const int dneed = (KC + kNW - 1) / kNW;
  if (dneed > 10 && wfmt != WF_BF16) return LLJ_EINVAL;
  c.q = (const bf16_t*)q; c.kc = (const bf16_t*)kcache; c.vc = (const bf16_t*)vcache; c.y = (bf16_t*)y;
  c.pos = pos; c.S = S; c.nh = n_head; c.n_att = n_head * M; c.sl2 = 1.4426950408889634f / sqrtf((float)hs);
  c.ctr = counters; c.err = err;
  const int grid = c.n_att + C / 16;
  size_t lds = gemv_smem(wfmt, AM_LDS, M, C);
  lds = std::max(lds, (size_t)(hs == 128 ? attention_lds_floats<128, 256>() : attention_lds_floats<64, 256>()) * 4);
  hipStream_t st = (hipStream_t)stream;
#define LLJ_AR(WF_, MB_, HS_)                                                         \
  (dneed <= 4 ? launch_attn_resid<WF_, MB_, HS_, 4>(c, lds, grid, st)                  \
   : dneed <= 8 ? launch_attn_resid<WF_, MB_, HS_, 8>(c, lds, grid, st)                \
                : launch_attn_resid<WF_, MB_, HS_, 10>(c, lds, grid, st))
#define LLJ_AR_HS(WF_, MB_) (hs == 128 ? LLJ_AR(WF_, MB_, 128) : LLJ_AR(WF_, MB_, 64))
  if (wfmt == WF_W4) return M == 1 ? LLJ_AR_HS(WF_W4, 1) : LLJ_AR_HS(WF_W4, 8);
  if (wfmt == WF_W8) return M == 1 ? LLJ_AR_HS(WF_W8, 1) : LLJ_AR_HS(WF_W8, 8);
  // bf16: 4 KiB per wave-chunk, the usual D = 4 chunks in flight (no register room for all)
  if (M == 1) return hs == 128 ? launch_attn_resid<WF_BF16, 1, 128, 4>(c, lds, grid, st)
                               : launch_attn_resid<WF_BF16, 1, 64, 4>(c, lds, grid, st);
  return hs == 128 ? launch_attn_resid<WF_BF16, 8, 128, 4>(c, lds, grid, st)
                   : launch_attn_resid<WF_BF16, 8, 64, 4>(c, lds, grid, st);
#undef LLJ_AR_HS
#undef LLJ_AR
}

int llj_decode_layer(const llj_layer* L, void* stream) {
  if (!L) return LLJ_EINVAL;
  const int M = L->M, C = L->C, H = L->H, nh = L->n_head, wf = L->wfmt;
  if (M < 1 || M > 8 || nh < 1 || C % nh || (wf != WF_W4 && wf != WF_BF16 && wf != WF_W8) || !L->counters ||
      !L->err)
    return LLJ_EINVAL;
  const int hs = C / nh;
  const int parts = C / 16;
  const bool chain = wf != WF_W8 && chain_prologue_ok(AM_NORM, M, C, parts) && chain_prologue_ok(AM_LDS, M, C, 0) &&
                     (hs == 64 || hs == 128) && (M > 1 || chain_prologue_ok(AM_LDS, M, H, 0));
  hipStream_t st = (hipStream_t)stream;
  if (!chain) {  // the same five ops as separate launches
    int e;
    if ((e = llj_norm_qkv_rope(wf, L->x, L->rms1, L->eps, L->w_qkv, L->sz_qkv, L->q, L->kcache, L->vcache, L->rope,
                               L->pos, M, 1, C, nh, L->S, 0, M, nullptr, L->nst_in, L->nst_in_parts, nullptr, stream)))
      return e;
    if ((e = llj_attention(L->q, L->kcache, L->vcache, L->y, L->pos, M, 1, nh, hs, L->S, stream))) return e;
    if ((e = llj_linear_resid(wf, L->y, C, L->w_proj, L->sz_proj, L->x, C, M, C, C, nullptr, 0, L->nst_mid, stream)))
      return e;
    if ((e = llj_norm_swiglu(wf, L->x, L->rms2, L->eps, L->w_fc1, L->sz_fc1, L->w_fc2, L->sz_fc2, L->h, M, H, C,
                             nullptr, 0, L->nst_mid, parts, nullptr, stream)))
      return e;
    return llj_linear_resid(wf, L->h, H, L->w_down, L->sz_down, L->x, C, M, C, H, nullptr, 0, L->nst_out, stream);
  }
  LayerChain c{};
  GemvParams& q = c.qkv;
  q.A = (const bf16_t*)L->x; q.lda = C; q.norm_w = (const bf16_t*)L->rms1; q.eps = L->eps;
  q.M = M; q.m0 = 0; q.N = 3 * C; q.K = C; q.W = L->w_qkv; q.sz = (const float2*)L->sz_qkv;
  q.q_out = (bf16_t*)L->q; q.kcache = (bf16_t*)L->kcache; q.vcache = (bf16_t*)L->vcache; q.rope = L->rope;
  q.pos = L->pos; q.n_head = nh; q.head_size = hs; q.S = L->S; q.T = 1;
  q.nst_in = L->nst_in; q.nst_parts = L->nst_in_parts;
  GemvParams& pr = c.cproj;
  pr.A = (const bf16_t*)L->y; pr.lda = C; pr.M = M; pr.N = C; pr.K = C; pr.W = L->w_proj;
  pr.sz = (const float2*)L->sz_proj; pr.C = (bf16_t*)L->x; pr.ldc = C; pr.nst_out = L->nst_mid;
  GemvParams& f = c.fc12;
  f.A = (const bf16_t*)L->x; f.lda = C; f.norm_w = (const bf16_t*)L->rms2; f.eps = L->eps; f.M = M; f.N = H;
  f.K = C; f.W = L->w_fc1; f.W2 = L->w_fc2; f.sz = (const float2*)L->sz_fc1; f.sz2 = (const float2*)L->sz_fc2;
  f.C = (bf16_t*)L->h; f.ldc = H; f.nst_in = L->nst_mid; f.nst_parts = parts;
  GemvParams& d = c.down;
  d.A = (const bf16_t*)L->h; d.lda = H; d.M = M; d.N = C; d.K = H; d.W = L->w_down;
  d.sz = (const float2*)L->sz_down; d.C = (bf16_t*)L->x; d.ldc = C; d.nst_out = L->nst_out;
  for (const GemvParams* g : {&c.qkv, &c.cproj, &c.fc12, &c.down})
    if (check_shape(wf, *g)) return LLJ_EINVAL;
  if (!L->nst_mid || (L->nst_in && L->nst_in_parts < 1)) return LLJ_EINVAL;
  c.q = (const bf16_t*)L->q; c.kc = (const bf16_t*)L->kcache; c.vc = (const bf16_t*)L->vcache;
  c.y = (bf16_t*)L->y; c.pos = L->pos; c.S = L->S; c.nh = nh; c.sl2 = 1.4426950408889634f / sqrtf((float)hs);
  c.n_qkv = 3 * C / 16; c.n_att = nh * M; c.n_cproj = C / 16; c.n_fc12 = H / 16;
  c.b_att = c.n_qkv; c.b_cproj = c.b_att + c.n_att; c.b_fc12 = c.b_cproj + c.n_cproj; c.b_down = c.b_fc12 + c.n_fc12;
  // M > 1: the (M, H) A image does not fit the LDS; a long-K down op runs with LLJ_NWR waves (not
  // the chain's 4): both as the separate launch below, so results stay those of the five launches
  c.has_down = M == 1 && !(LLJ_NWR != kNW && H >= LLJ_NWR_KMIN);
  c.ctr = L->counters; c.err = L->err;
  const int grid = c.b_down + (c.has_down ? C / 16 : 0);
  size_t lds = gemv_smem(wf, AM_NORM, M, C);
  lds = std::max(lds, gemv_smem(wf, AM_LDS, M, C));
  if (c.has_down) lds = std::max(lds, gemv_smem(wf, AM_LDS, M, H));
  lds = std::max(lds, (size_t)(hs == 128 ? attention_lds_floats<128, 256>() : attention_lds_floats<64, 256>()) * 4);
  if (lds > 160 * 1024) return LLJ_EINVAL;
  int e;
  if (wf == WF_W4) {
    if (M == 1) e = hs == 128 ? launch_chain<WF_W4, 1, 128>(c, lds, grid, st) : launch_chain<WF_W4, 1, 64>(c, lds, grid, st);
    else e = hs == 128 ? launch_chain<WF_W4, 8, 128>(c, lds, grid, st) : launch_chain<WF_W4, 8, 64>(c, lds, grid, st);
  } else {
    if (M == 1) e = hs == 128 ? launch_chain<WF_BF16, 1, 128>(c, lds, grid, st) : launch_chain<WF_BF16, 1, 64>(c, lds, grid, st);
    else e = hs == 128 ? launch_chain<WF_BF16, 8, 128>(c, lds, grid, st) : launch_chain<WF_BF16, 8, 64>(c, lds, grid, st);
  }
  if (e || c.has_down) return e;
  return llj_linear_resid(wf, L->h, H, L->w_down, L->sz_down, L->x, C, M, C, H, nullptr, 0, L->nst_out, stream);
}

}  // extern "C"

// C-ABI entry points of the weight-streaming GEMV family (device code: gemv_impl.h; the
// per-format instantiations: gemv_w4.hip, gemv_bf16.hip, gemv_w8.hip, gemv_i8.hip).
#include "gemv_impl.h"

namespace llj {

int g_tpw_max = LLJ_TPW_MAX;
int g_stream_a = 1;

template <int EP>
static int dispatch(int wf, int am, const GemvParams& p, hipStream_t s) {
  switch (wf) {
    case WF_W4: return gemv_launch_w4(am, EP, p, s);
    case WF_BF16: return gemv_launch_bf16(am, EP, p, s);
    case WF_W8: return gemv_launch_w8(am, EP, p, s);
    case WF_I8: return gemv_launch_i8(am, EP, p, s);
    case WF_W4G: return gemv_launch_w4g(am, EP, p, s);
  }
  return LLJ_EINVAL;
}

template <int EP>
static int run(int wfmt, GemvParams& p, void* stream) {
  // wfmt: weight format in bits [0, 8); WF_W4G carries its group size (in 128-deep chunks) above
  const int wf = wfmt & 0xff;
  p.gch = (wfmt >> 8) & 0xff;
  if (wf == WF_I8 && (wfmt & LLJ_WF_I8_ROWSTATS)) {  // i8ws is a decode hand-off block (AM_I8Q)
    if (!p.i8ws) return LLJ_EINVAL;
    p.i8st = (const uint32_t*)p.i8ws;
    p.i8ws = nullptr;
  }
  if (int e = check_shape(wf, p)) return e;
  // norm statistics hand-off: partial sums of squares [npart][16] (row slot = row of the call),
  // written by a residual op, read by the next norm-fused op; at most 16 rows, 2 partials per thread
  if (p.nstat_out && p.M > kNstRows) return LLJ_EINVAL;
  if (p.nstat && (!p.norm_w || wf == WF_I8 || p.M > kNstRows || p.npart < 1 || p.npart > 2 * kNW * 64))
    return LLJ_EINVAL;
  if (EP == EP_SWIGLU && wf != WF_BF16 && !p.sz2) return LLJ_EINVAL;
  const int am = pick_am(wf, p);
  if (am < 0) return LLJ_EINVAL;
  return dispatch<EP>(wf, am, p, (hipStream_t)stream);
}

}  // namespace llj

using namespace llj;

extern "C" {
// Cap on tiles per workgroup of the multi-tile GEMV forms (1 = one tile per workgroup);
// returns the previous cap. A host-side launch parameter only (no device state).
int llj_set_tpw_max(int tiles) {
  const int old = g_tpw_max;
  g_tpw_max = tiles < 1 ? 1 : tiles;
  return old;
}

// Streamed-A forms of the GEMVs (gemv_impl.h AM_STREAM / AM_SNORM): 1 (default) for batched rows
// 2 <= M <= 8, 2 for 1 <= M <= 8, 0 off (the LDS-image forms); returns the previous setting.
// Host-side only.
int llj_set_stream_a(int mode) {
  const int old = g_stream_a;
  g_stream_a = mode < 0 ? 0 : mode > 2 ? 2 : mode;
  return old;
}

// C[M,N] = A[M,K] . W^T (+bias); bf16 in/out, fp32 accumulation, M <= 16 (int8: <= 8) per call.
int llj_linear(int wfmt, const void* A, int lda, const void* W, const void* sz, const void* bias, void* C,
               int ldc, int M, int N, int K, const void* i8ws, int i8_row0, const float* rowsum, void* stream) {
  GemvParams p{};
  p.rowsum = rowsum;
  p.A = (const bf16_t*)A; p.lda = lda; p.M = M; p.N = N; p.K = K;
  p.W = W; p.sz = (const float2*)sz; p.bias = (const bf16_t*)bias; p.C = (bf16_t*)C; p.ldc = ldc;
  p.i8ws = i8ws; p.m0 = i8_row0;
  return run<EP_STORE>(wfmt, p, stream);
}

// out[M,N] = RMSNorm(x)[M,K] . W^T  (ln_f + lm_head, model.py:125-127); norm_w NULL = no norm.
int llj_norm_linear(int wfmt, const void* x, const void* norm_w, float eps, const void* W, const void* sz,
                    void* out, int ldo, int M, int N, int K, const void* i8ws, int i8_row0, const float* rowsum,
                    const float* nstat, int npart, void* stream) {
  GemvParams p{};
  p.rowsum = rowsum;
  p.nstat = nstat; p.npart = npart;
  p.A = (const bf16_t*)x; p.lda = K; p.norm_w = (const bf16_t*)norm_w; p.eps = eps; p.M = M; p.N = N; p.K = K;
  p.W = W; p.sz = (const float2*)sz; p.C = (bf16_t*)out; p.ldc = ldo;
  p.i8ws = i8ws; p.m0 = i8_row0;
  return run<EP_STORE>(wfmt, p, stream);
}

// x[M,N] += A[M,K] . W^T, bf16 residual add (attn.c_proj / mlp.c_proj + model.py:172-173).
int llj_linear_resid(int wfmt, const void* A, int lda, const void* W, const void* sz, void* x, int ldx, int M,
                     int N, int K, const void* i8ws, int i8_row0, float* nstat_out, void* stream) {
  GemvParams p{};
  p.nstat_out = nstat_out;
  p.A = (const bf16_t*)A; p.lda = lda; p.M = M; p.N = N; p.K = K;
  p.W = W; p.sz = (const float2*)sz; p.C = (bf16_t*)x; p.ldc = ldx;
  p.i8ws = i8ws; p.m0 = i8_row0;
  return run<EP_RESID>(wfmt, p, stream);
}

// h[M,H] = silu(RMSNorm(x) . W1^T) * (RMSNorm(x) . W2^T)  (rms_2 + model.py:258).
int llj_norm_swiglu(int wfmt, const void* x, const void* norm_w, float eps, const void* W1, const void* sz1,
                    const void* W2, const void* sz2, void* h, int M, int H, int K, const void* i8ws, int i8_row0,
                    const float* rowsum, const float* nstat, int npart, void* stream) {
  GemvParams p{};
  p.rowsum = rowsum;
  p.nstat = nstat; p.npart = npart;
  p.A = (const bf16_t*)x; p.lda = K; p.norm_w = (const bf16_t*)norm_w; p.eps = eps; p.M = M; p.N = H; p.K = K;
  p.W = W1; p.W2 = W2; p.sz = (const float2*)sz1; p.sz2 = (const float2*)sz2; p.C = (bf16_t*)h; p.ldc = H;
  p.i8ws = i8ws; p.m0 = i8_row0;
  return run<EP_SWIGLU>(wfmt, p, stream);
}

// rms_1 + c_attn + split + RoPE(q,k) + KV-cache write at slot pos % S (model.py:171,204-228).
// Rows m = b*T + t of x (B*T, C); this call handles rows [row0, row0 + rows), rows <= 8;
// q_out (B*T, C); caches (B, n_head, S, hs).
int llj_norm_qkv_rope(int wfmt, const void* x, const void* norm_w, float eps, const void* W, const void* sz,
                      void* q_out, void* kcache, void* vcache, const float* rope, const int* pos, int B, int T,
                      int C, int n_head, int S, int row0, int rows, const void* i8ws, const float* rowsum,
                      const float* nstat, int npart, void* stream) {
  GemvParams p{};
  p.rowsum = rowsum ? rowsum + row0 : nullptr;
  p.nstat = nstat ? nstat + row0 : nullptr; p.npart = npart;
  if (row0 < 0 || rows < 1 || row0 + rows > B * T || n_head < 1 || C % n_head || S < 1) return LLJ_EINVAL;
  p.A = (const bf16_t*)x + (size_t)row0 * C; p.lda = C; p.norm_w = (const bf16_t*)norm_w; p.eps = eps;
  p.M = rows; p.m0 = row0; p.N = 3 * C; p.K = C;
  p.W = W; p.sz = (const float2*)sz; p.q_out = (bf16_t*)q_out; p.kcache = (bf16_t*)kcache;
  p.vcache = (bf16_t*)vcache; p.rope = rope; p.pos = pos; p.n_head = n_head; p.head_size = C / n_head;
  p.S = S; p.T = T; p.i8ws = i8ws;
  if (p.head_size < 2 || (p.head_size & (p.head_size - 1)) || rows > 8) return LLJ_EINVAL;  // power of two
  return run<EP_QKV>(wfmt, p, stream);
}

// ---- LLM.int8() decode rows with handed-over statistics (i8ws.h kI8StFlags; M <= 8)
size_t llj_i8_rowstats_bytes(int K) { return (size_t)i8st_words(K) * 4; }

// x[M,N] += LLM.int8(A)[M,K] . CB^T: A bf16 rows quantized per K chunk inside the GEMV with the row
// statistics `stats` its producer wrote (llj_attention_i8 / llj_i8_swiglu_stats), the fp16 outlier
// side product from the streamed weights (attn.c_proj / mlp.c_proj + model.py:172-173).
int llj_i8_linear_resid(const void* A, int lda, const void* CB, const void* SCB, void* x, int ldx, int M, int N, int K,
                        const void* stats, void* stream) {
  if (!stats || M > 8 || (lda & 7)) return LLJ_EINVAL;
  GemvParams p{};
  p.A = (const bf16_t*)A; p.lda = lda; p.M = M; p.N = N; p.K = K;
  p.W = CB; p.sz = (const float2*)SCB; p.C = (bf16_t*)x; p.ldc = ldx;
  p.i8st = (const uint32_t*)stats;
  return run<EP_RESID>(WF_I8, p, stream);
}

// x[1,N] += y . W^T with y the decode attention output of one row, merged in the prologue from the
// nsplit interleaved key-split partials of llj_attention_part (no combine launch): attn.c_proj +
// model.py:172. Bitwise llj_linear_resid of attention_combine_kernel's y over the same partials.
int llj_linear_resid_attn(int wfmt, const void* part, int nsplit, int n_head, const void* W, const void* sz, void* x,
                          int ldx, int N, int K, float* nstat_out, void* stream) {
  if (!part || nsplit < 1 || nsplit > kMergeMax || n_head < 1 || K % n_head) return LLJ_EINVAL;
  GemvParams p{};
  p.nstat_out = nstat_out;
  p.apart = (const float*)part; p.asplit = nsplit; p.n_head = n_head; p.head_size = K / n_head;
  if (p.head_size < 8 || (p.head_size & (p.head_size - 1))) return LLJ_EINVAL;
  p.A = nullptr; p.lda = K; p.M = 1; p.N = N; p.K = K;
  p.W = W; p.sz = (const float2*)sz; p.C = (bf16_t*)x; p.ldc = ldx;
  return run<EP_RESID>(wfmt, p, stream);
}

// h = silu(xn . CB1^T) * (xn . CB2^T) for LLM.int8 decode rows -- xn's statistics either in i8ws
// (llj_i8_norm_stats) or as a hand-off block x_stats (llj_i8_norm_rowstats: rows quantized per chunk,
// AM_I8Q) -- that also writes the LLM.int8 statistics of h (h_stats, zeroed beforehand) and zeroes
// clr_words words at clr (the attention output's statistics block of the next layer).
int llj_i8_swiglu_stats(const void* x, const void* CB1, const void* SCB1, const void* CB2, const void* SCB2, void* h,
                        int M, int H, int K, const void* i8ws, const void* x_stats, void* h_stats, void* clr,
                        int clr_words, float threshold, void* stream) {
  if (!i8ws == !x_stats || !h_stats || M > 8 || clr_words < 0 || (clr_words && !clr)) return LLJ_EINVAL;
  GemvParams p{};
  p.A = (const bf16_t*)x; p.lda = K; p.M = M; p.N = H; p.K = K;
  p.W = CB1; p.W2 = CB2; p.sz = (const float2*)SCB1; p.sz2 = (const float2*)SCB2; p.C = (bf16_t*)h; p.ldc = H;
  p.i8ws = i8ws;  // the statistics launch's workspace (the LDS image of the quantized rows), or
  p.i8st = (const uint32_t*)x_stats;  // x's hand-off block (rows quantized per chunk)
  p.i8st_out = (uint32_t*)h_stats; p.clr = (uint32_t*)clr; p.clr_words = clr_words; p.thr = threshold;
  return run<EP_SWIGLU>(WF_I8, p, stream);
}

}  // extern "C"

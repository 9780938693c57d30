/* lit_llama_amd.h — C ABI of the MI355X (gfx950) quantized LLaMA decode path.
 *
 * Library: lit-llama-ja_amd/lit_llama/_lljamd.so (hipcc --offload-arch=gfx950).
 * Conventions: every pointer is a device pointer (HBM) except where noted; bf16 tensors
 * are raw 16-bit patterns; `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream
 * on the Python side, or 0). Every entry point only enqueues work (graph-capturable: no
 * allocation, no synchronisation) and returns 0 on success, a hipError_t, or
 * LLJ_EINVAL (1000) for a shape/argument the kernels do not support. The library owns no
 * memory; callers own every buffer.
 *
 * Reference = if001/lit-llama-ja @ 2025-02-05 (paths relative to its root).
 */
#ifndef LIT_LLAMA_AMD_H
#define LIT_LLAMA_AMD_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LLJ_EINVAL 1000

/* ---------------------------------------------------------------- int4 weight layout
 * Replaces the `quant_weight` buffer contract of ColBlockQuantizedLinear
 * (lit_llama/quantization.py:348-357, pack_weight 374-388): logical (N, K/2) uint8 stored
 * column-major (= physical row-major (K/2, N)), low nibble = even k. The GEMV consumes the
 * "W4P" tiling (1 KiB per 16 columns x 128 k). repack/unpack are exact inverses.
 * N % 16 == 0, K % 128 == 0. */
int llj_w4_repack(const void* qweight_ref, void* packed, int N, int K, void* stream);
int llj_w4_unpack(const void* packed, void* qweight_ref, int N, int K, void* stream);

/* sz[2n] = scales[n], sz[2n+1] = 128 + zeros[n] (fp32) from the module's (N, 1) `scales` /
 * `zeros` buffers (quantization.py:358-367; gptq.int4 is tile_cols = -1, utils.py:181).
 * dtype: 0 fp32, 1 bf16, 2 fp16. */
int llj_w4_scale_zero(const void* scales, const void* zeros, int dtype, void* sz, int N, void* stream);

/* ---------------------------------------------------------------- int8 (gptq.int8) weight layout
 * ColBlockQuantizedLinear(bits=8, tile_cols=-1) (quantization.py:338-409, utils.py:182-184):
 * `quant_weight` is the logical (N, K) uint8 tensor stored column-major (= physical row-major
 * (K, N)), one code per byte. The GEMV consumes "W8P": per 16 columns x 128 k, the W4P tile of
 * the low nibbles followed by the W4P tile of the high nibbles (2 KiB). `packed` holds N*K
 * bytes. sz[2n] = scales[n], sz[2n+1] = 2176 + zeros[n] (the W8P magic offset). */
int llj_w8_repack(const void* qweight_ref, void* packed, int N, int K, void* stream);
int llj_w8_scale_zero(const void* scales, const void* zeros, int dtype, void* sz, int N, void* stream);

/* Host-side tuning knob (no device work): at most `tiles` 16-column tiles per workgroup in the
 * int4 / gptq.int8 GEMVs (default 4; 1 = one tile per workgroup). Results do not depend on it
 * (tested bitwise). Returns the previous value. */
int llj_set_tpw_max(int tiles);

/* ---------------------------------------------------------------- linear layers
 * wfmt: 0 = int4 W4P (sz = (scale, 128+zero) pairs required), 1 = bf16 (N, K) row-major
 * (torch.nn.Linear.weight), 2 = LLM.int8() CB (N, K) int8 with sz = SCB (N) fp32,
 * 3 = gptq.int8 W8P (sz = (scale, 2176+zero) pairs, llj_w8_scale_zero); for
 * wfmt 2, `i8ws` is the statistics workspace llj_i8_stats filled for the whole activation
 * and `i8_row0` the index of this call's first row in it (NULL / 0 otherwise).
 * C[M, N] = A[M, K] . W^T (+ bias), bf16 in/out, fp32 (int8: int32) accumulation,
 * M <= 16 rows per call (int8: <= 8).
 * Replaces qlinear_4bit_weight / linear_kernel_4bit_weight (quantization.py:80-331),
 * ColBlockQuantizedLinear.forward (quantization.py:411-421), bnb Linear8bitLt.forward
 * (used by quantization.py:36-75) and, for wfmt 1, F.linear. */
int llj_linear(int wfmt, const void* A, int lda, const void* W, const void* sz, const void* bias, void* C, int ldc,
               int M, int N, int K, const void* i8ws, int i8_row0, const float* rowsum, void* stream);

/* ---------------------------------------------------------------- fused decode-layer ops
 * (Block.forward, lit_llama/model.py:162-175, split at its four Linear boundaries).
 * norm_w == NULL means the input is used as is (no fused RMSNorm); int8 (wfmt 2) takes
 * already-normalised input (its statistics are computed on it).
 * RMSNorm row statistics (optional, decode path, <= 8 rows): fp64 partial sums of
 * bf16(x^2) laid out [part][8 rows]. llj_embedding writes part 0 (whole rows);
 * llj_linear_resid writes part n/16 for its 16-column tile n (N/16 parts); the norm-fused
 * ops read `nstat_parts` parts (1 after the embedding, n_embd/16 after a residual GEMV)
 * instead of re-reducing the row in every workgroup. NULL = off (row reduced in-kernel).
 * rowsum (int4 only, optional): fp32 sum over k of each row of A exactly as the MFMA reads it
 * (i.e. after the RMSNorm when norm_w is given), from llj_rmsnorm_rows; used for the int4
 * offset term instead of a per-workgroup reduction. NULL = reduced in-kernel. */

/* rms_1 + attn.c_attn + split q/k/v + apply_rope(q, k) + KV-cache write
 * (model.py:171, 204-228, 312-329). x (B*T, C) rows m = b*T + t; q_out (B*T, C);
 * kcache/vcache (B, n_head, S, hs) with token at absolute position p stored in slot p % S
 * (ring form of the reference's roll-by-one sliding window, model.py:221-227);
 * rope (block_size, hs/2, 2) fp32 (build_rope_cache, model.py:286-309); pos (T) int32.
 * Handles rows [row0, row0 + rows) of the B*T rows; rows <= 8 (RMSNorm staged in LDS). */
int llj_norm_qkv_rope(int wfmt, const void* x, const void* norm_w, float eps, const void* W, const void* sz,
                      void* q_out, void* kcache, void* vcache, const float* rope, const int* pos, int B, int T,
                      int C, int n_head, int S, int row0, int rows, const void* i8ws, const double* nstat_in,
                      int nstat_parts, const float* rowsum, void* stream);

/* llj_norm_qkv_rope for one decode row (M = B = 1, T = 1) that also computes the attention of
 * every head (as llj_attention, model.py:237) into y (1, C): the workgroup completing a head's
 * last q / k / v tile runs it (per-head arrival counters att_ctr: n_head words, zero before the
 * first call and left zero). Bitwise equal to llj_norm_qkv_rope + llj_attention. wfmt 0, 1, 3. */
int llj_norm_qkv_rope_attn(int wfmt, const void* x, const void* norm_w, float eps, const void* W, const void* sz,
                           void* q_out, void* kcache, void* vcache, const float* rope, const int* pos, int C,
                           int n_head, int S, void* y, unsigned* att_ctr, void* stream);

/* Causal attention of q (B*T, C) over the cache slots each query may see
 * (F.scaled_dot_product_attention with the tril mask rows, model.py:101-104, 237):
 * positions <= p, or all S slots once p >= S. y (B*T, C) bf16. head_size 64 or 128. */
int llj_attention(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T,
                  int n_head, int head_size, int S, void* stream);

/* Split-K form of llj_attention for long caches: the valid keys of every (row, head) split into
 * nsplit equal ranges, one block each, writing unnormalized partials (outputs, max, sum) into
 * part_ws (llj_attention_ws_bytes(B*T, n_head, head_size, nsplit) bytes), merged in split order
 * by a second launch. nsplit <= 1 is llj_attention itself. Same softmax up to summation order. */
size_t llj_attention_ws_bytes(int rows, int n_head, int head_size, int nsplit);
int llj_attention_split(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T,
                        int n_head, int head_size, int S, int nsplit, void* part_ws, void* stream);

/* y = attention (as llj_attention, T = 1 decode rows, M = B <= 8) and then
 * x[M, C] += y . W_proj^T (as llj_linear_resid, attn.c_proj + residual, model.py:172,239-242),
 * in ONE launch: the c_proj workgroups load their weights while the attention runs and wait
 * for it on a completion counter. counters: 32 words the caller zeroes before every call;
 * err: set non-zero if the wait timed out (never expected). wfmt 0, 1 or 3. Bitwise equal
 * to llj_attention + llj_linear_resid. */
int llj_attn_resid(int wfmt, const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int M,
                   int n_head, int S, const void* W, const void* sz, void* x, int C, double* nstat_out,
                   unsigned* counters, unsigned* err, void* stream);

/* x[M, N] += A[M, K] . W^T (attn.c_proj / mlp.c_proj + residual add, model.py:172-173). */
int llj_linear_resid(int wfmt, const void* A, int lda, const void* W, const void* sz, void* x, int ldx, int M,
                     int N, int K, const void* i8ws, int i8_row0, double* nstat_out, void* stream);

/* The same, then the next RMSNorm of the updated rows (rms_2 after c_proj, the next layer's
 * rms_1 / ln_f after mlp.c_proj; model.py:173, 171, 125): xn[M, N] = RMSNorm(x) with scale
 * norm_w, rowsum[m] = fp32 sum of the normalized row (or NULL). Computed once, by the last
 * workgroup to finish (agent release/acquire + the completion `counter`, one word the caller
 * zeroes once; the kernel leaves it 0). M <= 8, wfmt 0 or 1. Batched decode (M >= 2) uses it
 * instead of a separate llj_rmsnorm_rows launch. */
int llj_linear_resid_norm(int wfmt, const void* A, int lda, const void* W, const void* sz, void* x, int ldx, int M,
                          int N, int K, const void* norm_w, float eps, void* xn, float* rowsum, unsigned* counter,
                          void* stream);

/* h[M, H] = silu(rms_2(x) . W1^T) * (rms_2(x) . W2^T)  (model.py:173, 258). M <= 8. */
int llj_norm_swiglu(int wfmt, const void* x, const void* norm_w, float eps, const void* W1, const void* sz1,
                    const void* W2, const void* sz2, void* h, int M, int H, int K, const void* i8ws, int i8_row0,
                    const double* nstat_in, int nstat_parts, const float* rowsum, void* stream);

/* out[M, N] = RMSNorm(x) . W^T  (ln_f + lm_head, model.py:125-127). M <= 8. */
int llj_norm_linear(int wfmt, const void* x, const void* norm_w, float eps, const void* W, const void* sz,
                    void* out, int ldo, int M, int N, int K, const void* i8ws, int i8_row0, const double* nstat_in,
                    int nstat_parts, const float* rowsum, void* stream);

/* ---------------------------------------------------------------- one decode layer, one launch
 * Block.forward (model.py:162-175) for a decode step (T = 1, M = B <= 8 rows) with int4 W4P
 * (wfmt 0), bf16 (wfmt 1) or int8 W8P (wfmt 3, always as separate launches) linears: rms_1 + c_attn + RoPE + KV write -> attention -> c_proj +
 * residual -> rms_2 + c_fc1/c_fc2 + silu*mul -> mlp.c_proj + residual. Same math and results
 * as the five entry points above; when the shapes allow, all five run in ONE launch whose
 * consumer workgroups start streaming their weights before their producer op has finished
 * (completion counters, sc1 write-through hand-offs), otherwise as separate launches.
 * counters: 128 words the caller zeroes before every call; err: set non-zero if a
 * dependency wait timed out (never expected; a diagnostic, results then invalid). */
typedef struct llj_layer {
  int wfmt, M, C, H, n_head, S;
  void* x;                       /* (M, C) residual stream, updated in place */
  const void* rms1;
  const void* rms2;
  float eps;
  const void* w_qkv;  const void* sz_qkv;
  const void* w_proj; const void* sz_proj;
  const void* w_fc1;  const void* sz_fc1;
  const void* w_fc2;  const void* sz_fc2;
  const void* w_down; const void* sz_down;
  void* q;                       /* (M, C) scratch */
  void* kcache; void* vcache;    /* (M, n_head, S, C/n_head), ring slot pos % S */
  const float* rope;
  const int* pos;                /* device position of the decode token */
  void* y;                       /* (M, C) attention output scratch */
  void* h;                       /* (M, H) MLP hidden scratch */
  const double* nst_in; int nst_in_parts;  /* RMSNorm statistics of x for rms_1 (or NULL) */
  double* nst_mid;               /* written by c_proj, read by rms_2: C/16 parts x 8 rows */
  double* nst_out;               /* written by mlp.c_proj for the next layer's rms_1 */
  unsigned* counters;
  unsigned* err;
} llj_layer;
int llj_decode_layer(const llj_layer* layer, void* stream);

/* ---------------------------------------------------------------- LLM.int8() */
/* Bytes of the activation-statistics workspace for an (M, K) activation (host function). */
size_t llj_i8_ws_bytes(int M, int K);
/* Outlier columns (any row |A16| >= threshold) and per-row absmax of the other elements of
 * A (M, K) bf16 into ws (bitsandbytes double_quant(A, threshold) as used by MatMul8bitLt). */
int llj_i8_stats(const void* A, int lda, int M, int K, float threshold, void* ws, void* stream);
/* CB = round(W16 * 127 / SCB), SCB = row absmax of W16 = W.half() (Linear8bitLt._quantize_weight,
 * quantization.py:67-75). W (N, K) of dtype 0 fp32 / 1 bf16 / 2 fp16. */
int llj_i8_quant_weight(const void* W, int dtype, void* CB, void* SCB, int N, int K, void* stream);

/* ---------------------------------------------------------------- GPTQ producer */
/* One 128-column block of GPTQQuantizer.quantize (reference quantization.py:568-596, groupsize
 * -1): for rows n < N, quantize columns i1 .. i1+127 in order with the per-row (scale, zero)
 * (quantize_weight, 470-473), propagate each column's error through the block with Hinv1 =
 * hinv[i1:i1+128, i1:i1+128] (593). wt: the (permuted, running) weight TRANSPOSED, (K, N) fp32,
 * its block rows updated in place; qt (K, N): reconstructions scale*(q - zero) of the block's
 * rows; err (128, N): Err1; loss[n] += Σ_i (w - q)² / d² (Losses1 before the / 2). hinv: (K, K)
 * fp32 upper Cholesky factor of H⁻¹. Requires i1 % 128 == 0, i1 + 128 <= K, bits in {2,4,8}.
 * Each fp32 op rounded on its own in the reference's order (bitwise the reference's loop). The
 * trailing update W[:, i2:] -= Err1 · Hinv[i1:i2, i2:] is a plain GEMM left to the caller. */
int llj_gptq_block(const float* hinv, int K, int i1, float* wt, int N, const float* scale, const float* zero,
                   int bits, float* qt, float* err, float* loss, void* stream);
/* ColBlockQuantizedLinear.pack_weight (quantization.py:374-388) from reconstructions qt (K, N)
 * fp32: code = uint8(clamp(q / scale + zero, 0, 2^bits - 1)) (truncating), entries_per_byte =
 * 8/bits codes per byte; qw is quant_weight in its column-major storage: byte (n, j) at j*N + n. */
int llj_colblock_pack(const float* qt, int K, int N, const float* scale, const float* zero, int bits,
                      unsigned char* qw, void* stream);

/* ---------------------------------------------------------------- small ops */
/* out[m] = wte[idx[m]] (model.py:110); if pos_inc != NULL, *pos_inc += 1 (device-side
 * decode position, so a captured decode step advances itself); nstat_out: per-row sum of
 * bf16(x^2) (see "RMSNorm row statistics" above) or NULL. */
int llj_embedding(const int* idx, const void* wte, void* out, int M, int C, int* pos_inc, double* nstat_out,
                  void* stream);

/* Standalone RMSNorm (model.py:276-283) for rows the fused prologue does not take. */
int llj_rmsnorm(const void* x, const void* w, float eps, void* y, int M, int C, void* stream);
/* The same, plus rowsum[m] = fp32 sum of the normalized bf16 row (the int4 GEMVs' offset
 * term): batched rows (M >= 2) are normalized once here instead of in every GEMV workgroup. */
int llj_rmsnorm_rows(const void* x, const void* w, float eps, void* y, float* rowsum, int M, int C, void* stream);

/* Greedy next token (generate.py:66-74 with top_k = 1): out_idx[m] = argmax logits[m, :V]
 * (lowest index on ties). If tokens_out != NULL also tokens_out[m*tok_stride + *pos + 1]. */
int llj_argmax(const void* logits, int ldl, int M, int V, int* out_idx, int* tokens_out, int tok_stride,
               const int* pos, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LIT_LLAMA_AMD_H */

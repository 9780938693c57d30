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
int llj_w8_unpack(const void* packed, void* qweight_ref, int N, int K, void* stream);
int llj_w8_scale_zero(const void* scales, const void* zeros, int dtype, void* sz, int N, void* stream);

/* ---------------------------------------------------------------- LLM.int8() weight layout
 * Linear8bitLt's CB (N, K) int8 row-major (quantization.py:36-75; llj_i8_quant_weight) <-> "I8P",
 * the tiling the int8 GEMV (wfmt 2) consumes: per 16 columns x 128 k, 2 KiB = two 1-KiB blocks (the
 * two 64-deep MFMA steps), lane l of a block holding row 16 nt + (l & 15), k = 64 t + 16 (l >> 4)
 * + 0 .. 15 of the chunk. packed and cb are distinct N*K-byte buffers. */
int llj_i8_repack(const void* cb, void* packed, int N, int K, void* stream);
int llj_i8_unpack(const void* packed, void* cb, int N, int K, void* stream);

/* Host-side tuning knob (no device work): at most `tiles` 16-column tiles per workgroup in the
 * int4 / gptq.int8 GEMVs (default 4; 1 = one tile per workgroup). Results do not depend on it
 * (tested bitwise). Returns the previous value. */
int llj_set_tpw_max(int tiles);

/* Host-side switch (no device work): 1 (default) = batched decode rows (2 <= M <= 8) of the
 * int4 / gptq.int8 / bf16 GEMVs stream their activation rows per K chunk (the fused RMSNorm then
 * takes the residual op's handed-over sums of squares, `nstat`); 2 = also single rows; 0 = the
 * LDS-image forms. Same rounding points either way. Returns the previous value. */
int llj_set_stream_a(int mode);

/* Host-side A/B options (no device work). Each starts from its environment variable (read once, at
 * first use; -1 = unset = the build default) and can be set per process; launches never read the
 * environment. Returns the previous value, or -1000 for an unknown option / out-of-range value.
 *   LLJ_OPT_ATT_SPEC_FULL  0..1  decode attention loads a whole (1) or half (0) key pass before the position (LLJ_ATT_SPEC)
 *   LLJ_OPT_FLASH_QB       1..2  flash prefill: 16-query blocks per wave (LLJ_FLASH_QB)
 *   LLJ_OPT_FLASH_PAIR     0..1  flash prefill: (long, short) query-block pairs per workgroup (LLJ_FLASH_PAIR)
 *   LLJ_OPT_GEMM_GLDS      0..1  prefill GEMMs: LDS-DMA (1) or register-staged (0) kernel for every format (LLJ_GEMM_GLDS)
 *   LLJ_OPT_GLDS_COST128   0..   LDS-DMA GEMM: cost of a 256 x 128 tile in % of a 256 x 256 one (LLJ_GLDS_COST128)
 *   LLJ_OPT_GEMV_LDS_A_KB  56..96 decode GEMVs: cap of the staged A image in KiB (LLJ_GEMV_LDS_A_KB)
 *   LLJ_OPT_ATT_SPEC_BATCH 0..1  decode attention: the half speculative key pass also past 64 blocks (LLJ_ATT_SPEC_BATCH)
 *   LLJ_OPT_GEMM_W4Z       0..1  prefill int4 GEMMs with LLJ_WF_ZINT: convert-once LDS-DMA kernel (1) or the int4 default (0) (LLJ_GEMM_W4Z) */
enum {
  LLJ_OPT_ATT_SPEC_FULL = 0,
  LLJ_OPT_FLASH_QB = 1,
  LLJ_OPT_FLASH_PAIR = 2,
  LLJ_OPT_GEMM_GLDS = 3,
  LLJ_OPT_GLDS_COST128 = 4,
  LLJ_OPT_GEMV_LDS_A_KB = 5,
  LLJ_OPT_ATT_SPEC_BATCH = 6,
  LLJ_OPT_GEMM_W4Z = 7,
  LLJ_OPT_COUNT = 8
};
int llj_set_option(int which, int value);

/* ---------------------------------------------------------------- linear layers
 * wfmt: 0 = int4 W4P (sz = (scale, 128+zero) pairs required), 1 = bf16 (N, K) row-major
 * (torch.nn.Linear.weight), 2 = LLM.int8() CB in the I8P tiling (llj_i8_repack) with sz = SCB (N) fp32,
 * 3 = gptq.int8 W8P (sz = (scale, 2176+zero) pairs, llj_w8_scale_zero),
 * 4 | (g / 128) << 8 = grouped int4 (ColBlockQuantizedLinear tile_cols = g, g % 128 == 0,
 * quantization.py:338-409 with scales (N, ceil(K / g))): W4P tiles with sz = (scale, 128+zero)
 * pairs per (group, column), group-major (ceil(K / g), N) (llj_w4_scale_zero over the transposed
 * buffers); the fused ops below take the same wfmt; for
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
 * nstat / npart (optional, norm-fused forms with M <= 16, not int8): the RMSNorm's sum of
 * squares of each row comes from npart <= 512 partials nstat[p * 16 + m] written by the residual
 * op that produced x (llj_linear_resid's nstat_out) instead of being recomputed from x in every
 * workgroup; NULL = computed from x.
 * (Block.forward, lit_llama/model.py:162-175, split at its four Linear boundaries).
 * norm_w == NULL means the input is used as is (no fused RMSNorm); int8 (wfmt 2) takes
 * already-normalised input (its statistics are computed on it).
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
                      int C, int n_head, int S, int row0, int rows, const void* i8ws, const float* rowsum,
                      const float* nstat, int npart, void* stream);

/* Causal attention of q (B*T, C) over the cache slots each query may see
 * (F.scaled_dot_product_attention with the tril mask rows, model.py:101-104, 237):
 * positions <= p, or all S slots once p >= S. y (B*T, C) bf16. head_size 64 or 128. */
int llj_attention(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T,
                  int n_head, int head_size, int S, void* stream);

/* Causal attention of T prompt rows per sequence on the MFMA units (flash-style: 64-query x
 * 64-key tiles, online softmax; csrc/attention_prefill.hip): query t of sequence b sits at position
 * pos[0] + t and attends cache slots 0 .. pos[0] + t. Requires contiguous positions pos[t] = pos[0]
 * + t with pos[0] + T <= S (no ring wrap; the caller checks). head_size 64 or 128. */
int llj_attention_prefill(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T,
                          int n_head, int head_size, int S, void* stream);

/* Split-K form of llj_attention for long caches: the valid keys of every (row, head) split into
 * nsplit equal ranges, one block each, writing unnormalized partials (outputs, max, sum) into
 * part_ws (llj_attention_ws_bytes(B*T, n_head, head_size, nsplit) bytes), merged in split order
 * by a second launch. nsplit <= 1 is llj_attention itself. Same softmax up to summation order. */
size_t llj_attention_ws_bytes(int rows, int n_head, int head_size, int nsplit);
/* Decode attention (model.py:237) as nsplit <= 4 interleaved key splits per (row, head) whose
 * unnormalized partials (outputs, max, sum; llj_attention_ws_bytes layout) go to part_ws with no
 * combine launch: llj_linear_resid_attn merges them in attn.c_proj's prologue (one row). */
int llj_attention_part(const void* q, const void* kcache, const void* vcache, const int* pos, int B, int T,
                       int n_head, int head_size, int S, int nsplit, void* part_ws, void* stream);
int llj_attention_split(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T,
                        int n_head, int head_size, int S, int nsplit, void* part_ws, void* stream);

/* x[M, N] += A[M, K] . W^T (attn.c_proj / mlp.c_proj + residual add, model.py:172-173).
 * nstat_out (optional, M <= 16, not int8): per 16-column tile t of the new x, the bf16-rounded
 * squares summed over the tile's columns, nstat_out[t * 16 + m] (fp32; N / 16 partials): the
 * statistics of the next RMSNorm (model.py:281), handed to the norm-fused op that follows. */
int llj_linear_resid(int wfmt, const void* A, int lda, const void* W, const void* sz, void* x, int ldx, int M,
                     int N, int K, const void* i8ws, int i8_row0, float* nstat_out, void* stream);
/* llj_linear_resid for one row whose A is the attention output merged from llj_attention_part's
 * partials in the prologue (attn.c_proj + model.py:172-173 without the combine launch); wfmt 0 / 1 / 3,
 * K = n_head * head_size < 8192. */
int llj_linear_resid_attn(int wfmt, const void* part, int nsplit, int n_head, const void* W, const void* sz, void* x,
                          int ldx, int N, int K, float* nstat_out, void* stream);
/* h[M, H] = silu(rms_2(x) . W1^T) * (rms_2(x) . W2^T)  (model.py:173, 258). M <= 8. */
int llj_norm_swiglu(int wfmt, const void* x, const void* norm_w, float eps, const void* W1, const void* sz1,
                    const void* W2, const void* sz2, void* h, int M, int H, int K, const void* i8ws, int i8_row0,
                    const float* rowsum, const float* nstat, int npart, void* stream);

/* out[M, N] = RMSNorm(x) . W^T  (ln_f + lm_head, model.py:125-127). M <= 8. */
int llj_norm_linear(int wfmt, const void* x, const void* norm_w, float eps, const void* W, const void* sz,
                    void* out, int ldo, int M, int N, int K, const void* i8ws, int i8_row0, const float* rowsum,
                    const float* nstat, int npart, void* stream);

/* ---------------------------------------------------------------- prefill GEMMs (many rows)
 * The same Linear layers for M >> 16 rows (a prompt, a perplexity window: LLaMA.forward over
 * T tokens, model.py:84-128), MFMA-tiled 128 x 128 per workgroup with the chunk tiles staged
 * through LDS (csrc/gemm.hip). wfmt 0 (int4 W4P, sz = (scale, 128 + zero)), 1 (bf16 (N, K)),
 * 3 (gptq.int8 W8P, sz = (scale, 2176 + zero)) or 4 | (g / 128) << 8 (grouped int4, sz per
 * (group, column) as for llj_linear; B fragments dequantized to bf16((q - z) * s)).
 * N % 128 == 0, K % 128 == 0, lda % 8 == 0; any M >= 1. Same epilogue semantics as the GEMVs.
 * wfmt 0 | LLJ_WF_ZINT: int4 whose zeros are all integers (GPTQ's round(-min / scale); the caller
 * checks): for M >= 256 each chunk's codes are converted once per workgroup into an exact bf16
 * (q - z) tile and the scale is applied in the epilogue, y = s * sum_k A (q - z) -- the reference
 * kernel's ((q - zero) * scale) . A (quantization.py:263-267) with the scale factored out. */
#define LLJ_WF_ZINT 0x20000
int llj_gemm_linear(int wfmt, const void* A, int lda, const void* W, const void* sz, void* C, int ldc, int M, int N,
                    int K, void* stream);
/* x[M, N] += A . W^T (bf16 residual add, model.py:172-173). */
int llj_gemm_resid(int wfmt, const void* A, int lda, const void* W, const void* sz, void* x, int ldx, int M, int N,
                   int K, void* stream);
/* llj_gemm_resid for prompts whose 256-row x 128-column tiles fill at most half the CUs (256..1024
 * rows at the 4096-wide residual GEMMs): the K range is split over up to 8 workgroups per tile, fp32
 * partials go to `ws` (llj_gemm_resid_ws_bytes(wfmt, M, N, K) bytes; 0 = no split, and then this call is
 * llj_gemm_resid), one reduce launch adds them in slice order and the residual. bf16 and integral-zero
 * int4 (0 | LLJ_WF_ZINT) weights, M >= 256. */
size_t llj_gemm_resid_ws_bytes(int wfmt, int M, int N, int K);
int llj_gemm_resid_ws(int wfmt, const void* A, int lda, const void* W, const void* sz, void* x, int ldx, int M, int N,
                      int K, void* ws, size_t ws_bytes, void* stream);
/* h[M, N] = bf16(silu(h)) * bf16(A . W^T), h holding bf16(rms_2(x) . W_fc1^T) from a llj_gemm_linear
 * pass (model.py:258; two passes instead of a dual-weight tile). */
int llj_gemm_silu_mul(int wfmt, const void* A, int lda, const void* W, const void* sz, void* h, int ldh, int M, int N,
                      int K, void* stream);
/* h[M, H] = bf16(silu(bf16(A . W1^T))) * bf16(A . W2^T) in ONE pass (model.py:258, c_fc1 and c_fc2 of
 * the SwiGLU MLP): int4 with integral zeros only (wfmt 0 | LLJ_WF_ZINT), M >= 256, H % 64 == 0; each
 * 256 x 64 tile stages one A tile for both weights. LLJ_EINVAL otherwise (then llj_gemm_linear +
 * llj_gemm_silu_mul). */
int llj_gemm_swiglu(int wfmt, const void* A, int lda, const void* W1, const void* sz1, const void* W2, const void* sz2,
                    void* h, int ldh, int M, int H, int K, void* stream);
/* llj_gemm_swiglu whose tiles leave a partial last wave over the CUs (7B: 2,048 or 512 rows x 11,008): that
 * wave's column tiles (the right end of h) run as two K halves into a caller-owned fp32 workspace and one
 * more launch finishes them; the rest is llj_gemm_swiglu on whole waves. 0 bytes = no split (then
 * llj_gemm_swiglu_ws is llj_gemm_swiglu). Same arguments as llj_gemm_swiglu + the workspace. */
size_t llj_gemm_swiglu_ws_bytes(int wfmt, int M, int H, int K);
int llj_gemm_swiglu_ws(int wfmt, const void* A, int lda, const void* W1, const void* sz1, const void* W2,
                       const void* sz2, void* h, int ldh, int M, int H, int K, void* ws, size_t ws_bytes, void* stream);
/* c_attn + split + RoPE(q, k) + KV-cache write for B*T pre-normalized rows x (as llj_norm_qkv_rope
 * with norm_w NULL; model.py:204-228). */
int llj_gemm_qkv_rope(int wfmt, const void* x, const void* W, const void* sz, void* q_out, void* kcache, void* vcache,
                      const float* rope, const int* pos, int B, int T, int C, int n_head, int S, void* stream);
/* LLM.int8() prompt rows (Linear8bitLt.forward for any M, reference quantization.py:36-75 over
 * bitsandbytes MatMul8bitLt): the four GEMMs above for CB (N, K) int8 in the I8P tiling and SCB
 * (N) fp32, with i8ws = llj_i8_stats / llj_i8_norm_stats of A (all M rows): int8 MFMA over the
 * quantized rows + the fp16 outlier side product, y = f16(f16(acc * SCA * SCB / 127^2) + side), then
 * the same epilogues. N % 128 == 0, K % 128 == 0. ao16 / w16 / kpad: llj_i8_gather_* (optional). */
int llj_gemm_i8_linear(const void* A, int lda, const void* CB, const void* SCB, const void* i8ws, const void* ao16,
                       const void* w16, int kpad, void* C, int ldc, int M, int N, int K, void* stream);
int llj_gemm_i8_resid(const void* A, int lda, const void* CB, const void* SCB, const void* i8ws, const void* ao16,
                      const void* w16, int kpad, void* x, int ldx, int M, int N, int K, void* stream);
int llj_gemm_i8_silu_mul(const void* A, int lda, const void* CB, const void* SCB, const void* i8ws, const void* ao16,
                         const void* w16, int kpad, void* h, int ldh, int M, int N, int K, void* stream);
int llj_gemm_i8_qkv_rope(const void* x, const void* CB, const void* SCB, const void* i8ws, const void* ao16,
                         const void* w16, int kpad, void* q_out, void* kcache, void* vcache, const float* rope,
                         const int* pos, int B, int T, int C, int n_head, int S, void* stream);
/* The outlier columns of an activation (its llj_i8_stats workspace) gathered as f16 rows
 * ao16[M][kpad] and of a weight (CB in I8P, SCB) as f16(CB * SCB / 127) rows w16[N][kpad], zero past
 * the outlier count up to the next multiple of 64: with both passed to llj_gemm_i8_* (else NULL,
 * NULL, 0) the fp16 outlier side product runs as a dense f16 GEMM over them (bitsandbytes' fp16
 * matmul of the outlier sub-matrices). kpad is a capacity in columns: kpad % 64 == 0, kpad >= 64,
 * (80 + kpad) * 4 <= 64 KiB (the gathers' LDS list); it may be smaller than K. When the activation
 * has more outlier columns than kpad, the gathers write nothing and the GEMM falls back to its
 * per-tile side product (same results). */
int llj_i8_gather_act(const void* A, int lda, int M, int K, const void* i8ws, void* ao16, int kpad, void* stream);
int llj_i8_gather_weight(const void* CB, const void* SCB, int N, int K, const void* i8ws, void* w16, int kpad,
                         void* stream);

/* ---------------------------------------------------------------- LLM.int8() */
/* Bytes of the activation-statistics workspace for an (M, K) activation (host function). */
size_t llj_i8_ws_bytes(int M, int K);
/* Outlier columns (any row |A16| >= threshold) and per-row absmax of the other elements of
 * A (M, K) bf16 into ws (bitsandbytes double_quant(A, threshold) as used by MatMul8bitLt). */
int llj_i8_stats(const void* A, int lda, int M, int K, float threshold, void* ws, void* stream);
/* The RMSNorm before an int8 Linear and llj_i8_stats of its output in two launches instead of
 * three: xn (M, K) = RMSNorm(x; norm_w, eps) bit-identical to llj_rmsnorm (model.py:276-283 on
 * bf16 tensors), then ws as llj_i8_stats(xn, K, M, K, threshold, ws). One-launch form for
 * M <= 16, K <= 8192 and M * (k-block width / 8) <= 256; otherwise the two ops it replaces. */
int llj_i8_norm_stats(const void* x, const void* norm_w, float eps, void* xn, int M, int K, float threshold, void* ws,
                      void* stream);
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
/* llj_gptq_block for GPTQQuantizer(blocksize=b) (quantization.py:437, 557-596): the column loop over
 * the b-column block [i1, i1 + b), b in {16, 32, 64, 128}; err (b, N). Requires i1 % b == 0,
 * i1 + b <= K. llj_gptq_block is this with b = 128. */
int llj_gptq_block_bs(const float* hinv, int K, int i1, int blocksize, float* wt, int N, const float* scale,
                      const float* zero, int bits, float* qt, float* err, float* loss, void* stream);
/* ColBlockQuantizedLinear.pack_weight (quantization.py:374-388) from reconstructions qt (K, N)
 * fp32: code = uint8(clamp(q / scale + zero, 0, 2^bits - 1)) (truncating), entries_per_byte =
 * 8/bits codes per byte; qw is quant_weight in its column-major storage: byte (n, j) at j*N + n. */
int llj_colblock_pack(const float* qt, int K, int N, const float* scale, const float* zero, int bits,
                      unsigned char* qw, void* stream);

/* ---------------------------------------------------------------- small ops */
/* out[m] = wte[idx[m]] (model.py:110), any C; if pos_inc != NULL, *pos_inc += 1 (device-side
 * decode position, so a captured decode step advances itself). */
int llj_embedding(const int* idx, const void* wte, void* out, int M, int C, int* pos_inc, void* stream);

/* Standalone RMSNorm (model.py:276-283) for rows the fused prologue does not take. */
int llj_rmsnorm(const void* x, const void* w, float eps, void* y, int M, int C, void* stream);
/* The same, plus rowsum[m] = fp32 sum of the normalized bf16 row (the int4 GEMVs' offset
 * term): batched rows (M >= 2) are normalized once here instead of in every GEMV workgroup. */
int llj_rmsnorm_rows(const void* x, const void* w, float eps, void* y, float* rowsum, int M, int C, void* stream);

/* Greedy next token (generate.py:66-74 with top_k = 1): out_idx[m] = argmax logits[m, :V]
 * (lowest index on ties). If tokens_out != NULL also tokens_out[m*tok_stride + *pos + 1]. */
int llj_argmax(const void* logits, int ldl, int M, int V, int* out_idx, int* tokens_out, int tok_stride,
               const int* pos, void* stream);

/* Sampled next token (generate.py:66-74, top_k > 1 or top_k <= 0 = None): x = bf16(logits /
 * temperature), keep x >= the top_k-th largest x (ties kept, torch.topk + torch.where),
 * probs = bf16(softmax(x)), then one draw: the first index whose running sum of probs (index
 * order) exceeds u * sum(probs). u in [0, 1): if u != NULL, u[(*pos + 1) * M + m] (a table of
 * uniforms per output position; u[m] when pos == NULL), otherwise a counter-based hash of
 * (seed, *pos, m), so a captured decode step draws a fresh u each step. Writes out_idx[m]
 * and, if tokens_out != NULL, tokens_out[m*tok_stride + *pos + 1]. One block per row. */
int llj_sample(const void* logits, int ldl, int M, int V, float temperature, int top_k, const float* u,
               unsigned long long seed, int* out_idx, int* tokens_out, int tok_stride, const int* pos, void* stream);

/* ---------------------------------------------------------------- any-shape path (csrc/generic.hip)
 * LLaMA configurations the streaming kernels do not tile (n_embd % 128 != 0, head size not 64 /
 * 128: the JA fork's 125M, n_embd 780 / head 78, reference lit_llama/model.py:48-51; the reference
 * test's n_embd 32 / head 2, tests/test_model.py:108-112), and every fp32 model. Plain kernels;
 * dt selects the activation type of every operand (and of dense weights, KV cache, logits):
 * 0 = bf16 with the reference's bf16 rounding points, 1 = fp32 with none (the reference's float32
 * model: evaluate/full.py:55, 84 default dtype, generate.py:121 on a host without a GPU).
 * LLaMA.forward and the decode session route such models here. */
/* out[m] = wte[idx[m]] (model.py:110), any C; bumps *pos_inc when not NULL (decode step). */
int llj_g_embedding(const int* idx, const void* wte, void* out, int M, int C, int* pos_inc, int dt, void* stream);
/* RMSNorm (model.py:276-283) of M rows of any width C (row strides ldx / ldy). */
int llj_g_rmsnorm(const void* x, int ldx, const void* w, float eps, void* y, int ldy, int M, int C, int dt, void* stream);
/* y[m, n] = x[m] . W[n] for M rows, or resid[m, n] + that when resid != NULL (may be y); rounded to
 * bf16 at the reference's points when dt = 0. wkind 1: dense W (N, K) row-major of the activation
 * type (nn.Linear). wkind 0: ColBlockQuantizedLinear's buffers as the reference stores them --
 * quant_weight column-major (byte (n, j) at j*N + n, 8/bits codes per byte, low bits first), scales
 * / zeros fp32 (N, G), G = ceil(K / group), group = tile_cols (K for tile_cols = -1); weight element
 * (q - zero) * scale in fp32 (quantization.py:250-267, 390-409). */
int llj_g_linear(int wkind, const void* x, int ldx, int M, int K, const void* W, const float* scales, const float* zeros,
                 int bits, int group, int N, void* y, int ldy, const void* resid, int ldr, int dt, void* stream);
/* c_attn output qkv (B*T, 3C) -> q_out (B*T, C) with RoPE, k (RoPE) / v into cache slot pos[t] % S
 * (model.py:204-228, 312-329); rope (block_size, hs/2, 2) fp32; head size even. */
int llj_g_rope_kv(const void* qkv, void* q_out, void* kcache, void* vcache, const float* rope, const int* pos, int B, int T,
                  int C, int n_head, int S, int dt, void* stream);
/* Causal attention as llj_attention, any head size ((S + hs) * 4 bytes of LDS <= 64 KiB). */
int llj_g_attention(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T, int C,
                    int n_head, int S, int dt, void* stream);
/* h[i] = silu(a1[i]) * a2[i], i < n (model.py:258-259; dt 0: bf16(bf16(silu(a1)) * a2)). */
int llj_g_silu_mul(const void* a1, const void* a2, void* h, size_t n, int dt, void* stream);
/* LLM.int8() (Linear8bitLt, quantization.py:36-75, threshold 6.0; bitsandbytes' algorithm restated)
 * for any K: outlier columns, row scales and the int8 / fp16 products in three plain launches; CB
 * (N, K) int8 row-major, SCB (N) fp32; x, y (or resid + y, resid may be y) of the activation type
 * dt (0 bf16, 1 fp32: as bitsandbytes, the input is cast to fp16 and the fp16 result back to fp32 --
 * a float32 model under --quantize llm.int8, evaluate/full.py's default dtype).
 * ws: llj_g_i8_ws_bytes(M, K) bytes. */
size_t llj_g_i8_ws_bytes(int M, int K);
int llj_g_i8_linear(const void* x, int ldx, int M, int K, const void* CB, const float* SCB, float threshold, void* ws, int N,
                    void* y, int ldy, const void* resid, int ldr, int dt, void* stream);
/* Greedy next token over fp32 logits (generate.py:66-74, top_k = 1), as llj_argmax. */
int llj_g_argmax(const float* logits, int ldl, int M, int V, int* out_idx, int* tokens_out, int tok_stride, const int* pos,
                 void* stream);
/* Sampled next token over fp32 logits (generate.py:66-74 on the reference's float32 model: x =
 * logits / temperature, the top_k threshold (ties kept), fp32 softmax, one inverse-CDF draw), as
 * llj_sample. */
int llj_g_sample(const float* logits, int ldl, int M, int V, float temperature, int top_k, const float* u,
                 unsigned long long seed, int* out_idx, int* tokens_out, int tok_stride, const int* pos, void* stream);

/* ---------------------------------------------------------------- LLM.int8() decode statistics hand-off
 * Decode rows (M <= 8) of an llm.int8 model skip the statistics launch of the attention output y and
 * of the SwiGLU output h (Linear8bitLt inputs of attn.c_proj / mlp.c_proj, quantization.py:36-75):
 * the producing op writes the LLM.int8 row statistics into a small block -- words [16 + 8 s + m]
 * (s < 64 slots) partial SCA[m] = max |f16(A[m, k])| below the threshold (the bits of the float;
 * SCA[m] = the max over the slots), words [528, 528 + ceil(K / 32)) the outlier columns (any row
 * |f16(A)| >= threshold) as bits -- with order-independent atomics (max / or: the values of
 * llj_i8_stats exactly), and the int8 GEMV quantizes its bf16 rows per K chunk from it,
 * taking the fp16 outlier side product from the streamed weights. A block must be zero before its
 * producer runs: llj_attention_i8 zeroes the (previous layer's) h block and llj_i8_swiglu_stats the
 * y block, so a decode step leaves both zero. */
size_t llj_i8_rowstats_bytes(int K);
/* llj_attention / llj_attention_split (nsplit <= 1: one block per (head, row)) + y's statistics. */
int llj_attention_i8(const void* q, const void* kcache, const void* vcache, void* y, const int* pos, int B, int T,
                     int n_head, int head_size, int S, int nsplit, void* part_ws, void* y_stats, void* clr,
                     int clr_words, float threshold, void* stream);
/* llj_norm_swiglu for wfmt 2 on decode rows x (M <= 8) with x's statistics in exactly one of i8ws
 * (llj_i8_norm_stats) and x_stats (a hand-off block, llj_i8_norm_rowstats) + h's statistics into
 * h_stats; zeroes clr_words words at clr. */
int llj_i8_swiglu_stats(const void* x, const void* CB1, const void* SCB1, const void* CB2, const void* SCB2, void* h,
                        int M, int H, int K, const void* i8ws, const void* x_stats, void* h_stats, void* clr,
                        int clr_words, float threshold, void* stream);
/* llj_i8_norm_stats for M <= 8 rows (norm_w NULL: llj_i8_stats of x) that also writes x's (or the
 * normalized rows') hand-off block st; any GEMV entry point takes it in place of i8ws with wfmt
 * 2 | LLJ_WF_I8_ROWSTATS (the rows then quantized per chunk inside the GEMV). */
#define LLJ_WF_I8_ROWSTATS 0x10000
int llj_i8_norm_rowstats(const void* x, const void* norm_w, float eps, void* xn, int M, int K, float threshold, void* ws,
                         void* st, void* stream);
/* x[M, N] += LLM.int8(A)[M, K] . CB^T (CB in I8P, SCB) with A's statistics `stats` (M <= 8). */
int llj_i8_linear_resid(const void* A, int lda, const void* CB, const void* SCB, void* x, int ldx, int M, int N, int K,
                        const void* stats, void* stream);

/* Measurement aid (no reference counterpart): reads `bytes` (a multiple of 16) at p once with
 * non-temporal 16-byte loads over `grid` workgroups of 256 and writes one float per workgroup to
 * out (grid floats). bench.py times it over a buffer far larger than the 256 MB MALL to report the
 * achievable HBM read bandwidth beside the 8 TB/s peak (roofline.achievable). */
int llj_stream_read(const void* p, size_t bytes, float* out, int grid, void* stream);


#ifdef __cplusplus
}
#endif
#endif /* LIT_LLAMA_AMD_H */

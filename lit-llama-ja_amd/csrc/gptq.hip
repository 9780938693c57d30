// GPTQ producer kernels (reference lit_llama/quantization.py:424-614,
// GPTQQuantizer.quantize). The calibration Hessian, its Cholesky factors and the trailing
// block update W[:, i2:] -= Err1 · Hinv[i1:i2, i2:] are plain GEMM / LAPACK work (library calls on
// the device, host side); what is specific to GPTQ is the sequential column loop inside a
// 128-column block (quantization.py:568-596) and the ColBlock packing (pack_weight, 374-388).
//
// llj_gptq_block(_bs): 8 or 4 lanes per weight row (rows are independent inside a block: the update of
// row r uses only its own error and the shared Hinv1 rows). The block's 128 columns of each row
// and Hinv1^T sit in LDS (32 or 64 rows per workgroup: 20 + 66 KiB); 16 columns at a time are quantized
// in registers, then the rest of the block takes their 16 updates per column in one LDS round
// trip, the columns split over the row's lanes. Weights are passed
// transposed (Wt: K x N, element (k, n) at k * N + n) so column i of 128 rows is one coalesced load.
// The block is the reference's `blocksize` (557; 16 / 32 / 64 / 128: whole 16-column register
// groups, at most the 128 columns the LDS holds).
// Every arithmetic step is the reference's fp32 op in the reference's order, rounded on its own
// (this file is built with -ffp-contract=off, lit_llama/_build.py), so a block reproduces the torch CPU
// loop bitwise given the same W1 and Hinv1.
#include "common.h"

namespace llj {

constexpr int kGptqBlock = 128;

constexpr int kGptqSub = 16;          // columns held in registers at a time
// Two shapes, picked by N at launch (both 256 threads, one workgroup per CU by LDS):
//   kGptqRows = 32 rows x 8 lanes, W1^T row stride 40: lane l's column j = b + 16 + l + 8k lands
//     40 l (mod 64) banks over -> the 8 lanes x 8 rows of a wavefront hit 64 distinct banks;
//   kGptqRows = 64 rows x 4 lanes, stride 80 (80 l mod 64 = 16 l; 16 rows per wavefront),
//     for N > 8192 so N / 64 workgroups still fit the 256 CUs in one round.
constexpr int kHs = kGptqBlock + 1;   // LDS row stride of Hinv1^T (odd: conflict-free staging)

// Each row's 16-column quantization group is computed redundantly by all kGptqLanes lanes of the
// row (identical inputs, identical fp32 ops -> identical e[u]); the trailing update of the block's
// remaining columns is split over the lanes (column j to lane (j - b - 16) % kGptqLanes). Every
// column still receives the same updates in the same order, so results are unchanged bit for bit;
// the serial chain per block shrinks from 16 + 112 updates to 16 + 14 (16 + 28) and N / 32
// (N / 64) workgroups fill the chip (N / 128 single-lane workgroups used 32-96 CUs at 7B shapes).
template <int kGptqRows, int kGptqLanes, int kWs>
__global__ __launch_bounds__(kGptqRows * kGptqLanes) void gptq_block_kernel(const float* __restrict__ hinv, int K, int i1,
                                                                  int blk,
                                                                  float* __restrict__ wt, int N,
                                                                  const float* __restrict__ scale,
                                                                  const float* __restrict__ zero, float maxq,
                                                                  float* __restrict__ qt, float* __restrict__ err,
                                                                  float* __restrict__ loss) {
  __shared__ float hsT[kGptqBlock * kHs];              // hsT[j * kHs + i] = Hinv1[i][j]
  __shared__ float ws[kGptqBlock * kWs];               // ws[j * kWs + t] = W1[row t][j]
  constexpr int kGptqThreads = kGptqRows * kGptqLanes;
  const int tid = threadIdx.x;
  const int t = tid / kGptqLanes, l = tid % kGptqLanes;
  for (int v = tid; v < blk * blk; v += kGptqThreads) {
    const int i = v / blk, j = v % blk;
    hsT[j * kHs + i] = hinv[(size_t)(i1 + i) * K + i1 + j];
  }
  const int n = blockIdx.x * kGptqRows + t;
  const int nn = n < N ? n : N - 1;  // clamped: loads stay in bounds, stores are guarded
  const float s = scale[nn], z = zero[nn];
  for (int j = l; j < blk; j += kGptqLanes) ws[j * kWs + t] = wt[(size_t)(i1 + j) * N + nn];
  __syncthreads();
  const bool writer = l == 0 && n < N;
  float lsum = 0.f;
  for (int b = 0; b < blk; b += kGptqSub) {
    float r[kGptqSub], e[kGptqSub];
#pragma unroll
    for (int u = 0; u < kGptqSub; ++u) r[u] = ws[(b + u) * kWs + t];
#pragma unroll
    for (int u = 0; u < kGptqSub; ++u) {
      const int i = b + u;
      const float w = r[u];
      const float d = hsT[i * kHs + i];
      // quantize_weight (quantization.py:470-473): clamp(round(x / scale) + zero, 0, maxq)
      const float qi = fminf(fmaxf(__fadd_rn(rintf(__fdiv_rn(w, s)), z), 0.f), maxq);
      const float q = __fmul_rn(s, __fsub_rn(qi, z));
      const float dq = __fsub_rn(w, q);
      lsum = __fadd_rn(lsum, __fdiv_rn(__fmul_rn(dq, dq), __fmul_rn(d, d)));  // Losses1 (590)
      e[u] = __fdiv_rn(dq, d);                                                  // err1 (592)
      if (writer) {
        qt[(size_t)(i1 + i) * N + n] = q;
        err[(size_t)i * N + n] = e[u];
      }
      // W1[:, i:] -= err1 (x) Hinv1[i, i:] (593) inside the register group (columns <= i are
      // never read again)
#pragma unroll
      for (int v = u + 1; v < kGptqSub; ++v) r[v] = __fsub_rn(r[v], __fmul_rn(e[u], hsT[(b + v) * kHs + i]));
    }
    __syncthreads();  // every lane has read the group's columns before any lane rewrites ws
    // the rest of the block, column by column: the group's updates in increasing i, as the
    // reference applies them one column i at a time
    for (int j = b + kGptqSub + l; j < blk; j += kGptqLanes) {
      float acc = ws[j * kWs + t];
      const float* hc = hsT + j * kHs + b;  // Hinv1[b .. b+15][j]
#pragma unroll
      for (int u = 0; u < kGptqSub; ++u) acc = __fsub_rn(acc, __fmul_rn(e[u], hc[u]));
      ws[j * kWs + t] = acc;
    }
    __syncthreads();  // the next group's columns are complete
  }
  if (writer) loss[n] += lsum;
}

// pack_weight (quantization.py:374-388) of reconstructed weights Qt (K x N, fp32):
// code = uint8(clamp(q / scale + zero, 0, 2^bits - 1)) (truncating cast, as the reference's
// .to(torch.uint8)), entries_per_byte = 8 / bits codes per byte, column epb*j + nr in bits
// [nr*bits, (nr+1)*bits) of byte (n, j); quant_weight is column-major: byte (n, j) at j * N + n.
__global__ __launch_bounds__(256) void colblock_pack_kernel(const float* __restrict__ qt, int K, int N,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ zero, int bits,
                                                            unsigned char* __restrict__ qw) {
  const int epb = 8 / bits;
  const int n = blockIdx.x * 256 + threadIdx.x;
  const int j = blockIdx.y;
  if (n >= N) return;
  const float s = scale[n], z = zero[n], maxq = (float)((1 << bits) - 1);
  unsigned v = 0;
  for (int nr = 0; nr < epb; ++nr) {
    const float x = qt[(size_t)(epb * j + nr) * N + n];
    const float c = fminf(fmaxf(__fadd_rn(__fdiv_rn(x, s), z), 0.f), maxq);
    v += ((unsigned)c) << (nr * bits);
  }
  qw[(size_t)j * N + n] = (unsigned char)v;
}

}  // namespace llj

using namespace llj;

extern "C" {

int llj_gptq_block_bs(const float* hinv, int K, int i1, int blocksize, float* wt, int N, const float* scale,
                      const float* zero, int bits, float* qt, float* err, float* loss, void* stream) {
  LLJ_REQUIRE(blocksize >= kGptqSub && blocksize <= kGptqBlock && blocksize % kGptqSub == 0);
  LLJ_REQUIRE(K > 0 && N > 0 && i1 >= 0 && i1 % blocksize == 0 && i1 + blocksize <= K);
  LLJ_REQUIRE(bits == 2 || bits == 4 || bits == 8);
  LLJ_REQUIRE(hinv && wt && scale && zero && qt && err && loss);
  const float maxq = (float)((1 << bits) - 1);
  if (N > 8192)
    hipLaunchKernelGGL((gptq_block_kernel<64, 4, 80>), dim3((N + 63) / 64), dim3(256), 0, (hipStream_t)stream, hinv,
                       K, i1, blocksize, wt, N, scale, zero, maxq, qt, err, loss);
  else
    hipLaunchKernelGGL((gptq_block_kernel<32, 8, 40>), dim3((N + 31) / 32), dim3(256), 0, (hipStream_t)stream, hinv,
                       K, i1, blocksize, wt, N, scale, zero, maxq, qt, err, loss);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_gptq_block(const float* hinv, int K, int i1, float* wt, int N, const float* scale, const float* zero,
                   int bits, float* qt, float* err, float* loss, void* stream) {
  return llj_gptq_block_bs(hinv, K, i1, kGptqBlock, wt, N, scale, zero, bits, qt, err, loss, stream);
}

int llj_colblock_pack(const float* qt, int K, int N, const float* scale, const float* zero, int bits,
                      unsigned char* qw, void* stream) {
  LLJ_REQUIRE(K > 0 && N > 0 && (bits == 2 || bits == 4 || bits == 8) && K % (8 / bits) == 0);
  LLJ_REQUIRE(qt && scale && zero && qw);
  hipLaunchKernelGGL(colblock_pack_kernel, dim3((N + 255) / 256, K / (8 / bits)), dim3(256), 0, (hipStream_t)stream,
                     qt, K, N, scale, zero, bits, qw);
  LLJ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

// int4 weight layout conversion between the reference's ColBlockQuantizedLinear buffer and
// the W4P streaming layout consumed by gemv.hip.
//
// Reference layout (quantization.py:348-357, pack_weight 374-388): `quant_weight` is the
// logical (N, K/2) uint8 tensor stored column-major, i.e. physically a row-major (K/2, N)
// byte array; byte [k/2][n] holds q[n, k] in its low nibble for even k and in its high
// nibble for odd k.
//
// W4P: tile (nt, kc) = 16 columns x 128 k = 1 KiB at byte offset (nt * K/128 + kc) * 1024.
// Lane l (0..63) owns bytes [16 l, 16 l + 16): dword t (0..3) holds the 8 codes of column
// 16 nt + (l & 15) for k = 128 kc + 32 (l >> 4) + 8 t + j, j = 0..7, with code j at bit
// 4 (j >> 1) + 16 (j & 1) so that ((dword >> 4 i) & 0x000F000F) is the (j = 2i, 2i+1) pair.
// Both conversions are exact inverses (tested bit-for-bit).
//
// W8P (gptq.int8, ColBlock bits=8): the reference buffer is the logical (N, K) uint8 tensor
// stored column-major = physically row-major (K, N), one code per byte. Tile (nt, kc) is 2 KiB
// at (nt * K/128 + kc) * 2048: the W4P tile of the low nibbles, then the W4P tile of the high
// nibbles (gemv.hip WF_W8 streams both with one 16-B load each per lane).
#include "common.h"

namespace llj {

__device__ __forceinline__ int w4p_bit(int j) { return 4 * (j >> 1) + 16 * (j & 1); }

__global__ void w4_repack_kernel(const uint8_t* __restrict__ ref, uint32_t* __restrict__ out, int N, int K) {
  const size_t total = (size_t)N * K / 8;  // dwords
  const int KC = K >> 7;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int t = (int)(i & 3);
    const int l = (int)((i >> 2) & 63);
    const size_t tile = i >> 8;
    const int kc = (int)(tile % KC);
    const int nt = (int)(tile / KC);
    const int n = nt * 16 + (l & 15);
    const int k0 = kc * 128 + 32 * (l >> 4) + 8 * t;
    uint32_t d = 0;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {  // 4 bytes = codes k0 + 2jj, k0 + 2jj + 1
      const uint32_t b = ref[(size_t)((k0 >> 1) + jj) * N + n];
      d |= (b & 0xF) << w4p_bit(2 * jj);
      d |= (b >> 4) << w4p_bit(2 * jj + 1);
    }
    out[i] = d;
  }
}

__global__ void w8_repack_kernel(const uint8_t* __restrict__ ref, uint32_t* __restrict__ out, int N, int K) {
  const size_t total = (size_t)N * K / 4;  // dwords (two nibble planes)
  const int KC = K >> 7;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int t = (int)(i & 3);
    const int l = (int)((i >> 2) & 63);
    const int hi = (int)((i >> 8) & 1);
    const size_t tile = i >> 9;
    const int kc = (int)(tile % KC);
    const int nt = (int)(tile / KC);
    const int n = nt * 16 + (l & 15);
    const int k0 = kc * 128 + 32 * (l >> 4) + 8 * t;
    uint32_t d = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t b = ref[(size_t)(k0 + j) * N + n];
      d |= (hi ? b >> 4 : b & 0xF) << w4p_bit(j);
    }
    out[i] = d;
  }
}

__global__ void w4_unpack_kernel(const uint32_t* __restrict__ in, uint8_t* __restrict__ ref, int N, int K) {
  const size_t total = (size_t)N * K / 2;  // bytes of the reference buffer
  const int KC = K >> 7;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int n = (int)(i % N);
    const int k = 2 * (int)(i / N);
    const int kc = k >> 7, w = k & 127;
    const int g = w >> 5, t = (w & 31) >> 3, j = w & 7;  // j even
    const int l = 16 * g + (n & 15);
    const uint32_t d = in[((size_t)((n >> 4) * KC + kc) * 64 + l) * 4 + t];
    ref[i] = (uint8_t)(((d >> w4p_bit(j)) & 0xF) | (((d >> w4p_bit(j + 1)) & 0xF) << 4));
  }
}

__global__ void w8_unpack_kernel(const uint32_t* __restrict__ in, uint8_t* __restrict__ ref, int N, int K) {
  const size_t total = (size_t)N * K;  // bytes of the reference buffer (one code each)
  const int KC = K >> 7;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int n = (int)(i % N);
    const int k = (int)(i / N);
    const int kc = k >> 7, w = k & 127;
    const int g = w >> 5, t = (w & 31) >> 3, j = w & 7;
    const int l = 16 * g + (n & 15);
    const size_t tile = (size_t)(n >> 4) * KC + kc;
    const uint32_t lo = in[(tile * 128 + l) * 4 + t];       // low-nibble plane
    const uint32_t hi = in[(tile * 128 + 64 + l) * 4 + t];  // high-nibble plane
    ref[i] = (uint8_t)(((lo >> w4p_bit(j)) & 0xF) | (((hi >> w4p_bit(j)) & 0xF) << 4));
  }
}

// sz[n] = (scale[n], off + zero[n]) in fp32 from the module's scale/zero buffers (any of
// fp32 / bf16 / fp16, given by dtype code 0/1/2; one group per row: tile_cols = -1); off is the
// magic-exponent offset of the format (W4P 128, W8P 128 + 2048).
// LLM.int8() CB (N, K) int8 row-major <-> "I8P": per (16-column tile nt, 128-deep chunk c) 2 KiB,
// [step t = 0: 64 lanes x 16 B][step t = 1: 64 lanes x 16 B]; lane l of step t holds
// CB[16 nt + (l & 15)][128 c + 64 t + 16 (l >> 4) + 0 .. 15] (the int8 MFMA 16x16x64 B fragment),
// so a wave reads 1 KiB contiguous per step (row-major CB: 16 rows x 64 B per wave load).
// One thread per 16-byte piece.
__global__ void i8_tile_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, int N, int K, int unpack) {
  const size_t total = (size_t)N * K / 16;
  const int KC = K / 128;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int l = (int)(i & 63), t = (int)((i >> 6) & 1);
    const size_t tc = i >> 7;  // (tile, chunk)
    const int c = (int)(tc % KC), nt = (int)(tc / KC);
    const int n = 16 * nt + (l & 15), k = 128 * c + 64 * t + 16 * (l >> 4);
    const size_t rm = ((size_t)n * K + k) / 16;  // row-major piece
    if (unpack) dst[rm] = src[i];
    else dst[i] = src[rm];
  }
}

__global__ void w4_sz_kernel(const void* scales, const void* zeros, int dtype, float2* sz, int N, float off) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s, z;
  if (dtype == 0) {
    s = ((const float*)scales)[n]; z = ((const float*)zeros)[n];
  } else if (dtype == 1) {
    s = bf2f(((const bf16_t*)scales)[n]); z = bf2f(((const bf16_t*)zeros)[n]);
  } else {
    s = (float)((const _Float16*)scales)[n]; z = (float)((const _Float16*)zeros)[n];
  }
  sz[n] = make_float2(s, off + z);
}

}  // namespace llj

using namespace llj;

extern "C" {

int llj_w4_repack(const void* qweight_ref, void* packed, int N, int K, void* stream) {
  LLJ_REQUIRE(N > 0 && K > 0 && N % 16 == 0 && K % 128 == 0);
  const size_t total = (size_t)N * K / 8;
  int grid = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(w4_repack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)qweight_ref,
                     (uint32_t*)packed, N, K);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_w4_unpack(const void* packed, void* qweight_ref, int N, int K, void* stream) {
  LLJ_REQUIRE(N > 0 && K > 0 && N % 16 == 0 && K % 128 == 0);
  const size_t total = (size_t)N * K / 2;
  int grid = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(w4_unpack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint32_t*)packed,
                     (uint8_t*)qweight_ref, N, K);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_w4_scale_zero(const void* scales, const void* zeros, int dtype, void* sz, int N, void* stream) {
  LLJ_REQUIRE(N > 0 && dtype >= 0 && dtype <= 2);
  hipLaunchKernelGGL(w4_sz_kernel, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, scales, zeros, dtype,
                     (float2*)sz, N, 128.f);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_w8_repack(const void* qweight_ref, void* packed, int N, int K, void* stream) {
  LLJ_REQUIRE(N > 0 && K > 0 && N % 16 == 0 && K % 128 == 0);
  const size_t total = (size_t)N * K / 4;
  int grid = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(w8_repack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)qweight_ref,
                     (uint32_t*)packed, N, K);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_w8_unpack(const void* packed, void* qweight_ref, int N, int K, void* stream) {
  LLJ_REQUIRE(N > 0 && K > 0 && N % 16 == 0 && K % 128 == 0);
  const size_t total = (size_t)N * K;
  int grid = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(w8_unpack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint32_t*)packed,
                     (uint8_t*)qweight_ref, N, K);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_i8_repack(const void* cb, void* packed, int N, int K, void* stream) {
  LLJ_REQUIRE(N > 0 && K > 0 && N % 16 == 0 && K % 128 == 0 && cb != packed);
  const size_t total = (size_t)N * K / 16;
  int grid = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(i8_tile_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint4*)cb, (uint4*)packed,
                     N, K, 0);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_i8_unpack(const void* packed, void* cb, int N, int K, void* stream) {
  LLJ_REQUIRE(N > 0 && K > 0 && N % 16 == 0 && K % 128 == 0 && cb != packed);
  const size_t total = (size_t)N * K / 16;
  int grid = (int)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(i8_tile_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint4*)packed, (uint4*)cb,
                     N, K, 1);
  LLJ_CHECK_LAUNCH();
  return 0;
}

int llj_w8_scale_zero(const void* scales, const void* zeros, int dtype, void* sz, int N, void* stream) {
  LLJ_REQUIRE(N > 0 && dtype >= 0 && dtype <= 2);
  hipLaunchKernelGGL(w4_sz_kernel, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, scales, zeros, dtype,
                     (float2*)sz, N, 2176.f);
  LLJ_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

// Micro-benchmark of the persistent engine's consumer inner loop (csrc/engine.hip consume_t): per
// CU one 512-thread workgroup, NCW consumer waves (+ idle waves up to 8), an LDS ring of 1 KiB W4P
// blocks filled once, the A fragments of 5 chunks in registers; every consumer wave runs `tiles`
// tiles of NM matrices x its chunks (c = w mod NCW of kc = 32), per tile: 5 x NM ring reads issued
// at once, then per chunk NM x (4 x dequant + MFMA 16x16x32 bf16), then one partial-sum store.
// Reports s_memtime cycles per block (1 KiB) per wave and per SIMD (the busiest pairing).
// Variants: 0 the engine's loop, 1 MFMA on the raw codes (no dequant VALU), 2 dequant only (no
// MFMA; results kept live), 3 dequant with 20 instead of 28 VALU ops per block (pairs 1/3 by
// v_and_or on a pre-shifted word: the layout a re-packed tile would need), 4 the engine's loop with
// the chunk's NM x 4 MFMAs issued after all its dequant, 5 the engine's loop with 4 independent
// accumulators per matrix (fragment t into accumulator t: no dependent MFMA chain), 6 with 2.
// Usage: consume_probe <variant> <consumer waves> <NM> <tiles>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t and_or(uint32_t x, uint32_t m, uint32_t c) { return (x & m) | c; }
__device__ __forceinline__ bf16x8 dequant(uint32_t w, uint32_t msk, uint32_t mag) {
  uint4 b = make_uint4(and_or(w, msk, mag), and_or(w >> 4, msk, mag), and_or(w >> 8, msk, mag), and_or(w >> 12, msk, mag));
  return __builtin_bit_cast(bf16x8, b);
}
// 5 ops per 8 codes: pairs 0 / 2 from w, pairs 1 / 3 from a second word holding w >> 4 (as if the
// tile stored both phases): and_or(w), and_or(w >> 8), and_or(v), and_or(v >> 8) with v = w >> 4
__device__ __forceinline__ bf16x8 dequant5(uint32_t w, uint32_t msk, uint32_t mag) {
  const uint32_t v = w >> 4;
  uint4 b = make_uint4(and_or(w, msk, mag), and_or(v, msk, mag), and_or(w >> 8, msk, mag), and_or(v >> 8, msk, mag));
  return __builtin_bit_cast(bf16x8, b);
}

constexpr int AREG_C = 5;
template <int VAR, int NM>
__global__ __launch_bounds__(512, 1) void probe(const uint4* __restrict__ fill, int ncw, int tiles, unsigned long long* out,
                                               float* sink) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < 120 * 1024 / 16; i += 512) reinterpret_cast<uint4*>(smem)[i] = fill[i & 4095];
  __syncthreads();
  if (w >= ncw) return;
  const int kc = 32, nch = (kc - w + ncw - 1) / ncw;
  const unsigned char* ring = smem;
  const unsigned char* A = smem + 104 * 1024;
  uint32_t msk = 0x000F000Fu, mag = 0x43004300u;
  asm volatile("" : "+s"(msk));
  asm volatile("" : "+v"(mag));
  bf16x8 ar[AREG_C][4];
#pragma unroll
  for (int ci = 0; ci < AREG_C; ++ci)
#pragma unroll
    for (int t = 0; t < 4; ++t)
      ar[ci][t] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(A + 256 * (ci * 7 + w) + 64 * (lane >> 4) + 16 * t));
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  uint32_t xo = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int j = 0; j < tiles; ++j) {
    const int tb = (j * kc * NM) % 96;
    u32x4 wt[AREG_C][NM];
#pragma unroll
    for (int ci = 0; ci < AREG_C; ++ci) {
      const int b = tb + (w + (ci < nch ? ci : 0) * ncw) * NM;
#pragma unroll
      for (int m = 0; m < NM; ++m) wt[ci][m] = *reinterpret_cast<const u32x4*>(ring + (size_t)((b + m) % 104) * 1024 + 16 * lane);
    }
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
    f32x4 q0[4] = {a0, a0, a0, a0}, q1[4] = {a0, a0, a0, a0};
#pragma unroll
    for (int ci = 0; ci < AREG_C; ++ci) {
      if (ci < nch) {
        if constexpr (VAR == 0) {
#pragma unroll
          for (int t = 0; t < 4; ++t) a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[ci][t], dequant(wt[ci][0][t], msk, mag), a0, 0, 0, 0);
          if constexpr (NM == 2) {
#pragma unroll
            for (int t = 0; t < 4; ++t) a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[ci][t], dequant(wt[ci][1][t], msk, mag), a1, 0, 0, 0);
          }
        } else if constexpr (VAR == 1) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const u32x4 r = u32x4{wt[ci][0][t], wt[ci][0][(t + 1) & 3], wt[ci][0][(t + 2) & 3], wt[ci][0][(t + 3) & 3]};
            a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[ci][t], __builtin_bit_cast(bf16x8, r), a0, 0, 0, 0);
          }
          if constexpr (NM == 2) {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              const u32x4 r = u32x4{wt[ci][1][t], wt[ci][1][(t + 1) & 3], wt[ci][1][(t + 2) & 3], wt[ci][1][(t + 3) & 3]};
              a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[ci][t], __builtin_bit_cast(bf16x8, r), a1, 0, 0, 0);
            }
          }
        } else if constexpr (VAR == 2) {
#pragma unroll
          for (int m = 0; m < NM; ++m)
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              const uint4 d = __builtin_bit_cast(uint4, dequant(wt[ci][m][t], msk, mag));
              xo ^= d.x ^ d.y ^ d.z ^ d.w;
            }
        } else if constexpr (VAR == 3) {
#pragma unroll
          for (int t = 0; t < 4; ++t) a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[ci][t], dequant5(wt[ci][0][t], msk, mag), a0, 0, 0, 0);
          if constexpr (NM == 2) {
#pragma unroll
            for (int t = 0; t < 4; ++t) a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[ci][t], dequant5(wt[ci][1][t], msk, mag), a1, 0, 0, 0);
          }
        } else if constexpr (VAR == 5 || VAR == 6) {
          constexpr int NA = VAR == 5 ? 4 : 2;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            q0[t % NA] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[ci][t], dequant(wt[ci][0][t], msk, mag), q0[t % NA], 0, 0, 0);
            if constexpr (NM == 2)
              q1[t % NA] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[ci][t], dequant(wt[ci][1][t], msk, mag), q1[t % NA], 0, 0, 0);
          }
        } else {
          bf16x8 d0[4], d1[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            d0[t] = dequant(wt[ci][0][t], msk, mag);
            if constexpr (NM == 2) d1[t] = dequant(wt[ci][1][t], msk, mag);
          }
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[ci][t], d0[t], a0, 0, 0, 0);
            if constexpr (NM == 2) a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[ci][t], d1[t], a1, 0, 0, 0);
          }
        }
      }
    }
    acc0 += a0 + (q0[0] + q0[1]) + (q0[2] + q0[3]);
    acc1 += a1 + (q1[0] + q1[1]) + (q1[2] + q1[3]);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    out[(size_t)blockIdx.x * 16 + w] = t1 - t0;
    out[(size_t)blockIdx.x * 16 + 8 + w] = r1 - r0;  // 100 MHz ticks: the clock the loop ran at
  }
  sink[(size_t)blockIdx.x * 512 + tid] = acc0[0] + acc1[1] + (float)(xo & 1);
}

template <int VAR, int NM>
static void run(int ncw, int tiles, const uint4* fill, unsigned long long* out, float* sink) {
  hipFuncSetAttribute((const void*)probe<VAR, NM>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL((probe<VAR, NM>), dim3(256), dim3(512), 120 * 1024, 0, fill, ncw, tiles, out, sink);
}

int main(int argc, char** argv) {
  const int var = argc > 1 ? atoi(argv[1]) : 0, ncw = argc > 2 ? atoi(argv[2]) : 7, nm = argc > 3 ? atoi(argv[3]) : 2,
            tiles = argc > 4 ? atoi(argv[4]) : 64;
  if (ncw < 1 || ncw > 8 || (nm != 1 && nm != 2)) return 2;
  uint4* fill;
  unsigned long long* out;
  float* sink;
  hipMalloc(&fill, 4096 * 16);
  hipMalloc(&out, 256 * 16 * 8);
  hipMalloc(&sink, 256 * 512 * 4);
  std::vector<uint32_t> h(4096 * 4);
  uint32_t s = 12345;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = (s & 0x0FFF0FFFu) | 0x3C003C00u; }
  hipMemcpy(fill, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipMemset(out, 0, 256 * 16 * 8);
  for (int rep = 0; rep < 2; ++rep) {
#define R(V) (nm == 1 ? run<V, 1>(ncw, tiles, fill, out, sink) : run<V, 2>(ncw, tiles, fill, out, sink))
    switch (var) {
      case 0: R(0); break;
      case 1: R(1); break;
      case 2: R(2); break;
      case 3: R(3); break;
      case 4: R(4); break;
      case 5: R(5); break;
      default: R(6); break;
    }
#undef R
    if (hipDeviceSynchronize() != hipSuccess) return 3;
  }
  std::vector<unsigned long long> ho(256 * 16);
  hipMemcpy(ho.data(), out, ho.size() * 8, hipMemcpyDeviceToHost);
  // per wave: cycles per block; per SIMD (waves w and w + 4 share SIMD w % 4): busiest
  double sum = 0, worst = 0, ghz = 0;
  int n = 0;
  for (int b = 0; b < 256; ++b)
    for (int w = 0; w < ncw; ++w) {
      const int nch = (32 - w + ncw - 1) / ncw;
      const double c = (double)ho[b * 16 + w] / ((double)tiles * nch * nm);
      sum += c;
      ghz += (double)ho[b * 16 + w] / ((double)ho[b * 16 + 8 + w] * 10.0);  // cycles per ns
      ++n;
      worst = std::max(worst, (double)ho[b * 16 + w]);
    }
  printf("clock %.2f GHz; ", ghz / n);
  const double tot_blocks = 32.0 * nm * tiles;  // per CU
  printf("variant %d consumers %d NM %d tiles %d: cycles/block/wave avg %.1f; CU wall %.0f cycles = %.1f cycles per block per CU "
         "(%.1f per SIMD)\n",
         var, ncw, nm, tiles, sum / n, worst, worst / tot_blocks, 4 * worst / tot_blocks);
  return 0;
}

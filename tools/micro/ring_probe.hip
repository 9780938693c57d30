// Micro-benchmark of the persistent engine's weight stream (csrc/engine.hip loader + consumers) in
// isolation: one workgroup per CU streams MB KiB of its own 1 KiB blocks from HBM into an LDS ring
// by global_load_lds_dwordx4 (nt) and NC consumer waves take every block (ds_read_b128 + 4 MFMA,
// like the engine's consume loop), with the engine's landed / freed LDS counters. Variants:
//   mode 0: loader only (no consumers; the ring is recycled without waiting)
//   mode 1: loader + consumers (engine protocol)
//   mode 2: every wave loads its own blocks to registers (global_load_dwordx4 nt, D in flight): the
//           GEMV's stream, for comparison
//   mode 3: mode 1 with s_sleep(1) in the consumers' landed spin (LDS polling pressure)
// Prints GB/s per CU and chip-wide for each mode. Usage: ./ring_probe [MB_per_CU_KiB]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);     \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ unsigned lds_ld(const unsigned* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_st(unsigned* p, unsigned v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

template <int NC, int D, int MODE>
__global__ __launch_bounds__(64 * (NC + 1), 1) void ring_kernel(const char* __restrict__ w, int nblk, int nb, float* out,
                                                                  unsigned long long* cycles) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned* ctl = reinterpret_cast<unsigned*>(smem);
  unsigned char* ring = smem + 256;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (threadIdx.x < 64) ctl[threadIdx.x] = 0;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const char* base = w + (size_t)blockIdx.x * nblk * 1024 + 16 * lane;
  if (MODE == 2) {  // register stream by every wave: blocks wave, wave + NW, ...
    constexpr int NW = NC + 1;
    f32x4 acc = {0, 0, 0, 0};
    u32x4 r[D];
    int i = wave;
#pragma unroll
    for (int d = 0; d < D; ++d) r[d] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + (size_t)(i + NW * d < nblk ? i + NW * d : 0) * 1024));
    for (; i < nblk; i += NW * D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        acc[0] += __builtin_bit_cast(float, r[d][0] & 0x3FF);
        const int j = i + NW * (d + D);
        r[d] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + (size_t)(j < nblk ? j : 0) * 1024));
      }
    }
    if (acc[0] == 1234.5f) out[threadIdx.x] = acc[1];
  } else if (wave == NC) {  // loader (the engine's: groups of 8 DMAs, one check / publish per group)
    const uint32_t rb = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ring);
    int pub = 0, limit = nb, slot = 0;
    for (int b = 0; b < nblk; b += 8) {
      if (MODE != 0 && b + 8 > limit) {
        for (;;) {
          int F = 0x7fffffff;
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            const int f = (int)lds_ld(ctl + 1 + c) * NC + c;
            F = f < F ? f : F;
          }
          limit = F + nb;
          if (limit >= b + 8) break;
          if (pub < b) {
            wait_vm<0>();
            pub = b;
            if (lane == 0) lds_st(ctl, (unsigned)pub);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        unsigned keep;
        const char* src = base + (size_t)(b + u) * 1024;
        const uint32_t dst = __builtin_amdgcn_readfirstlane(rb + (uint32_t)slot * 1024u);
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
        if (++slot == nb) slot = 0;
      }
      if (b + 8 - pub >= D + 8) {
        wait_vm<D>();
        pub = b + 8 - D;
        if (lane == 0) lds_st(ctl, (unsigned)pub);
      }
    }
    wait_vm<0>();
    if (lane == 0) lds_st(ctl, (unsigned)nblk);
  } else if (MODE == 1 || MODE == 3) {  // consumers
    f32x4 acc = {0, 0, 0, 0};
    const bf16x8 a = __builtin_bit_cast(bf16x8, u32x4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u});
    int landed = 0, slot = wave;
    for (int b = wave; b < nblk; b += NC) {
      while (landed <= b) {
        landed = (int)lds_ld(ctl);
        if (MODE == 3 && landed <= b) __builtin_amdgcn_s_sleep(1);
      }
      const u32x4 wv = *reinterpret_cast<const u32x4*>(ring + (size_t)slot * 1024 + 16 * lane);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t x = wv[t];
        const u32x4 d = {(x & 0x000F000Fu) | 0x43004300u, ((x >> 4) & 0x000F000Fu) | 0x43004300u,
                         ((x >> 8) & 0x000F000Fu) | 0x43004300u, ((x >> 12) & 0x000F000Fu) | 0x43004300u};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, d), acc, 0, 0, 0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) lds_st(ctl + 1 + wave, (unsigned)(b / NC + 1));
      slot += NC;
      if (slot >= nb) slot -= nb;
    }
    if (acc[0] == 1234.5f) out[threadIdx.x] = acc[1];
  } else if (MODE == 4) {  // consumers: blocks b and b + NC per trip, both reads issued first
    f32x4 acc = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0};
    const bf16x8 a = __builtin_bit_cast(bf16x8, u32x4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u});
    int landed = 0, slot = wave;
    for (int b = wave; b < nblk; b += 2 * NC) {
      const int b2 = b + NC < nblk ? b + NC : b;
      while (landed <= b2) landed = (int)lds_ld(ctl);
      int slot2 = slot + NC;
      if (slot2 >= nb) slot2 -= nb;
      const u32x4 wv = *reinterpret_cast<const u32x4*>(ring + (size_t)slot * 1024 + 16 * lane);
      const u32x4 wv2 = *reinterpret_cast<const u32x4*>(ring + (size_t)slot2 * 1024 + 16 * lane);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t x = wv[t], y = wv2[t];
        const u32x4 d = {(x & 0x000F000Fu) | 0x43004300u, ((x >> 4) & 0x000F000Fu) | 0x43004300u,
                         ((x >> 8) & 0x000F000Fu) | 0x43004300u, ((x >> 12) & 0x000F000Fu) | 0x43004300u};
        const u32x4 e = {(y & 0x000F000Fu) | 0x43004300u, ((y >> 4) & 0x000F000Fu) | 0x43004300u,
                         ((y >> 8) & 0x000F000Fu) | 0x43004300u, ((y >> 12) & 0x000F000Fu) | 0x43004300u};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, d), acc, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, e), acc2, 0, 0, 0);
      }
      if (lane == 0) lds_st(ctl + 1 + wave, (unsigned)(b2 / NC + 1));
      slot = slot2 + NC;
      if (slot >= nb) slot -= nb;
    }
    if (acc[0] + acc2[0] == 1234.5f) out[threadIdx.x] = acc[1];
  }
  if (threadIdx.x == 0) cycles[blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
}

template <int NC, int D, int MODE>
static int run(const char* w, int nblk, int nb, int G, float* out, unsigned long long* cyc, const char* name) {
  auto k = ring_kernel<NC, D, MODE>;
  const size_t lds = 256 + (size_t)nb * 1024;
  CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(k, dim3(G), dim3(64 * (NC + 1)), lds, 0, w, nblk, nb, out, cyc);
  CHECK(hipEventRecord(e0));
  const int R = 10;
  for (int it = 0; it < R; ++it) hipLaunchKernelGGL(k, dim3(G), dim3(64 * (NC + 1)), lds, 0, w, nblk, nb, out, cyc);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / R;
  const double bytes = (double)nblk * 1024 * G;
  printf("%-44s NC=%d D=%d: %8.1f us  %6.1f GB/s per CU  %6.2f TB/s chip\n", name, NC, D, us,
         (double)nblk * 1024 / us / 1e3, bytes / us / 1e6);
  return 0;
}

int main(int argc, char** argv) {
  const int kib = argc > 1 ? atoi(argv[1]) : 400;
  int G = 0;
  CHECK(hipDeviceGetAttribute(&G, hipDeviceAttributeMultiprocessorCount, 0));
  const int nblk = kib;
  char* w;
  float* out;
  unsigned long long* cyc;
  CHECK(hipMalloc(&w, (size_t)nblk * 1024 * G));
  CHECK(hipMemset(w, 0x11, (size_t)nblk * 1024 * G));
  CHECK(hipMalloc(&out, 4096));
  CHECK(hipMalloc(&cyc, 8 * 4096));
  const int nb = 100;
  printf("per CU %d KiB, %d CUs, ring %d KiB\n", kib, G, nb);
  run<3, 48, 0>(w, nblk, nb, G, out, cyc, "loader only");
  run<3, 48, 1>(w, nblk, nb, G, out, cyc, "loader + consumers");
  run<7, 48, 1>(w, nblk, nb, G, out, cyc, "loader + consumers");
  run<7, 48, 3>(w, nblk, nb, G, out, cyc, "loader + consumers (sleep in spin)");
  run<3, 48, 4>(w, nblk, nb, G, out, cyc, "loader + consumers (2 blocks / trip)");
  run<7, 48, 4>(w, nblk, nb, G, out, cyc, "loader + consumers (2 blocks / trip)");
  run<3, 8, 2>(w, nblk, nb, G, out, cyc, "register stream (all waves)");
  run<7, 4, 2>(w, nblk, nb, G, out, cyc, "register stream (all waves)");
  return 0;
}

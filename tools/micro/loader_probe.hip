// Which way of filling an LDS ring from HBM sustains the per-CU weight stream a persistent decode
// engine needs (~25 GB/s per CU)? One workgroup per CU streams N KiB of its own 1 KiB blocks into a
// 100-slot LDS ring, nothing consumes (the ring is recycled). Variants:
//   dma1    one loader wave, global_load_lds_dwordx4 nt, 8 DMAs per loop trip, vmcnt(D) window
//   dma1-rt the same without nt
//   dma2    two loader waves (even / odd blocks)
//   dma4    four loader waves
//   reg1    one wave: global_load_dwordx4 nt into VGPRs (D deep), ds_write_b128 into the ring
//   reg2    two such waves
// Prints GB/s per CU and chip-wide. Usage: ./loader_probe [KiB_per_CU]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <bool NT>
__device__ __forceinline__ void dma(const char* src, uint32_t dst) {
  unsigned keep;
  if (NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
}

// KIND 0: LDS-DMA by NL loader waves; KIND 1: register-staged by NL waves
template <int KIND, int NL, int D, bool NT>
__global__ __launch_bounds__(256, 1) void fill_kernel(const char* __restrict__ w, int nblk, int nb, float* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wave >= NL) return;
  const char* base = w + (size_t)blockIdx.x * nblk * 1024 + 16 * lane;
  const uint32_t rb = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
  if (KIND == 0) {
    int slot = wave;
    for (int b = wave; b < nblk; b += 8 * NL) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int bb = b + u * NL < nblk ? b + u * NL : b;
        dma<NT>(base + (size_t)bb * 1024, __builtin_amdgcn_readfirstlane(rb + (uint32_t)slot * 1024u));
        slot += NL;
        if (slot >= nb) slot -= nb;
      }
      wait_vm<D>();
    }
    wait_vm<0>();
  } else {
    u32x4 r[D];
    int slot = wave;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int b = wave + d * NL;
      r[d] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + (size_t)(b < nblk ? b : 0) * 1024));
    }
    for (int b0 = wave; b0 < nblk; b0 += D * NL) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        *reinterpret_cast<u32x4*>(smem + (size_t)slot * 1024 + 16 * lane) = r[d];
        slot += NL;
        if (slot >= nb) slot -= nb;
        const int b = b0 + (d + D) * NL;
        r[d] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + (size_t)(b < nblk ? b : 0) * 1024));
      }
    }
    if (r[0][0] == 12345u) out[threadIdx.x] = 1.f;
  }
}

template <int KIND, int NL, int D, bool NT>
static int run(const char* w, int nblk, int nb, int G, float* out, const char* name) {
  auto k = fill_kernel<KIND, NL, D, NT>;
  const size_t lds = (size_t)nb * 1024;
  CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(k, dim3(G), dim3(256), lds, 0, w, nblk, nb, out);
  CHECK(hipEventRecord(e0));
  const int R = 10;
  for (int it = 0; it < R; ++it) hipLaunchKernelGGL(k, dim3(G), dim3(256), lds, 0, w, nblk, nb, out);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / R;
  printf("%-10s NL=%d D=%2d: %8.1f us  %6.1f GB/s per CU  %6.2f TB/s chip\n", name, NL, D, us,
         (double)nblk * 1024 / us / 1e3, (double)nblk * 1024 * G / us / 1e6);
  return 0;
}

int main(int argc, char** argv) {
  const int nblk = argc > 1 ? atoi(argv[1]) : 2000;
  int G = 0;
  CHECK(hipDeviceGetAttribute(&G, hipDeviceAttributeMultiprocessorCount, 0));
  char* w;
  float* out;
  CHECK(hipMalloc(&w, (size_t)nblk * 1024 * G));
  CHECK(hipMemset(w, 0x11, (size_t)nblk * 1024 * G));
  CHECK(hipMalloc(&out, 4096));
  const int nb = 100;
  printf("per CU %d KiB, %d CUs\n", nblk, G);
  run<0, 1, 16, true>(w, nblk, nb, G, out, "dma1");
  run<0, 1, 32, true>(w, nblk, nb, G, out, "dma1");
  run<0, 1, 56, true>(w, nblk, nb, G, out, "dma1");
  run<0, 1, 32, false>(w, nblk, nb, G, out, "dma1-rt");
  run<0, 2, 16, true>(w, nblk, nb, G, out, "dma2");
  run<0, 2, 32, true>(w, nblk, nb, G, out, "dma2");
  run<0, 4, 16, true>(w, nblk, nb, G, out, "dma4");
  run<1, 1, 16, true>(w, nblk, nb, G, out, "reg1");
  run<1, 1, 32, true>(w, nblk, nb, G, out, "reg1");
  run<1, 2, 16, true>(w, nblk, nb, G, out, "reg2");
  run<1, 4, 8, true>(w, nblk, nb, G, out, "reg4");
  return 0;
}

// Which way of filling an LDS ring from HBM sustains the per-CU weight stream a persistent decode
// engine needs (~25 GB/s per CU)? One workgroup per CU streams N KiB of its own 1 KiB blocks into a
// 100-slot LDS ring, nothing consumes (the ring is recycled). Variants:
//   dma1    one loader wave, global_load_lds_dwordx4 nt, 8 DMAs per loop trip, vmcnt(D) window
//   dma1-rt the same without nt
//   dma2    two loader waves (even / odd blocks)
//   dma4    four loader waves
//   reg1    one wave: global_load_dwordx4 nt into VGPRs (D deep), ds_write_b128 into the ring
//   reg2    two such waves
//   tile    the decode engine's pattern: one loader wave, CU g streams tiles g, g + G, g + 2G, ...
//           of a [ntiles][kc] matrix of 1 KiB blocks (all CUs at the same chunk offset at once)
//   tile-rot  the same with each CU starting its tile at chunk (g mod kc) and wrapping
//   tile-blk  CU g owns tiles [g nt, (g + 1) nt) (contiguous nt kc KiB per CU)
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

// tile-pattern stream (KIND 2: strided tiles, 3: strided + rotated chunk start, 4: blocked tiles)
template <int KIND, int D>
__global__ __launch_bounds__(256, 1) void tile_kernel(const char* __restrict__ w, int kc, int nt, float* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wave) return;
  const int G = gridDim.x, g = blockIdx.x, nb = 100;
  const uint32_t rb = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
  const char* base = w + 16 * lane;
  int slot = 0;
  const int rot = KIND == 3 ? g % kc : 0;
  for (int j = 0; j < nt; ++j) {
    const size_t tile = KIND == 4 ? (size_t)g * nt + j : (size_t)g + (size_t)j * G;
    for (int c0 = 0; c0 < kc; c0 += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        int c = c0 + u + rot;
        if (c >= kc) c -= kc;
        dma<true>(base + (tile * kc + c) * 1024, __builtin_amdgcn_readfirstlane(rb + (uint32_t)slot * 1024u));
        if (++slot == nb) slot = 0;
      }
      wait_vm<D>();
    }
  }
  wait_vm<0>();
}

template <int KIND, int D>
static int run_tile(const char* w, int kc, int nt, int G, float* out, const char* name) {
  auto k = tile_kernel<KIND, D>;
  CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(k, dim3(G), dim3(256), 100 * 1024, 0, w, kc, nt, out);
  CHECK(hipEventRecord(e0));
  const int R = 10;
  for (int it = 0; it < R; ++it) hipLaunchKernelGGL(k, dim3(G), dim3(256), 100 * 1024, 0, w, kc, nt, out);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / R, kib = (double)kc * nt;
  printf("%-10s kc=%3d nt=%2d D=%2d: %8.1f us  %6.1f GB/s per CU  %6.2f TB/s chip\n", name, kc, nt, D, us,
         kib * 1024 / us / 1e3, kib * 1024 * G / us / 1e6);
  return 0;
}

// the engine's whole step stream over LLaMA-7B-shaped int4 matrices, one allocation per matrix
// (as a framework allocates them): per layer QKV, O, fc1 + fc2 (interleaved), down; tiles g + j G
struct ModelTbl {
  const char* w[32][5];
};
template <int D>
__global__ __launch_bounds__(256, 1) void model_kernel(const ModelTbl* __restrict__ T, int nl, int C, int H) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wave) return;
  const int G = gridDim.x, g = blockIdx.x, nb = 100;
  const uint32_t rb = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
  int slot = 0, cnt = 0;
  for (int l = 0; l < nl; ++l) {
    for (int op = 0; op < 4; ++op) {
      const int ntile = op == 0 ? 3 * C / 16 : op == 2 ? H / 16 : C / 16;
      const int kc = (op == 3 ? H : C) / 128, nm = op == 2 ? 2 : 1;
      const char* w0 = T->w[l][op == 3 ? 4 : op] + 16 * lane;
      const char* w1 = T->w[l][op == 2 ? 3 : op == 3 ? 4 : op] + 16 * lane;
      for (int tile = g; tile < ntile; tile += G) {
        for (int c = 0; c < kc; ++c) {
          for (int m = 0; m < nm; ++m) {
            dma<true>((m ? w1 : w0) + ((size_t)tile * kc + c) * 1024, __builtin_amdgcn_readfirstlane(rb + (uint32_t)slot * 1024u));
            if (++slot == nb) slot = 0;
            if ((++cnt & 7) == 0) wait_vm<D>();
          }
        }
      }
    }
  }
  wait_vm<0>();
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
  {
    const int C = 4096, H = 11008, NL = 32;
    ModelTbl t;
    size_t tot = 0;
    for (int l = 0; l < NL; ++l)
      for (int k = 0; k < 5; ++k) {
        const size_t sz = k == 0 ? (size_t)3 * C * C / 2 : k == 1 ? (size_t)C * C / 2 : (size_t)C * H / 2;
        char* p;
        CHECK(hipMalloc(&p, sz));
        CHECK(hipMemset(p, 0x11, sz));
        t.w[l][k] = p;
        tot += sz;
      }
    ModelTbl* dt;
    CHECK(hipMalloc(&dt, sizeof(ModelTbl)));
    CHECK(hipMemcpy(dt, &t, sizeof t, hipMemcpyHostToDevice));
    auto k = model_kernel<48>;
    CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int it = 0; it < 2; ++it) hipLaunchKernelGGL(k, dim3(G), dim3(256), 100 * 1024, 0, dt, NL, C, H);
    CHECK(hipEventRecord(e0));
    for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(k, dim3(G), dim3(256), 100 * 1024, 0, dt, NL, C, H);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / 5;
    printf("model-7B  160 allocations, %.2f GB: %8.1f us  %6.1f GB/s per CU  %6.2f TB/s chip\n", tot / 1e9, us,
           tot / (double)G / us / 1e3, tot / us / 1e6);
  }
  // the engine's patterns over a 7B-like SwiGLU-sized matrix (kc 32, 172 tiles per 256 CUs ~ 8 per CU here)
  for (int kc : {32, 86}) {
    const int nt = nblk / kc;
    run_tile<2, 48>(w, kc, nt, G, out, "tile");
    run_tile<3, 48>(w, kc, nt, G, out, "tile-rot");
    run_tile<4, 48>(w, kc, nt, G, out, "tile-blk");
  }
  return 0;
}

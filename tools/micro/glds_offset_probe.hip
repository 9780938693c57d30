// Does global_load_lds_dwordx4's immediate offset move the LDS destination too? One wave DMAs
// 1 KiB from src + 1024 (offset:1024, saddr form) with M0 = LDS byte 0, then dumps LDS[0, 4 KiB)
// as the block index found at each 1 KiB (src block b is filled with the value b).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void probe(const char* src, unsigned* out) {
  __shared__ __attribute__((aligned(16))) unsigned lds[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = 0xFFFFFFFFu;
  __syncthreads();
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds);
  const uint32_t voff = threadIdx.x * 16;
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 offset:1024\n\t"
               "s_waitcnt vmcnt(0)\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(src), "s"(dst) : "memory");
  __syncthreads();
  if (threadIdx.x < 4) out[threadIdx.x] = lds[threadIdx.x * 256];
}

int main() {
  char* src;
  unsigned* out;
  hipMalloc(&src, 8192);
  hipMalloc(&out, 16);
  unsigned h[2048];
  for (int i = 0; i < 2048; ++i) h[i] = i / 256;  // block b (1 KiB) holds b
  hipMemcpy(src, h, 8192, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, src, out);
  unsigned r[4];
  hipMemcpy(r, out, 16, hipMemcpyDeviceToHost);
  printf("LDS KiB 0..3 hold source block: %d %d %d %d  (0xffffffff = untouched)\n", (int)r[0], (int)r[1], (int)r[2], (int)r[3]);
  printf(r[1] == 1u ? "offset applies to BOTH the global and the LDS address\n"
                    : r[0] == 1u ? "offset applies to the global address only\n" : "unexpected\n");
  return 0;
}

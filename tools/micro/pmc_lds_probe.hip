// Probe for the rocprofv3 --pmc rc 139: does a counter pass die on a plain launch
// with more than 64 KiB of dynamic LDS (hipFuncSetAttribute(MaxDynamicSharedMemorySize))?
// Usage: pmc_lds_probe <lds_kib> <attr_kib> <launches>   (attr 0: no attribute call)
// Prints one line per variant; exit 0 when every launch completed and the sums check.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void lds_touch(const float* __restrict__ in, float* __restrict__ out, int n_lds) {
  extern __shared__ float s[];
  for (int i = threadIdx.x; i < n_lds; i += 256) s[i] = in[(blockIdx.x * 256 + i) & 65535];
  __syncthreads();
  float acc = 0.f;
  for (int i = threadIdx.x; i < n_lds; i += 256) acc += s[(i * 7) % n_lds];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const int lds_kib = argc > 1 ? atoi(argv[1]) : 96;
  const int attr_kib = argc > 2 ? atoi(argv[2]) : 160;
  const int launches = argc > 3 ? atoi(argv[3]) : 4;
  const int grid = 512;
  float *in, *out;
  if (hipMalloc(&in, 65536 * 4) != hipSuccess || hipMalloc(&out, grid * 256 * 4) != hipSuccess) return 2;
  hipMemset(in, 0, 65536 * 4);
  if (attr_kib > 0) {
    hipError_t e = hipFuncSetAttribute((const void*)lds_touch, hipFuncAttributeMaxDynamicSharedMemorySize, attr_kib * 1024);
    printf("hipFuncSetAttribute(%d KiB) -> %d\n", attr_kib, (int)e);
  }
  const size_t lds = (size_t)lds_kib * 1024;
  for (int i = 0; i < launches; ++i) {
    hipLaunchKernelGGL(lds_touch, dim3(grid), dim3(256), lds, 0, in, out, (int)(lds / 4));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      printf("launch %d: error %d\n", i, (int)e);
      return 3;
    }
  }
  hipError_t e = hipDeviceSynchronize();
  printf("lds %d KiB attr %d KiB launches %d: sync %d\n", lds_kib, attr_kib, launches, (int)e);
  return e == hipSuccess ? 0 : 4;
}

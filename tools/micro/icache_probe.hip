// Instruction-fetch probe (profiling aid, not product code): does a decode GEMV pay for cold
// instruction cache at every launch? A kernel executes N `s_nop 0` either as straight-line code
// (4 N bytes) or as a loop over a 64-nop body (256 bytes); two instances of each alternate in a
// graph, like the five different kernels of a decode layer. The difference between the two
// forms is the cost of fetching the straight-line code.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int N, int TAG>
__global__ void straight_k(int* out) {
#pragma unroll
  for (int i = 0; i < N / 16; ++i)
    asm volatile("s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n"
                 "s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n");
  if (out && threadIdx.x == 9999) out[TAG] = 1;
}

template <int N, int TAG>
__global__ void loop_k(int* out, int iters) {
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      asm volatile("s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n"
                   "s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n");
  }
  if (out && threadIdx.x == 9999) out[TAG] = 1;
}

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(err_), __LINE__); return 1; } } while (0)

template <int N>
static int run(hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  const int L = 128;
  for (int grid : {256, 1024}) {
    for (int form : {0, 1}) {
      hipGraph_t g; hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int i = 0; i < L; ++i) {
        if (form == 0) {
          if (i & 1) hipLaunchKernelGGL((straight_k<N, 1>), dim3(grid), dim3(256), 0, s, nullptr);
          else hipLaunchKernelGGL((straight_k<N, 0>), dim3(grid), dim3(256), 0, s, nullptr);
        } else {
          if (i & 1) hipLaunchKernelGGL((loop_k<N, 1>), dim3(grid), dim3(256), 0, s, nullptr, N / 64);
          else hipLaunchKernelGGL((loop_k<N, 0>), dim3(grid), dim3(256), 0, s, nullptr, N / 64);
        }
      }
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      float best = 1e30f;
      for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(e0, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      printf("{\"probe\": \"icache\", \"nops\": %d, \"code_bytes\": %d, \"grid\": %d, \"form\": \"%s\", \"us\": %.3f}\n", N,
             form == 0 ? 4 * N : 256, grid, form == 0 ? "straight" : "loop", best * 1e3 / L);
      fflush(stdout);
      CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
  }
  return 0;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  if (run<256>(s, e0, e1) || run<1024>(s, e0, e1) || run<2048>(s, e0, e1) || run<4096>(s, e0, e1) ||
      run<8192>(s, e0, e1))
    return 1;
  return 0;
}

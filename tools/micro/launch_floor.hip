// Launch-floor probe (profiling aid, not product code): time per kernel of a captured HIP graph
// of N back-to-back dependent launches, for an empty body and for a body whose every workgroup
// reads an 8 KB activation row (L2/MALL) and writes 16 columns, at 256 / 768 workgroups of 256
// threads. Tells how much of a decode GEMV's time is the kernel boundary itself.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void empty_k(int* p) { if (p && threadIdx.x == 9999) p[0] = 1; }

__global__ void rowread_k(const uint4* __restrict__ a, uint32_t* __restrict__ out) {
  // every workgroup reads the same 8 KB row (the A prologue of a GEMV) and writes 64 B
  const int t = threadIdx.x;
  uint4 v0 = a[t], v1 = a[t + 256];
  uint32_t s = v0.x ^ v0.y ^ v0.z ^ v0.w ^ v1.x ^ v1.y ^ v1.z ^ v1.w;
  __shared__ uint32_t r[256];
  r[t] = s;
  __syncthreads();
  if (t < 16) out[blockIdx.x * 16 + t] = r[t] + r[t + 16];
}

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
__global__ void stream_k(const uint4* __restrict__ w_, uint32_t* __restrict__ out, int per_wg16) {
  const u32x4v* w = reinterpret_cast<const u32x4v*>(w_);
  // every workgroup streams per_wg16 x 16 B of weights (non-temporal), all loads in flight
  const int t = threadIdx.x;
  const u32x4v* base = w + (size_t)blockIdx.x * per_wg16;
  uint32_t s = 0;
  for (int i = t; i < per_wg16; i += 256) {
    u32x4v v = __builtin_nontemporal_load(base + i);
    s ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  __shared__ uint32_t r[256];
  r[t] = s;
  __syncthreads();
  if (t < 16) out[blockIdx.x * 16 + t] = r[t] ^ r[t + 16];
}

template <int U>
__global__ void stream_u_k(const uint4* __restrict__ w_, uint32_t* __restrict__ out, int per_wg16) {
  // U independent 16-B loads per thread in flight before any use
  const u32x4v* w = reinterpret_cast<const u32x4v*>(w_) + (size_t)blockIdx.x * per_wg16;
  const int t = threadIdx.x, nt = blockDim.x;
  uint32_t s = 0;
  for (int i0 = t; i0 < per_wg16; i0 += U * nt) {
    u32x4v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * nt;
      v[u] = __builtin_nontemporal_load(w + (i < per_wg16 ? i : t));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) s ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  __shared__ uint32_t r[1024];
  r[t] = s;
  __syncthreads();
  if (t < 16) out[blockIdx.x * 16 + t] = r[t] ^ r[t + 16];
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  uint4* a; uint32_t* out; uint4* w;
  CK(hipMalloc(&a, 1 << 20));
  CK(hipMalloc(&out, 1 << 22));
  const size_t wbytes = (size_t)1 << 30;  // 1 GiB of "weights": every launch streams its own slice
  CK(hipMalloc(&w, wbytes));
  CK(hipMemset(w, 1, wbytes));
  CK(hipMemset(a, 1, 1 << 20));
  const int N = 160;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int kind = 0; kind < 5; ++kind) {
    for (int grid : {32, 256, 768}) {
      // kind 0 empty, 1 row read, 2..4 stream 8 / 25 / 45 MB per launch (c_proj / QKV / SwiGLU sizes)
      const size_t mb[5] = {0, 0, 8400000, 25200000, 45200000};
      if (kind >= 2 && grid == 32) continue;
      const int per_wg16 = kind >= 2 ? (int)(mb[kind] / 16 / grid) : 0;
      hipGraph_t g; hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int i = 0; i < N; ++i) {
        if (kind == 0) hipLaunchKernelGGL(empty_k, dim3(grid), dim3(256), 0, s, nullptr);
        else if (kind == 1) hipLaunchKernelGGL(rowread_k, dim3(grid), dim3(256), 0, s, a, out);
        else {
          const size_t off16 = ((size_t)i * mb[kind] / 16) % (wbytes / 16 - mb[kind] / 16);
          hipLaunchKernelGGL(stream_k, dim3(grid), dim3(256), 0, s, w + off16, out, per_wg16);
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
      const double us = best * 1e3 / N;
      printf("{\"kind\": %d, \"grid\": %d, \"bytes\": %zu, \"us_per_launch\": %.3f, \"GBps\": %.1f}\n", kind, grid,
             mb[kind], us, kind >= 2 ? mb[kind] / us / 1e3 : 0.0);
      CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
  }
  // sweep: bytes x grid x threads x loads in flight
  for (size_t bytes : {(size_t)8400000, (size_t)22500000, (size_t)25200000, (size_t)45200000}) {
    for (int grid : {256, 512, 768, 1024, 2048}) {
      for (int nt : {256, 512}) {
        for (int U : {4, 8}) {
          const int per_wg16 = (int)(bytes / 16 / grid);
          hipGraph_t g; hipGraphExec_t ge;
          CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
          for (int i = 0; i < N; ++i) {
            const size_t off16 = ((size_t)i * bytes / 16) % (wbytes / 16 - bytes / 16);
            if (U == 4) hipLaunchKernelGGL(stream_u_k<4>, dim3(grid), dim3(nt), 0, s, w + off16, out, per_wg16);
            else hipLaunchKernelGGL(stream_u_k<8>, dim3(grid), dim3(nt), 0, s, w + off16, out, per_wg16);
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
          const double us = best * 1e3 / N;
          printf("{\"sweep\": 1, \"bytes\": %zu, \"grid\": %d, \"threads\": %d, \"U\": %d, \"us_per_launch\": %.3f, \"GBps\": %.1f}\n",
                 bytes, grid, nt, U, us, bytes / us / 1e3);
          CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
        }
      }
    }
  }
  return 0;
}

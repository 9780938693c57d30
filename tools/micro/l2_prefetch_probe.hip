// L2 prefetch probe (profiling aid, not product code). The MALL probe showed that a slice read
// once is fast on a second pass only while it fits the 8 x 4 MB L2s, and that a prefetch from
// workgroups on the wrong XCD does not help. Here every prefetch is XCD-matched: the prefetching
// workgroup sits on the XCD (blockIdx % 8) of the workgroup that will read the slice.
//  (a) latency-bound launch + XCD-matched prefetch of fraction f of the next stream's slices;
//  (b) stream A whose workgroups, after their own loads, prefetch fraction f of stream B's slice
//      of the same-numbered workgroup (same XCD), then stream B.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t stream_slice(const u32x4v* base, int n, int t, bool nt) {
  uint32_t s = 0;
  for (int i0 = t; i0 < n; i0 += 4 * 256) {
    u32x4v v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * 256;
      const u32x4v* p = base + (i < n ? i : t);
      v[u] = nt ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) s ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  return s;
}

// stream kernel: WG b reads per_wg16 x 16 B at w + b*per_wg16 (non-temporal); then, if pf != null,
// plain-loads the first pf_n16 x 16 B of slice b of `pf` (the next launch's slice for WG b).
__global__ void stream_pf_k(const u32x4v* __restrict__ w, uint32_t* __restrict__ out, int per_wg16,
                            const u32x4v* __restrict__ pf, int pf_n16) {
  const int t = threadIdx.x;
  uint32_t s = stream_slice(w + (size_t)blockIdx.x * per_wg16, per_wg16, t, true);
  if (pf) s ^= stream_slice(pf + (size_t)blockIdx.x * per_wg16, pf_n16, t, false);
  __shared__ uint32_t r[256];
  r[t] = s;
  __syncthreads();
  if (t < 16) out[blockIdx.x * 16 + t] = r[t] ^ r[t + 16];
}

// latency stand-in: WGs < 32 walk 8 dependent rounds; WG j >= 32 (XCD j % 8) prefetches the first
// pf_n16 of the slices of stream WGs b = x + 8*(q + nq*r) (same XCD x, q = its rank on that XCD).
__global__ void latency_pf_k(const u32x4v* __restrict__ kv, uint32_t* __restrict__ out,
                             const u32x4v* __restrict__ pf, int per_wg16, int pf_n16, int stream_grid) {
  const int t = threadIdx.x;
  __shared__ uint32_t r[256];
  if (blockIdx.x < 32) {
    const u32x4v* base = kv + (size_t)blockIdx.x * 2560;
    uint32_t s = 0;
    for (int round = 0; round < 8; ++round) {
      const int i = (round * 320 + t + (int)(s & 1)) % 2560;
      u32x4v v = base[i];
      s += v[0] ^ v[1];
      r[t] = s;
      __syncthreads();
      s += r[(t + 1) & 255];
      __syncthreads();
    }
    if (t < 16) out[blockIdx.x * 16 + t] = s;
    return;
  }
  const int j = blockIdx.x - 32, x = blockIdx.x % 8, nq = (gridDim.x - 32) / 8, q = j / 8;
  uint32_t s = 0;
  for (int b = x + 8 * q; b < stream_grid; b += 8 * nq)
    s ^= stream_slice(pf + (size_t)b * per_wg16, pf_n16, t, false);
  if (s == 0x9e3779b9u) out[8192 + blockIdx.x] = s;
}

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(err_), __LINE__); return 1; } } while (0)

static float time_graph(hipGraphExec_t ge, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0, s);
    hipGraphLaunch(ge, s);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  uint32_t* out; u32x4v* w; u32x4v* kv;
  CK(hipMalloc(&out, 1 << 22));
  const size_t wbytes = (size_t)4 << 30;
  CK(hipMalloc(&w, wbytes));
  CK(hipMalloc(&kv, 32 << 20));
  CK(hipMemset(w, 1, wbytes));
  CK(hipMemset(kv, 1, 32 << 20));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int N = 128, grid = 1024;
  // (a)
  for (size_t bytes : {(size_t)8400000, (size_t)25200000}) {
    for (int frac8 : {0, 2, 4, 8}) {
      for (int pfwg : {256, 512}) {
        if (frac8 == 0 && pfwg != 256) continue;
        const int per_wg16 = (int)(bytes / 16 / grid), pf_n16 = per_wg16 * frac8 / 8;
        hipGraph_t g; hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < N; ++i) {
          const size_t off16 = ((size_t)i * bytes / 16) % (wbytes / 16 - bytes / 16);
          hipLaunchKernelGGL(latency_pf_k, dim3(frac8 ? 32 + pfwg : 32), dim3(256), 0, s, kv, out, w + off16,
                             per_wg16, pf_n16, grid);
          hipLaunchKernelGGL(stream_pf_k, dim3(grid), dim3(256), 0, s, w + off16, out, per_wg16,
                             (const u32x4v*)nullptr, 0);
        }
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        const double us = time_graph(ge, s, e0, e1) * 1e3 / N;
        printf("{\"probe\": \"latency_xcd_prefetch\", \"bytes\": %zu, \"frac\": %.3f, \"pf_wgs\": %d, \"us_pair\": %.3f}\n",
               bytes, frac8 / 8.0, frac8 ? pfwg : 0, us);
        fflush(stdout);
        CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
      }
    }
  }
  // (b) chain of N stream launches over consecutive slices; launch i prefetches fraction f of launch i+1's
  for (size_t bytes : {(size_t)8400000, (size_t)25200000, (size_t)45200000}) {
    for (int frac8 : {0, 1, 2, 4}) {
      const int per_wg16 = (int)(bytes / 16 / grid), pf_n16 = per_wg16 * frac8 / 8;
      hipGraph_t g; hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int i = 0; i < N; ++i) {
        const size_t off16 = ((size_t)i * bytes / 16) % (wbytes / 16 - 2 * bytes / 16);
        hipLaunchKernelGGL(stream_pf_k, dim3(grid), dim3(256), 0, s, w + off16, out, per_wg16,
                           frac8 ? (const u32x4v*)(w + off16 + bytes / 16) : (const u32x4v*)nullptr, pf_n16);
      }
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      const double us = time_graph(ge, s, e0, e1) * 1e3 / N;
      printf("{\"probe\": \"stream_tail_prefetch\", \"bytes\": %zu, \"frac\": %.3f, \"us\": %.3f, \"GBps\": %.1f}\n", bytes,
             frac8 / 8.0, us, bytes / us / 1e3);
      fflush(stdout);
      CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
  }
  return 0;
}

// Infinity-cache (MALL) probe (profiling aid, not product code). Questions for the bs=1 decode
// layer, whose GEMVs stream 101 MB of weights with ~20 us per layer of kernel boundaries and
// latency-bound work in between:
//  1. does a streamed slice stay resident (second pass of the same 8.4 / 25 / 45 MB faster)?
//     with non-temporal and with plain loads;
//  2. does prefetching the next kernel's slice from extra workgroups of a latency-bound launch
//     (the attention) make that next kernel faster;
//  3. does a prefetch branch running one kernel ahead on a second stream of the graph shorten a
//     chain shaped like one decode layer.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

template <int NT_LOAD>
__global__ void stream_k(const u32x4v* __restrict__ w, uint32_t* __restrict__ out, int per_wg16) {
  const u32x4v* base = w + (size_t)blockIdx.x * per_wg16;
  const int t = threadIdx.x;
  uint32_t s = 0;
  for (int i0 = t; i0 < per_wg16; i0 += 4 * 256) {
    u32x4v v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * 256;
      const u32x4v* p = base + (i < per_wg16 ? i : t);
      v[u] = NT_LOAD ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) s ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  __shared__ uint32_t r[256];
  r[t] = s;
  __syncthreads();
  if (t < 16) out[blockIdx.x * 16 + t] = r[t] ^ r[t + 16];
}

// Latency-bound stand-in for bs=1 attention: `lat_wg` workgroups each walk 8 dependent rounds
// over 40 KB; workgroups beyond lat_wg prefetch pf16 x 16 B of the next kernel's slice (plain
// loads, result folded into a store nobody reads).
__global__ void latency_k(const u32x4v* __restrict__ kv, uint32_t* __restrict__ out, int lat_wg,
                          const u32x4v* __restrict__ pf, int pf16) {
  const int t = threadIdx.x;
  __shared__ uint32_t r[256];
  if ((int)blockIdx.x < lat_wg) {
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
  const int nwg = gridDim.x - lat_wg, wg = blockIdx.x - lat_wg;
  const int per = (pf16 + nwg - 1) / nwg;
  const u32x4v* base = pf + (size_t)wg * per;
  const int n = min(per, pf16 - wg * per);
  uint32_t s = 0;
  for (int i0 = t; i0 < n; i0 += 4 * 256) {
    u32x4v v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * 256;
      v[u] = base[i < n ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) s ^= v[u][0];
  }
  if (s == 0x9e3779b9u) out[4096 + blockIdx.x] = s;  // keeps the loads alive
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

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
  hipStream_t s, s2;
  CK(hipStreamCreate(&s)); CK(hipStreamCreate(&s2));
  uint32_t* out; u32x4v* w; u32x4v* kv;
  CK(hipMalloc(&out, 1 << 22));
  const size_t wbytes = (size_t)4 << 30;  // 4 GiB: larger than the 7B int4 weights
  CK(hipMalloc(&w, wbytes));
  CK(hipMalloc(&kv, 32 << 20));
  CK(hipMemset(w, 1, wbytes));
  CK(hipMemset(kv, 1, 32 << 20));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int N = 128;

  // 1. residency: N launches over the same slice (hot) vs consecutive slices (cold)
  for (size_t bytes : {(size_t)8400000, (size_t)25200000, (size_t)45200000, (size_t)101000000}) {
    for (int nt : {1, 0}) {
      for (int hot : {0, 1}) {
        const int grid = 1024, per_wg16 = (int)(bytes / 16 / grid);
        hipGraph_t g; hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < N; ++i) {
          const size_t off16 = hot ? 0 : ((size_t)i * bytes / 16) % (wbytes / 16 - bytes / 16);
          if (nt) hipLaunchKernelGGL(stream_k<1>, dim3(grid), dim3(256), 0, s, w + off16, out, per_wg16);
          else hipLaunchKernelGGL(stream_k<0>, dim3(grid), dim3(256), 0, s, w + off16, out, per_wg16);
        }
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        const double us = time_graph(ge, s, e0, e1) * 1e3 / N;
        printf("{\"probe\": \"residency\", \"bytes\": %zu, \"nontemporal\": %d, \"hot\": %d, \"us\": %.3f, \"GBps\": %.1f}\n",
               bytes, nt, hot, us, bytes / us / 1e3);
        fflush(stdout);
        CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
      }
    }
  }

  // 2. latency kernel (32 workgroups) then an 8.4 MB stream; extra workgroups of the latency
  //    launch prefetch 0 / 8.4 MB of the stream's slice. Consecutive slices (cold otherwise).
  for (int nt : {1, 0}) {
    for (int extra : {0, 224, 480}) {
      const size_t bytes = 8400000;
      const int grid = 1024, per_wg16 = (int)(bytes / 16 / grid);
      hipGraph_t g; hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int i = 0; i < N; ++i) {
        const size_t off16 = ((size_t)i * bytes / 16) % (wbytes / 16 - bytes / 16);
        hipLaunchKernelGGL(latency_k, dim3(32 + extra), dim3(256), 0, s, kv, out, 32, w + off16,
                           extra ? (int)(bytes / 16) : 0);
        if (nt) hipLaunchKernelGGL(stream_k<1>, dim3(grid), dim3(256), 0, s, w + off16, out, per_wg16);
        else hipLaunchKernelGGL(stream_k<0>, dim3(grid), dim3(256), 0, s, w + off16, out, per_wg16);
      }
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      const double us = time_graph(ge, s, e0, e1) * 1e3 / N;
      printf("{\"probe\": \"latency_then_stream\", \"nontemporal\": %d, \"prefetch_wgs\": %d, \"us_pair\": %.3f}\n", nt,
             extra, us);
      fflush(stdout);
      CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
  }
  // latency kernel alone, with and without prefetch workgroups
  for (int extra : {0, 224}) {
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < N; ++i) {
      const size_t off16 = ((size_t)i * 8400000 / 16) % (wbytes / 16 - 8400000 / 16);
      hipLaunchKernelGGL(latency_k, dim3(32 + extra), dim3(256), 0, s, kv, out, 32, w + off16,
                         extra ? 8400000 / 16 : 0);
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    const double us = time_graph(ge, s, e0, e1) * 1e3 / N;
    printf("{\"probe\": \"latency_alone\", \"prefetch_wgs\": %d, \"us\": %.3f}\n", extra, us);
    fflush(stdout);
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
  }

  // 3. a decode-layer-shaped chain: stream 25.2 MB, latency, 8.4, 45.2, 22.6 MB; layers use
  //    consecutive slices. Variant 1: a second stream prefetches kernel k+1's slice while kernel k
  //    runs (branch waits on kernel k-1's completion event). Variant 2: the prefetch branch runs a
  //    whole layer ahead.
  const size_t lb[5] = {25200000, 0, 8400000, 45200000, 22600000};
  size_t loff[5]; size_t layer_bytes = 0;
  for (int k = 0; k < 5; ++k) { loff[k] = layer_bytes; layer_bytes += lb[k]; }
  const int L = 32;
  for (int variant : {0, 1, 2}) {
    for (int nt : {1, 0}) {
      for (int pfw : {64, 128}) {
        if (variant == 0 && pfw != 64) continue;
        hipGraph_t g; hipGraphExec_t ge;
        std::vector<hipEvent_t> done(5 * L + 1);
        for (auto& ev : done) CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        CK(hipEventRecord(done[5 * L], s));
        CK(hipStreamWaitEvent(s2, done[5 * L], 0));
        for (int l = 0; l < L; ++l) {
          for (int k = 0; k < 5; ++k) {
            const int idx = l * 5 + k;
            // prefetch branch: the slice of kernel idx + ahead, launched once kernel idx - 1 is done
            const int ahead = variant == 1 ? 1 : 5;
            const int tgt = idx + ahead;
            if (variant > 0 && tgt < 5 * L && lb[tgt % 5] > 0) {
              if (idx > 0) CK(hipStreamWaitEvent(s2, done[idx - 1], 0));
              const u32x4v* p = w + ((size_t)(tgt / 5) * layer_bytes + loff[tgt % 5]) / 16;
              hipLaunchKernelGGL(latency_k, dim3(pfw), dim3(256), 0, s2, kv, out, 0, p, (int)(lb[tgt % 5] / 16));
            }
            if (lb[k] == 0) {
              hipLaunchKernelGGL(latency_k, dim3(32), dim3(256), 0, s, kv, out, 32, w, 0);
            } else {
              const int grid = 1024, per_wg16 = (int)(lb[k] / 16 / grid);
              const u32x4v* p = w + ((size_t)l * layer_bytes + loff[k]) / 16;
              if (nt) hipLaunchKernelGGL(stream_k<1>, dim3(grid), dim3(256), 0, s, p, out, per_wg16);
              else hipLaunchKernelGGL(stream_k<0>, dim3(grid), dim3(256), 0, s, p, out, per_wg16);
            }
            CK(hipEventRecord(done[idx], s));
          }
        }
        CK(hipEventRecord(done[5 * L], s2));
        CK(hipStreamWaitEvent(s, done[5 * L], 0));
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        const double us = time_graph(ge, s, e0, e1) * 1e3 / L;
        printf("{\"probe\": \"layer_chain\", \"variant\": %d, \"nontemporal\": %d, \"prefetch_wgs\": %d, \"us_per_layer\": %.3f}\n",
               variant, nt, pfw, us);
        fflush(stdout);
        CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
        for (auto& ev : done) CK(hipEventDestroy(ev));
      }
    }
  }
  return 0;
}

// Persistent decode-layer probe (profiling aid, not product code). One launch streams the byte
// pattern of 32 decode layers (25.2 MB QKV, attention on 32 workgroups, 8.4 MB c_proj, 45.2 MB
// c_fc1/c_fc2, 22.6 MB mlp.c_proj) with 256 workgroups x 16 waves, a grid-wide completion
// counter between ops instead of a kernel boundary, and each op's weight loads issued BEFORE
// waiting for the previous op (the weights do not depend on the activations). Compared with the
// same pattern as separate launches. Every spin is bounded (the grid always drains).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
constexpr int NOPS = 5, NL = 32, NWG = 256, NT = 1024, MAXV = 12;  // MAXV 16-B loads per lane per op
constexpr size_t c_bytes[NOPS] = {25200000, 0, 8400000, 45200000, 22600000};

struct Ctl {
  unsigned int cnt[8];    // per-XCD arrival counters (monotonic)
  unsigned int gcnt;      // global counter (monotonic)
  unsigned int timeouts;
};

template <int MODE>  // bit 0: per-XCD counters (else one global counter); bit 1: no fence; bit 2: no barrier at all
__device__ __forceinline__ void arrive(Ctl* ctl) {
  if (MODE & 4) return;
  if (!(MODE & 2)) __threadfence();
  if (!(MODE & 1)) __hip_atomic_fetch_add(&ctl->gcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else __hip_atomic_fetch_add(&ctl->cnt[blockIdx.x & 7], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int MODE>
__device__ __forceinline__ void wait_all(Ctl* ctl, unsigned int target_per_wg) {
  // thread 0 of the workgroup polls; target = (ops done) * NWG arrivals
  if (MODE & 4) return;
  for (int it = 0; it < (1 << 20); ++it) {
    unsigned int tot = 0;
    if (!(MODE & 1)) {
      tot = __hip_atomic_load(&ctl->gcnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
#pragma unroll
      for (int x = 0; x < 8; ++x) tot += __hip_atomic_load(&ctl->cnt[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tot >= target_per_wg * NWG) return;
    __builtin_amdgcn_s_sleep(1);
  }
  __hip_atomic_fetch_add(&ctl->timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int MODE>
__global__ __launch_bounds__(NT) void persist_k(const u32x4v* __restrict__ w, const u32x4v* __restrict__ kv,
                                                uint32_t* __restrict__ out, Ctl* ctl, unsigned int epoch) {
  const int t = threadIdx.x;
  const size_t gt = (size_t)blockIdx.x * NT + t, nthr = (size_t)NWG * NT;
  __shared__ uint32_t r[NT];
  uint32_t s = 0;
  u32x4v v[MAXV];
  size_t off16 = 0;
  int nv = 0;
  unsigned int done = epoch;  // ops completed before this launch (x NWG arrivals each)
  auto issue = [&](int op) {
    const size_t n16 = c_bytes[op] / 16;
    nv = (int)((n16 + nthr - 1) / nthr);
#pragma unroll
    for (int u = 0; u < MAXV; ++u) {
      const size_t i = gt + (size_t)u * nthr;
      if (u < nv) v[u] = __builtin_nontemporal_load(w + off16 + (i < n16 ? i : 0));
    }
    off16 += n16;
  };
  auto consume = [&]() {
#pragma unroll
    for (int u = 0; u < MAXV; ++u)
      if (u < nv) s ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  };
  for (int l = 0; l < NL; ++l) {
#pragma unroll
    for (int op = 0; op < NOPS; ++op) {
      if (c_bytes[op] > 0) issue(op);  // weights first: independent of the previous op's output
      if (t == 0) wait_all<MODE>(ctl, done);
      __syncthreads();
      if (c_bytes[op] > 0) {
        consume();
      } else if (blockIdx.x < 32) {  // attention stand-in: 8 dependent rounds over 40 KB per head
        const u32x4v* base = kv + (size_t)blockIdx.x * 2560;
        for (int round = 0; round < 8; ++round) {
          const int i = (round * 320 + (t & 255) + (int)(s & 1)) % 2560;
          u32x4v a = base[i];
          s += a[0] ^ a[1];
          r[t] = s;
          __syncthreads();
          s += r[(t + 1) & (NT - 1)];
          __syncthreads();
        }
      }
      if (t < 16) out[blockIdx.x * 16 + t] = s;  // the op's "output"
      __syncthreads();
      if (t == 0) arrive<MODE>(ctl);
      ++done;
    }
  }
}

__global__ void stream_k(const u32x4v* __restrict__ w, uint32_t* __restrict__ out, int per_wg16) {
  const u32x4v* base = w + (size_t)blockIdx.x * per_wg16;
  const int t = threadIdx.x;
  uint32_t s = 0;
  for (int i0 = t; i0 < per_wg16; i0 += 4 * 256) {
    u32x4v v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * 256;
      v[u] = __builtin_nontemporal_load(base + (i < per_wg16 ? i : t));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) s ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  __shared__ uint32_t r[256];
  r[t] = s;
  __syncthreads();
  if (t < 16) out[blockIdx.x * 16 + t] = r[t] ^ r[t + 16];
}
__global__ void latency_k(const u32x4v* __restrict__ kv, uint32_t* __restrict__ out) {
  const int t = threadIdx.x;
  __shared__ uint32_t r[256];
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
}

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(err_), __LINE__); return 1; } } while (0)

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  uint32_t* out; u32x4v* w; u32x4v* kv; Ctl* ctl;
  CK(hipMalloc(&out, 1 << 22));
  const size_t wbytes = (size_t)4 << 30;
  CK(hipMalloc(&w, wbytes));
  CK(hipMalloc(&kv, 32 << 20));
  CK(hipMalloc(&ctl, sizeof(Ctl)));
  CK(hipMemset(w, 1, wbytes));
  CK(hipMemset(kv, 1, 32 << 20));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const size_t bytes[NOPS] = {25200000, 0, 8400000, 45200000, 22600000};
  // separate launches
  {
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    size_t off16 = 0;
    for (int l = 0; l < NL; ++l)
      for (int op = 0; op < NOPS; ++op) {
        if (bytes[op] == 0) { hipLaunchKernelGGL(latency_k, dim3(32), dim3(256), 0, s, kv, out); continue; }
        const int grid = 1024, per = (int)(bytes[op] / 16 / grid);
        hipLaunchKernelGGL(stream_k, dim3(grid), dim3(256), 0, s, w + off16, out, per);
        off16 += bytes[op] / 16;
      }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s));
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0, s)); CK(hipGraphLaunch(ge, s)); CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = ms < best ? ms : best;
    }
    printf("{\"probe\": \"separate_launches\", \"us_per_layer\": %.3f}\n", best * 1e3 / NL);
    fflush(stdout);
  }
  for (int mode : {0, 1, 2, 3, 4}) {
    CK(hipMemset(ctl, 0, sizeof(Ctl)));
    unsigned int epoch = 0;
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
      CK(hipEventRecord(e0, s));
      if (mode == 0) hipLaunchKernelGGL(persist_k<0>, dim3(NWG), dim3(NT), 0, s, w, kv, out, ctl, epoch);
      else if (mode == 1) hipLaunchKernelGGL(persist_k<1>, dim3(NWG), dim3(NT), 0, s, w, kv, out, ctl, epoch);
      else if (mode == 2) hipLaunchKernelGGL(persist_k<2>, dim3(NWG), dim3(NT), 0, s, w, kv, out, ctl, epoch);
      else if (mode == 3) hipLaunchKernelGGL(persist_k<3>, dim3(NWG), dim3(NT), 0, s, w, kv, out, ctl, epoch);
      else hipLaunchKernelGGL(persist_k<4>, dim3(NWG), dim3(NT), 0, s, w, kv, out, ctl, epoch);
      CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
      epoch += NL * NOPS;
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0) best = ms < best ? ms : best;
    }
    Ctl h;
    CK(hipMemcpy(&h, ctl, sizeof(Ctl), hipMemcpyDeviceToHost));
    printf("{\"probe\": \"persistent\", \"mode\": %d, \"us_per_layer\": %.3f, \"timeouts\": %u}\n", mode, best * 1e3 / NL,
           h.timeouts);
    fflush(stdout);
  }
  return 0;
}

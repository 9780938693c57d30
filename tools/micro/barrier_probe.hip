// Grid-barrier latency probe (profiling aid, not product code): 256 workgroups (one per CU),
// NB back-to-back barriers, three implementations: one global counter; per-group counters whose
// last arriver bumps a global counter; per-workgroup flags read by one wave of every waiter.
// Every spin is bounded (the grid always drains).
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int NWG = 256, SPIN = 1 << 20;
struct Ctl {
  unsigned int gcnt;
  unsigned int pad0[31];
  unsigned int grp[8][32];  // one counter per 128-B line
  unsigned int flag[NWG];
  unsigned int timeouts;
};

__device__ __forceinline__ unsigned int ld_agent(const unsigned int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int IMPL, int SLEEP>
__global__ __launch_bounds__(256) void barrier_k(Ctl* ctl, int nb, unsigned int base) {
  const int t = threadIdx.x;
  for (int b = 0; b < nb; ++b) {
    const unsigned int ep = base + b + 1;  // barriers completed after this one
    __syncthreads();
    if (IMPL == 0) {
      if (t == 0) {
        __hip_atomic_fetch_add(&ctl->gcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int it = 0;
        for (; it < SPIN && ld_agent(&ctl->gcnt) < ep * NWG; ++it) if (SLEEP) __builtin_amdgcn_s_sleep(1);
        if (it == SPIN) __hip_atomic_fetch_add(&ctl->timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else if (IMPL == 1) {
      if (t == 0) {
        const int g = blockIdx.x & 7;
        const unsigned int old = __hip_atomic_fetch_add(&ctl->grp[g][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1 == ep * (NWG / 8))
          __hip_atomic_fetch_add(&ctl->gcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int it = 0;
        for (; it < SPIN && ld_agent(&ctl->gcnt) < ep * 8; ++it) if (SLEEP) __builtin_amdgcn_s_sleep(1);
        if (it == SPIN) __hip_atomic_fetch_add(&ctl->timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      if (t == 0) __hip_atomic_store(&ctl->flag[blockIdx.x], ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t < 64) {
        int it = 0;
        for (; it < SPIN; ++it) {
          bool ok = true;
#pragma unroll
          for (int j = 0; j < 4; ++j) ok &= ld_agent(&ctl->flag[t * 4 + j]) >= ep;
          if (__all(ok)) break;
          if (SLEEP) __builtin_amdgcn_s_sleep(1);
        }
        if (it == SPIN && t == 0) __hip_atomic_fetch_add(&ctl->timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();
  }
}

#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(err_), __LINE__); return 1; } } while (0)

template <int IMPL, int SLEEP>
static int run(hipStream_t s, Ctl* ctl, hipEvent_t e0, hipEvent_t e1) {
  CK(hipMemset(ctl, 0, sizeof(Ctl)));
  const int nb = 2000;
  unsigned int base = 0;
  float best = 1e30f;
  for (int r = 0; r < 4; ++r) {
    CK(hipEventRecord(e0, s));
    hipLaunchKernelGGL((barrier_k<IMPL, SLEEP>), dim3(NWG), dim3(256), 0, s, ctl, nb, base);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    base += nb;
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (r > 0) best = ms < best ? ms : best;
  }
  Ctl h;
  CK(hipMemcpy(&h, ctl, sizeof(Ctl), hipMemcpyDeviceToHost));
  printf("{\"probe\": \"grid_barrier\", \"impl\": %d, \"sleep\": %d, \"us_per_barrier\": %.3f, \"timeouts\": %u}\n", IMPL,
         SLEEP, best * 1e3 / nb, h.timeouts);
  fflush(stdout);
  return 0;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  Ctl* ctl;
  CK(hipMalloc(&ctl, sizeof(Ctl)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  if (run<0, 1>(s, ctl, e0, e1) || run<0, 0>(s, ctl, e0, e1) || run<1, 1>(s, ctl, e0, e1) || run<1, 0>(s, ctl, e0, e1) ||
      run<2, 1>(s, ctl, e0, e1) || run<2, 0>(s, ctl, e0, e1))
    return 1;
  return 0;
}

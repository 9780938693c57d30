// Dataflow chaining of ops inside one launch (see gemv.hip llj_decode_layer).
#pragma once
#include "common.h"

namespace llj {

// ---- dataflow chaining inside one launch (llj_decode_layer, end of file). Producer and
// consumer ops share one grid; consumers (higher blockIdx, so dispatched after every
// producer workgroup) start their weight stream, then poll the producer's completion
// counter. The per-XCD L2s are not coherent with each other, so handed-off bytes follow
// the gfx950 write-through protocol: every store of them is sc1 (4/8/16 B), every storing
// wave drains (s_waitcnt vmcnt(0)) before ONE lane's agent-scope atomic add, the consumer
// polls with relaxed agent-scope (sc1) loads and reads the bytes only with sc1 loads.
struct ChainCtl {
  const unsigned* dep;  // the producer op's counter block (nullptr: no producer in this launch)
  int dep_nwg;          // producer workgroups
  unsigned* sig;        // this op's counter block (nullptr: nobody waits for it)
  int sig_nwg;          // this op's workgroups
  unsigned* err;        // set to 1 if a poll timed out (results are then garbage, the launch ends)
  int local;            // this workgroup's index within its op
};
// Counter block of one op: 16 shards (workgroup i adds to shard i % 16, so no word takes more
// than nwg/16 arrivals) and at word 16 a top counter that the LAST arriver of each shard
// (told by its add's return value) increments. Consumers poll only the top word.
constexpr int kShards = 16;
constexpr int kCtrWords = 32;  // per op (128 B: shards + top on their own lines)
__device__ __forceinline__ unsigned shard_target(int nwg, int s) {
  return (unsigned)(nwg / kShards + (s < nwg % kShards ? 1 : 0));
}
__device__ __forceinline__ unsigned top_target(int nwg) { return (unsigned)(nwg < kShards ? nwg : kShards); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7FFFFFFF, 0x00020000);
}
constexpr int kSC1 = 16;  // buffer instruction cache-policy bit: system coherent (write-through / L2 bypass)
__device__ __forceinline__ u32x4 ld16_sc1(const void* base, unsigned byte_off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc_of(base), byte_off, 0, kSC1));
}
__device__ __forceinline__ uint32_t ld4_sc1(const void* base, unsigned byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b32(rsrc_of(base), byte_off, 0, kSC1);
}
__device__ __forceinline__ uint2 ld8_sc1(const void* base, unsigned byte_off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc_of(base), byte_off, 0, kSC1);
  return make_uint2(v[0], v[1]);
}
__device__ __forceinline__ double ld8d_sc1(const void* base, unsigned byte_off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsrc_of(base), byte_off, 0, kSC1));
}
__device__ __forceinline__ void st4_sc1(void* base, unsigned byte_off, uint32_t v) {
  __builtin_amdgcn_raw_buffer_store_b32(v, rsrc_of(base), byte_off, 0, kSC1);
}
__device__ __forceinline__ void st8d_sc1(void* base, unsigned byte_off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v),
                                        rsrc_of(base), byte_off, 0, kSC1);
}

// Poll the producer's top counter (one lane, relaxed agent-scope = sc1 load, s_sleep between
// polls so waiting workgroups do not flood the fabric), bounded (50 ms), then release the
// workgroup through a barrier.
__device__ __forceinline__ void chain_wait(const ChainCtl& cc) {
  if (cc.dep) {
    if (threadIdx.x == 0) {
      const unsigned tgt = top_target(cc.dep_nwg);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(cc.dep + kShards, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < tgt) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 5000000ull) {
          __hip_atomic_store(cc.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(8);
      }
    }
    __syncthreads();
  }
}
// After this wave's sc1 stores (every storing wave of the workgroup must have drained before
// the signalling lane runs): count the workgroup done; the shard's last arriver bumps the top.
__device__ __forceinline__ void chain_count_done(const ChainCtl& cc) {
  if (cc.sig) {
    const int sh = cc.local % kShards;
    const unsigned old = __hip_atomic_fetch_add(cc.sig + sh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == shard_target(cc.sig_nwg, sh))
      __hip_atomic_fetch_add(cc.sig + kShards, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ void chain_signal(const ChainCtl& cc) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) chain_count_done(cc);
}

}  // namespace llj

// Shared device helpers for the lit-llama MI355X (gfx950) decode path.
// Wave64 everywhere; MFMA 16x16x32 bf16 / 16x16x64 i8 operand maps per the CDNA4 guide:
//   A: lane l holds A[row l&15][k = 8*(l>>4) + j], B: lane l holds B[k = 8*(l>>4) + j][col l&15]
//   C/D: lane l, reg r holds C[row 4*(l>>4) + r][col l&15]
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace llj {

#ifndef LLJ_TRACE
#define LLJ_TRACE 0  // profiling only: per-workgroup phase timestamps (s_memrealtime, 100 MHz)
#endif
#if LLJ_TRACE
// [workgroup][8]: 6 phase stamps, then HW_ID (CU / SE of the workgroup) and XCC_ID at stamp 0
static __device__ unsigned long long g_trace[8192 * 8];  // per translation unit
#define LLJ_STAMP(k)                                                                             \
  if (threadIdx.x == 0 && blockIdx.x < 8192) {                                                   \
    g_trace[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();                            \
    if ((k) == 0) {                                                                              \
      g_trace[blockIdx.x * 8 + 6] = __builtin_amdgcn_s_getreg((31 << 11) | 4);  /* HW_ID */   \
      g_trace[blockIdx.x * 8 + 7] = __builtin_amdgcn_s_getreg((31 << 11) | 20); /* XCC_ID */  \
    }                                                                                            \
  }
// per translation unit: extern "C" llj_trace_copy_<tu>(host_dst, bytes)
#define LLJ_TRACE_EXPORT(tu)                                                                     \
  int llj_trace_copy_##tu(void* host_dst, size_t bytes) {                                        \
    return (int)hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(llj::g_trace), bytes, 0, hipMemcpyDeviceToHost); \
  }
#else
#define LLJ_STAMP(k)
#define LLJ_TRACE_EXPORT(tu)
#endif

typedef uint16_t bf16_t;  // raw bf16 bits in HBM
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(bf16_t b) { return __uint_as_float(((uint32_t)b) << 16); }
__device__ __forceinline__ float bflo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bfhi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }

// fp32 -> bf16 round-to-nearest-even (lowers to v_cvt_pk_bf16_f32 on gfx950; keeps NaN)
__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, __float2bfloat16(f));
}
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}
__device__ __forceinline__ float round_bf(float f) { return bf2f(f2bf(f)); }
// fp32 -> fp16 -> fp32 (bitsandbytes' A16 = A.half())
__device__ __forceinline__ float f16r(float x) { return (float)(_Float16)x; }

// packed pairs: one v_pk_mul_f32 / v_cvt_pk_bf16_f32 for two values
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 unpk(uint32_t w) { return f32x2{bflo(w), bfhi(w)}; }
__device__ __forceinline__ uint32_t cvt_pk(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));
}

// (x & m) | c: the compiler selects one v_and_or_b32 when m is in an SGPR (pass it through
// uniform()). Not inline asm: the hazard recognizer cannot see inside asm blocks, and an asm
// VALU write to a VGPR an in-flight MFMA still reads as its B operand is a WAR hazard that
// corrupted results when the writes were scheduled right after the MFMA.
__device__ __forceinline__ uint32_t and_or(uint32_t x, uint32_t m_sgpr, uint32_t c) { return (x & m_sgpr) | c; }

__device__ __forceinline__ f32x4 mfma_bf16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ i32x4 mfma_i8(i32x4 a, i32x4 b, i32x4 c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}


#ifndef LLJ_OUT_STORE
#define LLJ_OUT_STORE 1  // 1 agent-scope relaxed atomic store (sc1, write-through; measured 7B: bs=1 1.167 -> 1.151 ms, bs=8 1.819 -> 1.789), 0 plain, 2 non-temporal
#endif
// 4-byte store of an epilogue output (a bf16 column pair) through a vector store
__device__ __forceinline__ void st_out32(void* dst, uint32_t v) {
  uint32_t* p = reinterpret_cast<uint32_t*>(dst);
#if LLJ_OUT_STORE == 1
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#elif LLJ_OUT_STORE == 2
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

// host-side A/B options (options.hip, llj_set_option): -1 = the site's build default
int opt(int which);

__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// A zero in a VGPR that the compiler cannot see through. Added to the index of a load from a
// wave-uniform address it keeps the value in VGPRs: the compiler moves a uniform value to SGPRs
// with a readfirstlane right after its load -- a vmcnt wait for that load, and for every load
// issued before it, at the point of issue (a prefetch that waits for itself).
__device__ __forceinline__ int vzero() {
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return z;
}// Cross-lane moves inside a DPP row (16 lanes) as one VALU op each, instead of __shfl_xor's
// ds_bpermute (an LDS round trip plus a wait).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __builtin_bit_cast(float, dpp_u32<CTRL>(__builtin_bit_cast(uint32_t, v)));
}
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppRowMirror = 0x140;  // lane i <- 15 - i
constexpr int kDppHalfMirror = 0x141; // lane i <- 7 - i within each half row
__device__ __forceinline__ uint32_t lane_xor1(uint32_t v) { return dpp_u32<kDppXor1>(v); }
__device__ __forceinline__ float lane_xor1(float v) { return dpp_f32<kDppXor1>(v); }
// Sum over the 16 lanes of a row; every step pairs lanes symmetrically, so all 16 lanes end
// with the bitwise-same total (as an xor butterfly would).
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f32<kDppHalfMirror>(v);
  v += dpp_f32<kDppRowMirror>(v);
  v += dpp_f32<kDppXor1>(v);
  v += dpp_f32<kDppXor2>(v);
  return v;
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f32<kDppHalfMirror>(v));
  v = fmaxf(v, dpp_f32<kDppRowMirror>(v));
  v = fmaxf(v, dpp_f32<kDppXor1>(v));
  v = fmaxf(v, dpp_f32<kDppXor2>(v));
  return v;
}
// The other half of each 32-lane pair of rows (lane i <- i ^ 16) and of the wave (i <- i ^ 32),
// as the two halves that gfx950's v_permlane16_swap / v_permlane32_swap hand back: a VALU move
// instead of __shfl_xor's ds_bpermute (an LDS round trip each). Inline asm: the ROCm 7.2
// builtins (__builtin_amdgcn_permlane{16,32}_swap) miscompile here, the second result read
// back as the first (lo + hi emitted as lo + lo). The asm pads its own hazards: s_nop 1 after
// the VALU write of its operands and before their next VALU read.
template <bool WIDE>
__device__ __forceinline__ void lane_halves(float v, float& lo, float& hi) {
  float a = v, b = v;
  if constexpr (WIDE)
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
  else
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
  lo = a;
  hi = b;
}
// Sum / max over the 64 lanes of the wave, the same value (bitwise) in every lane: DPP inside
// each 16-lane row, then rows (0+1, 2+3) and halves (lo+hi), in one order for all lanes.
// RMSNorm output pair g * bf16(x * r), each product rounded to bf16 (model.py:283 on bf16 tensors)
__device__ __forceinline__ uint32_t norm_pair(uint32_t a, uint32_t g, float r) {
  return pack2bf(round_bf(bflo(g) * round_bf(bflo(a) * r)), round_bf(bfhi(g) * round_bf(bfhi(a) * r)));
}

__device__ __forceinline__ float wave_sum(float v) {
  float lo, hi;
  v = row16_sum(v);
  lane_halves<false>(v, lo, hi);
  v = lo + hi;
  lane_halves<true>(v, lo, hi);
  return lo + hi;
}
__device__ __forceinline__ float wave_max(float v) {
  float lo, hi;
  v = row16_max(v);
  lane_halves<false>(v, lo, hi);
  v = fmaxf(lo, hi);
  lane_halves<true>(v, lo, hi);
  return fmaxf(lo, hi);
}

}  // namespace llj

// Error convention for the C ABI: 0 = ok, otherwise a hipError_t or one of these.
#define LLJ_EINVAL 1000
#define LLJ_CHECK_LAUNCH()                         \
  do {                                             \
    hipError_t e__ = hipGetLastError();            \
    if (e__ != hipSuccess) return (int)e__;        \
  } while (0)
#define LLJ_REQUIRE(c) \
  do {                 \
    if (!(c)) return LLJ_EINVAL; \
  } while (0)

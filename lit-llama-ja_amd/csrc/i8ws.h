// LLM.int8() activation workspace (filled by llj_i8_stats, read by the int8 GEMV).
//
//   [0, 16)        header {mtot, K, nsb, kb}
//   aq[M][K]       the activation quantized once: round(A16 * 127 / SCA), outlier columns 0 -- first,
//                  so that row r is at 16 + r * K whatever M is (the streamed int8 GEMV, AM_I8S,
//                  addresses its rows before it has read the header)
//   part[nsb][M]   fp32 per-(k-block, row) absmax of the non-outlier elements
//   cnt[nsb]       outlier columns found in each k-block
//   list[nsb][kb]  their column indices (ascending within a block)
//   sca[M]         SCA[m] = max over the k-blocks of part
//   flag[K]        1 for an outlier column
//   avh[4]         avh[0] = 1 when aval below is valid (the one-launch decode prep, M <= 8), else 0
//   aval[nsb][kb]  f16(A) of rows 0..7 of each listed outlier column (16 B, list order; rows >= M 0):
//                  the int8 GEMV's in-stream fp16 side product reads them with the chunk's weights
// Quantizing once here (instead of in every GEMV workgroup) is what keeps the batched int8
// GEMV weight-streaming.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace llj {

constexpr int kNSB = 32;  // statistics blocks (k-ranges)

struct I8WsHeader {
  int mtot, K, nsb, kb;
};

// k-block width: a multiple of 32, so a block's outlier flags are whole 32-bit words of the
// hand-off block below
__host__ __device__ inline int i8_kb(int K) { return ((K + kNSB - 1) / kNSB + 31) & ~31; }

__host__ __device__ inline size_t i8_align16(size_t x) { return (x + 15) & ~(size_t)15; }

// A count or a list entry read back from a workspace is bounded by what it indexes before use: a
// stale or corrupt workspace (a count past kb, a column outside [0, K)) then gives wrong numbers,
// never an out-of-bounds read (the r05i fault: a prep variant that skipped the list compaction left
// the counts stale and the side product walked past the list)
__host__ __device__ inline int i8_cnt_clamp(int c, int kb) { return c < 0 ? 0 : (c > kb ? kb : c); }
__host__ __device__ inline int i8_col_clamp(int k, int K) { return k < 0 ? 0 : (k >= K ? K - 1 : k); }
__host__ __device__ inline int i8_nsb_clamp(int nsb) { return nsb < 0 ? 0 : (nsb > kNSB ? kNSB : nsb); }

// byte offsets of the arrays (the layout above)
struct I8Offsets {
  size_t part, cnt, list, sca, flag, aq, avh, aval, total;
};
__host__ __device__ inline I8Offsets i8_offsets(int M, int K) {
  I8Offsets o;
  o.aq = 16;
  o.part = i8_align16(o.aq + (size_t)M * K);
  o.cnt = o.part + sizeof(float) * (size_t)kNSB * M;
  o.list = o.cnt + sizeof(int) * kNSB;
  o.sca = o.list + sizeof(int) * (size_t)kNSB * i8_kb(K);
  o.flag = i8_align16(o.sca + sizeof(float) * (size_t)M);
  o.avh = i8_align16(o.flag + (size_t)K);
  o.aval = o.avh + 16;
  o.total = o.aval + (size_t)16 * kNSB * i8_kb(K);
  return o;
}

struct I8Layout {
  float* part;
  int* cnt;
  int* list;
  float* sca;
  uint8_t* flag;  // flag[k] = 1 for an outlier column
  int8_t* aq;
  int* avh;
  uint4* aval;
};

__host__ __device__ inline I8Layout i8_layout(const void* ws, int M, int K) {
  char* b = const_cast<char*>(reinterpret_cast<const char*>(ws));
  const I8Offsets o = i8_offsets(M, K);
  return I8Layout{reinterpret_cast<float*>(b + o.part), reinterpret_cast<int*>(b + o.cnt),
                  reinterpret_cast<int*>(b + o.list), reinterpret_cast<float*>(b + o.sca),
                  reinterpret_cast<uint8_t*>(b + o.flag), reinterpret_cast<int8_t*>(b + o.aq),
                  reinterpret_cast<int*>(b + o.avh), reinterpret_cast<uint4*>(b + o.aval)};
}

// LLM.int8() row statistics of a decode activation (M <= 8 rows) handed from the op that produces
// it to the int8 GEMV that consumes it, instead of a statistics launch in between (attention -> y,
// SwiGLU -> h). Words [kI8StSca, kI8StSca + 8 kI8StSlots): SCA partials -- slot s, row m at
// kI8StSca + 8 s + m: the max |f16(A[m, k])| below the threshold over the producer workgroups that
// map to slot s (as the bits of the non-negative float, atomicMax); SCA[m] = max over the slots.
// Words [kI8StFlags, kI8StFlags + ceil(K / 32)): the outlier columns (any row |f16(A)| >= threshold),
// bit k % 32 of word k / 32 (atomicOr). Max and or are order-independent, so the values are the
// statistics launch's exactly; the slots keep the atomics off a few hot addresses (688 SwiGLU
// workgroups on 8 words took 47 us). Zeroed before the producer runs.
constexpr int kI8StSca = 16;
constexpr int kI8StSlots = 64;
constexpr int kI8StFlags = kI8StSca + 8 * kI8StSlots;
__host__ __device__ inline int i8st_words(int K) { return kI8StFlags + (K + 31) / 32; }

}  // namespace llj

// Host-side A/B options of the library (no device state): each is read from the environment ONCE,
// at its first use, validated, and settable per process through llj_set_option (tests, A/B runs).
// -1 = the build default of the site that reads it. Launch paths read a table entry, never getenv.
#include <cstdlib>

#include "common.h"
#include "lit_llama_amd.h"

namespace llj {

namespace {
struct OptSpec {
  const char* env;
  int lo, hi;
};
// index = LLJ_OPT_* (lit_llama_amd.h)
constexpr OptSpec kOpts[LLJ_OPT_COUNT] = {
    {"LLJ_ATT_SPEC", 0, 1},          // decode attention's speculative first pass: 0 half (default), 1 whole ("full")
    {"LLJ_FLASH_QB", 1, 2},          // flash prefill: 16-query blocks per wave
    {"LLJ_FLASH_PAIR", 0, 1},        // flash prefill: (long, short) query-block pairs per workgroup
    {"LLJ_GEMM_GLDS", 0, 1},         // prefill GEMMs (M >= 256): 1 LDS-DMA kernel, 0 register-staged, for every format
    {"LLJ_GLDS_COST128", 0, 100000}, // LDS-DMA GEMM: cost of a 256 x 128 tile in % of a 256 x 256 one
    {"LLJ_GEMV_LDS_A_KB", 56, 96},   // decode GEMVs: cap of the staged A image (KiB)
    {"LLJ_ATT_SPEC_BATCH", 0, 1},    // decode attention: the half speculative pass also for large grids
    {"LLJ_GEMM_W4Z", 0, 1},          // prefill int4 GEMMs with integral zeros: the convert-once LDS-DMA kernel
};

int env_value(int i) {
  const char* e = getenv(kOpts[i].env);
  if (!e || !e[0]) return -1;
  long v;
  if (i == LLJ_OPT_ATT_SPEC_FULL) v = (e[0] == 'f' || e[0] == '1') ? 1 : 0;  // "full" / "half"
  else v = atol(e);
  return v < kOpts[i].lo ? kOpts[i].lo : v > kOpts[i].hi ? kOpts[i].hi : (int)v;
}

int* table() {
  static int t[LLJ_OPT_COUNT] = {};
  static const bool init = [] {
    for (int i = 0; i < LLJ_OPT_COUNT; ++i) t[i] = env_value(i);
    return true;
  }();
  (void)init;
  return t;
}
}  // namespace

int opt(int which) { return which >= 0 && which < LLJ_OPT_COUNT ? table()[which] : -1; }

}  // namespace llj

extern "C" int llj_set_option(int which, int value) {
  using namespace llj;
  if (which < 0 || which >= LLJ_OPT_COUNT) return -1000;
  if (value != -1 && (value < kOpts[which].lo || value > kOpts[which].hi)) return -1000;
  int* t = table();
  const int old = t[which];
  t[which] = value;
  return old;
}

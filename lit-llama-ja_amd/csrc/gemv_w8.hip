// Instantiations of the GEMV kernels for weight format WF_W8 (gemv_impl.h).
#include "gemv_impl.h"

namespace llj {
int gemv_launch_w8(int am, int ep, const GemvParams& p, hipStream_t s) { return launch_fmt<WF_W8>(am, ep, p, s); }
}  // namespace llj

extern "C" {
LLJ_TRACE_EXPORT(w8)
}

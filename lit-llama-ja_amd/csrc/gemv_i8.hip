// Instantiations of the GEMV kernels for weight format WF_I8 (gemv_impl.h).
#include "gemv_impl.h"

namespace llj {
int gemv_launch_i8(int am, int ep, const GemvParams& p, hipStream_t s) { return launch_fmt<WF_I8>(am, ep, p, s); }
}  // namespace llj

extern "C" {
LLJ_TRACE_EXPORT(i8)
}

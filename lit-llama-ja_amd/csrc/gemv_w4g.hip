// Instantiations of the GEMV kernels for weight format WF_W4G (grouped int4, gemv_impl.h).
#include "gemv_impl.h"

namespace llj {
int gemv_launch_w4g(int am, int ep, const GemvParams& p, hipStream_t s) { return launch_fmt<WF_W4G>(am, ep, p, s); }
}  // namespace llj

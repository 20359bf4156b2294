// rtg_trace_s.hip — instantiates the trace kernels for ONE stack capacity,
// RTG_S (set by the Makefile: one object per S = 1..16, built in parallel).
#include "rtg_trace_kernels.h"

#ifndef RTG_S
#error "RTG_S (stack capacity) must be defined"
#endif
#define RTG_CAT2(a, b) a##b
#define RTG_CAT(a, b) RTG_CAT2(a, b)

namespace rtg {
TraceFn RTG_CAT(trace_fn_s, RTG_S)(bool lds, int variant, bool bvh, int list) {
  return trace_fn<RTG_S>(lds, variant, bvh, list);
}
}  // namespace rtg

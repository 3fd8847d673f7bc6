// Batched k-means (placeholder until the kernel lands).
#include <hip/hip_runtime.h>

#include "ccmi_internal.h"

extern "C" size_t cc_kmeans_workspace_bytes(int, int, int, int, const int32_t*, int, int, int, int) {
  return 0;
}

extern "C" int cc_kmeans_batched(const float*, const float*, int, int, int, const int32_t*, int, int,
                                 int, int, const int32_t*, int, int, int, double, const double*,
                                 int, const int32_t*, int8_t*, int, float*, int32_t*,
                                 unsigned long long*, void*, size_t, void*) {
  cc::set_error("cc_kmeans_batched: not built yet");
  return CC_ERR_UNSUPPORTED;
}

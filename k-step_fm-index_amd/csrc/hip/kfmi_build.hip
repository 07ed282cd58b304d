/*
 * kfmi_build.hip -- GPU index builder (placeholder until the device suffix
 * sort lands; the host builder in csrc/host/fmi_build.c is complete).
 */
#include <hip/hip_runtime.h>
#include "../kfmi_internal.h"

extern "C" int32_t kfmi_build_index_gpu(const char* text, uint64_t n, uint32_t k, uint32_t d,
                                        int32_t want_host_image, void** index)
{
  (void) want_host_image;
  return kfmi_build_index_cpu(text, n, k, d, index);
}

/*
 * kfmi_devguard.h -- keeps the caller's current HIP device across the
 * library's entry points (shared by every translation unit that selects
 * devices).
 */
#ifndef KFMI_DEVGUARD_H_
#define KFMI_DEVGUARD_H_

#include <hip/hip_runtime.h>

namespace kfmi {

/* The caller's current HIP device, put back when an entry point returns.  The
 * library selects devices internally (the index's, the results', each group
 * member's); none of that leaks: a HIP or torch call the caller makes next
 * lands on the device it had selected.  (The reference leaves DEVICE selected
 * after transferCPUtoGPU, fmIndexGPU-Coop-2Step.cu:256; its driver makes no
 * HIP call of its own, so it cannot tell.)  No-op without a HIP device. */
struct DeviceGuard {
  int dev = -1;
  DeviceGuard()
  {
    if (hipGetDevice(&dev) != hipSuccess) {
      (void) hipGetLastError();
      dev = -1;
    }
  }
  ~DeviceGuard()
  {
    int now = -1;
    if (dev >= 0 && hipGetDevice(&now) == hipSuccess && now != dev) (void) hipSetDevice(dev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

}  // namespace kfmi

#endif  // KFMI_DEVGUARD_H_

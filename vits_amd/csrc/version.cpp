// Library introspection entry points.
#include <hip/hip_runtime.h>
#include <string.h>

#include "common.h"

extern "C" const char* vits_amd_version(void) { return "vits_amd 0.1.0 gfx950"; }

extern "C" int vits_amd_device_arch(char* buf, int len) {
  if (!buf || len <= 0) return VITS_E_ARG;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return VITS_E_ARG;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return VITS_E_ARG;
  strncpy(buf, prop.gcnArchName, (size_t)len - 1);
  buf[len - 1] = 0;
  return VITS_OK;
}

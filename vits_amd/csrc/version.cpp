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

#include <atomic>

namespace {
std::atomic<int64_t> g_counts[VITS_CNT_N];
}

void vits_count(int which, int n) {
  if (which >= 0 && which < VITS_CNT_N) g_counts[which].fetch_add(n, std::memory_order_relaxed);
}

extern "C" int64_t vits_dispatch_count(int which) {
  if (which < 0 || which >= VITS_CNT_N) return -1;
  return g_counts[which].load(std::memory_order_relaxed);
}

extern "C" void vits_dispatch_count_reset(void) {
  for (auto& c : g_counts) c.store(0, std::memory_order_relaxed);
}

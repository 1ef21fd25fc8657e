// Shared helpers for the gfx950 kernels of libvits_amd.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vits_amd.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define VITS_CHECK_ARG(cond)  \
  do {                        \
    if (!(cond)) return VITS_E_ARG; \
  } while (0)
#define VITS_CHECK_SHAPE(cond)  \
  do {                          \
    if (!(cond)) return VITS_E_SHAPE; \
  } while (0)

static inline int vits_launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? VITS_OK : (int)e;
}

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

__device__ __forceinline__ float vits_sigmoid(float x) { return 1.0f / (1.0f + __expf(-x)); }

// tanh with full fp32 accuracy (torch CPU uses an accurate tanh; the fast
// exp-based form loses ~1e-7 relative near 0, which is fine, but we keep the
// libm form to stay within a few ulp of the reference).
__device__ __forceinline__ float vits_tanh(float x) { return tanhf(x); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// host-side dispatch counters (vits_dispatch_count, include/vits_amd.h)
void vits_count(int which, int n = 1);
static inline int count_ok(int rc, int which, int n = 1) {
  if (rc == VITS_OK) vits_count(which, n);
  return rc;
}

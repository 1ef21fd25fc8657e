// mfma_probe.hip - what the split-fp32 conv's k-step loop can reach on
// MI355X: bf16 MFMA loops shaped like conv1d_impl.h's F32P loop (a 64 x 64
// wave tile, six products per fragment pair = 24 v_mfma_f32_32x32x16_bf16
// per 16-deep k-step), two 256-thread workgroups per CU (two waves per
// SIMD), random operands, against the same work as v_mfma_f32_16x16x32_bf16
// (96 per step), each with and without the loop's operand traffic (6 A
// fragments from global memory / L2 and 6 B fragments from LDS per step,
// issued one step ahead).  Prints TFLOP/s and the in-kernel clock.
//   hipcc --offload-arch=gfx950 -O3 -o build/mfma_probe tools/mfma_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int STEPS = 4096;
constexpr int ABUF = 1 << 20;  // bf16x8 entries of the A buffer (16 MB: L2 / MALL resident)

// SHAPE 0: 32x32x16 (4 accumulators, 6 products each per step)
// SHAPE 1: 16x16x32 (16 accumulators, 6 products each per 32-deep step = two 16-deep steps)
template <int SHAPE, bool LOADS>
__global__ __launch_bounds__(256, 2) void probe(const bf16x8* __restrict__ abuf, float* out,
                                                long long* clk) {
  __shared__ bf16x8 lds[4096];
  const int tid = threadIdx.x;
  for (int i = tid; i < 4096; i += 256) lds[i] = abuf[(blockIdx.x * 4096 + i) & (ABUF - 1)];
  __syncthreads();
  bf16x8 a[2][6], b[2][6];
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    a[0][q] = abuf[(tid * 7 + q * 131 + blockIdx.x * 977) & (ABUF - 1)];
    b[0][q] = lds[(tid * 3 + q * 67) & 4095];
    a[1][q] = a[0][q];
    b[1][q] = b[0][q];
  }
  const long long t0 = __builtin_amdgcn_s_memtime();
  const long long r0 = __builtin_amdgcn_s_memrealtime();
  float sum = 0.f;
  if constexpr (SHAPE == 0) {
    f32x16 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    for (int s = 0; s < STEPS; s += 2) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        bf16x8* ac = a[h];
        bf16x8* bc = b[h];
        if constexpr (LOADS) {
          bf16x8* an = a[h ^ 1];
          bf16x8* bn = b[h ^ 1];
          const int base = ((s + h + 1) * 1024 + blockIdx.x * 64 + (tid & 63)) & (ABUF - 1);
#pragma unroll
          for (int q = 0; q < 6; ++q) an[q] = abuf[(base + q * 64 * 4096) & (ABUF - 1)];
#pragma unroll
          for (int q = 0; q < 6; ++q) bn[q] = lds[((s + h) * 37 + tid + q * 256) & 4095];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni) {
            f32x16 c = acc[mi * 2 + ni];
#pragma unroll
            for (int p = 0; p < 6; ++p)
              c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ac[mi * 3 + p / 2], bc[ni * 3 + p % 3], c,
                                                          0, 0, 0);
            acc[mi * 2 + ni] = c;
          }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) sum += acc[i][r];
  } else {
    f32x4 acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][r] = 0.f;
    // 16x16x32: a 32-deep step covers two 16-deep k-steps of the 32x32 loop;
    // per 32-deep step 4 x 4 sub-tiles x 6 products = 96 MFMAs = the FLOPs
    // of 2 x 24 32x32x16; the operands: 4 A + 4 B fragments x 3 planes
    for (int s = 0; s < STEPS; s += 2) {
      bf16x8* ac = a[0];
      bf16x8* bc = b[0];
      if constexpr (LOADS) {
        const int base = ((s + 1) * 1024 + blockIdx.x * 64 + (tid & 63)) & (ABUF - 1);
#pragma unroll
        for (int q = 0; q < 6; ++q) a[1][q] = abuf[(base + q * 64 * 4096) & (ABUF - 1)];
#pragma unroll
        for (int q = 0; q < 6; ++q) b[1][q] = lds[(s * 37 + tid + q * 256) & 4095];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          f32x4 c = acc[mi * 4 + ni];
#pragma unroll
          for (int p = 0; p < 6; ++p)
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ac[(mi + p) % 6], bc[(ni + p) % 6], c, 0, 0,
                                                        0);
          acc[mi * 4 + ni] = c;
        }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (LOADS) {
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          a[0][q] = a[1][q];
          b[0][q] = b[1][q];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) sum += acc[i][r];
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  const long long r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + tid] = sum;
  if (tid == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int SHAPE, bool LOADS>
void run(const char* name, const bf16x8* abuf, float* out, long long* clk, int blocks) {
  hipLaunchKernelGGL((probe<SHAPE, LOADS>), dim3(blocks), dim3(256), 0, 0, abuf, out, clk);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = 20;
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((probe<SHAPE, LOADS>), dim3(blocks), dim3(256), 0, 0, abuf, out, clk);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  std::vector<long long> c(2 * blocks);
  hipMemcpy(c.data(), clk, sizeof(long long) * 2 * blocks, hipMemcpyDeviceToHost);
  double ghz = 0;
  for (int i = 0; i < blocks; ++i) ghz += (double)c[2 * i] / (double)c[2 * i + 1] * 0.1;
  ghz /= blocks;
  // FLOP: per wave and step 24 x (2 * 32 * 32 * 16)
  const double flop = (double)blocks * 4 * STEPS * 24 * 2.0 * 32 * 32 * 16;
  printf("%-34s %8.3f ms  %7.1f TF/s bf16  (= %6.1f TF/s split fp32)  clock %.2f GHz\n", name, ms,
         flop / ms / 1e9, flop / ms / 1e9 / 6, ghz);
}

int main() {
  bf16x8* abuf;
  float* out;
  long long* clk;
  hipMalloc(&abuf, sizeof(bf16x8) * ABUF);
  const int blocks = 512;  // two per CU
  hipMalloc(&out, sizeof(float) * blocks * 256);
  hipMalloc(&clk, sizeof(long long) * 2 * blocks);
  std::vector<__bf16> h(8 * (size_t)ABUF);
  srand(1);
  for (auto& v : h) v = (__bf16)((float)rand() / RAND_MAX - 0.5f);
  hipMemcpy(abuf, h.data(), sizeof(bf16x8) * ABUF, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) {
    run<0, false>("32x32x16, registers only", abuf, out, clk, blocks);
    run<1, false>("16x16x32, registers only", abuf, out, clk, blocks);
    run<0, true>("32x32x16 + A global / B LDS", abuf, out, clk, blocks);
    run<1, true>("16x16x32 + A global / B LDS", abuf, out, clk, blocks);
  }
  return 0;
}

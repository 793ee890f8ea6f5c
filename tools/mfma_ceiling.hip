// mfma_ceiling.hip — sustained fp32-MFMA rate and shader clock on this GPU.
//
// Register-only v_mfma_f32_32x32x2_f32 loop (4 independent accumulators per
// wave, random operands), every CU busy with the GEMM's occupancy (2 blocks x
// 4 waves per CU), timed with hipEvents over ~1 s; the in-kernel clock is
// Δs_memtime / Δs_memrealtime x 100 MHz (MI355X_MICROARCH.md, DVFS give-back).
// This is the ceiling the fp32 GEMM's roofline fraction should be read
// against (spec peak 157.3 TF assumes 2.4 GHz).
//
//   hipcc --offload-arch=gfx950 -O3 -o build/mfma_ceiling tools/mfma_ceiling.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void __launch_bounds__(256, 2) mfma_loop(float* out, unsigned long long* clk, int iters, float seed) {
  const int lane = threadIdx.x;
  float a = seed + lane * 1e-3f, b = seed - lane * 2e-3f;
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, b, c3, 0, 0, 0);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  out[blockIdx.x * blockDim.x + lane] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount * 2, threads = 256;
  float* out;
  unsigned long long* clk;
  hipMalloc(&out, sizeof(float) * blocks * threads);
  hipMalloc(&clk, sizeof(unsigned long long) * 2 * blocks);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  // warm-up ~2 s of back-to-back launches (DVFS settles)
  for (int w = 0; w < 120; ++w) hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(threads), 0, 0, out, clk, iters, 0.5f);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  const int reps = 120;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(threads), 0, 0, out, clk, iters, 0.25f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = (double)reps * blocks * (threads / 64) * iters * 16 * (2.0 * 32 * 32 * 2);
  std::vector<unsigned long long> h(2 * blocks);
  hipMemcpy(h.data(), clk, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  std::vector<double> mhz;
  for (int b = 0; b < blocks; ++b) mhz.push_back(h[2 * b] / (double)h[2 * b + 1] * 100.0);
  std::sort(mhz.begin(), mhz.end());
  printf("{\"cus\": %d, \"tflops\": %.2f, \"ms\": %.2f, \"clock_mhz_median\": %.0f, \"clock_mhz_min\": %.0f, "
         "\"clock_mhz_max\": %.0f, \"peak_at_clock_tflops\": %.2f}\n",
         p.multiProcessorCount, flops / (ms * 1e-3) / 1e12, ms, mhz[mhz.size() / 2], mhz.front(), mhz.back(),
         p.multiProcessorCount * 4 * 64.0 * mhz[mhz.size() / 2] * 1e6 / 1e12);
  return 0;
}

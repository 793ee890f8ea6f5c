// gemm_x3_probe.hip — speed and accuracy of the 3xbf16-split GEMM against the
// fp32-MFMA GEMM, both checked against an fp64 reference on sampled rows.
//   hipcc --offload-arch=gfx950 -O3 -I include -o tools/gemm_x3_probe tools/gemm_x3_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "../task-vector-replication_amd/csrc/gemm_x3bf16.hpp"

using namespace tvr;

__global__ void fill_normal(float* p, size_t n, unsigned seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)(i * 2654435761u) ^ seed, y = (unsigned)((i >> 32) * 40503u) ^ (seed * 7919u);
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15; y ^= x; y ^= y >> 13; y *= 0x5bd1e995u; y ^= y >> 15;
    const float u1 = ((x & 0xffffff) + 0.5f) / 16777216.0f, u2 = ((y & 0xffffff) + 0.5f) / 16777216.0f;
    p[i] = scale * sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
  }
}

// fp64 reference for rows rows[0..nr) : out[r][n] = sum_k A[row][k] W[n][k]; also sum |a||w|
__global__ void ref64(const float* A, const float* W, const int* rows, int nr, int N, int K, double* out, double* mag) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= nr * N) return;
  const int r = idx / N, n = idx % N;
  const float* a = A + (size_t)rows[r] * K;
  const float* w = W + (size_t)n * K;
  double s = 0, m = 0;
  for (int k = 0; k < K; ++k) { s += (double)a[k] * (double)w[k]; m += fabs((double)a[k] * (double)w[k]); }
  out[idx] = s;
  mag[idx] = m;
}

int main() {
  struct Shape { const char* name; int M, N, K; };
  std::vector<Shape> shapes = {{"qkv_mlpin", 90000, 17920, 2560}, {"o_mlpout", 90000, 2560, 12800}};
  for (auto& s : shapes) {
    float *A, *W, *C1, *C2;
    uint16_t* Wp;
    hipMalloc(&A, sizeof(float) * (size_t)s.M * s.K);
    hipMalloc(&W, sizeof(float) * (size_t)s.N * s.K);
    hipMalloc(&Wp, sizeof(uint16_t) * 3 * (size_t)s.N * s.K);
    hipMalloc(&C1, sizeof(float) * (size_t)s.M * s.N);
    hipMalloc(&C2, sizeof(float) * (size_t)s.M * s.N);
    hipLaunchKernelGGL(fill_normal, dim3(8192), dim3(256), 0, 0, A, (size_t)s.M * s.K, 11u, 1.0f);
    hipLaunchKernelGGL(fill_normal, dim3(8192), dim3(256), 0, 0, W, (size_t)s.N * s.K, 29u, 0.02f);
    hipLaunchKernelGGL(split_planes_kernel, dim3(8192), dim3(256), 0, 0, W, Wp, (size_t)s.N * s.K);
    GemmEpi e1{}; e1.out0 = C1; e1.ld0 = s.N;
    GemmEpi e2{}; e2.out0 = C2; e2.ld0 = s.N;
    auto run_f32 = [&]() {
      hipLaunchKernelGGL((gemm_f32_nt_kernel<EPI_BIAS, TileLarge>), dim3(gemm_grid<TileLarge>(s.M, s.N)),
                         dim3(TileLarge::THREADS), 0, 0, A, s.K, W, s.K, s.M, s.N, s.K, e1);
    };
    auto run_x3 = [&]() {
      hipLaunchKernelGGL((gemm_x3bf16_nt_kernel<EPI_BIAS, X3Large>), dim3(gemm_x3_grid<X3Large>(s.M, s.N)), dim3(X3Large::THREADS), 0, 0,
                         A, s.K, Wp, s.K, (size_t)s.N * s.K, s.M, s.N, s.K, e2);
    };
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    auto time_it = [&](auto fn) {
      fn(); hipDeviceSynchronize();
      hipEventRecord(a); fn(); hipEventRecord(b); hipEventSynchronize(b);
      float ms1; hipEventElapsedTime(&ms1, a, b);
      const int reps = std::max(2, (int)(1500.f / ms1));
      for (int i = 0; i < reps; ++i) fn();
      hipEventRecord(a);
      for (int i = 0; i < reps; ++i) fn();
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      return ms / reps;
    };
    const float ms_f32 = time_it(run_f32);
    const float ms_x3 = time_it(run_x3);
    run_f32(); run_x3(); hipDeviceSynchronize();
    // accuracy on 64 sampled rows x all N
    const int nr = 64;
    std::vector<int> hrows(nr);
    for (int i = 0; i < nr; ++i) hrows[i] = (int)((i * 1403ll + 17) % s.M);
    int* drows; double *ref, *mag;
    hipMalloc(&drows, nr * sizeof(int)); hipMalloc(&ref, sizeof(double) * nr * s.N); hipMalloc(&mag, sizeof(double) * nr * s.N);
    hipMemcpy(drows, hrows.data(), nr * sizeof(int), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(ref64, dim3((nr * s.N + 255) / 256), dim3(256), 0, 0, A, W, drows, nr, s.N, s.K, ref, mag);
    std::vector<double> hr(nr * s.N), hm(nr * s.N);
    hipMemcpy(hr.data(), ref, hr.size() * 8, hipMemcpyDeviceToHost);
    hipMemcpy(hm.data(), mag, hm.size() * 8, hipMemcpyDeviceToHost);
    double e1max = 0, e2max = 0, e1rms = 0, e2rms = 0, refrms = 0;
    std::vector<float> row(s.N);
    for (int pass = 0; pass < 2; ++pass) {
      for (int i = 0; i < nr; ++i) {
        hipMemcpy(row.data(), (pass ? C2 : C1) + (size_t)hrows[i] * s.N, s.N * 4, hipMemcpyDeviceToHost);
        for (int n = 0; n < s.N; ++n) {
          const double err = fabs(row[n] - hr[i * s.N + n]) / hm[i * s.N + n];
          if (pass) { e2max = std::max(e2max, err); e2rms += err * err; }
          else { e1max = std::max(e1max, err); e1rms += err * err; refrms += hr[i * s.N + n] * hr[i * s.N + n]; }
        }
      }
    }
    const double cnt = (double)nr * s.N;
    const double fl = 2.0 * s.M * (double)s.N * s.K;
    printf("{\"shape\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"f32_tflops\": %.1f, \"x3bf16_tflops\": %.1f, "
           "\"speedup\": %.3f, \"f32_err_max\": %.3e, \"x3_err_max\": %.3e, \"f32_err_rms\": %.3e, \"x3_err_rms\": %.3e, "
           "\"err_unit\": \"|C - C_fp64| / sum_k |a_k w_k|\"}\n",
           s.name, s.M, s.N, s.K, fl / (ms_f32 * 1e-3) / 1e12, fl / (ms_x3 * 1e-3) / 1e12, ms_f32 / ms_x3, e1max, e2max,
           sqrt(e1rms / cnt), sqrt(e2rms / cnt));
    fflush(stdout);
    hipFree(A); hipFree(W); hipFree(Wp); hipFree(C1); hipFree(C2); hipFree(drows); hipFree(ref); hipFree(mag);
  }
  return 0;
}

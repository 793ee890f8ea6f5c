// attention_probe.hip — time the engine's attention_mfma_kernel at the C3
// staircase shape (Pythia-2.8B: d 2560, 32 heads of 80, T = 15, fp32 qkv in,
// 2-plane fp16 z out) on synthetic data; achieved GB/s on the algorithmic
// bytes (Q, K, V fp32 + z planes = 16 B per row per model dim).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I task-vector-replication_amd/csrc \
//       -o tools/attention_probe tools/attention_probe.hip
//   tools/attention_probe [repeats]
// Variants measured with it in r02 (profiles/attention_variants_r02.json):
// coalesced 64-B Q/K loads, z through LDS, XCD-contiguous block order, no
// rotary / no stores (timing only).
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../task-vector-replication_amd/csrc/attention_mfma.hpp"

using namespace tvr;

__global__ void fill(float* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)(i * 2654435761u) ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = ((x & 0xffff) / 65536.0f - 0.5f) * 2.0f;
  }
}

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
  const int repeats = argc > 1 ? std::atoi(argv[1]) : 2;
  const int d = 2560, H = 32, DH = 80, T = 15, K2 = 12800, rd = 20;
  const int n_seq = 6144;  // 12 prompts x 32 heads x 16 entry layers: the middle of the C3 staircase
  const int R = n_seq * T;
  float *qkv, *cs, *sn;
  uint16_t* z;
  unsigned* flag;
  SeqDesc* sd;
  CHECK(hipMalloc(&qkv, sizeof(float) * (size_t)R * 3 * d));
  CHECK(hipMalloc(&z, sizeof(uint16_t) * (size_t)R * 2 * K2));
  CHECK(hipMalloc(&cs, sizeof(float) * 128 * rd));
  CHECK(hipMalloc(&sn, sizeof(float) * 128 * rd));
  CHECK(hipMalloc(&flag, 4));
  CHECK(hipMalloc(&sd, sizeof(SeqDesc) * n_seq));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, qkv, (size_t)R * 3 * d, 17u);
  std::vector<float> hc(128 * rd), hs(128 * rd);
  for (int p = 0; p < 128; ++p)
    for (int i = 0; i < rd; ++i) {
      const double f = std::pow(10000.0, -2.0 * (i % (rd / 2)) / rd);
      hc[p * rd + i] = (float)std::cos(p * f);
      hs[p * rd + i] = (float)std::sin(p * f);
    }
  CHECK(hipMemcpy(cs, hc.data(), hc.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(sn, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
  std::vector<SeqDesc> hsd(n_seq);
  for (int s = 0; s < n_seq; ++s) hsd[s] = SeqDesc{s * T, T, 0, -1, 0, 0};
  CHECK(hipMemcpy(sd, hsd.data(), hsd.size() * sizeof(SeqDesc), hipMemcpyHostToDevice));
  CHECK(hipMemset(flag, 0, 4));
  const int pairs = n_seq * H;
  const dim3 grid((pairs + ATTM_WAVES - 1) / ATTM_WAVES), block(64 * ATTM_WAVES);
  const float inv = 1.0f / std::sqrt((float)DH);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int rep = 0; rep < repeats; ++rep) {
    auto launch = [&]() {
      hipLaunchKernelGGL((attention_mfma_kernel<ACT_X2F16, 80, 1>), grid, block, 0, 0, qkv, 3 * d,
                         (const float*)nullptr, 3 * d, sd, n_seq, H, (void*)z, K2, (float*)nullptr, d, 0, INT_MAX,
                         flag, cs, sn, d, inv);
    };
    for (int i = 0; i < 3; ++i) launch();
    CHECK(hipDeviceSynchronize());
    const int reps = 20;
    CHECK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    const double bytes = 16.0 * R * d;
    printf("{\"kernel\": \"attention_mfma_kernel<ACT_X2F16, 80, 1>\", \"seqs\": %d, \"T\": %d, \"us\": %.1f, "
           "\"alg_bytes\": %.0f, \"gbps\": %.1f}\n", n_seq, T, ms * 1e3, bytes, bytes / (ms * 1e-3) / 1e9);
  }
  return 0;
}

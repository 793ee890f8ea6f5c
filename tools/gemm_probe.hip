// gemm_probe.hip — the engine's fp32 GEMM kernel alone at the Pythia-2.8B
// staircase shapes, ~2 s of back-to-back launches per shape (DVFS settled),
// reporting TFLOP/s and the in-kernel shader clock (Δs_memtime/Δs_memrealtime).
//   hipcc --offload-arch=gfx950 -O3 -I include -o tools/gemm_probe tools/gemm_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "../task-vector-replication_amd/csrc/gemm_f32.hpp"

using namespace tvr;
using Tile256x128k16 = GemmTile<256, 128, 2, 2, 16>;  // 4 waves, 2 blocks/CU (probe-only variant)
using Tile256x256k16 = GemmTile<256, 256, 2, 4, 16>;

template <class TL>
void launch_tile(int epi, int nblk, const float* A, const float* W, int M, int N, int K, const GemmEpi& ep) {
  if (epi == EPI_SPLIT_GELU)
    hipLaunchKernelGGL((gemm_f32_nt_kernel<EPI_SPLIT_GELU, TL>), dim3(nblk), dim3(TL::THREADS), 0, 0, A, K, W, K, M, N, K, ep);
  else
    hipLaunchKernelGGL((gemm_f32_nt_kernel<EPI_RESID, TL>), dim3(nblk), dim3(TL::THREADS), 0, 0, A, K, W, K, M, N, K, ep);
}

__global__ void fill(float* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = ((x & 0xffffff) / 16777216.0f - 0.5f) * 0.2f;
  }
}

int main(int argc, char** argv) {
  struct Shape { const char* name; int M, N, K, epi, tile; };
  // tile: 0 = engine choice, 1 = 256x256 BK32, 2 = 128x128, 3 = 256x128 BK16, 4 = 256x256 BK16
  std::vector<Shape> shapes;
  for (int tile : {1, 3, 4, 2}) {
    shapes.push_back({"qkv_mlpin M=90k", 90000, 17920, 2560, EPI_SPLIT_GELU, tile});
    shapes.push_back({"o_mlpout M=90k", 90000, 2560, 12800, EPI_RESID, tile});
  }
  shapes.push_back({"qkv_mlpin M=5760", 5760, 17920, 2560, EPI_SPLIT_GELU, 0});
  shapes.push_back({"o_mlpout M=5760", 5760, 2560, 12800, EPI_RESID, 0});
  for (auto& s : shapes) {
    float *A, *W, *C, *C2, *b;
    unsigned long long* stamps;
    int tile = s.tile ? s.tile : (gemm_use_large(s.M, s.N) ? 1 : 2);
    const int nblk = tile == 1 ? gemm_grid<TileLarge>(s.M, s.N) : tile == 2 ? gemm_grid<TileSmall>(s.M, s.N)
                   : tile == 3 ? gemm_grid<Tile256x128k16>(s.M, s.N) : gemm_grid<Tile256x256k16>(s.M, s.N);
    const char* tname = tile == 1 ? "256x256k32" : tile == 2 ? "128x128k32" : tile == 3 ? "256x128k16" : "256x256k16";
    hipMalloc(&A, sizeof(float) * (size_t)s.M * s.K);
    hipMalloc(&W, sizeof(float) * (size_t)s.N * s.K);
    hipMalloc(&C, sizeof(float) * (size_t)s.M * s.N);
    hipMalloc(&C2, sizeof(float) * (size_t)s.M * 10240);
    hipMalloc(&b, sizeof(float) * s.N);
    hipMalloc(&stamps, sizeof(unsigned long long) * 2 * nblk);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, A, (size_t)s.M * s.K, 1u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, W, (size_t)s.N * s.K, 2u);
    hipLaunchKernelGGL(fill, dim3(64), dim3(256), 0, 0, b, (size_t)s.N, 3u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, C, (size_t)s.M * s.N, 4u);
    GemmEpi ep{};
    ep.bias = b; ep.out0 = C; ep.ld0 = (s.epi == EPI_SPLIT_GELU) ? 7680 : s.N; ep.out1 = C2; ep.ld1 = 10240;
    ep.n_split = 7680; ep.resid = C; ep.ldr = s.N;
    auto launch = [&](unsigned long long* st) {
      ep.stamps = st;
      switch (tile) {
        case 1: launch_tile<TileLarge>(s.epi, nblk, A, W, s.M, s.N, s.K, ep); break;
        case 2: launch_tile<TileSmall>(s.epi, nblk, A, W, s.M, s.N, s.K, ep); break;
        case 3: launch_tile<Tile256x128k16>(s.epi, nblk, A, W, s.M, s.N, s.K, ep); break;
        default: launch_tile<Tile256x256k16>(s.epi, nblk, A, W, s.M, s.N, s.K, ep); break;
      }
    };
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    launch(nullptr);
    hipEventRecord(e0); launch(nullptr); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms1 = 0; hipEventElapsedTime(&ms1, e0, e1);
    const int reps = std::max(2, (int)(1500.0f / ms1));
    for (int i = 0; i < reps; ++i) launch(nullptr);  // ~2 s warm (DVFS settles)
    hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) launch(i == reps - 1 ? stamps : nullptr);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0; hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> h(2 * nblk);
    hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> mhz;
    for (int i = 0; i < nblk; ++i) if (h[2 * i + 1]) mhz.push_back(h[2 * i] / (double)h[2 * i + 1] * 100.0);
    std::sort(mhz.begin(), mhz.end());
    const double tf = 2.0 * s.M * (double)s.N * s.K * reps / (ms * 1e-3) / 1e12;
    printf("{\"tile\": \"%s\", \"shape\": \"%s\", \"tflops\": %.2f, \"ms_per_launch\": %.3f, \"clock_mhz_median\": %.0f, "
           "\"peak_at_clock\": %.1f, \"frac_of_clock_peak\": %.3f}\n", tname, s.name, tf, ms / reps, mhz[mhz.size() / 2],
           1024 * 64.0 * mhz[mhz.size() / 2] * 1e6 / 1e12, tf / (1024 * 64.0 * mhz[mhz.size() / 2] * 1e6 / 1e12));
    hipFree(A); hipFree(W); hipFree(C); hipFree(C2); hipFree(b); hipFree(stamps);
  }
  return 0;
}

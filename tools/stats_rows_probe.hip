// Unit probe of the EPI_STATS row reduction (gemm_pingpong.hpp pp_stats_rows) on synthetic LDS halves:
// one 512-thread block per case fills the 128-row LDS half from global memory and reduces it; the host
// compares max / sum exp / top-K / target logit with a double reference of the same rows.
//   hipcc --offload-arch=gfx950 -O3 -I include -o tools/stats_rows_probe tools/stats_rows_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#ifndef PP_HEADER
#define PP_HEADER "../task-vector-replication_amd/csrc/gemm_pingpong.hpp"
#endif
#include PP_HEADER

using namespace tvr;

#ifndef GEMM_ONLY
__global__ void __launch_bounds__(PP_THREADS) stats_probe_kernel(const float* src, int rows, int Nlim, int col0,
                                                                 float acc_scale, GemmEpi ep) {
  extern __shared__ float L[];
  for (int i = threadIdx.x; i < 128 * PP_EPI_LDR; i += blockDim.x) {
    const int r = i / PP_EPI_LDR, c = i % PP_EPI_LDR;
    L[i] = (r < rows && c < 256) ? src[r * 256 + c] : 0.f;
  }
  __syncthreads();
  pp_stats_rows(ep, L, 0, col0, rows, Nlim, threadIdx.x, acc_scale);
}
#endif

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e = (x);                                            \
    if (e != hipSuccess) {                                         \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                    \
    }                                                              \
  } while (0)

int main() {
  const int rows = 128, K = 5, rec = 2 + 2 * K, tiles = 2;
  int bad = 0;
#ifndef GEMM_ONLY
  for (int Nlim : {256, 128, 100, 4, 640}) {
    for (int tile = 0; tile < 2; ++tile) {
      const int col0 = tile * 256;
      const float scale = tile ? 0.5f : 1.0f;
      std::vector<float> a(128 * 256), bias(512);
      unsigned s = 12345u + Nlim + tile;
      auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xFFFF) / 65536.0f - 0.5f; };
      for (auto& x : a) x = 20.f * rnd();
      for (int r = 0; r < 128; ++r) a[r * 256 + (r % 7)] = a[r * 256 + 200 % std::max(Nlim, 1)];  // ties
      for (auto& x : bias) x = rnd();
      std::vector<int> tg(128);
      for (int r = 0; r < 128; ++r) tg[r] = col0 + (r * 37) % 300;
      float *d_a, *d_b, *d_st, *d_tl;
      int* d_tg;
      CK(hipMalloc(&d_a, a.size() * 4));
      CK(hipMalloc(&d_b, bias.size() * 4));
      CK(hipMalloc(&d_st, (size_t)128 * tiles * rec * 4));
      CK(hipMalloc(&d_tl, 128 * 4));
      CK(hipMalloc(&d_tg, 128 * 4));
      CK(hipMemcpy(d_a, a.data(), a.size() * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(d_b, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(d_tg, tg.data(), 128 * 4, hipMemcpyHostToDevice));
      CK(hipMemset(d_st, 0, (size_t)128 * tiles * rec * 4));
      CK(hipMemset(d_tl, 0, 128 * 4));
      GemmEpi ep{};
      ep.bias = d_b;
      ep.stats = d_st;
      ep.stats_k = K;
      ep.stats_tiles = tiles;
      ep.targets = d_tg;
      ep.tlogit = d_tl;
      hipLaunchKernelGGL(stats_probe_kernel, dim3(1), dim3(PP_THREADS), 128 * PP_EPI_LDR * 4, 0, d_a, rows, Nlim, col0,
                         scale, ep);
      CK(hipDeviceSynchronize());
      std::vector<float> st((size_t)128 * tiles * rec), tl(128);
      CK(hipMemcpy(st.data(), d_st, st.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(tl.data(), d_tl, 128 * 4, hipMemcpyDeviceToHost));
      double worst_se = 0;
      int bad_case = 0;
      for (int r = 0; r < rows; ++r) {
        std::vector<std::pair<float, int>> v;
        for (int c = 0; c < std::min(Nlim, 256); ++c) v.push_back({a[r * 256 + c] * scale + bias[col0 + c], col0 + c});
        float mx = -INFINITY;
        for (auto& p : v) mx = std::max(mx, p.first);
        double se = 0;
        for (auto& p : v) se += std::exp((double)p.first - mx);
        std::stable_sort(v.begin(), v.end(), [](auto& x, auto& y) { return x.first > y.first || (x.first == y.first && x.second < y.second); });
        const float* o = &st[((size_t)r * tiles + tile) * rec];
        if (o[0] != mx || std::fabs(o[1] - se) > 1e-5 * se) {
          if (bad_case < 3) printf("row %d: max %g want %g, sum %g want %g\n", r, o[0], mx, o[1], se);
          ++bad_case;
        }
        worst_se = std::max(worst_se, std::fabs(o[1] - se) / se);
        for (int j = 0; j < K; ++j) {
          const bool have = j < (int)v.size();
          const float ev = have ? v[j].first : -INFINITY;
          const int ei = have ? v[j].second : 0x7fffffff;
          int gi;
          std::memcpy(&gi, &o[2 + K + j], 4);
          if (o[2 + j] != ev || gi != ei) {
            if (bad_case < 3) printf("row %d j %d: got %g/%d want %g/%d\n", r, j, o[2 + j], gi, ev, ei);
            ++bad_case;
          }
        }
        const int tc = tg[r] - col0;
        if (tc < std::min(Nlim, 256) && tl[r] != a[r * 256 + tc] * scale + bias[tg[r]]) {
          if (bad_case < 3) printf("row %d: tlogit %g want %g\n", r, tl[r], a[r * 256 + tc] * scale + bias[tg[r]]);
          ++bad_case;
        }
        if (tc >= std::min(Nlim, 256) && tl[r] != 0.f) ++bad_case;
      }
      printf("{\"Nlim\": %d, \"tile\": %d, \"bad\": %d, \"se_rel_err_max\": %.3e}\n", Nlim, tile, bad_case, worst_se);
      bad += bad_case + (worst_se > 1e-5);
      hipFree(d_a); hipFree(d_b); hipFree(d_st); hipFree(d_tl); hipFree(d_tg);
    }
  }
#endif
  // the whole bf16 stats GEMM (gemm_pingpong_kernel<EPI_STATS, ACT_BF16>) on small-integer operands (exact
  // fp32 logits), M = 200 (a partial second half), N = 512 + 128 (a partial last tile), K = 128
  {
    const int M = 200, N = 640, Kd = 128, KS = 3, NT = (N + 255) / 256, recs = 2 + 2 * KS;
    std::vector<uint16_t> A((size_t)M * Kd), W((size_t)N * Kd);
    std::vector<float> Af(A.size()), Wf(W.size()), bias(N);
    unsigned s = 777u;
    auto rnd = [&](int lo, int hi) { s = s * 1664525u + 1013904223u; return lo + (int)((s >> 8) % (unsigned)(hi - lo + 1)); };
    auto bf = [](float x) { uint32_t u; std::memcpy(&u, &x, 4); return (uint16_t)(u >> 16); };
    for (size_t i = 0; i < A.size(); ++i) { Af[i] = (float)rnd(-3, 3); A[i] = bf(Af[i]); }
    for (size_t i = 0; i < W.size(); ++i) { Wf[i] = (float)rnd(-3, 3); W[i] = bf(Wf[i]); }
    for (auto& x : bias) x = (float)rnd(-8, 8) * 0.25f;
    std::vector<int> tg(M);
    for (int m = 0; m < M; ++m) tg[m] = (m * 97) % N;
    uint16_t *dA, *dW;
    float *dB, *dS, *dT;
    int* dG;
    CK(hipMalloc(&dA, A.size() * 2));
    CK(hipMalloc(&dW, W.size() * 2));
    CK(hipMalloc(&dB, N * 4));
    CK(hipMalloc(&dS, (size_t)M * NT * recs * 4));
    CK(hipMalloc(&dT, M * 4));
    CK(hipMalloc(&dG, M * 4));
    CK(hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dW, W.data(), W.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, bias.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dG, tg.data(), M * 4, hipMemcpyHostToDevice));
    CK(hipMemset(dT, 0, M * 4));
    GemmEpi ep{};
    ep.bias = dB;
    ep.stats = dS;
    ep.stats_k = KS;
    ep.stats_tiles = NT;
    ep.targets = dG;
    ep.tlogit = dT;
    hipLaunchKernelGGL((gemm_pingpong_kernel<EPI_STATS, ACT_BF16, true>), dim3(gemm_pingpong_grid(M, N)), dim3(PP_THREADS), 0,
                       0, dA, Kd, (size_t)0, dW, Kd, (size_t)0, 1.0f, M, N, Kd, ep);
    CK(hipDeviceSynchronize());
    std::vector<float> st((size_t)M * NT * recs), tl(M);
    CK(hipMemcpy(st.data(), dS, st.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(tl.data(), dT, M * 4, hipMemcpyDeviceToHost));
    int gbad = 0;
    for (int m = 0; m < M; ++m) {
      std::vector<float> row(N);
      for (int n = 0; n < N; ++n) {
        double acc = 0;
        for (int k = 0; k < Kd; ++k) acc += (double)Af[(size_t)m * Kd + k] * Wf[(size_t)n * Kd + k];
        row[n] = (float)acc + bias[n];
      }
      if (tl[m] != row[tg[m]]) {
        if (gbad < 5) printf("gemm row %d: tlogit %g want %g\n", m, tl[m], row[tg[m]]);
        ++gbad;
      }
      for (int t = 0; t < NT; ++t) {
        const float* o = &st[((size_t)m * NT + t) * recs];
        const int c1 = std::min(N, 256 * t + 256);
        float mx = -INFINITY;
        for (int n = 256 * t; n < c1; ++n) mx = std::max(mx, row[n]);
        double se = 0;
        for (int n = 256 * t; n < c1; ++n) se += std::exp((double)row[n] - mx);
        if (o[0] != mx || std::fabs(o[1] - se) > 1e-5 * se) {
          if (gbad < 5) printf("gemm row %d tile %d: max %g want %g, sum %g want %g\n", m, t, o[0], mx, o[1], se);
          ++gbad;
        }
      }
    }
    printf("{\"gemm_stats_bf16\": {\"M\": %d, \"N\": %d, \"bad\": %d}}\n", M, N, gbad);
    bad += gbad;
  }
  printf(bad ? "FAIL\n" : "OK\n");
  return bad ? 1 : 0;
}

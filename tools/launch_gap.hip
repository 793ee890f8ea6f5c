// launch_gap.hip — per-dispatch cost of back-to-back dependent launches on one
// stream (the C2 sweep runs ~256 small dispatches: how much of its span is
// dispatch overhead rather than kernel work?).  Diagnostic only.
//   hipcc --offload-arch=gfx950 -O2 -o tools/launch_gap tools/launch_gap.hip && ./tools/launch_gap
// Prints us per launch for: an empty 1-block kernel; a 256-block kernel that
// writes `mb` MB (dirty lines the end-of-kernel release must write back); the
// same sequence captured in a hipGraph and replayed.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));                      \
      return 1;                                                                \
    }                                                                          \
  } while (0)

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1024) p[0] = 1;  // never true: keeps the argument
}

__global__ void write_kernel(float4* p, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int N = 2000;
  float* buf;
  const size_t bytes = (size_t)64 << 20;
  CK(hipMalloc(&buf, bytes));
  auto run = [&](const char* name, auto&& body) -> int {
    for (int i = 0; i < 50; ++i) body();  // warm
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(a, st));
    for (int i = 0; i < N; ++i) body();
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("{\"case\": \"%s\", \"us_per_launch\": %.3f}\n", name, ms * 1e3 / N);
    return 0;
  };
  run("empty 1 block", [&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, nullptr); });
  run("empty 256 blocks x 512", [&] { hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(512), 0, st, nullptr); });
  for (int mb : {1, 8, 32}) {
    const size_t n4 = ((size_t)mb << 20) / 16;
    char name[64];
    std::snprintf(name, sizeof name, "write %d MB, 256 x 512", mb);
    run(name, [&] { hipLaunchKernelGGL(write_kernel, dim3(256), dim3(512), 0, st, (float4*)buf, n4); });
  }
  // graph replay of 100 empty 256-block launches
  {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(512), 0, st, nullptr);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(a, st));
    for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("{\"case\": \"graph: empty 256 blocks x 512\", \"us_per_launch\": %.3f}\n", ms * 1e3 / 2000);
  }
  CK(hipFree(buf));
  return 0;
}

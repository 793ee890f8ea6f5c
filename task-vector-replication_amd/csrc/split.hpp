// split.hpp — the activation side of the TVR_GEMM_X2F16 format.
//
// In X2F16 mode every GEMM input activation (LayerNorm outputs, attention z,
// GELU(h)) is written by its producer as two fp16 planes of 16 * a, interleaved
// per row: logical [R][K] -> halves [R][2][K] (row stride 2K halves, plane
// offset K), the same bytes as fp32.  a * 16 = x0 + x1, x0 = fp16(16 a),
// x1 = fp16(16 a - x0): 22 significand bits; the GEMM's LDS-DMA staging then
// copies the planes unchanged (gemm_x2f16.hpp).  |16 a| >= 65520 would round
// x0 to infinity: producers of unbounded values (z, GELU) raise *flag, which
// the engine reports as TVR_ERR_RANGE (LayerNorm outputs are bounded by
// sqrt(d) and need no check).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tvr {

constexpr float X2_ASCALE = 16.0f;
constexpr float X2_FP16_OVERFLOW = 65520.0f;  // fp16(x) is inf from here (round to nearest)

struct SplitF16 {
  uint16_t h0, h1;
};

__device__ __forceinline__ SplitF16 split_f16(float a) {
  const float x = a * X2_ASCALE;
  const _Float16 x0 = (_Float16)x;
  return {__builtin_bit_cast(uint16_t, x0), __builtin_bit_cast(uint16_t, (_Float16)(x - (float)x0))};
}

// store element a at p (plane 0) and p + plane (plane 1); NaN passes through
__device__ __forceinline__ void store_split(uint16_t* p, int plane, float a, unsigned* flag) {
  const SplitF16 s = split_f16(a);
  p[0] = s.h0;
  p[plane] = s.h1;
  if (fabsf(a) * X2_ASCALE >= X2_FP16_OVERFLOW && flag) atomicOr(flag, 1u);
}

// fp32 rows a [rows][lda] -> the split format with K logical columns
__global__ void split_rows_f16_kernel(const float* __restrict__ a, int lda, uint16_t* __restrict__ out, int rows,
                                      int K, unsigned* __restrict__ flag) {
  const size_t n = (size_t)rows * K;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / K, c = i % K;
    store_split(out + r * 2 * K + c, K, a[r * lda + c], flag);
  }
}

}  // namespace tvr

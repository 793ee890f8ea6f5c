// split.hpp — activation formats of the planar GEMM paths.
//
// ACT_X2F16 (TVR_GEMM_X2F16), described below, and ACT_BF16 (TVR_GEMM_BF16):
// bf16(a) in plane 0 of the same [R][2][K]-halves layout (plane 1 unused),
// round to nearest even, no range limit.
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

// Butterfly reductions over one 64-lane wave (fixed order: deterministic).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// (value desc, index asc) argmax merge: torch.argmax's first-occurrence rule
__device__ __forceinline__ void argmax_merge(float& bv, int& bi, float ov, int oi) {
  if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
}
__device__ __forceinline__ void wave_argmax(float& bv, int& bi) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    argmax_merge(bv, bi, ov, oi);
  }
}


// ACT_F16: one fp16 plane, read from plane 1 of a TVR_GEMM_BF16 LayerNorm
// output (store_ln4): the operand format of that mode's attention-score
// projections (Q, K columns of W1), see engine.hip launch_w1.
enum ActFmt { ACT_F32 = 0, ACT_X2F16 = 1, ACT_BF16 = 2, ACT_F16 = 3 };

#ifndef TVR_X2_ASCALE
#define TVR_X2_ASCALE 16.0f
#endif
constexpr float X2_ASCALE = TVR_X2_ASCALE;
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

__device__ __forceinline__ uint16_t bf16_bits(float a) { return __builtin_bit_cast(uint16_t, (__bf16)a); }

// one element in activation format FMT (ACT_X2F16 / ACT_BF16)
template <int FMT>
__device__ __forceinline__ void store_act(uint16_t* p, int plane, float a, unsigned* flag) {
  if constexpr (FMT == ACT_X2F16)
    store_split(p, plane, a, flag);
  else
    p[0] = bf16_bits(a);
}

typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));

// split_f16 of two elements with packed conversions (v_pk_mul_f32,
// v_cvt_pk_f16_f32 x2, two v_cvt_f32_f16, one v_pk_fma_f32: 6 instructions per
// pair); the same values as split_f16 element by element.  *m is raised to
// the pair's max |16 a| (the range check).
__device__ __forceinline__ void split_f16x2(float a, float b, unsigned& h0, unsigned& h1, float& m) {
  const f32x2v x = f32x2v{a, b} * X2_ASCALE;
  const f16x2v x0 = __builtin_convertvector(x, f16x2v);
  const f16x2v x1 = __builtin_convertvector(x - __builtin_convertvector(x0, f32x2v), f16x2v);
  h0 = __builtin_bit_cast(unsigned, x0);
  h1 = __builtin_bit_cast(unsigned, x1);
  m = fmaxf(m, fmaxf(fabsf(x.x), fabsf(x.y)));
}

// four consecutive elements (p 8-B aligned)
template <int FMT>
__device__ __forceinline__ void store_act4(uint16_t* p, int plane, float a, float b, float c, float d,
                                           unsigned* flag) {
  if constexpr (FMT == ACT_X2F16) {
    unsigned l0, l1, h0, h1;
    float m = 0.f;
    split_f16x2(a, b, l0, h0, m);
    split_f16x2(c, d, l1, h1, m);
    *(uint2*)p = make_uint2(l0, l1);
    *(uint2*)(p + plane) = make_uint2(h0, h1);
    if (m >= X2_FP16_OVERFLOW && flag) atomicOr(flag, 1u);
  } else {
    *(uint2*)p = make_uint2(bf16_bits(a) | ((unsigned)bf16_bits(b) << 16), bf16_bits(c) | ((unsigned)bf16_bits(d) << 16));
  }
}

// LayerNorm outputs (|a| <= sqrt(d): no range check).  TVR_GEMM_BF16 writes
// fp16(a) into the otherwise unused plane 1 as well: the Q / K projections
// read it (bf16 rounding of the score operands, amplified by the softmax at
// peaked attention, was the dominant error of bf16 extraction: 2.7e-2 of
// max |mean| with bf16 Q / K, 1.4e-2 with fp16 Q / K in a CPU emulation at
// Pythia-6.9B width, tests/test_gpu_headline_shapes.py's weights).
template <int FMT>
__device__ __forceinline__ void store_ln4(uint16_t* p, int plane, float a, float b, float c, float d) {
  store_act4<FMT>(p, plane, a, b, c, d, nullptr);
  if constexpr (FMT == ACT_BF16) {
    const f16x2v lo = __builtin_convertvector(f32x2v{a, b}, f16x2v);
    const f16x2v hi = __builtin_convertvector(f32x2v{c, d}, f16x2v);
    *(uint2*)(p + plane) = make_uint2(__builtin_bit_cast(unsigned, lo), __builtin_bit_cast(unsigned, hi));
  }
}

// eight consecutive elements (p 16-B aligned): one 16-B store per plane; the
// X2F16 range check is folded into *mx (the caller raises the flag once, after
// all its stores: no per-store divergent branch) when mx is given, else done here
template <int FMT, bool NT = false>
__device__ __forceinline__ void store_act8(uint16_t* p, int plane, const float (&v)[8], unsigned* flag,
                                           float* mx = nullptr) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  auto st = [](uint16_t* q, u32x4 x) {
    if constexpr (NT)
      __builtin_nontemporal_store(x, (u32x4*)q);
    else
      *(u32x4*)q = x;
  };
  if constexpr (FMT == ACT_X2F16) {
    unsigned lo[4], hi[4];
    float m = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) split_f16x2(v[2 * k], v[2 * k + 1], lo[k], hi[k], m);
    st(p, u32x4{lo[0], lo[1], lo[2], lo[3]});
    st(p + plane, u32x4{hi[0], hi[1], hi[2], hi[3]});
    if (mx)
      *mx = fmaxf(*mx, m);
    else if (m >= X2_FP16_OVERFLOW && flag)
      atomicOr(flag, 1u);
  } else {
    unsigned w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = bf16_bits(v[2 * k]) | ((unsigned)bf16_bits(v[2 * k + 1]) << 16);
    st(p, u32x4{w[0], w[1], w[2], w[3]});
  }
}

// fp32 rows a [rows][lda] -> activation format FMT with K logical columns
template <int FMT>
__global__ void act_rows_kernel(const float* __restrict__ a, int lda, uint16_t* __restrict__ out, int rows, int K,
                                unsigned* __restrict__ flag) {
  const size_t n = (size_t)rows * K;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / K, c = i % K;
    store_act<FMT>(out + r * 2 * K + c, K, a[r * lda + c], flag);
  }
}

// fp32 rows a [rows][lda] -> the bf16 activation format with plane 1 holding
// fp16(a) (as store_ln4: TVR_GEMM_BF16's Q / K products read it): the
// linearised entry's vectors, K logical columns
__global__ void act_rows_bf16_f16_kernel(const float* __restrict__ a, int lda, uint16_t* __restrict__ out, int rows,
                                         int K) {
  const size_t n = (size_t)rows * K;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / K, c = i % K;
    const float v = a[r * lda + c];
    out[r * 2 * K + c] = bf16_bits(v);
    out[r * 2 * K + K + c] = __builtin_bit_cast(uint16_t, (_Float16)v);
  }
}

// W [n] fp32 -> one bf16 plane (TVR_GEMM_BF16 weights, load time)
// (trunc: round toward zero — a diagnostic, the negative control of the bf16 parity bars)
__global__ void bf16_plane_kernel(const float* __restrict__ w, uint16_t* __restrict__ out, size_t n, int trunc) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = trunc ? (uint16_t)(__float_as_uint(w[i]) >> 16) : bf16_bits(w[i]);
}

// W [n] fp32 -> one fp16 plane of scale * W (scale a power of two putting
// max |W| in [2^14, 2^15]: the TVR_GEMM_BF16 Q / K weights, load time)
__global__ void f16_plane_kernel(const float* __restrict__ w, float scale, uint16_t* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = __builtin_bit_cast(uint16_t, (_Float16)(w[i] * scale));
}

}  // namespace tvr

// gemm_x2f16.hpp — fp32-accurate GEMM on fp16 matrix cores, three products.
//
//   C[M][N] = A[M][K] @ W[N][K]^T (+ the epilogues of gemm_f32.hpp)
//
// Each operand is split into two fp16 planes, x = x0 + x1, x0 = fp16(x) and
// x1 = fp16(x - x0): 2 x 11 significand bits, within 2^-22 of x.  The product
// keeps a0w0 + a0w1 + a1w0 (the dropped a1w1 is <= 2^-22 relative); each term
// is exact in fp32 and accumulates into the fp32 accumulator of
// v_mfma_f32_32x32x16_f16.  This is the fp16 analogue of "3xTF32" (fp16 and
// TF32 share the 11-bit significand); measured error against an fp64
// reference is at or below the fp32 MFMA GEMM's (tools/gemm_split_probe.hip,
// DESIGN.md section 3).  Half the MFMA work of the 3-plane bf16 split.
//
// fp16 has a 5-bit exponent, so both operands are scaled by powers of two
// (exact) into its range and the accumulator is scaled back in the epilogue:
//   * W planes are built once at load time with a per-matrix scale s_w that
//     maps max|W| to [2^14, 2^15] (x1 stays a normal number for every weight
//     within 2^-10 of the largest);
//   * A is split while it is staged into LDS, scaled by X2_ASCALE = 2^4 (the
//     residual plane of |a| >= 2^-7 stays normal).  |a| * 2^4 must stay below
//     the fp16 overflow threshold 65520, i.e. |a| < 4095: every GEMM input of
//     the Pythia forward is a LayerNorm output (|x| <= sqrt(d)), an attention
//     mix of V rows or GELU(h).  A launch that sees a larger |a| raises
//     *range_flag (the engine reports TVR_ERR_RANGE instead of a result).
//
// Layout / schedule (gfx950): BK = 32 (two k-groups of 16), 256x256 block tile
// of 8 waves (128x64 each, 4 x 2 accumulators) for large launches, 128x128 of
// 4 waves below that; LDS rows of 32 fp16 (64 B) with the 16-B chunk index
// XOR-swizzled by bits 2-3 of the row, which makes the fragment reads
// (ds_read_b128), the A writes (ds_write_b64) and the W writes
// (ds_write_b128) bank-conflict free; 2 buffers x 2 operands x 2 planes
// = 128 KB.  Global -> register prefetch one K step ahead (one register
// set: two do not fit beside 128 accumulators), one barrier per K step,
// XCD-aware bijective block remap + grouped raster.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>

#include "gemm_f32.hpp"
#include "split.hpp"

namespace tvr {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

template <int BM_, int BN_, int WM_, int WN_>
struct X2TileT {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, BK = 32;
  static constexpr int THREADS = WM * WN * 64;
  static constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static constexpr int LOADS_A = BM * BK / 4 / THREADS;  // float4 of A per thread per K step
  static constexpr int LOADS_W = BN * BK / 8 / THREADS;  // 16-B chunks of W per thread per plane
  static constexpr int PLANE = BM * BK;                  // fp16 elements per LDS plane
  static_assert(BM == BN, "one LDS plane size for A and W");
  static_assert(LOADS_A * THREADS * 4 == BM * BK && LOADS_W * THREADS * 8 == BN * BK, "staging map");
  static_assert(GEMM_BK % BK == 0, "BK must divide the host K granule");
};
using X2Large = X2TileT<256, 256, 2, 4>;  // 8 waves of 128x64, 128 KB LDS
using X2Small = X2TileT<128, 128, 2, 2>;  // 4 waves of 64x64, 64 KB LDS

// fp16 offset of (row, 16-B chunk) in a swizzled [rows][32] plane
__device__ __forceinline__ int x2_swz(int row, int chunk) { return row * 32 + ((chunk ^ ((row >> 2) & 3)) << 3); }

template <int EPI, class TL>
__global__ void __launch_bounds__(TL::THREADS, 2)
gemm_x2f16_nt_kernel(const float* __restrict__ A, int lda, const uint16_t* __restrict__ W, int ldw,
                     size_t wps, float acc_scale, unsigned* __restrict__ range_flag, int M, int N, int K,
                     GemmEpi ep) {
  constexpr int BM = TL::BM, BN = TL::BN, TM = TL::TM, TN = TL::TN, NT = TL::THREADS;
  constexpr int BK = TL::BK, PL = TL::PLANE;
  const unsigned long long st0 = ep.stamps ? __builtin_amdgcn_s_memtime() : 0;
  const unsigned long long sr0 = ep.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
  // [buf][A0 A1 W0 W1][row][32] — one __shared__ object
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * 4 * PL];
  auto sA = [&](int b, int p) { return lds + (size_t)(b * 4 + p) * PL; };
  auto sB = [&](int b, int p) { return lds + (size_t)(b * 4 + 2 + p) * PL; };

  const int nbm = (M + BM - 1) / BM, nbn = (N + BN - 1) / BN, nwg = nbm * nbn;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int per_group = GEMM_GROUP_M * nbn;
  const int grp = wg / per_group;
  const int first_m = grp * GEMM_GROUP_M;
  const int gsz = min(nbm - first_m, GEMM_GROUP_M);
  const int in_grp = wg - grp * per_group;
  const int m0 = (first_m + in_grp % gsz) * BM, n0 = (in_grp / gsz) * BN;

  const int t = threadIdx.x;
  // A staging: float4 f = t + NT*i -> row f/8, k = (f%8)*4; written as 2 x 4 fp16 (ds_write_b64)
  const float* ga[TL::LOADS_A];
  int sa[TL::LOADS_A];
#pragma unroll
  for (int i = 0; i < TL::LOADS_A; ++i) {
    const int f = t + NT * i, row = f >> 3, c4 = f & 7;
    const int am = min(m0 + row, M - 1);
    ga[i] = A + (size_t)(ep.a_rows ? ep.a_rows[am] : am) * lda + c4 * 4;
    sa[i] = x2_swz(row, c4 >> 1) + (c4 & 1) * 4;
  }
  // W staging: 16-B chunk f = t + NT*i -> row f/4, chunk f%4 (ds_write_b128)
  const uint16_t* gw[TL::LOADS_W];
  int sw[TL::LOADS_W];
#pragma unroll
  for (int i = 0; i < TL::LOADS_W; ++i) {
    const int f = t + NT * i, row = f >> 2, c = f & 3;
    gw[i] = W + (size_t)min(n0 + row, N - 1) * ldw + c * 8;
    sw[i] = x2_swz(row, c);
  }

  const int wave = t >> 6, lane = t & 63;
  const int wr = wave / TL::WN, wc = wave % TL::WN;
  const int lr = lane & 31, lh = lane >> 5;
  // fragment offsets per k-group (tile i / j adds i*32 rows: the swizzle bits are unchanged)
  int aoff[2], boff[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    aoff[g] = x2_swz(wr * (BM / TL::WM) + lr, 2 * g + lh);
    boff[g] = x2_swz(wc * (BN / TL::WN) + lr, 2 * g + lh);
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
  float amax = 0.0f;

  f32x4 ra[TL::LOADS_A];
  u32x4_t rw[2][TL::LOADS_W];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < TL::LOADS_A; ++i) ra[i] = *(const f32x4*)(ga[i] + k0);
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int i = 0; i < TL::LOADS_W; ++i) rw[p][i] = *(const u32x4_t*)(gw[i] + p * wps + k0);
  };
  auto stage = [&](int b) {
#pragma unroll
    for (int i = 0; i < TL::LOADS_A; ++i) {
      f16x4 h0, h1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = ra[i][e] * X2_ASCALE;
        amax = fmaxf(amax, fabsf(x));
        const _Float16 x0 = (_Float16)x;
        h0[e] = x0;
        h1[e] = (_Float16)(x - (float)x0);
      }
      *(f16x4*)(sA(b, 0) + sa[i]) = h0;
      *(f16x4*)(sA(b, 1) + sa[i]) = h1;
    }
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int i = 0; i < TL::LOADS_W; ++i) *(u32x4_t*)(sB(b, p) + sw[i]) = rw[p][i];
  };
  auto compute = [&](int b) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      f16x8 fb[2][TN];
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[p][j] = *(const f16x8*)(sB(b, p) + boff[g] + j * 32 * 32);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const f16x8 a0 = *(const f16x8*)(sA(b, 0) + aoff[g] + i * 32 * 32);
        const f16x8 a1 = *(const f16x8*)(sA(b, 1) + aoff[g] + i * 32 * 32);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          // small terms first into the running sum; the big a0*w0 term last
          f32x16 c = acc[i][j];
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, fb[0][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, fb[1][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, fb[0][j], c, 0, 0, 0);
          acc[i][j] = c;
        }
      }
    }
  };

  // One register set, one K step ahead: after tile kt's MFMAs the registers
  // (tile kt+1) go to the other LDS buffer, whose last readers (step kt-1)
  // passed the previous barrier; tile kt+2's loads are issued right behind.
  const int nk = K / BK;
  gload(0);
  stage(0);
  if (nk > 1) gload(BK);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int b = kt & 1;
    compute(b);
    if (kt + 1 < nk) {
      stage(b ^ 1);
      if (kt + 2 < nk) gload((kt + 2) * BK);
      __syncthreads();
    }
  }
  if (range_flag && amax >= X2_FP16_OVERFLOW) atomicOr(range_flag, 1u);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] *= acc_scale;
  gemm_epilogue<EPI, TM, TN>(ep, acc, M, N, m0 + wr * (BM / TL::WM), n0 + wc * (BN / TL::WN), lr, lh);
  if (ep.stamps && t == 0) {
    ep.stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - st0;
    ep.stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - sr0;
  }
}

// max |w| over n elements -> *out (as the uint bits of a non-negative float; *out zeroed by the caller)
__global__ void absmax_kernel(const float* __restrict__ w, size_t n, unsigned* __restrict__ out) {
  float m = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(w[i]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));
}

// W [N][K] fp32 -> 2 fp16 planes [2][N][K] of w * scale (load time)
__global__ void split_planes_f16_kernel(const float* __restrict__ w, float scale, uint16_t* __restrict__ out,
                                        size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float x = w[i] * scale;
    const _Float16 h0 = (_Float16)x;
    const _Float16 h1 = (_Float16)(x - (float)h0);
    out[i] = __builtin_bit_cast(uint16_t, h0);
    out[n + i] = __builtin_bit_cast(uint16_t, h1);
  }
}

// Power-of-two weight scale for a matrix whose largest magnitude is wmax:
// maps wmax into [2^14, 2^15] (fp16 max 65504).
inline float x2_weight_scale(float wmax) {
  if (!(wmax > 0.0f) || !std::isfinite(wmax)) return 1.0f;
  int e = 0;
  (void)std::frexp(wmax, &e);  // wmax = f * 2^e, f in [0.5, 1)
  return std::ldexp(1.0f, 15 - e);
}

// A [M][K] fp32 -> 2 fp16 planes [2][M][K] of a * X2_ASCALE (probe / tests)
__global__ void split_act_f16_kernel(const float* __restrict__ a, uint16_t* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float x = a[i] * X2_ASCALE;
    const _Float16 h0 = (_Float16)x;
    out[i] = __builtin_bit_cast(uint16_t, h0);
    out[n + i] = __builtin_bit_cast(uint16_t, (_Float16)(x - (float)h0));
  }
}

template <class TL>
inline int gemm_x2_grid(int M, int N) {
  return ((M + TL::BM - 1) / TL::BM) * ((N + TL::BN - 1) / TL::BN);
}

}  // namespace tvr

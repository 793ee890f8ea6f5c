// gemm_planar.hpp — the engine's GEMM for pre-formatted activations.
//
//   C[M][N] = A[M][K] @ W[N][K]^T (+ fused epilogue)
//
// A arrives in an activation format its producer already wrote (split.hpp):
//   ACT_X2F16  two fp16 planes of 16a (fp32-accurate split, TVR_GEMM_X2F16):
//              C = a0 w0 + a0 w1 + a1 w0 on v_mfma_f32_16x16x32_f16, W planes
//              of s_w W (gemm_x2f16.hpp has the numerics), BK = 32
//   ACT_BF16   one bf16 plane (TVR_GEMM_BF16): C = a w on
//              v_mfma_f32_16x16x32_bf16, W one bf16 plane, BK = 64
// so staging is a pure copy and both operands go global -> LDS by LDS-DMA
// (global_load_lds_dwordx4: no VGPRs, no ds_write).  Both formats use 64 B
// (x2f16) or 128 B (bf16) of K per plane row and the same LDS budget: 2
// stages x 2 operands x 256 rows x 128 B = 128 KB; per K step each of the 8
// waves issues 8 x 1 KB pieces.  The 16-B chunk of row r is stored at chunk
// c ^ g(r) (64-B rows: g = 2 * bit 3 of r; 128-B rows: g = bits 1-3 of r),
// which makes every 16x16x32 fragment read (lane l: row l & 15, chunk l >> 4
// of its 32-wide k group) bank-conflict free; the swizzle is applied on the
// per-lane SOURCE address because a DMA piece's LDS image is lane-linear.
// Tile k+1's pieces fly while tile k's MFMAs run; one barrier per K step
// (its vmcnt(0) retires them).
//
// The MFMA is issued as D = W A^T (weights as the A operand), so lane l ends
// with C[m = 16-row slice + (l & 15)][n = 16-col slice + 4 (l >> 4) + r],
// r = 0..3: four consecutive columns of one row -> 16-B fp32 / 8-B
// activation-format vector stores in the fused epilogues.
//
// Measured (tools/gemm_split_probe.hip, profiles/gemm_x2_variants_r01.json):
// ACT_X2F16 405/423 TFLOP/s of fp32 work at the qkv / o_mlpout shapes
// (M = 90,000) with error at or below the fp32 MFMA GEMM's; 16x16x32 beats
// 32x32x16 by 6-13 % (the chip holds a higher clock on it: MI355X_MICROARCH.md,
// DVFS item 7).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gemm_f32.hpp"
#include "split.hpp"

namespace tvr {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

template <int FMT>
struct PlanarFmt;
template <>
struct PlanarFmt<ACT_X2F16> {
  static constexpr int NPL = 2, BK = 32;
  using frag = f16x8;
};
template <>
struct PlanarFmt<ACT_BF16> {
  static constexpr int NPL = 1, BK = 64;
  using frag = bf16x8_t;
};
template <>
struct PlanarFmt<ACT_F16> {  // one fp16 plane (TVR_GEMM_BF16's Q / K columns), v_mfma_f32_16x16x32_f16
  static constexpr int NPL = 1, BK = 64;
  using frag = f16x8;
};

// One 16-B-per-lane LDS-DMA (global_load_lds_dwordx4): lane l's 16 bytes land
// at lds_base + 16 l.  (A non-template wrapper: referenced directly from a
// kernel template, the builtin suppresses the host-side launch stub.)
__device__ __forceinline__ void glds16(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds(g, lds_base, 16, 0, 0);
}

// chunk swizzle of a plane row with CPR 16-B chunks (4: 64-B rows, 8: 128-B rows)
template <int CPR>
__device__ __forceinline__ int planar_g(int row) {
  if constexpr (CPR == 4)
    return ((row >> 3) & 1) << 1;
  else
    return (row >> 1) & 7;
}

// 16-B store, optionally non-temporal (streamed past the caches: the GEMM
// outputs are far larger than L2 / MALL and would evict the K loop's operands)
template <bool NT>
__device__ __forceinline__ void st16(float* p, f32x4 v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, (f32x4*)p);
  else
    *(f32x4*)p = v;
}

// Four consecutive output columns of one row (VEC epilogue; N, the strides
// and n_split are multiples of 4).
template <int EPI, int FMT, bool NT = false>
__device__ __forceinline__ void epi_store4(const GemmEpi& ep, size_t orow, int n0, f32x4 v) {
  if constexpr (EPI == EPI_BIAS) {
    st16<NT>(ep.out0 + orow * ep.ld0 + n0, v);
    if (ep.out0m && orow < (size_t)ep.mirror_rows) st16<false>(ep.out0m + orow * ep.ld0 + n0, v);
  } else if constexpr (EPI == EPI_SPLIT_GELU_ACT) {
    if (n0 < ep.n_split) {  // n_split % 4 == 0: a group never straddles it
      st16<NT>(ep.out0 + orow * ep.ld0 + n0, v);
      if (ep.out0m && orow < (size_t)ep.mirror_rows) st16<false>(ep.out0m + orow * ep.ld0 + n0, v);
    } else {
      if (ep.raw && orow < (size_t)ep.raw_rows) st16<false>(ep.raw + orow * ep.ld_raw + (n0 - ep.n_split), v);
      const f32x2 g01 = gelu_erf2(f32x2{v[0], v[1]}), g23 = gelu_erf2(f32x2{v[2], v[3]});
      store_act4<FMT>(ep.out1h + orow * ep.ld1h + (n0 - ep.n_split), ep.ps1h, g01.x, g01.y, g23.x, g23.y,
                      ep.range_flag);
    }
  } else {
    static_assert(EPI == EPI_RESID, "planar epilogues: bias, split-GELU (activation format), residual");
    const f32x4 rr = *(const f32x4*)(ep.resid + orow * ep.ldr + n0);
    st16<NT>(ep.out0 + orow * ep.ld0 + n0, v + rr);
  }
}

// VEC (chosen on the host by planar_epilogue_vec): a 4-column group is either
// wholly in range or out.  Without it, element-wise stores (one path per
// instantiation: both in one body exceed the unroller's budget and the
// accumulators go to scratch).
// Every global load (the gathered output rows, the bias, the residual) is
// issued ahead of the stores it feeds: s_waitcnt vmcnt counts loads and
// stores together in issue order, so a load between two stores makes the
// second wait for the first to reach memory.  The lane's output rows and
// column biases are loaded once; the residual of row tile i + 1 is loaded
// before row tile i is stored.
template <int EPI, int FMT, bool VEC, int TM, int TN>
__device__ __forceinline__ void gemm_epilogue16t(const GemmEpi& ep, const f32x4 (&acc)[TM][TN], int M, int N,
                                                 int row_base, int col_base, int lane) {
  int orow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = min(row_base + i * 16 + (lane & 15), M - 1);
    orow[i] = ep.out_rows ? ep.out_rows[m] : m;
  }
  f32x4 b4[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n0 = col_base + j * 16 + 4 * (lane >> 4);
    b4[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (ep.bias) {
#pragma unroll
      for (int r = 0; r < 4; ++r) b4[j][r] = n0 + r < N ? ep.bias[n0 + r] : 0.f;
    }
  }
  f32x4 rr[2][TN];
  auto load_resid = [&](int i, f32x4 (&q)[TN]) {
    if constexpr (EPI == EPI_RESID && VEC) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n0 = min(col_base + j * 16 + 4 * (lane >> 4), N - 4);
        q[j] = *(const f32x4*)(ep.resid + (size_t)orow[i] * ep.ldr + n0);
      }
    }
  };
  load_resid(0, rr[0]);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    if (i + 1 < TM) load_resid(i + 1, rr[(i + 1) & 1]);
    const int m = row_base + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n0 = col_base + j * 16 + 4 * (lane >> 4);
      if (n0 >= N) continue;
      const f32x4 v = acc[i][j] + b4[j];
      if constexpr (VEC) {
        if constexpr (EPI == EPI_RESID)
          st16<false>(ep.out0 + (size_t)orow[i] * ep.ld0 + n0, v + rr[i & 1][j]);
        else
          epi_store4<EPI, FMT>(ep, orow[i], n0, v);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n0 + r < N) epi_store<EPI, FMT>(ep, orow[i], n0 + r, v[r]);
      }
    }
  }
}

inline bool planar_epilogue_vec(int EPI, const GemmEpi& ep, int N) {
  int m = N | ep.ld0;
  if (EPI == EPI_RESID) m |= ep.ldr;
  if (EPI == EPI_SPLIT_GELU_ACT) m |= ep.ld1h | ep.ps1h | ep.n_split;
  return (m & 3) == 0;
}

}  // namespace tvr

// gemm_skinny.hpp — planar GEMM for M <= 64 rows (the linearised entry
// layer's G = v W1^T: one row per distinct patch vector, 32 at C3, 40 at C5).
//
//   C[M][N] = A[M][K] @ W[N][K]^T * acc_scale + bias,   EPI_BIAS semantics
//   (A rows gathered through ep.a_rows), A and W in a planar activation format
//   (split.hpp / gemm_planar.hpp: ACT_X2F16 2 fp16 planes, ACT_BF16 1 plane).
//
// Why not gemm_pingpong_kernel: its 256-row tile computes 256 rows for 32 (8x
// the MFMA work) and 70 column tiles need a split-K partial round trip; such a
// launch is a weight stream (N K 4 B: 183 MB per 2.8B layer), so this kernel
// reads every weight element once, straight into registers, and spends its
// MFMAs on 16-row tiles of the real rows only.  It streams W at ~2.5 TB/s
// (16 rows x 64 B per load instruction), so it wins only where the 256-row
// tile wastes the most: see SK_USE_M.  A variant reading 64 B per lane and
// plane per 4 k-steps without the register double buffer ran slower still
// (profiles/r02o/skinny_ab.txt).
// Block = 4 waves over 32 output columns; wave w takes k-steps [w S / 4,
// (w + 1) S / 4) of the S = K / 32 and all M rows: per k-step 2 W fragments
// and MT A fragments (16 B per lane per plane, global -> VGPR, the next
// k-step's issued before this one's MFMAs), D = W A^T on
// v_mfma_f32_16x16x32 (x2f16: the pingpong kernel's three products in its
// order, small terms first).  The four k-partials are summed in wave order
// through LDS (deterministic), then wave 0 adds the bias and stores 16 B per
// lane (4 consecutive columns of one row).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gemm_planar.hpp"

namespace tvr {

constexpr int SK_THREADS = 256;  // 4 waves
constexpr int SK_NT = 2;         // 16-column tiles per block (every wave computes all of them)
constexpr int SK_COLS = 16 * SK_NT;
constexpr int SK_MAX_M = 64;
// The engine's policy (launch_gemm, ep.skinny launches): this kernel at most
// 16 rows, the split-K pingpong launch above.  C3 rocprof (tag r02p): 72 us
// at 32 rows against 59 us for the pingpong G; rank 0 of an 8-way head split
// (4 rows): ~55 us against ~75 us.
constexpr int SK_USE_M = 16;

inline int gemm_skinny_grid(int N) { return (N + SK_COLS - 1) / SK_COLS; }

template <int FMT, int MT>
__global__ void __launch_bounds__(SK_THREADS)
gemm_skinny_kernel(const uint16_t* __restrict__ A, int lda, size_t aps, const uint16_t* __restrict__ W, int ldw,
                   size_t wps, float acc_scale, int M, int N, int K, GemmEpi ep) {
  using F = PlanarFmt<FMT>;
  using frag = typename F::frag;
  constexpr int NPL = F::NPL;
  __shared__ f32x4 red[3][SK_NT][MT][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n0 = blockIdx.x * SK_COLS;
  const int steps = K / 32;
  const int kb = wave * steps / 4, ke = (wave + 1) * steps / 4;
  const int r16 = lane & 15, kq = (lane >> 4) * 8;  // fragment row / first k of this lane

  const uint16_t* wp[SK_NT];
  const uint16_t* ap[MT];
#pragma unroll
  for (int j = 0; j < SK_NT; ++j) wp[j] = W + (size_t)min(n0 + 16 * j + r16, N - 1) * ldw + kq;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = min(16 * i + r16, M - 1);
    ap[i] = A + (size_t)(ep.a_rows ? ep.a_rows[m] : m) * lda + kq;
  }
  f32x4 acc[SK_NT][MT];
#pragma unroll
  for (int j = 0; j < SK_NT; ++j)
#pragma unroll
    for (int i = 0; i < MT; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  frag w[2][SK_NT][NPL], a[2][MT][NPL];
  auto load = [&](int buf, int ks) {
    const int ko = ks * 32;
#pragma unroll
    for (int j = 0; j < SK_NT; ++j)
#pragma unroll
      for (int p = 0; p < NPL; ++p) w[buf][j][p] = *(const frag*)(wp[j] + p * wps + ko);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int p = 0; p < NPL; ++p) a[buf][i][p] = *(const frag*)(ap[i] + p * aps + ko);
  };
  auto mfma = [&](int buf) {
#pragma unroll
    for (int j = 0; j < SK_NT; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        f32x4 c = acc[j][i];
        if constexpr (FMT == ACT_X2F16) {
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(w[buf][j][0], a[buf][i][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(w[buf][j][1], a[buf][i][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(w[buf][j][0], a[buf][i][0], c, 0, 0, 0);
        } else {
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[buf][j][0], a[buf][i][0], c, 0, 0, 0);
        }
        acc[j][i] = c;
      }
  };
  // two register buffers, the loop unrolled by two so each buffer index is a constant
  if (kb < ke) load(0, kb);
  int ks = kb;
  for (; ks + 1 < ke; ks += 2) {
    load(1, ks + 1);
    mfma(0);
    if (ks + 2 < ke) load(0, ks + 2);
    mfma(1);
  }
  if (ks < ke) mfma(0);

  if (wave > 0) {
#pragma unroll
    for (int j = 0; j < SK_NT; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i) red[wave - 1][j][i][lane] = acc[j][i];
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int j = 0; j < SK_NT; ++j) {
    const int n = n0 + 16 * j + 4 * (lane >> 4);  // D[n][m]: 4 consecutive columns n.. of row m
    if (n >= N) continue;
    f32x4 b4 = {0.f, 0.f, 0.f, 0.f};
    if (ep.bias) b4 = f32x4{ep.bias[n], ep.bias[n + 1], ep.bias[n + 2], ep.bias[n + 3]};
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int m = 16 * i + r16;
      if (m >= M) continue;
      const f32x4 s = ((acc[j][i] + red[0][j][i][lane]) + red[1][j][i][lane]) + red[2][j][i][lane];
      *(f32x4*)(ep.out0 + (size_t)m * ep.ld0 + n) = s * acc_scale + b4;
    }
  }
}

}  // namespace tvr

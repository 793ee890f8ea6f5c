// gemm_f32.hpp — fp32 GEMM on CDNA4 matrix cores (v_mfma_f32_32x32x2_f32).
//
//   C[M][N] = A[M][K] @ W[N][K]^T  (+ fused epilogue)
//
// Every projection of the patched Pythia forward goes through this kernel:
// the fused QKV+MLP-in projection (epilogue: bias, exact-erf GELU on the MLP
// columns, split into two destinations), the fused O+MLP-out projection
// (epilogue: bias + parallel residual add) and the last-row unembed.
// The reference runs the same contractions as batch-1 fp32 einsums inside
// TransformerLens (scratch2.py:96,123,191 → TL attention/MLP).
//
// Design (gfx950):
//   * 128x128 block tile, BK = 32, 256 threads = 4 waves in a 2x2 grid, each
//     wave owns a 64x64 sub-tile = 2x2 accumulators of 32x32 (64 AGPRs).
//   * f32-in MFMA is exact fp32 (bit-for-bit a k-ordered fmaf chain), 64
//     FLOP/clk/SIMD, so this is the only matrix path that keeps the
//     reference's fp32 numerics.
//   * Both operands are K-contiguous ([row][k]); LDS rows are padded to
//     BK+4 floats so the fragment reads (ds_read_b128, 16 distinct rows per
//     lane group) are bank-conflict free.  Lane half h supplies k = 4h..4h+3
//     of every 8-wide k group, so one ds_read_b128 feeds four MFMAs.
//   * Register-staged double buffer: the next tile's global loads are issued
//     before the current tile's MFMAs and written to the other LDS buffer
//     after them; one barrier per K step.
//   * XCD-aware bijective block remap + grouped raster so neighbouring tiles
//     (which share A and W panels) run on the same XCD's L2.
//   * K must be a multiple of 32 (every Pythia K is); M and N are arbitrary:
//     out-of-range rows/cols load clamped addresses and are never stored.
#pragma once
#include <hip/hip_runtime.h>

namespace tvr {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

enum GemmEpiKind {
  EPI_BIAS = 0,        // out0 = acc + bias
  EPI_SPLIT_GELU = 1,  // col < n_split: out0 = acc + bias ; else out1 = gelu(acc + bias)
  EPI_RESID = 2,       // out0 = acc + bias + resid   (in place allowed: out0 == resid)
};

struct GemmEpi {
  const float* bias;  // [N] or nullptr
  float* out0;
  int ld0;
  float* out1;
  int ld1;
  int n_split;
  const float* resid;
  int ldr;
  // Diagnostics only (tools/gemm_probe.hip; the engine passes nullptr): per
  // block {Δs_memtime, Δs_memrealtime} to read the shader clock under load.
  unsigned long long* stamps;
};

__device__ __forceinline__ float gelu_erf(float x) {
  // torch.nn.functional.gelu (approximate='none'), TransformerLens act_fn "gelu"
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}

constexpr int GEMM_BM = 128;
constexpr int GEMM_BN = 128;
constexpr int GEMM_BK = 32;
constexpr int GEMM_LDK = GEMM_BK + 4;  // padded LDS row (floats)
constexpr int GEMM_GROUP_M = 8;
constexpr int GEMM_THREADS = 256;

template <int EPI>
__global__ void __launch_bounds__(GEMM_THREADS, 2)
gemm_f32_nt_kernel(const float* __restrict__ A, int lda,
                   const float* __restrict__ W, int ldw, int M, int N, int K,
                   GemmEpi ep) {
  const unsigned long long st0 = ep.stamps ? __builtin_amdgcn_s_memtime() : 0;
  const unsigned long long sr0 = ep.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
  __shared__ __attribute__((aligned(16))) float sA[2][GEMM_BM * GEMM_LDK];
  __shared__ __attribute__((aligned(16))) float sB[2][GEMM_BN * GEMM_LDK];

  const int nbm = (M + GEMM_BM - 1) / GEMM_BM;
  const int nbn = (N + GEMM_BN - 1) / GEMM_BN;
  const int nwg = nbm * nbn;
  const int bid = blockIdx.x;
  // Blocks b and b+8 share an XCD (round-robin dispatch): give each of the 8
  // classes a contiguous range of tiles.  Bijective for any nwg.
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int per_group = GEMM_GROUP_M * nbn;
  const int grp = wg / per_group;
  const int first_m = grp * GEMM_GROUP_M;
  const int gsz = min(nbm - first_m, GEMM_GROUP_M);
  const int in_grp = wg - grp * per_group;
  const int tm = first_m + in_grp % gsz;
  const int tn = in_grp / gsz;
  const int m0 = tm * GEMM_BM, n0 = tn * GEMM_BN;

  const int t = threadIdx.x;
  // staging map: 4 float4 of A and 4 of W per thread per K step
  const float* ga[4];
  const float* gw[4];
  int soff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int f = t + GEMM_THREADS * i;
    const int row = f >> 3, c = (f & 7) * 4;
    const int am = min(m0 + row, M - 1);
    const int wn = min(n0 + row, N - 1);
    ga[i] = A + (size_t)am * lda + c;
    gw[i] = W + (size_t)wn * ldw + c;
    soff[i] = row * GEMM_LDK + c;
  }

  const int wave = t >> 6, lane = t & 63;
  const int wr = wave >> 1, wc = wave & 1;
  const int lr = lane & 31, lh = lane >> 5;
  const int aoff = (wr * 64 + lr) * GEMM_LDK + lh * 4;
  const int boff = (wc * 64 + lr) * GEMM_LDK + lh * 4;

  f32x16 acc00 = {}, acc01 = {}, acc10 = {}, acc11 = {};
  f32x4 ra[4], rb[4];

#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ra[i] = *(const f32x4*)(ga[i]);
    rb[i] = *(const f32x4*)(gw[i]);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    *(f32x4*)(&sA[0][soff[i]]) = ra[i];
    *(f32x4*)(&sB[0][soff[i]]) = rb[i];
  }
  __syncthreads();

  const int nk = K / GEMM_BK;
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = (kt + 1) < nk;
    if (more) {
      const int k1 = (kt + 1) * GEMM_BK;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ra[i] = *(const f32x4*)(ga[i] + k1);
        rb[i] = *(const f32x4*)(gw[i] + k1);
      }
    }
    const float* pa = &sA[buf][aoff];
    const float* pb = &sB[buf][boff];
#pragma unroll
    for (int kk = 0; kk < GEMM_BK / 8; ++kk) {
      const f32x4 a0 = *(const f32x4*)(pa + kk * 8);
      const f32x4 a1 = *(const f32x4*)(pa + 32 * GEMM_LDK + kk * 8);
      const f32x4 b0 = *(const f32x4*)(pb + kk * 8);
      const f32x4 b1 = *(const f32x4*)(pb + 32 * GEMM_LDK + kk * 8);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b0[s], acc00, 0, 0, 0);
        acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b1[s], acc01, 0, 0, 0);
        acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b0[s], acc10, 0, 0, 0);
        acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b1[s], acc11, 0, 0, 0);
      }
    }
    if (more) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        *(f32x4*)(&sA[buf ^ 1][soff[i]]) = ra[i];
        *(f32x4*)(&sB[buf ^ 1][soff[i]]) = rb[i];
      }
    }
    __syncthreads();
    buf ^= 1;
  }

  // Epilogue.  32x32 C/D map: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
  auto store = [&](const f32x16& acc, int mi, int ni) {
    const int col = n0 + wc * 64 + ni * 32 + lr;
    if (col >= N) return;
    const float b = ep.bias ? ep.bias[col] : 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + wr * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (row >= M) continue;
      const float v = acc[r] + b;
      if constexpr (EPI == EPI_BIAS) {
        ep.out0[(size_t)row * ep.ld0 + col] = v;
      } else if constexpr (EPI == EPI_SPLIT_GELU) {
        if (col < ep.n_split)
          ep.out0[(size_t)row * ep.ld0 + col] = v;
        else
          ep.out1[(size_t)row * ep.ld1 + (col - ep.n_split)] = gelu_erf(v);
      } else {
        ep.out0[(size_t)row * ep.ld0 + col] = v + ep.resid[(size_t)row * ep.ldr + col];
      }
    }
  };
  store(acc00, 0, 0);
  store(acc01, 0, 1);
  store(acc10, 1, 0);
  store(acc11, 1, 1);
  if (ep.stamps && t == 0) {
    ep.stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - st0;
    ep.stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - sr0;
  }
}

inline int gemm_grid(int M, int N) {
  return ((M + GEMM_BM - 1) / GEMM_BM) * ((N + GEMM_BN - 1) / GEMM_BN);
}

}  // namespace tvr

// gemm_x3bf16.hpp — fp32-accurate GEMM on bf16 matrix cores.
//
//   C[M][N] = A[M][K] @ W[N][K]^T (+ the epilogues of gemm_f32.hpp)
//
// Both operands are split into three bf16 planes, x = x0 + x1 + x2 with each
// plane the round-to-nearest bf16 of what the previous ones leave (three 8-bit
// significands cover fp32's 24).  The product keeps the six terms with
// i + j <= 2 (a0w0, a0w1, a1w0, a0w2, a1w1, a2w0); the three dropped ones are
// <= 2^-23 relative per product, below the fp32 rounding of the K-long sum
// itself.  Every term is exact in fp32 (8 x 8-bit significands) and
// accumulates into the same fp32 accumulator of v_mfma_f32_32x32x16_bf16.
// bf16 MFMA runs at 16x the fp32 MFMA rate, so the six terms take 3/8 of the
// fp32 kernel's MFMA time.
//
//   * W is pre-split once at load time: 3 planes [N][K] bf16, plane stride
//     `wps` elements.  A (activations) stays fp32 in HBM and is split while it
//     is staged into LDS (each element once per block).
//   * BK = 16 (one MFMA k-group per plane).  256x256 block tile, 8 waves of
//     128x64 (4 x 2 accumulators); LDS: 2 buffers x 2 operands x 3 planes x 256
//     rows x 48 B (16 bf16 + 8 pad: conflict-free ds_read_b128) = 144 KB.
//     A 128x128 / 4-wave variant covers small M (same 512-tile rule as f32).
//   * Measured (profiles/gemm_x3_probe_r01.jsonl, M=90000): 211 TF/s of
//     algorithmic fp32 work = 1.55x the fp32 MFMA GEMM, max error 2.8e-7 vs
//     3.4e-7 of sum|a*w| (fp64 truth).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gemm_f32.hpp"

namespace tvr {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));  // 8 bf16 in flight (native vector: stays in VGPRs)

__device__ __forceinline__ void split3(float x, __bf16& h0, __bf16& h1, __bf16& h2) {
  h0 = (__bf16)x;
  const float r1 = x - (float)h0;
  h1 = (__bf16)r1;
  h2 = (__bf16)(r1 - (float)h1);
}

template <int BM_, int BN_, int WM_, int WN_>
struct X3TileT {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, BK = 16;
  static constexpr int LDK = BK + 8;  // bf16 elements per LDS row (48 B)
  static constexpr int THREADS = WM * WN * 64;
  static constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static constexpr int LOADS_A = BM * BK / 4 / THREADS;  // float4 of A per thread
  static constexpr int PLANE = BM * LDK;                 // bf16 elements per LDS plane
  static_assert(BM == BN, "one LDS plane size for A and W");
  static_assert(BN * BK / 8 == THREADS, "one 16-B W chunk per thread per plane");
  static_assert(LOADS_A * THREADS * 4 == BM * BK, "A tile covered by float4 loads");
};
using X3Large = X3TileT<256, 256, 2, 4>;  // 8 waves of 128x64, 144 KB LDS
using X3Small = X3TileT<128, 128, 2, 2>;  // 4 waves of 64x64, 72 KB LDS (small M)

template <int EPI, class TL>
__global__ void __launch_bounds__(TL::THREADS, 2)
gemm_x3bf16_nt_kernel(const float* __restrict__ A, int lda, const uint16_t* __restrict__ W, int ldw,
                      size_t wps, int M, int N, int K, GemmEpi ep) {
  constexpr int BM = TL::BM, BN = TL::BN, TM = TL::TM, TN = TL::TN, NT = TL::THREADS;
  constexpr int BK = TL::BK, LDK = TL::LDK, PL = TL::PLANE;
  const unsigned long long st0 = ep.stamps ? __builtin_amdgcn_s_memtime() : 0;
  const unsigned long long sr0 = ep.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
  // [buf][plane][row][LDK] for A then B, one array (hipcc LDS trap: keep one __shared__ object)
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * 3 * (BM + BN) * LDK];
  auto sA = [&](int b, int p) { return lds + (size_t)(b * 6 + p) * PL; };
  auto sB = [&](int b, int p) { return lds + (size_t)(b * 6 + 3 + p) * PL; };

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
  const float* ga[TL::LOADS_A];
  int sa[TL::LOADS_A];
#pragma unroll
  for (int i = 0; i < TL::LOADS_A; ++i) {
    const int f = t + NT * i, row = f / (BK / 4), c = (f % (BK / 4)) * 4;
    const int am = min(m0 + row, M - 1);
    ga[i] = A + (size_t)(ep.a_rows ? ep.a_rows[am] : am) * lda + c;
    sa[i] = row * LDK + c;
  }
  const int wrow = t >> 1, wcol = (t & 1) * 8;
  const uint16_t* gw = W + (size_t)min(n0 + wrow, N - 1) * ldw + wcol;
  const int sbo = wrow * LDK + wcol;

  const int wave = t >> 6, lane = t & 63;
  const int wr = wave / TL::WN, wc = wave % TL::WN;
  const int lr = lane & 31, lh = lane >> 5;
  const int aoff = (wr * (BM / TL::WM) + lr) * LDK + lh * 8;
  const int boff = (wc * (BN / TL::WN) + lr) * LDK + lh * 8;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
  // Global -> register prefetch runs TWO K steps ahead (a K step is only
  // ~1.5k MFMA cycles per wave, shorter than an HBM round trip under load):
  // register set s holds the tile of every step with kt % 2 == s; the loop is
  // unrolled by 2 so the sets are indexed statically (nk = K/16 is even).
  f32x4 ra0[TL::LOADS_A], ra1[TL::LOADS_A];
  u32x4 rw0[3], rw1[3];

  auto gload = [&](int k0, f32x4 (&ra)[TL::LOADS_A], u32x4 (&rw)[3]) {
#pragma unroll
    for (int i = 0; i < TL::LOADS_A; ++i) ra[i] = *(const f32x4*)(ga[i] + k0);
#pragma unroll
    for (int p = 0; p < 3; ++p) rw[p] = *(const u32x4*)(gw + p * wps + k0);
  };
  auto stage = [&](int b, const f32x4 (&ra)[TL::LOADS_A], const u32x4 (&rw)[3]) {
#pragma unroll
    for (int i = 0; i < TL::LOADS_A; ++i) {
      bf16x4 h0, h1, h2;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        __bf16 x0, x1, x2;
        split3(ra[i][e], x0, x1, x2);
        h0[e] = x0; h1[e] = x1; h2[e] = x2;
      }
      *(bf16x4*)(sA(b, 0) + sa[i]) = h0;
      *(bf16x4*)(sA(b, 1) + sa[i]) = h1;
      *(bf16x4*)(sA(b, 2) + sa[i]) = h2;
    }
#pragma unroll
    for (int p = 0; p < 3; ++p) *(u32x4*)(sB(b, p) + sbo) = rw[p];
  };
  auto compute = [&](int b) {
    bf16x8 fb[3][TN];
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[p][j] = *(const bf16x8*)(sB(b, p) + boff + j * 32 * LDK);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const bf16x8 a0 = *(const bf16x8*)(sA(b, 0) + aoff + i * 32 * LDK);
      const bf16x8 a1 = *(const bf16x8*)(sA(b, 1) + aoff + i * 32 * LDK);
      const bf16x8 a2 = *(const bf16x8*)(sA(b, 2) + aoff + i * 32 * LDK);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        // small terms first into the running sum; the big a0*w0 term last
        f32x16 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, fb[0][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, fb[1][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, fb[2][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, fb[0][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, fb[1][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, fb[0][j], c, 0, 0, 0);
        acc[i][j] = c;
      }
    }
  };

  const int nk = K / BK;  // even: the host requires K % 32 == 0
  gload(0, ra0, rw0);
  if (nk > 1) gload(BK, ra1, rw1);
  stage(0, ra0, rw0);
  __syncthreads();
  for (int kt = 0; kt < nk; kt += 2) {
    // even step kt: buffer 0 holds tile kt; set 1 holds tile kt+1 (in flight)
    if (kt + 2 < nk) gload((kt + 2) * BK, ra0, rw0);
    compute(0);
    stage(1, ra1, rw1);  // tile kt+1 (nk even: always exists)
    __syncthreads();
    // odd step kt+1: buffer 1 holds tile kt+1; set 0 holds tile kt+2
    if (kt + 3 < nk) gload((kt + 3) * BK, ra1, rw1);
    compute(1);
    if (kt + 2 < nk) stage(0, ra0, rw0);
    __syncthreads();
  }
  gemm_epilogue<EPI, TM, TN>(ep, acc, M, N, m0 + wr * (BM / TL::WM), n0 + wc * (BN / TL::WN), lr, lh);
  if (ep.stamps && t == 0) {
    ep.stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - st0;
    ep.stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - sr0;
  }
}

// W [N][K] fp32 -> 3 bf16 planes [3][N][K] (load time)
__global__ void split_planes_kernel(const float* __restrict__ w, uint16_t* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    __bf16 h0, h1, h2;
    split3(w[i], h0, h1, h2);
    out[i] = __builtin_bit_cast(uint16_t, h0);
    out[n + i] = __builtin_bit_cast(uint16_t, h1);
    out[2 * n + i] = __builtin_bit_cast(uint16_t, h2);
  }
}

template <class TL>
inline int gemm_x3_grid(int M, int N) {
  return ((M + TL::BM - 1) / TL::BM) * ((N + TL::BN - 1) / TL::BN);
}

}  // namespace tvr

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

template <int BM_, int BN_, int WM_, int WN_>
struct PlanarTile {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
  static constexpr int THREADS = WM * WN * 64;
  static constexpr int TM = BM / WM / 16, TN = BN / WN / 16;  // 16x16 accumulators per wave
  static_assert(BM == BN, "one LDS plane size for A and W");
};
using PlanarLarge = PlanarTile<256, 256, 2, 4>;  // 8 waves of 128x64, 1 block per CU (128 KB LDS)
using PlanarSmall = PlanarTile<128, 128, 2, 2>;  // 4 waves of 64x64 (launches below 512 large tiles)

template <class TL>
inline int gemm_planar_grid(int M, int N) {
  return ((M + TL::BM - 1) / TL::BM) * ((N + TL::BN - 1) / TL::BN);
}

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
  } else if constexpr (EPI == EPI_SPLIT_GELU_ACT) {
    if (n0 < ep.n_split) {  // n_split % 4 == 0: a group never straddles it
      st16<NT>(ep.out0 + orow * ep.ld0 + n0, v);
    } else {
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
template <int EPI, int FMT, bool VEC, int TM, int TN>
__device__ __forceinline__ void gemm_epilogue16t(const GemmEpi& ep, const f32x4 (&acc)[TM][TN], int M, int N,
                                                 int row_base, int col_base, int lane) {
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n0 = col_base + j * 16 + 4 * (lane >> 4);
    if (n0 >= N) continue;
    f32x4 b4 = {0.f, 0.f, 0.f, 0.f};
    if (ep.bias) {
#pragma unroll
      for (int r = 0; r < 4; ++r) b4[r] = n0 + r < N ? ep.bias[n0 + r] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = row_base + i * 16 + (lane & 15);
      if (m >= M) continue;
      const size_t orow = ep.out_rows ? (size_t)ep.out_rows[m] : (size_t)m;
      const f32x4 v = acc[i][j] + b4;
      if constexpr (VEC) {
        epi_store4<EPI, FMT>(ep, orow, n0, v);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n0 + r < N) epi_store<EPI, FMT>(ep, orow, n0 + r, v[r]);
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

// A: activation format FMT, plane p of row m at A + p * aps + m * lda (halves)
// W: planes of the same format, plane p of row n at W + p * wps + n * ldw
// acc_scale: 1 / (s_w * 16) for ACT_X2F16, 1 for ACT_BF16
// PIPE 2 is a diagnostic build (tools/gemm_split_probe x2pt): per-wave cycles
// in the K loop, the vmcnt(0) drain and the barrier, to ep.stamps.
template <int EPI, class TL, int FMT, bool VEC = true, int PIPE = 0>
__global__ void __launch_bounds__(TL::THREADS, 2)
gemm_planar_kernel(const uint16_t* __restrict__ A, int lda, size_t aps, const uint16_t* __restrict__ W, int ldw,
                   size_t wps, float acc_scale, int M, int N, int K, GemmEpi ep) {
  using F = PlanarFmt<FMT>;
  using frag = typename F::frag;
  constexpr int BM = TL::BM, BN = TL::BN, NT = TL::THREADS, TM = TL::TM, TN = TL::TN;
  constexpr int NPL = F::NPL, BK = F::BK, KG = BK / 32;  // planes, K per step, 32-wide k groups per step
  constexpr int CPR = BK / 8;                             // 16-B chunks per plane row
  constexpr int RPP = 64 / CPR;                           // rows per 1 KB piece
  constexpr int PL = BM * BK;                             // halves per plane per stage
  constexpr int SLOTS = 2 * NPL;                          // (operand, plane) pairs
  constexpr int PPS = BM / RPP;                           // pieces per slot
  constexpr int PER_WAVE = SLOTS * PPS / (NT / 64);
  static_assert(PER_WAVE * (NT / 64) == SLOTS * PPS && PPS % PER_WAVE == 0, "piece map");
  static_assert(2 * SLOTS * PL * 2 <= 160 * 1024, "LDS budget");
  const unsigned long long st0 = ep.stamps ? __builtin_amdgcn_s_memtime() : 0;
  const unsigned long long sr0 = ep.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
  // [stage][A planes | W planes][row][BK] — one __shared__ object
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * SLOTS * PL];
  auto sA = [&](int b, int p) { return lds + (size_t)(b * SLOTS + p) * PL; };
  auto sB = [&](int b, int p) { return lds + (size_t)(b * SLOTS + NPL + p) * PL; };

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
  const int wave = t >> 6, lane = t & 63;
  // this wave's pieces: slot (operand*NPL + plane), rows [prow0, prow0 + RPP*PER_WAVE)
  const int first = wave * PER_WAVE;
  const int slot = first / PPS;
  const int prow0 = (first % PPS) * RPP;
  const bool is_w = slot >= NPL;
  const int plane = is_w ? slot - NPL : slot;
  const int lrow = lane / CPR, lch = lane % CPR;
  const uint16_t* src[PER_WAVE];
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int row = prow0 + RPP * i + lrow;
    const int chunk = lch ^ planar_g<CPR>(row);
    if (is_w) {
      src[i] = W + plane * wps + (size_t)min(n0 + row, N - 1) * ldw + chunk * 8;
    } else {
      const int am = min(m0 + row, M - 1);
      src[i] = A + plane * aps + (size_t)(ep.a_rows ? ep.a_rows[am] : am) * lda + chunk * 8;
    }
  }
  const int dst0 = slot * PL + prow0 * BK;
  auto issue = [&](int k0, int b) {
    uint16_t* d = lds + (size_t)b * SLOTS * PL + dst0;
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) glds16(src[i] + k0, d + i * RPP * BK);
  };

  const int wr = wave / TL::WN, wc = wave % TL::WN;
  // fragment offsets per k group (16-row slices add multiples of 16 rows: g unchanged)
  int aoff[KG], boff[KG];
#pragma unroll
  for (int g = 0; g < KG; ++g) {
    const int ra = wr * (BM / TL::WM) + (lane & 15), rb = wc * (BN / TL::WN) + (lane & 15);
    const int c = 4 * g + (lane >> 4);
    aoff[g] = ra * BK + ((c ^ planar_g<CPR>(ra)) << 3);
    boff[g] = rb * BK + ((c ^ planar_g<CPR>(rb)) << 3);
  }
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{};

  auto step = [&](int b) {
#pragma unroll
    for (int g = 0; g < KG; ++g) {
      frag fb[NPL][TN];
#pragma unroll
      for (int p = 0; p < NPL; ++p)
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[p][j] = *(const frag*)(sB(b, p) + boff[g] + j * 16 * BK);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        frag fa[NPL];
#pragma unroll
        for (int p = 0; p < NPL; ++p) fa[p] = *(const frag*)(sA(b, p) + aoff[g] + i * 16 * BK);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          // W fragment as the A operand, activations as B: D = W A^T (gemm_epilogue16t)
          f32x4 c = acc[i][j];
          if constexpr (FMT == ACT_X2F16) {  // small terms first; the big a0*w0 last
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[0][j], fa[1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[1][j], fa[0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[0][j], fa[0], c, 0, 0, 0);
          } else {
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[0][j], fa[0], c, 0, 0, 0);
          }
          acc[i][j] = c;
        }
      }
    }
  };

  const int nk = K / BK;
  issue(0, 0);
  __syncthreads();
  unsigned long long c_vm = 0, c_bar = 0, tl = 0;
  if constexpr (PIPE == 2) tl = __builtin_amdgcn_s_memtime();
  for (int kt = 0; kt < nk; ++kt) {
    const int b = kt & 1;
    if (kt + 1 < nk) issue((kt + 1) * BK, b ^ 1);
    step(b);
    if constexpr (PIPE == 2) {
      const unsigned long long t0 = __builtin_amdgcn_s_memtime();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned long long t1 = __builtin_amdgcn_s_memtime();
      __syncthreads();
      const unsigned long long t2 = __builtin_amdgcn_s_memtime();
      c_vm += t1 - t0;
      c_bar += t2 - t1;
    } else {
      __syncthreads();
    }
  }
  if constexpr (PIPE == 2) {
    const unsigned long long c_loop = __builtin_amdgcn_s_memtime() - tl;
    if (lane == 0 && (wave == 0 || wave == NT / 64 - 1)) {
      unsigned long long* o = ep.stamps + 6 * blockIdx.x + (wave ? 3 : 0);
      o[0] = c_loop;
      o[1] = c_vm;
      o[2] = c_bar;
    }
  }
  if (acc_scale != 1.0f) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] *= acc_scale;
  }
  gemm_epilogue16t<EPI, FMT, VEC, TM, TN>(ep, acc, M, N, m0 + wr * (BM / TL::WM), n0 + wc * (BN / TL::WN), lane);
  if (PIPE != 2 && ep.stamps && t == 0) {
    ep.stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - st0;
    ep.stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - sr0;
  }
}

}  // namespace tvr

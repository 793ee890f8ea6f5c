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
//   * Two block tiles (BK = 32, each wave owns TM x TN accumulators of 32x32):
//       large 256x256, 512 threads = 8 waves (2 x 4), wave tile 128x64, 1 block/CU
//       small 128x128, 256 threads = 4 waves (2 x 2), wave tile 64x64, 2 blocks/CU
//     The large tile halves the bytes streamed per FLOP: with most panel reads
//     missing L2 (blocks drift apart in k), the 128x128 tile's ~8 B/clk/CU of
//     beyond-L2 demand capped it at ~78% of the (measured, DVFS-free) fp32
//     MFMA peak; the small tile serves launches too small to fill 256 CUs.
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
#include <stdint.h>

#include "split.hpp"

namespace tvr {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

enum GemmEpiKind {
  EPI_BIAS = 0,        // out0 = acc + bias
  EPI_SPLIT_GELU = 1,  // col < n_split: out0 = acc + bias ; else out1 = gelu(acc + bias)
  EPI_RESID = 2,       // out0 = acc + bias + resid   (in place allowed: out0 == resid)
  EPI_SPLIT_GELU_ACT = 3,  // EPI_SPLIT_GELU with the GELU columns in the planar activation format (split.hpp)
  // Fused unembed statistics (gemm_pingpong_kernel only): no logits written.
  // Per (row, 256-column tile) of acc + bias: the max, sum(exp(x - max)) and
  // the top stats_k (value, column) candidates to stats, and the target
  // column's logit to tlogit; stats_merge_kernel combines the tiles.
  EPI_STATS = 4,
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
  // Optional row indirection (the trimmed last layer): A row m is read from
  // a_rows[m], output row m (and its residual) lives at out_rows[m].
  const int32_t* a_rows;
  const int32_t* out_rows;
  // EPI_SPLIT_GELU_ACT: GELU column c of row r goes to out1h + r*ld1h + c
  // (plane 0) and + ps1h (plane 1), both in halves; range_flag as split.hpp.
  uint16_t* out1h;
  int ld1h;
  int ps1h;
  unsigned* range_flag;
  // Diagnostics only (tools/gemm_probe.hip; the engine passes nullptr): per
  // block {Δs_memtime, Δs_memrealtime} to read the shader clock under load.
  unsigned long long* stamps;
  // gemm_pingpong_kernel launch shape (engine: small launches, last rounds):
  // tiles [tile_base, tile_base + tile_count) of the grouped raster (count 0:
  // all); k_split > 1 runs count x k_split blocks, each writing its fp32
  // partial tile to out0 + (split * count + tile) * 256 * 256 (EPI_BIAS, bias
  // nullptr), which splitk_reduce_kernel sums in order under the real epilogue.
  int k_split;
  int tile_base;
  int tile_count;
  int group_m;  // gemm_pingpong_kernel raster: m-blocks per group (0: GEMM_GROUP_M)
  // Stream-K (gemm_pingpong_kernel, sk_blocks > 0; EPI_BIAS, bias nullptr):
  // sk_blocks blocks share the tile_count x (K / BK) k-iterations of tiles
  // [tile_base, tile_base + tile_count) evenly, block g taking iterations
  // [g I / G, (g + 1) I / G) (at most two tile segments: sk_blocks >=
  // tile_count); segment j of block g stores its fp32 partial tile at
  // out0 + (2 g + j) * 256 * 256, which splitk_sk_reduce_kernel sums per tile
  // in k order under the real epilogue.
  int sk_blocks;
  // EPI_STATS: record of (row m, column tile t) at stats + (m * stats_tiles + t) * (2 + 2 stats_k):
  // {max, sum exp, value[stats_k], column[stats_k] (int bits)}; targets[m] (may be null) selects
  // the logit written to tlogit[m].
  float* stats;
  int stats_k;
  int stats_tiles;
  const int32_t* targets;
  float* tlogit;
  // EPI_SPLIT_GELU_ACT: rows m < raw_rows also store their GELU columns'
  // pre-activation (fp32, bias added) at raw + m * ld_raw + (c - n_split) — the
  // clean rows' y_c that lin_entry.hpp reads in the same sweep.
  float* raw;
  int raw_rows;
  int ld_raw;
  // fp32 (out0) columns of output rows < mirror_rows also go to out0m (same
  // row stride ld0): a fused clean + patch sweep's clean rows into the trace's
  // K / V cache (EPI_BIAS, EPI_SPLIT_GELU, EPI_SPLIT_GELU_ACT below n_split)
  float* out0m;
  int mirror_rows;
  // gemm_pingpong_kernel: tiles whose first column is >= a2_col stage their A rows from a2 instead of A
  // (same row / plane strides): the exact-fp16-weight QKV + MLP-in launch, whose Q | K | V columns read
  // LN1's gamma-scaled rows and whose MLP-in columns read LN2's (engine.hip, exact16)
  const uint16_t* a2;
  int a2_col;
  // EPI_BIAS planar launches of at most SK_MAX_M rows that opt in run
  // gemm_skinny.hpp (the linearised entry's G); the unembed keeps the pingpong
  // kernel so its logits path and fused statistics share one GEMM
  int skinny;
};

// torch.nn.functional.gelu (approximate='none'), TransformerLens act_fn "gelu":
// x Phi(x) = max(x, 0) - |x| h,  h = erfc(|x| / sqrt 2) / 2,  with
// erfc(z) = t (a1 + a2 t + ... + a5 t^4) exp(-z^2),  t = 1 / (1 + p z)
// (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7 on erfc), the 1/2 folded into
// the exponent: h = t P(t) exp2(-x^2 log2(e) / 2 - 1).  One reciprocal, one
// exp2, five polynomial steps, no branch or select (the GEMM epilogue applies
// it to every lane and is VALU-bound on it: it replaced Press's degree-9 erfcc
// form, 9 steps and a select).  |error| <= 1.7e-7 max(1, |x|) in fp32 against
// the exact GELU (numpy fp32 emulation over |x| <= 12; the Press form: 1.4e-7).
constexpr float GELU_P = 0.3275911f * 0.70710678118654752440f;  // p / sqrt 2 (t from |x|)
constexpr float GELU_Q = -0.5f * 1.44269504088896341f;          // -log2(e) / 2
constexpr float GELU_A1 = 0.254829592f, GELU_A2 = -0.284496736f, GELU_A3 = 1.421413741f,
                GELU_A4 = -1.453152027f, GELU_A5 = 1.061405429f;
__device__ __forceinline__ float gelu_erf(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(ax, GELU_P, 1.0f));
  float p = GELU_A5;
  p = fmaf(p, t, GELU_A4);
  p = fmaf(p, t, GELU_A3);
  p = fmaf(p, t, GELU_A2);
  p = fmaf(p, t, GELU_A1);
  p *= t;
  const float h = p * __builtin_amdgcn_exp2f(fmaf(ax, ax * GELU_Q, -1.0f));
  return fmaf(-ax, h, fmaxf(x, 0.0f));
}

// gelu_erf on two values with packed fp32 math (v_pk_fma_f32 / v_pk_mul_f32:
// the polynomial at half the VALU issue cycles); identical arithmetic.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
  const f32x2 ax = {fabsf(x.x), fabsf(x.y)};
  const f32x2 d = __builtin_elementwise_fma(ax, f32x2{GELU_P, GELU_P}, f32x2{1.0f, 1.0f});
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = {GELU_A5, GELU_A5};
  p = __builtin_elementwise_fma(p, t, f32x2{GELU_A4, GELU_A4});
  p = __builtin_elementwise_fma(p, t, f32x2{GELU_A3, GELU_A3});
  p = __builtin_elementwise_fma(p, t, f32x2{GELU_A2, GELU_A2});
  p = __builtin_elementwise_fma(p, t, f32x2{GELU_A1, GELU_A1});
  p *= t;
  const f32x2 e = __builtin_elementwise_fma(ax, ax * GELU_Q, f32x2{-1.0f, -1.0f});
  const f32x2 h = p * f32x2{__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
  return __builtin_elementwise_fma(-ax, h, f32x2{fmaxf(x.x, 0.0f), fmaxf(x.y, 0.0f)});
}

// One output element of the fused epilogues (v = acc + bias already); FMT is
// the activation format of EPI_SPLIT_GELU_ACT's GELU columns.
template <int EPI, int FMT = ACT_X2F16>
__device__ __forceinline__ void epi_store(const GemmEpi& ep, size_t orow, int col, float v) {
  const bool mirror = ep.out0m && orow < (size_t)ep.mirror_rows;
  if constexpr (EPI == EPI_BIAS) {
    ep.out0[orow * ep.ld0 + col] = v;
    if (mirror) ep.out0m[orow * ep.ld0 + col] = v;
  } else if constexpr (EPI == EPI_SPLIT_GELU) {
    if (col < ep.n_split) {
      ep.out0[orow * ep.ld0 + col] = v;
      if (mirror) ep.out0m[orow * ep.ld0 + col] = v;
    } else {
      ep.out1[orow * ep.ld1 + (col - ep.n_split)] = gelu_erf(v);
    }
  } else if constexpr (EPI == EPI_SPLIT_GELU_ACT) {
    if (col < ep.n_split) {
      ep.out0[orow * ep.ld0 + col] = v;
      if (mirror) ep.out0m[orow * ep.ld0 + col] = v;
    } else {
      if (ep.raw && orow < (size_t)ep.raw_rows) ep.raw[orow * ep.ld_raw + (col - ep.n_split)] = v;
      store_act<FMT>(ep.out1h + orow * ep.ld1h + (col - ep.n_split), ep.ps1h, gelu_erf(v), ep.range_flag);
    }
  } else {
    ep.out0[orow * ep.ld0 + col] = v + ep.resid[orow * ep.ldr + col];
  }
}

// Shared epilogue of every GEMM kernel: wave tile of TM x TN 32x32
// accumulators at (row_base, col_base).  32x32 C/D map (dtype-independent on
// gfx950): col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
template <int EPI, int TM, int TN>
__device__ __forceinline__ void gemm_epilogue(const GemmEpi& ep, const f32x16 (&acc)[TM][TN], int M, int N,
                                              int row_base, int col_base, int lr, int lh) {
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col_base + j * 32 + lr;
    if (col >= N) continue;
    const float bcol = ep.bias ? ep.bias[col] : 0.0f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = row_base + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row >= M) continue;
        const size_t orow = ep.out_rows ? (size_t)ep.out_rows[row] : (size_t)row;
        epi_store<EPI>(ep, orow, col, acc[i][j][r] + bcol);
      }
    }
  }
}

constexpr int GEMM_BK = 32;  // K granule the host must respect (every tile's BK divides it)
constexpr int GEMM_GROUP_M = 8;

template <int BM_, int BN_, int WM_, int WN_, int BK_>
struct GemmTile {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, BK = BK_;
  static constexpr int LDK = BK + 4;  // padded LDS row (floats): conflict-free ds_read_b128
  static constexpr int THREADS = WM * WN * 64;
  static constexpr int TM = BM / WM / 32;  // 32x32 accumulators per wave (M)
  static constexpr int TN = BN / WN / 32;  // (N)
  static constexpr int KK = BK / 8;        // k-groups of 8 per K step (one ds_read_b128 = 4 MFMAs)
  static constexpr int C4 = BK / 4;        // float4 per staged row
  static constexpr int LOADS_A = BM * BK / 4 / THREADS;  // float4 per thread per K step
  static constexpr int LOADS_B = BN * BK / 4 / THREADS;
  static_assert(LOADS_A * THREADS * 4 == BM * BK && LOADS_B * THREADS * 4 == BN * BK, "staging map");
  static_assert(GEMM_BK % BK == 0, "BK must divide the host K granule");
};
using TileLarge = GemmTile<256, 256, 2, 4, 32>;
using TileSmall = GemmTile<128, 128, 2, 2, 32>;

// 2 waves per SIMD for every tile (8 waves per CU).
// SLICE_KT > 0 (sliced accumulation, the 6.9B / 12B models: K up to 25,600):
// the MFMA chain of every SLICE_KT k-tiles (SLICE_KT * 16 fused products per
// output) runs in a fresh accumulator that is then added to the running sum
// once — K / (32 SLICE_KT) roundings of the large running sum instead of K / 2
// (the exact-product chain is one fp32 rounding per product pair); the second
// accumulator set fits the small tile only (64 + 64 VGPRs), so the host pairs
// it with TileSmall.  Same idea as gemm_pingpong.hpp's sliced x2f16 form.
#ifndef TVR_F32_SLICE_KT
#define TVR_F32_SLICE_KT 4
#endif
constexpr int F32_SLICE_KT = TVR_F32_SLICE_KT;  // k-tiles (32 deep) per fresh-accumulator slice
template <int EPI, class TL, int SLICE_KT = 0>
__global__ void __launch_bounds__(TL::THREADS, 2)
gemm_f32_nt_kernel(const float* __restrict__ A, int lda,
                   const float* __restrict__ W, int ldw, int M, int N, int K,
                   GemmEpi ep) {
  constexpr int BM = TL::BM, BN = TL::BN, TM = TL::TM, TN = TL::TN, NT = TL::THREADS;
  constexpr int BK = TL::BK, LDK = TL::LDK, KK = TL::KK;
  const unsigned long long st0 = ep.stamps ? __builtin_amdgcn_s_memtime() : 0;
  const unsigned long long sr0 = ep.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
  __shared__ __attribute__((aligned(16))) float sA[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) float sB[2][BN * LDK];

  const int nbm = (M + BM - 1) / BM;
  const int nbn = (N + BN - 1) / BN;
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
  const int m0 = tm * BM, n0 = tn * BN;

  const int t = threadIdx.x;
  // staging map: row = f / C4, 4 floats at column (f % C4) * 4 of the BK slice
  const float* ga[TL::LOADS_A];
  const float* gw[TL::LOADS_B];
  int sa[TL::LOADS_A], sb[TL::LOADS_B];
#pragma unroll
  for (int i = 0; i < TL::LOADS_A; ++i) {
    const int f = t + NT * i, row = f / TL::C4, c = (f % TL::C4) * 4;
    const int am = min(m0 + row, M - 1);
    ga[i] = A + (size_t)(ep.a_rows ? ep.a_rows[am] : am) * lda + c;
    sa[i] = row * LDK + c;
  }
#pragma unroll
  for (int i = 0; i < TL::LOADS_B; ++i) {
    const int f = t + NT * i, row = f / TL::C4, c = (f % TL::C4) * 4;
    gw[i] = W + (size_t)min(n0 + row, N - 1) * ldw + c;
    sb[i] = row * LDK + c;
  }

  const int wave = t >> 6, lane = t & 63;
  const int wr = wave / TL::WN, wc = wave % TL::WN;
  const int lr = lane & 31, lh = lane >> 5;
  const int aoff = (wr * (BM / TL::WM) + lr) * LDK + lh * 4;
  const int boff = (wc * (BN / TL::WN) + lr) * LDK + lh * 4;

  f32x16 acc[TM][TN];
  f32x16 sum[SLICE_KT > 0 ? TM : 1][SLICE_KT > 0 ? TN : 1];  // the running sum of the sliced form
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
  if constexpr (SLICE_KT > 0) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) sum[i][j] = f32x16{};
  }
  f32x4 ra[TL::LOADS_A], rb[TL::LOADS_B];
  f32x4 fa[TM], fb[TN];  // fragments of the k-group being multiplied

  auto frags = [&](int b, int kk, f32x4 (&xa)[TM], f32x4 (&xb)[TN]) {
    const float* pa = &sA[b][aoff + kk * 8];
    const float* pb = &sB[b][boff + kk * 8];
#pragma unroll
    for (int i = 0; i < TM; ++i) xa[i] = *(const f32x4*)(pa + i * 32 * LDK);
#pragma unroll
    for (int j = 0; j < TN; ++j) xb[j] = *(const f32x4*)(pb + j * 32 * LDK);
  };
  auto stage = [&](int b) {
#pragma unroll
    for (int i = 0; i < TL::LOADS_A; ++i) *(f32x4*)(&sA[b][sa[i]]) = ra[i];
#pragma unroll
    for (int i = 0; i < TL::LOADS_B; ++i) *(f32x4*)(&sB[b][sb[i]]) = rb[i];
  };

#pragma unroll
  for (int i = 0; i < TL::LOADS_A; ++i) ra[i] = *(const f32x4*)(ga[i]);
#pragma unroll
  for (int i = 0; i < TL::LOADS_B; ++i) rb[i] = *(const f32x4*)(gw[i]);
  stage(0);
  __syncthreads();
  frags(0, 0, fa, fb);

  // Software-pipelined K loop: the fragments of k-group kk+1 are read before
  // kk's MFMAs; at the last k-group the next tile is staged, the block
  // synchronises and the NEXT step's first fragments are read, all ahead of
  // the last group's MFMAs, whose 4*TM*TN MFMAs then cover the LDS latency.
  const int nk = K / BK;
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = (kt + 1) < nk;
    if (more) {
      const int k1 = (kt + 1) * BK;
#pragma unroll
      for (int i = 0; i < TL::LOADS_A; ++i) ra[i] = *(const f32x4*)(ga[i] + k1);
#pragma unroll
      for (int i = 0; i < TL::LOADS_B; ++i) rb[i] = *(const f32x4*)(gw[i] + k1);
    }
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      f32x4 na[TM], nb[TN];
      if (kk + 1 < KK) {
        frags(buf, kk + 1, na, nb);
      } else if (more) {
        stage(buf ^ 1);
        __syncthreads();
        frags(buf ^ 1, 0, na, nb);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = na[i];
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = nb[j];
    }
    buf ^= 1;
    if constexpr (SLICE_KT > 0) {
      if ((kt + 1) % SLICE_KT == 0 || !more) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            sum[i][j] += acc[i][j];
            acc[i][j] = f32x16{};
          }
      }
    }
  }

  if constexpr (SLICE_KT > 0)
    gemm_epilogue<EPI, TM, TN>(ep, sum, M, N, m0 + wr * (BM / TL::WM), n0 + wc * (BN / TL::WN), lr, lh);
  else
    gemm_epilogue<EPI, TM, TN>(ep, acc, M, N, m0 + wr * (BM / TL::WM), n0 + wc * (BN / TL::WN), lr, lh);
  if (ep.stamps && t == 0) {
    ep.stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - st0;
    ep.stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - sr0;
  }
}

template <class TL>
inline int gemm_grid(int M, int N) {
  return ((M + TL::BM - 1) / TL::BM) * ((N + TL::BN - 1) / TL::BN);
}

// The large tile once it fills every CU at least twice, else the small one.
inline bool gemm_use_large(int M, int N) { return gemm_grid<TileLarge>(M, N) >= 512; }

}  // namespace tvr

// gemm_pingpong.hpp — the planar GEMM (gemm_planar.hpp: same operands, same
// LDS image, same fused epilogues) on a phase-split, two-group schedule.
//
//   C[M][N] = A[M][K] @ W[N][K]^T (+ fused epilogue), A and W in a planar
//   activation format (ACT_X2F16: 2 fp16 planes, BK 32; ACT_BF16: 1 bf16
//   plane, BK 64) — 128 B of K per row per k-tile in both.
//
// Block 256 x 256, 8 waves as 2 (rows, wr) x 4 (columns, wc), 128 x 64 output
// per wave (8 x 4 accumulators of 16 x 16, D = W A^T as in gemm_planar.hpp).
// Why a new schedule: in gemm_planar_kernel both waves of a SIMD read LDS and
// issue MFMAs at the same time and meet at one barrier per k-tile; the older
// wave wins issue, finishes first and waits at the barrier 36 % of its loop
// (profiles/gemm_x2_variants_r01.json) — the SIMD's MFMA pipe is 55 % busy.
// Here each k-tile is 4 phases, one output quadrant each:
//     q1  Q(A_lo, W_lo)   reads A_lo (8 fragments) + W_lo (4)
//     q2  Q(A_lo, W_hi)   reads W_hi (4)
//     q3  Q(A_hi, W_hi)   reads A_hi (8)
//     q4  Q(A_hi, W_lo)   no reads (W_lo still in registers)
// and every phase is  [ds_reads, LDS-DMA issue] barrier [MFMA cluster] barrier.
// Waves 4-7 (wr = 1) pass one extra barrier before the loop, so on every SIMD
// one wave runs its MFMA cluster while its partner reads LDS and issues its
// loads: the MFMA pipe always has a wave to feed it.
//
// Staging (LDS-DMA, 2 buffers): a k-tile is 4 regions of 16 KB (A_lo = rows
// 0-63 of each wave-row's 128, A_hi, W_lo = columns 0-31 of each wave-column's
// 64, W_hi), each 16 x 1 KB pieces, 2 per wave.  Exactly one region is staged
// per phase — q1 A_hi(t+1), q2 W_hi(t+1), q3 A_lo(t+2), q4 W_lo(t+2) — so no
// read segment carries more than 2 glds (their issue cost, not LDS bandwidth,
// is what makes a read segment outlast its partner's 24-MFMA cluster; 4 glds in
// one segment cost 1-3 % of the loop, tools/gemm_split_probe x2pp9 in r02).
// Each region is restaged >= 2 phases after its last read (the WAR margin the
// one-barrier group offset needs: a wave of the other group may still be
// reading one segment later), lands >= 3 phases after it is issued, and is
// retired one phase before its first read by a COUNTED wait (the glds issued
// since): vmcnt(4) in q1 (W_hi), vmcnt(8) in q2 (A_hi), vmcnt(6) in q4 (A_lo,
// W_lo), then the phase's barrier; nothing in the loop waits vmcnt(0) and no
// __syncthreads() (its fence would drain the DMA).  Past the last k-tile the
// stage still issues (same counts) into a 1 KB LDS region nobody reads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "gemm_planar.hpp"

namespace tvr {

constexpr int PP_THREADS = 512;
constexpr int PP_TILE_ELEMS = 256 * 256;  // one tile's fp32 partial product (split-K workspace unit)

inline int gemm_pingpong_grid(int M, int N) { return ((M + 255) / 256) * ((N + 255) / 256); }

// Tile wg of the grouped raster: GEMM_GROUP_M m-blocks walked fastest, then
// the next column of blocks (blocks b and b + 8 of a launch share an XCD
// after the remap, so neighbours share A rows / W columns in one L2).
__host__ __device__ inline void pp_tile_coords(int wg, int nbm, int nbn, int& m0, int& n0, int gm = GEMM_GROUP_M) {
  const int per_group = gm * nbn;
  const int grp = wg / per_group;
  const int first_m = grp * gm;
  const int gsz = nbm - first_m < gm ? nbm - first_m : gm;
  const int in_grp = wg - grp * per_group;
  m0 = (first_m + in_grp % gsz) * 256;
  n0 = (in_grp / gsz) * 256;
}

// Epilogue through LDS (after the K loop, the staging buffers are free): the
// accumulators' natural layout gives each store instruction 16 rows x 32-64 B
// (a 16-column slice per row; 32 B per plane for the split activation format),
// and 256 lockstep blocks writing such partial lines ran the QKV+MLP-in
// epilogue at half the HBM write rate of full lines.  Here each 128-row half
// of the tile goes to LDS (row stride 260 floats: conflict-free 16-B writes),
// then all 512 threads store whole rows: 1 KB (fp32) or 2 x 512 B (planes)
// contiguous per row.  Rows [row0, row0 + Mlim) / columns [col0, col0 + Nlim)
// of the output; ep's out0 / out1h / resid / out_rows / bias index globally.
constexpr int PP_EPI_LDR = 260;                   // floats per LDS row
#ifndef TVR_PP_NT
#define TVR_PP_NT 1
#endif
// QKV + MLP-in outputs (qkv fp32, GELU planes: 72 KB per row) stored non-temporal:
// +2 % on that GEMM (the residual / unembed outputs measured no better); A/B: -DTVR_PP_NT=0
constexpr bool PP_NT_STORES = TVR_PP_NT;
// x2f16 sliced accumulation (template SL): each 32-deep k-slice's three products (a1 w0, a0 w1, a0 w0) are
// summed in a fresh MFMA accumulator and added to the tile's accumulator once (one fp32 rounding of the
// running sum per slice instead of three).  The running sum's roundings are the path's dominant error at
// large K (Pythia-12B's O + MLP-out GEMM: K = 25,600 -> 2,400 roundings per output before, 800 now;
// DESIGN.md §2, the accumulation term of tools/precision_probe.py).  Cost: 8 adds (20 VALU instructions)
// per 24 MFMAs: 454 -> 399 TF/s on the C3 GEMMs with every launch sliced (r04i; 394 with the adds placed
// by the compiler, 363 with them after the cluster, 396 with a finer 2 MFMA / 2 VALU interleave, 403 with
// no sched_group_barrier (r04r); summing only the two small products in t and the big
// one straight into the tile sum: 401 TF/s but 12B at 6.8e-5 instead of 3.8e-5 of max |CIE|).  So the
// host asks for it only where the fp32 bar needs it: every x2f16 GEMM of a model whose O + MLP-out K
// reaches PP_SLICE_MIN_K (6.9B, 12B: slicing that GEMM alone left 12B at 0.99e-4 of max |CIE|, all of
// them 0.38e-4); 2.8B (K = 12,800) runs unsliced at 0.36e-4.  A/B: -DTVR_PP_SLICE_MIN_K=<K>.
#ifndef TVR_PP_SLICE_MIN_K
#define TVR_PP_SLICE_MIN_K 16384
#endif
constexpr int PP_SLICE_MIN_K = TVR_PP_SLICE_MIN_K;
// Placement of the sliced form's adds: 2 (round 5) scalar adds, two in each of the next pair's last four MFMA
// gaps, the last pair carried into the next phase (+2.2 % on the probe's sliced shapes, C5 1,286 -> 1,317
// patched/s, profiles/r05/slice_form2_ab_r05n.txt: form 1 spread them 2, 2, 1, 1, 1, 1 and its first adds
// read results too soon after their MFMA, which the compiler paid for with an s_nop 3 three times per
// cluster); 1 that form; 0 (round 4) the pair's packed adds after the next pair's MFMAs.  Same adds in the
// same order in every form: bit-identical results.
#ifndef TVR_PP_SLICE_FORM
#define TVR_PP_SLICE_FORM 2
#endif
// The sliced form with one-plane weights (WX): 2 (default) the scheduled pairs below with the two tiles'
// product chains interleaved (a1 w0 of tile 0, of tile 1, then a0 w0 of each), the previous pair's adds two
// per MFMA gap: 592 / 601 TF on the probe's shapes; 1 tile 0's chain then tile 1's (each chain's second MFMA
// right behind its first: 577 / 587, profiles/r05/slice_form_wx2_ab_r05as.txt); 0 the compiler-placed loop.
#ifndef TVR_PP_SLICE_FORM_WX
#define TVR_PP_SLICE_FORM_WX 2
#endif
// One-plane weights: 1 stage the 2-piece activation regions in the read-light phases (pp_tile), 0 (default)
// the 3-product order.  Measured within noise (qkv / o probe shapes 654 / 672 vs 651 / 671 TF, sliced 578 /
// 582 vs 578 / 580, identical results: profiles/r05/wx_stage_ab_r05ab.txt), so the proven order stays.
#ifndef TVR_PP_WX_STAGE
#define TVR_PP_WX_STAGE 0
#endif
// One-plane weights: the wide wave tile (pp_tile_wt: 4 x 2 waves of 64 x 128, balanced read segments) —
// 2 (default) two phases per k-tile when unsliced, 1 four phases, 0 pp_tile's 2 x 4 waves of 128 x 64.
// Probe, one box, 3 interleaved rounds (profiles/r06/wide_tile_probe_r06c.txt): qkv / o shapes 641 / 655 TF
// (pp_tile) -> 651 / 661 (wide) -> 661 / 663 (wide, two phases); sliced 577 / 584 -> 601 / 610 (wide); PMC:
// MFMA busy 73.7 -> 77.2 -> 78.3 % at 1.69 -> 1.63 -> 1.62 GHz (the power cap gives back most of the cycles)
#ifndef TVR_PP_WX_WIDE
#define TVR_PP_WX_WIDE 2
#endif
// bf16 / fp16 operands (one plane each, BK 64): 1 the wide four-phase tile (pp_tile_wt: reads per phase 8 / 8
// / 4 / 4 fragments against pp_tile's 12 / 4 / 8 / 0), 0 (default) pp_tile.  The wide form holds 8 weight
// column tiles x 2 k-groups (+32 VGPRs: 256 with 11 spilled) and measured slower on the probe's shapes, qkv / o
// 1,193 / 1,250 vs 1,258 / 1,351 TF (profiles/r06/bf16_wide_probe_r06g.txt), so pp_tile stays
#ifndef TVR_PP_BF16_WIDE
#define TVR_PP_BF16_WIDE 0
#endif
// One-plane weights, unsliced: 1 the two-phase, three-buffer K loop (pp_tile P2), 0 the four-phase one
#ifndef TVR_PP_WX_2PHASE
#define TVR_PP_WX_2PHASE 0
#endif
// pp_tile, two-plane operands (bf16 / fp16, unsliced x2f16): 1 read the NEXT k-tile's first two A row tiles
// in q4 (into 4 extra fragments, +16 VGPRs), so the read segments are 8 / 4 / 8 / 4 fragments instead of
// 12 / 4 / 8 / 0 (A_lo(t+1) is then retired in q3: one more counted wait); 0 the plain order.  VAR 21 flips it
#ifndef TVR_PP_PF
#define TVR_PP_PF 1
#endif
// (The add as four v_add_f32 in inline asm, to keep the SLP vectorizer from packing it into v_pk_add_f32,
// read the MFMA results without the MFMA -> VALU wait states the compiler inserts for its own code: every
// x2f16 result came out wrong on the GPU.  Plain C++: the compiler packs and places the waits.)
__device__ __forceinline__ f32x4 slice_add(f32x4 c, f32x4 t) { return c + t; }
constexpr int PP_EPI_LDS = 128 * PP_EPI_LDR * 2;  // halves

// EPI_STATS: the rows of one LDS half (acc * acc_scale, row stride
// PP_EPI_LDR) reduced to the per-tile statistics of GemmEpi::stats instead of
// being stored: per row the max, sum(exp(x - max)) and stats_k rounds of (value
// desc, column asc) argmax.  Four threads per row (512 threads, 128 rows): the
// quad's thread q scans columns 16 i + 4 q (i = 0 .. 15, + bias) in ascending
// order from LDS, and the quad combines with two DPP steps — one pass for the
// max, one for the exp sum and the first argmax, one more per further round,
// whose candidates are the columns ordered after the previous winner.  (Round
// 5's form, one wave per row with a 64-lane shuffle butterfly per statistic and
// round, spent most of the epilogue in dependent ds_bpermute chains: 32 rows
// per wave, 12 + 12 K shuffles each.)  The tile's columns are [col0, col0 +
// min(Nlim, 256)), Nlim % 4 == 0 (host-checked).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
constexpr int DPP_QUAD_X1 = 0xB1, DPP_QUAD_X2 = 0x4E;  // quad_perm [1,0,3,2], [2,3,0,1]
__device__ __forceinline__ void quad_argmax(float& bv, int& bi) {
  argmax_merge(bv, bi, dpp_f<DPP_QUAD_X1>(bv), dpp_i<DPP_QUAD_X1>(bi));
  argmax_merge(bv, bi, dpp_f<DPP_QUAD_X2>(bv), dpp_i<DPP_QUAD_X2>(bi));
}
__device__ __forceinline__ void pp_stats_rows(const GemmEpi& ep, const float* L, int grow0, int col0, int rows,
                                              int Nlim, int t, float acc_scale) {
  const int r = t >> 2, q = t & 3;
  if (r >= rows) return;  // quad-uniform
  Nlim = min(Nlim, 256);  // (N - col0: the tile's own columns)
  const int K = ep.stats_k, rec = 2 + 2 * K, tile = col0 >> 8;
  const float* Lr = L + r * PP_EPI_LDR;
  const float* bias = ep.bias ? ep.bias + col0 : nullptr;
  // the accumulators are stored unscaled (scaling all 128 of a wave's in registers before the first half's
  // reduction spilled 28-41 VGPRs): acc * acc_scale, then + bias, each rounded as the other epilogues do
  auto elem = [&](float a, float b) { return __fadd_rn(__fmul_rn(a, acc_scale), b); };
  auto chunk = [&](int i) {  // columns 16 i + 4 q .. + 3 (+ bias)
    const int c = 16 * i + 4 * q;
    const f32x4 a = *(const f32x4*)(Lr + c);
    const f32x4 b = bias ? *(const f32x4*)(bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    return f32x4{elem(a[0], b[0]), elem(a[1], b[1]), elem(a[2], b[2]), elem(a[3], b[3])};
  };
  const int nc = (Nlim - 4 * q + 15) >> 4;  // this thread's live chunks
  float mx = -INFINITY;
#pragma unroll 2
  for (int i = 0; i < nc; ++i) {
    const f32x4 v = chunk(i);
    mx = fmaxf(mx, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
  }
  mx = fmaxf(mx, dpp_f<DPP_QUAD_X1>(mx));
  mx = fmaxf(mx, dpp_f<DPP_QUAD_X2>(mx));
  float se = 0.f, bv = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll 2
  for (int i = 0; i < nc; ++i) {
    const f32x4 v = chunk(i);
    se += (expf(v[0] - mx) + expf(v[1] - mx)) + (expf(v[2] - mx) + expf(v[3] - mx));
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (v[e] > bv) {  // ascending columns: the first of equal values stays
        bv = v[e];
        bi = col0 + 16 * i + 4 * q + e;
      }
  }
  se += dpp_f<DPP_QUAD_X1>(se);  // (a + b) == (b + a): every lane of the quad holds the same sum
  se += dpp_f<DPP_QUAD_X2>(se);
  const int m = grow0 + r;
  float* o = ep.stats + ((size_t)m * ep.stats_tiles + tile) * rec;
  if (q == 0) {
    o[0] = mx;
    o[1] = se;
    if (ep.targets && ep.tlogit) {
      const int tc = ep.targets[m] - col0;
      if (tc >= 0 && tc < Nlim) ep.tlogit[m] = elem(Lr[tc], bias ? bias[tc] : 0.f);
    }
  }
  for (int j = 0; j < K; ++j) {
    if (j > 0) {  // the best column after the previous winner (pv, pi) in (value desc, column asc) order
      const float pv = bv;
      const int pi = bi;
      bv = -INFINITY;
      bi = 0x7fffffff;
#pragma unroll 2
  for (int i = 0; i < nc; ++i) {
        const f32x4 v = chunk(i);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = col0 + 16 * i + 4 * q + e;
          if ((v[e] < pv || (v[e] == pv && c > pi)) && v[e] > bv) {
            bv = v[e];
            bi = c;
          }
        }
      }
    }
    quad_argmax(bv, bi);
    if (q == 0) {
      o[2 + j] = bv;
      o[2 + K + j] = __int_as_float(bi);
    }
  }
}

// TM x TN accumulators per wave: 8 x 4 (waves 2 rows x 4 columns of 128 x 64) or 4 x 8 (the wide-tile
// one-plane form, pp_tile_wt: waves 4 rows x 2 columns of 64 x 128); half p of the tile (rows 128 p ..)
// comes from the waves whose rows lie in it
template <int EPI, int FMT, bool NOSTORE = false, int TM = 8, int TN = 4>
__device__ __forceinline__ void pp_epilogue_lds(const GemmEpi& ep, const f32x4 (&acc)[TM][TN], float* L, int row0,
                                                int col0, int Mlim, int Nlim, int wr, int wc, int lane, int t,
                                                float acc_scale) {
  static_assert((TM == 8 && TN == 4) || (TM == 4 && TN == 8), "wave tile 128 x 64 or 64 x 128");
  // A thread's columns are the same in every row it stores (the row step, 512
  // threads, is a multiple of the threads per row), so the bias is loaded once
  // before the row loops: no global load inside them, only LDS reads and stores.
  bool split8 = false;
  if constexpr (EPI == EPI_SPLIT_GELU_ACT) split8 = col0 >= ep.n_split && Nlim >= 256;
  float range_mx = 0.f;  // X2F16 GELU planes: the largest scaled magnitude stored, checked once at the end
  const int c8 = (t & 31) * 8, c4 = (t & 63) * 4;
  float b8[8];
  f32x4 b4 = {0.f, 0.f, 0.f, 0.f};
  if (split8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) b8[k] = ep.bias ? ep.bias[col0 + c8 + k] : 0.f;
  } else if (EPI != EPI_STATS && ep.bias && c4 < Nlim) {  // (EPI_STATS adds the bias per chunk)
#pragma unroll
    for (int k = 0; k < 4; ++k) b4[k] = ep.bias[col0 + c4 + k];
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    if ((TM == 8 ? wr : wr >> 1) == p) {
      const int r0 = TM == 8 ? 0 : (wr & 1) * 64;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          *(f32x4*)(L + (r0 + i * 16 + (lane & 15)) * PP_EPI_LDR + wc * (16 * TN) + j * 16 + 4 * (lane >> 4)) =
              EPI == EPI_STATS ? acc[i][j] : acc[i][j] * acc_scale;  // (EPI_STATS scales as it reads)
    }
    __syncthreads();
    const int rows = min(128, Mlim - p * 128);
    // No global load may sit between two of a thread's row stores: s_waitcnt
    // vmcnt counts loads and stores together in issue order, so waiting for a
    // load issued after a store waits for that store to reach memory, and a
    // per-row load (out_rows[m], the residual) turned the row loop into one
    // store round trip per row.  The gathered row indices and the residual
    // rows are therefore loaded for all of the thread's rows of the half
    // before its first store (rows past `rows` read a valid row and store
    // nothing): a half's stores wait for memory once per batch of rows at
    // most (twice per GELU half), not once per row.
    if constexpr (EPI == EPI_STATS) {
      pp_stats_rows(ep, L, row0 + p * 128, col0, rows, Nlim, t, acc_scale);
    } else if (split8) {  // GELU columns: 8 per thread, one 16-B store per plane
      constexpr int RPT = 128 / (PP_THREADS / 32);  // rows per thread (8)
      const int rb = t >> 5;
      int orow[RPT];
#pragma unroll
      for (int i = 0; i < RPT; ++i) orow[i] = row0 + p * 128 + min(rb + i * (PP_THREADS / 32), max(rows - 1, 0));
      if (ep.out_rows) {
#pragma unroll
        for (int i = 0; i < RPT; ++i) orow[i] = ep.out_rows[orow[i]];
      }
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const int r = rb + i * (PP_THREADS / 32);
        if (r >= rows) break;
        const float* src = L + r * PP_EPI_LDR + c8;
        const f32x4 x0 = *(const f32x4*)src, x1 = *(const f32x4*)(src + 4);
        float v[8] = {x0[0] + b8[0], x0[1] + b8[1], x0[2] + b8[2], x0[3] + b8[3],
                      x1[0] + b8[4], x1[1] + b8[5], x1[2] + b8[6], x1[3] + b8[7]};
        const int m = row0 + p * 128 + r;
        if (ep.raw && m < ep.raw_rows) {  // the clean rows' pre-GELU values (lin_entry.hpp)
          float* q = ep.raw + (size_t)m * ep.ld_raw + (col0 + c8 - ep.n_split);
          *(f32x4*)q = f32x4{v[0], v[1], v[2], v[3]};
          *(f32x4*)(q + 4) = f32x4{v[4], v[5], v[6], v[7]};
        }
#pragma unroll
        for (int k = 0; k < 8; k += 2) {
          const f32x2 g = gelu_erf2(f32x2{v[k], v[k + 1]});
          v[k] = g.x;
          v[k + 1] = g.y;
        }
        if (!NOSTORE || v[0] == 1.2345e-30f)  // NOSTORE (diagnostic): the LDS pass and math without the stores
          store_act8<FMT, PP_NT_STORES>(ep.out1h + (size_t)orow[i] * ep.ld1h + (col0 + c8 - ep.n_split), ep.ps1h, v,
                                        ep.range_flag, &range_mx);
      }
    } else if (c4 < Nlim) {
      // 16 rows per thread, in two batches of 8: the residual rows of a batch
      // (32 VGPRs; the waves of the other half still hold their accumulators)
      // are loaded before its stores, so a half waits for memory twice, not
      // once per row
      constexpr int RB = 8, NB = 128 / (PP_THREADS / 64) / RB;
      const int rb = t >> 6;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        int orow[RB];
        f32x4 rr[RB];
#pragma unroll
        for (int i = 0; i < RB; ++i) orow[i] = row0 + p * 128 + min(rb + (b * RB + i) * (PP_THREADS / 64), max(rows - 1, 0));
        if (ep.out_rows) {
#pragma unroll
          for (int i = 0; i < RB; ++i) orow[i] = ep.out_rows[orow[i]];
        }
        if constexpr (EPI == EPI_RESID) {
#pragma unroll
          for (int i = 0; i < RB; ++i) rr[i] = *(const f32x4*)(ep.resid + (size_t)orow[i] * ep.ldr + col0 + c4);
        }
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int r = rb + (b * RB + i) * (PP_THREADS / 64);
          if (r >= rows) break;
          f32x4 v = *(const f32x4*)(L + r * PP_EPI_LDR + c4) + b4;
          if (!NOSTORE || v[0] == 1.2345e-30f) {
            if constexpr (EPI == EPI_RESID)
              st16<false>(ep.out0 + (size_t)orow[i] * ep.ld0 + col0 + c4, v + rr[i]);
            else
              epi_store4<EPI, FMT, PP_NT_STORES && EPI == EPI_SPLIT_GELU_ACT>(ep, orow[i], col0 + c4, v);
          }
        }
      }
    }
    __syncthreads();
  }
  if constexpr (EPI == EPI_SPLIT_GELU_ACT && FMT == ACT_X2F16)
    if (range_mx >= X2_FP16_OVERFLOW && ep.range_flag) atomicOr(ep.range_flag, 1u);
}

// K must be a multiple of BK (host-checked); any M, N.
// VAR (diagnostic builds, tools/gemm_split_probe): 1 no staging in the loop
// (stale LDS: timing only), 2 no s_setprio, 13 s_setprio 1 once for waves 4-7, 14 the cluster flips in the
// sliced form too, 3 no group offset, 4 no vmcnt
// waits in the loop (racy: timing only), 6 per-block stamps (start, loop
// start, loop end, end) of wave 0 to ep.stamps[4 block + i], 7 the register
// epilogue (no LDS pass), 8 the stamps of 6 with the epilogue's global stores
// skipped (timing only), 12 every k-tile staged from k-tile 0 (L2-hot operands,
// same instruction stream: timing only).
// LDS of one block: 2 stages x (A, W) planes + a 1 KB staging sink, or the
// epilogue's 128-row half, whichever is larger
template <int FMT>
struct PpLds {
  using F = PlanarFmt<FMT>;
  static constexpr int BUF = 2 * F::NPL * 256 * F::BK;
  static constexpr int HALVES = (2 * BUF + 512) > PP_EPI_LDS ? (2 * BUF + 512) : PP_EPI_LDS;
};

// One output tile (m0, n0) over k-tiles [kbeg, kbeg + nk) of this block:
// prologue, the phase-split K loop, epilogue.  has_part: the fp32 partial
// tile (acc * acc_scale, no bias) goes to part as a dense 256 x 256 tile
// (split-K / stream-K), else the launch's fused epilogue.  (A separate int
// flag: testing the pointer itself made hipcc spill 26-66 VGPRs.)
template <int EPI, int FMT, bool VEC, int VAR, bool SL, bool WX = false, bool PFOK = true>
__device__ __forceinline__ void pp_tile(const uint16_t* __restrict__ A, int lda, size_t aps,
                                        const uint16_t* __restrict__ W, int ldw, size_t wps, float acc_scale, int M,
                                        int N, const GemmEpi& ep, int m0, int n0, int kbeg, int nk, float* part, int has_part,
                                        unsigned long long st0, unsigned long long sr0) {
  using F = PlanarFmt<FMT>;
  using frag = typename F::frag;
  constexpr int NPL = F::NPL, BK = F::BK, KG = BK / 32;
  constexpr int CPR = BK / 8;          // 16-B chunks per plane row
  constexpr int RPP = 64 / CPR;        // rows per 1 KB piece
  constexpr int PPP = 128 / RPP;       // pieces per plane per region (128 rows)
  constexpr int PL = 256 * BK;         // halves per plane per buffer
  // WX (x2f16 only): the weights are exact in fp16 (their residual plane is zero), so only plane 0 is
  // staged and read and the a0 w1 product is dropped: 2 products per 32-deep slice instead of 3
  static_assert(!WX || FMT == ACT_X2F16, "one-plane weights: x2f16 activations only");
  constexpr int WNPL = WX ? 1 : NPL;   // weight planes staged
  constexpr int BUF = (NPL + WNPL) * PL; // halves per buffer: A planes, then W planes
  // P2 (one-plane weights, unsliced, TVR_PP_WX_2PHASE): 2 phases per k-tile of 32 MFMAs each and 3 LDS
  // buffers (3 x 48 KB: the one-plane buffer is 3/4 of the two-plane one), kloop below
  constexpr bool P2 = WX && !SL && TVR_PP_WX_2PHASE;
  constexpr int NBUF = P2 ? 3 : 2;
  constexpr int DUMMY = NBUF * BUF;    // 1 KB staging sink past the last k-tile
  constexpr int LDS_HALVES = P2 ? (NBUF * BUF + 512 > PP_EPI_LDS ? NBUF * BUF + 512 : PP_EPI_LDS)
                                : PpLds<FMT>::HALVES;
  static_assert(LDS_HALVES * 2 <= 160 * 1024, "LDS budget (P2)");
  static_assert(NPL * KG == 2, "two fragments per 16-row slice per k-tile");
  static_assert(PpLds<FMT>::HALVES * 2 <= 160 * 1024, "LDS budget");
  // ONE __shared__ object (a second one can make hipcc drain vmcnt before
  // ds_reads), declared here so every access is a known LDS address (a
  // generic pointer parameter costs VGPRs: 64-bit flat addresses)
  __shared__ __attribute__((aligned(16))) uint16_t lds[LDS_HALVES];

  // the thread index through an empty asm: a stream-K block's two inlined
  // tiles then recompute their lane addresses instead of one copy holding the
  // other's live across its K loop (VGPR spills)
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  const int wave = t >> 6, lane = t & 63;
  const int wr = wave >> 2, wc = wave & 3;

  // ---- staging map: region R (0 A_lo, 1 A_hi, 2 W_lo, 3 W_hi), pieces 2 wave + s.
  // The piece geometry is wave-uniform (readfirstlane): the LDS destinations
  // (M0) are then scalar, so a stage costs one VALU address add per piece
  // instead of five (add, select, shift, readfirstlane for M0, address).
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  const uint16_t* Ab = ep.a2 != nullptr && n0 >= ep.a2_col ? ep.a2 : A;  // this tile's A operand
  const uint16_t* src[4][2];
  int dst[4][2];
#pragma unroll
  for (int R = 0; R < 4; ++R) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      // pieces of a one-plane weight region (WX): one per wave (s = 0), plane 0
      const int pi = (WX && R >= 2) ? wave_s : 2 * wave_s + s;
      const int plane = pi / PPP, x0 = (pi % PPP) * RPP;  // region row of the piece's first row
      int trow0;                                          // tile row of it
      if (R < 2)
        trow0 = ((x0 >> 6) << 7) + (x0 & 63) + 64 * R;
      else
        trow0 = ((x0 >> 5) << 6) + (x0 & 31) + 32 * (R - 2);
      const int row = trow0 + lane / CPR;
      const int chunk = (lane % CPR) ^ planar_g<CPR>(row);
      if (R < 2) {
        const int am = min(m0 + row, M - 1);
        src[R][s] = Ab + plane * aps + (size_t)(ep.a_rows ? ep.a_rows[am] : am) * lda + chunk * 8;
        dst[R][s] = plane * PL + trow0 * BK;
      } else {
        src[R][s] = W + plane * wps + (size_t)min(n0 + row, N - 1) * ldw + chunk * 8;
        dst[R][s] = (NPL + plane) * PL + trow0 * BK;
      }
    }
  }
  auto stage = [&](int R, int kt) {
    if (VAR == 1 && kt >= 2) return;
    const bool live = kt < nk;
    const int koff = live && VAR != 12 ? (kbeg + kt) * BK : 0;  // VAR 12: every k-tile re-reads k-tile 0 (L2-hot)
    const int boff = (P2 ? kt % 3 : kt & 1) * BUF;
#pragma unroll
    for (int s = 0; s < ((WX && R >= 2) ? 1 : 2); ++s) glds16(src[R][s] + koff, lds + (live ? boff + dst[R][s] : DUMMY));
  };

  // ---- fragment offsets (halves, within a buffer); f = plane (x2f16) or k group (bf16)
  int aoff[2], boff[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int p = NPL == 2 ? f : 0, g = NPL == 2 ? 0 : f;
    const int ra = wr * 128 + (lane & 15), rb = wc * 64 + (lane & 15);
    const int c = 4 * g + (lane >> 4);
    aoff[f] = p * PL + ra * BK + ((c ^ planar_g<CPR>(ra)) << 3);
    boff[f] = (NPL + p) * PL + rb * BK + ((c ^ planar_g<CPR>(rb)) << 3);
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};
  frag fa[4][2], fwl[2][2], fwh[2][2];
  constexpr bool PF = PFOK && ((TVR_PP_PF != 0) != (VAR == 21)) && !P2 && !WX && !(FMT == ACT_X2F16 && SL);
  [[maybe_unused]] frag fx[2][2];  // PF: row tiles 0-1 of A_lo, read one phase early

  // 16-row slices of this wave's 128 rows that hold real rows (A rows past M
  // are staged as copies of row M - 1).  A wave with fewer than 8 runs the
  // K loop's PART copy, which skips the fragment reads and MFMAs of the padding
  // slices (the staging and the barriers stay: the other group needs them):
  // the last m-block of every launch, and most blocks of the small-M layer
  // sweeps (C2: M = 156 + 52 l rows in 256-row tiles).
  const int vi = __builtin_amdgcn_readfirstlane(min(8, max(0, (M - m0 - wr * 128 + 15) >> 4)));  // wave-uniform
  auto read_a = [&](const uint16_t* base, int i0, auto part, int ifirst = 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i >= ifirst && (!decltype(part)::value || i0 + i < vi))
#pragma unroll
        for (int f = 0; f < 2; ++f) fa[i][f] = *(const frag*)(base + aoff[f] + (i0 + i) * 16 * BK);
  };
  auto read_fx = [&](const uint16_t* base, auto part) {  // PF: A row tiles 0-1 into fx
#pragma unroll
    for (int i = 0; i < 2; ++i)
      if (!decltype(part)::value || i < vi)
#pragma unroll
        for (int f = 0; f < 2; ++f) fx[i][f] = *(const frag*)(base + aoff[f] + i * 16 * BK);
  };
  auto read_w = [&](const uint16_t* base, int j0, frag (&fw)[2][2], auto part) {
    if (decltype(part)::value && vi == 0) return;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int f = 0; f < (WX ? 1 : 2); ++f) fw[j][f] = *(const frag*)(base + boff[f] + (j0 + j) * 16 * BK);
  };
  // sliced form, all 8 tiles live: the slice sums of the cluster's LAST tile pair are carried into the next
  // phase's cluster (tc, for acc[ci][cj + 0..1]) and added there, while its first MFMAs run
  [[maybe_unused]] f32x4 tc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  auto mfma_quadrant = [&](int i0, int j0, const frag (&fw)[2][2], auto part, int ci, int cj) {
#if TVR_PP_SLICE_FORM_WX >= 1
    if constexpr (FMT == ACT_X2F16 && SL && WX && !decltype(part)::value) {
      // sliced, one-plane weights: per tile pair (i, 0..1) the two slices' products (form 2: a1 w0 of both
      // tiles, then a0 w0 of both; form 1: tile 0's chain, then tile 1's), two of the previous pair's 8
      // slice-sum adds after each MFMA (tile 0's sums first); the last pair carried into the next phase (tc),
      // as the 3-product form 2
      f32x4 t[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int di = i == 0 ? ci : i0 + i - 1, dj = i == 0 ? cj : j0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          // MFMA q: product pz of tile j (0: a1 w0, 1: a0 w0); form 2 interleaves the two tiles' chains
          const int j = TVR_PP_SLICE_FORM_WX == 2 ? (q & 1) : (q >> 1), pz = TVR_PP_SLICE_FORM_WX == 2 ? (q >> 1) : (q & 1);
          t[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][0], fa[i][pz == 0 ? 1 : 0],
                                                             pz == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : t[i][j], 0, 0, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
#pragma unroll
          for (int e = 2 * q; e < 2 * q + 2; ++e)
            acc[di][dj + (e >> 2)][e & 3] += i == 0 ? tc[e >> 2][e & 3] : t[i - 1][e >> 2][e & 3];
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
      }
      tc[0] = t[3][0];
      tc[1] = t[3][1];
      return;
    }
#endif
    if constexpr (FMT == ACT_X2F16 && SL && !WX && !decltype(part)::value) {
#if TVR_PP_SLICE_FORM >= 1
      // tile pairs (i, 0..1) in turn — the pair's first products, second, third (two independent chains back
      // to back) — and the previous pair's 8 slice-sum adds (the carried pair's for i = 0) spread 2, 2, 1, 1,
      // 1, 1 over its six MFMA gaps as SCALAR v_add_f32 (the engine builds with -fno-slp-vectorize: packed
      // v_pk_add_f32 beside MFMAs costs far more than its issue slot, MI355X_MICROARCH.md 'price of one
      // filler'); two v_add_f32 fit a 16x16x32 gap's free issue cycles, so the adds ride on the MFMA pipe's
      // time instead of extending the cluster
      f32x4 t[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int di = i == 0 ? ci : i0 + i - 1, dj = i == 0 ? cj : j0;  // the previous pair's tiles
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          const int j = q & 1, p = q >> 1;  // MFMA q: product p of tile j (p 0: a1 w0, 1: a0 w1, 2: a0 w0)
          t[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][p == 1 ? 1 : 0], fa[i][p == 0 ? 1 : 0],
                                                             p == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : t[i][j], 0, 0, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          // adds after MFMA q: elements e0 .. e1 of the previous pair's 8 (tile e / 4, element e % 4)
#if TVR_PP_SLICE_FORM == 2
          // form 2: none after q0 / q1, two after q2 .. q5, so that every add reads a result >= 9 issue slots after
          // the MFMA that wrote it (form 1's adds after q0 read the previous pair's tile-0 sum 5 slots after its
          // last MFMA: the compiler pads each with s_nop 3, 3 per cluster)
          const int e0 = q < 2 ? 0 : 2 * (q - 2), e1 = q < 2 ? 0 : 2 * (q - 2) + 2;
#else
          const int e0 = q < 2 ? 2 * q : q + 2, e1 = q < 2 ? 2 * q + 2 : q + 3;
#endif
#pragma unroll
          for (int e = e0; e < e1; ++e)
            acc[di][dj + (e >> 2)][e & 3] += i == 0 ? tc[e >> 2][e & 3] : t[i - 1][e >> 2][e & 3];
          if (e1 - e0 == 2)
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          else if (e1 - e0 == 1)
            __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        }
      }
      tc[0] = t[3][0];
      tc[1] = t[3][1];
      return;
#else
      // (round-4 form) tile pairs in turn, each pair's two slice sums added while the NEXT pair's MFMAs
      // run (6 MFMAs, then the pair's adds); the last pair's adds after the cluster
      (void)ci;
      (void)cj;
      f32x4 t[4][2];
#pragma unroll
      for (int i = 0; i <= 4; ++i) {
        if (i < 4) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
            t[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][0], fa[i][1], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
          for (int j = 0; j < 2; ++j) t[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][1], fa[i][0], t[i][j], 0, 0, 0);
#pragma unroll
          for (int j = 0; j < 2; ++j) t[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][0], fa[i][0], t[i][j], 0, 0, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
        }
        if (i > 0) {
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i0 + i - 1][j0 + j] = slice_add(acc[i0 + i - 1][j0 + j], t[i - 1][j]);
          __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
        }
      }
      return;
#endif
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (decltype(part)::value && i0 + i >= vi) continue;
        f32x4 c = acc[i0 + i][j0 + j];
        const bool x = PF && i0 == 0 && i < 2;  // PF: row tiles 0-1 live in fx
        const frag a0 = x ? fx[i & 1][0] : fa[i][0], a1 = x ? fx[i & 1][1] : fa[i][1];
        if constexpr (FMT == ACT_X2F16 && SL) {  // the slice's sum first, then one add (see above)
          f32x4 t = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][0], a1, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          if constexpr (!WX) t = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][1], a0, t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][0], a0, t, 0, 0, 0);
          c = slice_add(c, t);
        } else if constexpr (FMT == ACT_X2F16) {  // small terms first; the big a0*w0 last
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][0], a1, c, 0, 0, 0);
          if constexpr (VAR != 15 && !WX)  // (VAR 15, probe timing: the product dropped on full staging)
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][1], a0, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][0], a0, c, 0, 0, 0);
        } else if constexpr (FMT == ACT_F16) {
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][0], a0, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][1], a1, c, 0, 0, 0);
        } else {
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[j][0], a0, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[j][1], a1, c, 0, 0, 0);
        }
        acc[i0 + i][j0 + j] = c;
      }
  };
  // [MFMA cluster] between this phase's two barriers, at s_setprio 1 — except in the sliced form, whose
  // clusters carry the slice-sum adds: there the flips cost 1.3-1.6 % on the probe's 2.8B-width shapes (370 ->
  // 375-380 TF/s without them; unsliced within noise either way: profiles/r05/gemm_prio_ab_r05k.jsonl), +0.2 %
  // (noise) on C5's 12B GEMMs (profiles/r05/c5_prio_ab_r05l.txt)
  constexpr bool prio = VAR == 14 || (VAR != 2 && VAR != 13 && !(FMT == ACT_X2F16 && SL));
#define TVR_PP_CLUSTER(...)                  \
  __builtin_amdgcn_s_barrier();              \
  __builtin_amdgcn_sched_barrier(0);         \
  if (prio) __builtin_amdgcn_s_setprio(1);   \
  __VA_ARGS__;                               \
  if (prio) __builtin_amdgcn_s_setprio(0);   \
  __builtin_amdgcn_sched_barrier(0);         \
  __builtin_amdgcn_s_barrier();              \
  __builtin_amdgcn_sched_barrier(0)

  // ---- prologue: the stage history of tiles -2 and -1 in loop order (A_lo W_lo
  // A_hi W_hi of tile 0, A_lo W_lo of tile 1), then retire A_lo(0) / W_lo(0).
  // One-plane weights (WX, TVR_PP_WX_STAGE): a weight region is 1 piece per wave and an activation region 2,
  // so the 2-piece regions are staged in the phases with few fragment reads (q2: 2 reads, q4: none) and the
  // 1-piece ones in the read-heavy q1 / q3:  q1 W_hi(t+1), q2 A_hi(t+1), q3 W_lo(t+2), q4 A_lo(t+2) — each
  // still >= 2 phases after its region's last read and retired one phase before its first
  constexpr bool XS = WX && TVR_PP_WX_STAGE && !P2;
  if constexpr (P2) {
    // tiles 0 and 1 in loop order (R1: A_lo, W_lo, W_hi; R2: A_hi), then retire tile 0's R1 regions:
    // 2 + 4 + 2 pieces issued after them
    stage(0, 0);
    stage(2, 0);
    stage(3, 0);
    stage(1, 0);
    stage(0, 1);
    stage(2, 1);
    stage(3, 1);
    stage(1, 1);
  } else if constexpr (XS) {
    stage(2, 0);
    stage(0, 0);
    stage(3, 0);
    stage(1, 0);
    stage(2, 1);
    stage(0, 1);
  } else {
    stage(0, 0);
    stage(2, 0);
    stage(1, 0);
    stage(3, 0);
    stage(0, 1);
    stage(2, 1);
  }
  // counted waits: the pieces issued after the awaited region (2 per wave per region; 1 for a WX weight region)
  if constexpr (P2)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (WX)
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (PF) read_fx(lds, std::integral_constant<bool, false>{});  // A_lo(0) rows 0-1 (retired above)
  if (wr == 1 && VAR != 3) {  // the group offset: waves 4-7 run one barrier behind
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }

  if (VAR == 13 && wave_s >= 4) __builtin_amdgcn_s_setprio(1);  // VAR 13: static priority for the younger half (wave-uniform test)
  unsigned long long d_loop0 = 0, d_loop1 = 0;
  if constexpr (VAR == 6 || VAR == 8) d_loop0 = __builtin_amdgcn_s_memtime();
  auto kloop = [&](auto part) {
    if constexpr (P2) {
      // k-tile kt in 3-buffer rotation; per wave group: R1 [read A_lo, W_lo, W_hi; retire A_hi(kt); stage
      // A_lo / W_lo / W_hi of kt + 2] barrier [32 MFMAs: rows 0-63] barrier, R2 [read A_hi; retire the R1
      // regions of kt + 1; stage A_hi(kt + 2)] barrier [32 MFMAs: rows 64-127] barrier.  Buffer (kt + 2) % 3
      // held k-tile kt - 1, whose last reads (the lagging group's, one segment late) are >= 3 segments
      // before these stages; every region is retired one phase before its first read and >= 3 segments
      // after it was issued (counted waits: 4 + 2 pieces issued since)
      for (int kt = 0; kt < nk; ++kt) {
        const uint16_t* cur = lds + (kt % 3) * BUF;
        read_a(cur, 0, part);
        read_w(cur, 0, fwl, part);
        read_w(cur, 2, fwh, part);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // A_hi(kt) (R2 of kt - 2), read in R2
        stage(0, kt + 2);
        stage(2, kt + 2);
        stage(3, kt + 2);
        TVR_PP_CLUSTER(mfma_quadrant(0, 0, fwl, part, 7, 0); mfma_quadrant(0, 2, fwh, part, 3, 0));
        read_a(cur, 4, part);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // A_lo, W_lo, W_hi of kt + 1 (R1 of kt - 1)
        stage(1, kt + 2);
        TVR_PP_CLUSTER(mfma_quadrant(4, 0, fwl, part, 7, 2); mfma_quadrant(4, 2, fwh, part, 3, 2));
      }
      return;
    }
    for (int kt = 0; kt < nk; ++kt) {
      const uint16_t* cur = lds + (kt & 1) * BUF;
      // q1: Q(A_lo, W_lo)
      read_a(cur, 0, part, PF ? 2 : 0);
      read_w(cur, 0, fwl, part);
      if constexpr (XS) {
        asm volatile("s_waitcnt vmcnt(5)" ::: "memory");  // W_hi(kt) (q1 of kt-1), read in q2
        stage(3, kt + 1);
      } else {
        if constexpr (WX) {
          asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        } else {
          if (VAR != 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // W_hi(kt) (issued in q2 of kt-1), read in q2
        }
        stage(1, kt + 1);
      }
      TVR_PP_CLUSTER(mfma_quadrant(0, 0, fwl, part, 7, 0));  // (ci, cj): the carried pair of the previous phase
      // q2: Q(A_lo, W_hi)
      read_w(cur, 2, fwh, part);
      if constexpr (XS) {
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // A_hi(kt) (q2 of kt-1), read in q3
        stage(1, kt + 1);
      } else {
        if constexpr (WX) {
          asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        } else {
          if (VAR != 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // A_hi(kt) (q1 of kt-1), read in q3
        }
        stage(3, kt + 1);
      }
      TVR_PP_CLUSTER(mfma_quadrant(0, 2, fwh, part, 3, 0));
      // q3: Q(A_hi, W_hi)
      read_a(cur, 4, part);
      if constexpr (PF) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // A_lo(kt+1) (q3 of kt-1), read in q4
      stage(XS ? 2 : 0, kt + 2);
      TVR_PP_CLUSTER(mfma_quadrant(4, 2, fwh, part, 3, 2));
      // q4: Q(A_hi, W_lo)
      if constexpr (XS) {
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // A_lo(kt+1) (q4 of kt-1), W_lo(kt+1) (q3 of kt-1), read in q1
      } else if constexpr (WX) {
        asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      } else {
        if (VAR != 4) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // A_lo(kt+1), W_lo(kt+1) (q3 / q4 of kt-1), read in q1
      }
      if constexpr (PF) read_fx(lds + ((kt + 1) & 1) * BUF, part);  // A_lo(kt+1) rows 0-1, retired in q3
      stage(XS ? 0 : 2, kt + 2);
      TVR_PP_CLUSTER(mfma_quadrant(4, 0, fwl, part, 7, 2));
    }
  };
  if (vi == 8) {
    kloop(std::integral_constant<bool, false>{});
#if TVR_PP_SLICE_FORM >= 1
    if constexpr (FMT == ACT_X2F16 && SL && (!WX || TVR_PP_SLICE_FORM_WX >= 1)) {  // the last cluster's carried pair (q4: tiles (7, 0..1))
      acc[7][0] = slice_add(acc[7][0], tc[0]);
      acc[7][1] = slice_add(acc[7][1], tc[1]);
    }
#endif
  } else {
    kloop(std::integral_constant<bool, true>{});
  }
#undef TVR_PP_CLUSTER
  if constexpr (VAR == 6 || VAR == 8) d_loop1 = __builtin_amdgcn_s_memtime();
  if (wr == 0 && VAR != 3) __builtin_amdgcn_s_barrier();  // balance the group offset
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the sink's DMAs retire before the block ends

  if constexpr (VEC && VAR != 7) {  // epilogue through LDS (VAR 7: the register epilogue, for A/B)
    __syncthreads();  // every wave's DMA retired (vmcnt(0) above) and last LDS reads done
    float* L = reinterpret_cast<float*>(lds);
    if (has_part) {
      GemmEpi pe = ep;
      pe.out0 = part;
      pe.ld0 = 256;
      pe.out_rows = nullptr;  // partial tiles are stored densely; the reduce applies out_rows
      pp_epilogue_lds<EPI, FMT, VAR == 8>(pe, acc, L, 0, 0, M - m0, N - n0, wr, wc, lane, t, acc_scale);
    } else {
      pp_epilogue_lds<EPI, FMT, VAR == 8>(ep, acc, L, m0, n0, M - m0, N - n0, wr, wc, lane, t, acc_scale);
    }
    if ((VAR == 6 || VAR == 8) && ep.stamps && t == 0) {
      unsigned long long* o = ep.stamps + 4 * blockIdx.x;
      o[0] = st0;
      o[1] = d_loop0;
      o[2] = d_loop1;
      o[3] = __builtin_amdgcn_s_memtime();
    }
    return;
  }
  if constexpr (EPI == EPI_STATS) {  // the statistics exist in the LDS epilogue only (host-checked)
    return;
  } else {
    if (acc_scale != 1.0f) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] *= acc_scale;
    }
    if (has_part) {  // partial product of (split, tile) as a 256 x 256 fp32 tile (EPI_BIAS launches; host-checked)
      GemmEpi pe = ep;
      pe.out0 = part;
      pe.ld0 = 256;
      gemm_epilogue16t<EPI, FMT, VEC, 8, 4>(pe, acc, M - m0, N - n0, wr * 128, wc * 64, lane);
    } else {
      gemm_epilogue16t<EPI, FMT, VEC, 8, 4>(ep, acc, M, N, m0 + wr * 128, n0 + wc * 64, lane);
    }
    if (VAR == 6 && ep.stamps && t == 0) {
      unsigned long long* o = ep.stamps + 4 * blockIdx.x;
      o[0] = st0;
      o[1] = d_loop0;
      o[2] = d_loop1;
      o[3] = __builtin_amdgcn_s_memtime();
    } else if (ep.stamps && t == 0) {
      ep.stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - st0;
      ep.stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - sr0;
    }
  }
}

// The one-plane (WX) tile on a WIDE wave tile: 8 waves as 4 (rows, wr) x 2 (columns, wc) of 64 x 128 each
// (acc[4][8]) instead of 2 x 4 of 128 x 64.  With two activation planes and one weight plane a wave's
// fragment reads per k-tile are (rows / 16) x 2 + columns / 16: 16 here against 20 (8 x 2 + 4), and the
// four phases' read segments are balanced — 4 fragments each — by reading the NEXT k-tile's first two row
// tiles in q4, whose cluster needs nothing read in its own segment:
//     q1  rows 0-31 x cols 0-63     reads W_lo(t)    stages A_hi(t+1)   (2 pieces per wave)
//     q2  rows 0-31 x cols 64-127   reads W_hi(t)    stages A_lo(t+2)   (2)
//     q3  rows 32-63 x cols 64-127  reads A_hi(t)    stages W_lo(t+2)   (1)
//     q4  rows 32-63 x cols 0-63    reads A_lo(t+1)  stages W_hi(t+2)   (1)
// (pp_tile's q1 reads 10 fragments + 2 pieces and q3 8 + 2, longer than the partner's 16-MFMA cluster;
// q2 and q4 2 and 0.)  Regions: A_lo / A_hi = rows 0-31 / 32-63 of every wave row's 64 (2 planes, 16 KB),
// W_lo / W_hi = columns 0-63 / 64-127 of every wave column's 128 (8 KB).  Every region is restaged 2 phases
// after its last read, issued 6 phases before its first read and retired one phase before it by
// vmcnt(6) (the pieces issued since: 1 + 2 + 2 + 1 in every phase), as pp_tile's rules.  Per output
// element the MFMA sequence is pp_tile's (a1 w0, then a0 w0, k-slice by k-slice; sliced: the slice's sum
// added once): bit-identical results.  A/B: TVR_PP_WX_WIDE=0, or VAR 16 / 17 (probe).  TWO (unsliced x2f16):
// two phases of 32 MFMAs over three LDS buffers (the loop below).  FMT bf16 / fp16 (TVR_PP_BF16_WIDE, off):
// the same schedule with one plane per operand at BK 64 (2 weight pieces per wave per region, vmcnt(8)).
// Per-block anatomy (probe, VAR 6; profiles/r06/wide_tile_anatomy_r06l.jsonl): 2,143-2,365 cycles per
// k-tile against 2,048 of MFMA issue, a QKV + MLP-in tile 2.6 % prologue / 84 % loop / 13.4 % epilogue.
// TVR_WT_SGB=0 drops the sliced form's sched_group_barriers (A/B of the placement)
#ifndef TVR_WT_SGB
#define TVR_WT_SGB 1
#endif
template <int EPI, int FMT, bool VEC, int VAR, bool SL, bool TWO = false>
__device__ __forceinline__ void pp_tile_wt(const uint16_t* __restrict__ A, int lda, size_t aps,
                                           const uint16_t* __restrict__ W, int ldw, float acc_scale, int M, int N,
                                           const GemmEpi& ep, int m0, int n0, int kbeg, int nk, float* part,
                                           int has_part, unsigned long long st0, unsigned long long sr0) {
  // FMT: ACT_X2F16 with one exact weight plane (two activation planes, BK 32), or one bf16 / fp16 plane of each
  // operand (BK 64: the fragments' second index is the k-group instead of the plane); both 2 A fragments per
  // 16-row tile per k-tile, the weight 1 (x2f16) or 2 (bf16 / fp16) per 16-column tile
  using F = PlanarFmt<FMT>;
  using frag = typename F::frag;
  constexpr int NPL = F::NPL;          // activation planes (2 x2f16, 1 bf16 / fp16)
  constexpr int BK = F::BK;            // halves per plane row per k-tile: 128 B of K in both forms
  constexpr int KG = BK / 32;          // k-groups (fragments along K) per k-tile
  constexpr int CPR = BK / 8;          // 16-B chunks per plane row
  constexpr int RPP = 64 / CPR;        // rows per 1 KB piece
  constexpr int PPP = 128 / RPP;       // pieces per plane per region
  constexpr int WP = PPP / 8;          // weight pieces per wave per region (1 x2f16, 2 bf16)
  constexpr int PL = 256 * BK;         // halves per plane per buffer
  constexpr int BUF = (NPL + 1) * PL;  // activation planes + one weight plane
  constexpr int NBUF = TWO ? 3 : 2;    // TWO: the two-phase loop's three buffers (below)
  static_assert(!TWO || FMT == ACT_X2F16, "three 64 KB bf16 buffers do not fit the LDS");
  static_assert(NPL * KG == 2, "two A fragments per 16-row tile per k-tile");
  static_assert(!SL || FMT == ACT_X2F16, "the sliced accumulation is an x2f16 form");
  // vmcnt of every phase: the pieces issued after the awaited region (two activation regions of 2 pieces and
  // two weight regions of WP per k-tile; four phases: 4 + 2 WP, the prologue's first wait 4 + 3 WP)
  constexpr int VM = 4 + 2 * WP, VM0 = 4 + 3 * WP;
  constexpr int DUMMY = NBUF * BUF;
  constexpr int LDS_HALVES = (NBUF * BUF + 512) > PP_EPI_LDS ? (NBUF * BUF + 512) : PP_EPI_LDS;
  static_assert(LDS_HALVES * 2 <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint16_t lds[LDS_HALVES];

  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  const int wave = t >> 6, lane = t & 63;
  const int wr = wave >> 1, wc = wave & 1;
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  const uint16_t* Ab = ep.a2 != nullptr && n0 >= ep.a2_col ? ep.a2 : A;

  // staging map: region R (0 A_lo, 1 A_hi, 2 W_lo, 3 W_hi); A regions 2 pieces per wave, W regions 1
  const uint16_t* src[4][2];
  int dst[4][2];
#pragma unroll
  for (int R = 0; R < 4; ++R) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int pi = R >= 2 ? WP * wave_s + (WP > 1 ? s : 0) : 2 * wave_s + s;
      const int plane = pi / PPP, x0 = (pi % PPP) * RPP;  // region row of the piece's first row
      const int trow0 = R < 2 ? ((x0 >> 5) << 6) + (x0 & 31) + 32 * R : ((x0 >> 6) << 7) + (x0 & 63) + 64 * (R - 2);
      const int row = trow0 + lane / CPR;
      const int chunk = (lane % CPR) ^ planar_g<CPR>(row);
      if (R < 2) {
        const int am = min(m0 + row, M - 1);
        src[R][s] = Ab + plane * aps + (size_t)(ep.a_rows ? ep.a_rows[am] : am) * lda + chunk * 8;
        dst[R][s] = plane * PL + trow0 * BK;
      } else {
        src[R][s] = W + (size_t)min(n0 + row, N - 1) * ldw + chunk * 8;
        dst[R][s] = NPL * PL + trow0 * BK;
      }
    }
  }
  auto stage = [&](int R, int kt) {
    const bool live = kt < nk;
    const int koff = live ? (kbeg + kt) * BK : 0;
    const int boff = (TWO ? kt % 3 : kt & 1) * BUF;
#pragma unroll
    for (int s = 0; s < (R >= 2 ? WP : 2); ++s) glds16(src[R][s] + koff, lds + (live ? boff + dst[R][s] : DUMMY));
  };

  // fragment offsets: fragment f (x2f16: plane f; bf16: k-group f) of the wave's first row tile, k-group g of
  // the weight plane at its first column tile
  int aoff[2], woff[KG];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int p = NPL == 2 ? f : 0, g = NPL == 2 ? 0 : f;
    const int ra = wr * 64 + (lane & 15), c = 4 * g + (lane >> 4);
    aoff[f] = p * PL + ra * BK + ((c ^ planar_g<CPR>(ra)) << 3);
  }
#pragma unroll
  for (int g = 0; g < KG; ++g) {
    const int rb = wc * 128 + (lane & 15), c = 4 * g + (lane >> 4);
    woff[g] = NPL * PL + rb * BK + ((c ^ planar_g<CPR>(rb)) << 3);
  }

  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{};
  frag fa[4][2], fw[8][KG];

  // live 16-row slices of the wave's 64 rows (rows past M are copies of row M - 1): the PART loop skips the
  // padding slices' fragment reads and MFMAs (staging and barriers stay)
  const int vi = __builtin_amdgcn_readfirstlane(min(4, max(0, (M - m0 - wr * 64 + 15) >> 4)));
  auto read_a = [&](const uint16_t* base, int i0, auto part) {
#pragma unroll
    for (int i = i0; i < i0 + 2; ++i)
      if (!decltype(part)::value || i < vi)
#pragma unroll
        for (int f = 0; f < 2; ++f) fa[i][f] = *(const frag*)(base + aoff[f] + i * 16 * BK);
  };
  auto read_w = [&](const uint16_t* base, int j0, auto part) {
    if (decltype(part)::value && vi == 0) return;
#pragma unroll
    for (int j = j0; j < j0 + 4; ++j)
#pragma unroll
      for (int g = 0; g < KG; ++g) fw[j][g] = *(const frag*)(base + woff[g] + j * 16 * BK);
  };
  [[maybe_unused]] f32x4 tc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  // one phase's cluster: row tiles i0, i0 + 1 x column tiles j0 .. j0 + NJ - 1 (4, or 8 in the two-phase
  // loop), two products each
  constexpr int NJ = TWO ? 8 : 4, NP = NJ / 2;  // column tiles, tile pairs per row
  auto cluster = [&](int i0, int j0, auto part, int ci, int cj) {
    if constexpr (SL && !decltype(part)::value) {
      // sliced: tile pairs (i, j..j+1) in turn, the two tiles' chains interleaved (a1 w0 of both, then a0 w0
      // of both), two of the previous pair's 8 slice-sum adds after each MFMA; the cluster's last pair is
      // carried into the next phase (tc) — pp_tile's form 2
      f32x4 s[2][2];  // pair q's slice sums in s[q & 1] (the previous pair's are added while it runs)
#pragma unroll
      for (int q = 0; q < 2 * NP; ++q) {
        const int i = i0 + q / NP, j = j0 + 2 * (q % NP);  // pair q: tiles (i, j), (i, j + 1)
        const int pi = q == 0 ? ci : i0 + (q - 1) / NP, pj = q == 0 ? cj : j0 + 2 * ((q - 1) % NP);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int jj = u & 1, pz = u >> 1;  // MFMA u: product pz (0: a1 w0, 1: a0 w0) of tile (i, j + jj)
          s[q & 1][jj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j + jj][0], fa[i][pz == 0 ? 1 : 0],
                                                                 pz == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : s[q & 1][jj],
                                                                 0, 0, 0);
          if (TVR_WT_SGB) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
#pragma unroll
          for (int e = 2 * u; e < 2 * u + 2; ++e)
            acc[pi][pj + (e >> 2)][e & 3] += q == 0 ? tc[e >> 2][e & 3] : s[(q - 1) & 1][e >> 2][e & 3];
          if (TVR_WT_SGB) __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
        if (NP == 4 && q == NP - 1) __builtin_amdgcn_sched_barrier(0);  // two-phase: schedule each row's pairs apart
      }
      tc[0] = s[(2 * NP - 1) & 1][0];
      tc[1] = s[(2 * NP - 1) & 1][1];
      return;
    }
#pragma unroll
    for (int i = i0; i < i0 + 2; ++i)
#pragma unroll
      for (int j = j0; j < j0 + NJ; ++j) {
        if (decltype(part)::value && i >= vi) continue;
        f32x4 c = acc[i][j];
        if constexpr (SL) {
          f32x4 s = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][0], fa[i][1], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          s = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][0], fa[i][0], s, 0, 0, 0);
          c = slice_add(c, s);
        } else if constexpr (FMT == ACT_X2F16) {
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][0], fa[i][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][0], fa[i][0], c, 0, 0, 0);
        } else if constexpr (FMT == ACT_F16) {  // k-group 0, then 1 (pp_tile's order)
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][0], fa[i][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fw[j][KG - 1], fa[i][1], c, 0, 0, 0);
        } else {
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[j][0], fa[i][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[j][KG - 1], fa[i][1], c, 0, 0, 0);
        }
        acc[i][j] = c;
      }
  };
  constexpr bool prio = !SL;
#define TVR_PP_CLUSTER(...)                  \
  __builtin_amdgcn_s_barrier();              \
  __builtin_amdgcn_sched_barrier(0);         \
  if (prio) __builtin_amdgcn_s_setprio(1);   \
  __VA_ARGS__;                               \
  if (prio) __builtin_amdgcn_s_setprio(0);   \
  __builtin_amdgcn_sched_barrier(0);         \
  __builtin_amdgcn_s_barrier();              \
  __builtin_amdgcn_sched_barrier(0)

  // prologue, the loop's stage history.  Four phases: A_lo(0) W_lo(0) W_hi(0) A_hi(0) A_lo(1) W_lo(1) W_hi(1),
  // retire A_lo(0) / W_lo(0) (7 pieces issued after them).  Two phases: A_lo W_lo A_hi W_hi of k-tiles 0 and
  // 1, retire k-tile 0 (6 pieces after W_hi(0)).  Then read A_lo(0): the last phase's read of k-tile -1
  if constexpr (TWO) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      stage(0, k);
      stage(2, k);
      stage(1, k);
      stage(3, k);
    }
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    stage(0, 0);
    stage(2, 0);
    stage(3, 0);
    stage(1, 0);
    stage(0, 1);
    stage(2, 1);
    stage(3, 1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM0) : "memory");
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (vi == 4)
    read_a(lds, 0, std::integral_constant<bool, false>{});
  else
    read_a(lds, 0, std::integral_constant<bool, true>{});
  if (wr >= 2) {  // the group offset: waves 4-7 run one barrier behind
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  unsigned long long d_loop0 = 0, d_loop1 = 0;
  if constexpr (VAR == 6 || VAR == 8) d_loop0 = __builtin_amdgcn_s_memtime();
  auto kloop = [&](auto part) {
    if constexpr (TWO) {
      // Two phases per k-tile, 32 MFMAs each, three LDS buffers (k-tile t in buffer t % 3):
      //   P1  rows 0-31 x all 128 cols   reads W_lo, W_hi(t)          stages A_lo(t+2), W_lo(t+2)  (3 pieces)
      //   P2  rows 32-63 x all 128 cols  reads A_hi(t), A_lo(t+1)     stages A_hi(t+2), W_hi(t+2)  (3 pieces)
      // Each region is restaged >= 2 phases after its last read (buffer t % 3 held k-tile t - 1... t - 3's
      // regions, last read >= 2 phases before) and retired one phase before its first read, >= 2 phases (of
      // ~512 MFMA cycles) after its issue: vmcnt(4) in P1 (A_lo(t+1), A_hi(t): 4 pieces issued after
      // A_lo(t+1)), vmcnt(3) in P2 (W_hi(t+1): 3 after it)
      for (int kt = 0; kt < nk; ++kt) {
        const uint16_t* cur = lds + (kt % 3) * BUF;
        read_w(cur, 0, part);
        read_w(cur, 4, part);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // A_lo(kt+1) (P1 of kt-1), A_hi(kt): read in P2
        stage(0, kt + 2);
        stage(2, kt + 2);
        TVR_PP_CLUSTER(cluster(0, 0, part, 3, 6));  // the previous cluster's carried pair: tiles (3, 6..7)
        read_a(cur, 2, part);
        read_a(lds + ((kt + 1) % 3) * BUF, 0, part);
        asm volatile("s_waitcnt vmcnt(3)" ::: "memory");  // W_hi(kt+1) (P2 of kt-1), W_lo(kt+1): read in P1
        stage(1, kt + 2);
        stage(3, kt + 2);
        TVR_PP_CLUSTER(cluster(2, 0, part, 1, 6));
      }
      return;
    }
    for (int kt = 0; kt < nk; ++kt) {
      const uint16_t* cur = lds + (kt & 1) * BUF;
      // q1: rows 0-31 x cols 0-63
      read_w(cur, 0, part);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");  // W_hi(kt) (q4 of kt-2), read in q2
      stage(1, kt + 1);
      TVR_PP_CLUSTER(cluster(0, 0, part, 3, 2));  // (ci, cj): the previous phase's carried pair (q4: tiles (3, 2..3))
      // q2: rows 0-31 x cols 64-127
      read_w(cur, 4, part);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");  // A_hi(kt) (q1 of kt-1), read in q3
      stage(0, kt + 2);
      TVR_PP_CLUSTER(cluster(0, 4, part, 1, 2));
      // q3: rows 32-63 x cols 64-127
      read_a(cur, 2, part);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");  // A_lo(kt+1) (q2 of kt-1), read in q4
      stage(2, kt + 2);
      TVR_PP_CLUSTER(cluster(2, 4, part, 1, 6));
      // q4: rows 32-63 x cols 0-63; reads the next k-tile's A_lo (its cluster needs nothing read here)
      read_a(lds + ((kt + 1) & 1) * BUF, 0, part);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");  // W_lo(kt+1) (q3 of kt-1), read in q1
      stage(3, kt + 2);
      TVR_PP_CLUSTER(cluster(2, 0, part, 3, 6));
    }
  };
  if (vi == 4) {
    kloop(std::integral_constant<bool, false>{});
    if constexpr (SL) {  // the last cluster's carried pair (q4: tiles (3, 2..3); two-phase: (3, 6..7))
      acc[3][TWO ? 6 : 2] = slice_add(acc[3][TWO ? 6 : 2], tc[0]);
      acc[3][TWO ? 7 : 3] = slice_add(acc[3][TWO ? 7 : 3], tc[1]);
    }
  } else {
    kloop(std::integral_constant<bool, true>{});
  }
#undef TVR_PP_CLUSTER
  if constexpr (VAR == 6 || VAR == 8) d_loop1 = __builtin_amdgcn_s_memtime();
  if (wr < 2) __builtin_amdgcn_s_barrier();  // balance the group offset
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  if constexpr (VEC) {
    __syncthreads();
    float* L = reinterpret_cast<float*>(lds);
    if (has_part) {
      GemmEpi pe = ep;
      pe.out0 = part;
      pe.ld0 = 256;
      pe.out_rows = nullptr;
      pp_epilogue_lds<EPI, FMT, VAR == 8, 4, 8>(pe, acc, L, 0, 0, M - m0, N - n0, wr, wc, lane, t, acc_scale);
    } else {
      pp_epilogue_lds<EPI, FMT, VAR == 8, 4, 8>(ep, acc, L, m0, n0, M - m0, N - n0, wr, wc, lane, t, acc_scale);
    }
    if ((VAR == 6 || VAR == 8) && ep.stamps && t == 0) {
      unsigned long long* o = ep.stamps + 4 * blockIdx.x;
      o[0] = st0;
      o[1] = d_loop0;
      o[2] = d_loop1;
      o[3] = __builtin_amdgcn_s_memtime();
    }
    return;
  }
  if constexpr (EPI == EPI_STATS) {
    return;
  } else {
    if (acc_scale != 1.0f) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] *= acc_scale;
    }
    if (has_part) {
      GemmEpi pe = ep;
      pe.out0 = part;
      pe.ld0 = 256;
      gemm_epilogue16t<EPI, FMT, VEC, 4, 8>(pe, acc, M - m0, N - n0, wr * 64, wc * 128, lane);
    } else {
      gemm_epilogue16t<EPI, FMT, VEC, 4, 8>(ep, acc, M, N, m0 + wr * 64, n0 + wc * 128, lane);
    }
    if (ep.stamps && t == 0) {
      ep.stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - st0;
      ep.stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - sr0;
    }
  }
}

// One tile of a launch: the wide-tile form for one-plane weights (TVR_PP_WX_WIDE 1: four phases, 2: two;
// VAR 16 / 20 force the four / two-phase wide tile, 17 pp_tile), else pp_tile
template <int EPI, int FMT, bool VEC, int VAR, bool SL, bool WX, bool SKM>
__device__ __forceinline__ void pp_tile_any(const uint16_t* __restrict__ A, int lda, size_t aps,
                                            const uint16_t* __restrict__ W, int ldw, size_t wps, float acc_scale,
                                            int M, int N, const GemmEpi& ep, int m0, int n0, int kbeg, int nk,
                                            float* part, int has_part, unsigned long long st0,
                                            unsigned long long sr0) {
  // bf16 / fp16 (one plane each): the wide four-phase tile when TVR_PP_BF16_WIDE (VAR 16 / 17 force it / pp_tile)
  constexpr bool wide = (WX && FMT == ACT_X2F16 &&
                         (VAR == 16 || VAR == 20 || (VAR != 17 && TVR_PP_WX_WIDE && (VAR == 0 || VAR == 6 || VAR == 8)))) ||
                        ((FMT == ACT_BF16 || FMT == ACT_F16) &&
                         (VAR == 16 || (VAR != 17 && TVR_PP_BF16_WIDE && (VAR == 0 || VAR == 6 || VAR == 8))));
  // (the sliced form stays on four phases: the two-phase cluster keeps all 8 weight fragments live through
  // both clusters, 16 VGPRs more than the 252 the sliced four-phase form holds — it spilled 38)
  constexpr bool two = FMT == ACT_X2F16 && (VAR == 20 || (VAR != 16 && TVR_PP_WX_WIDE == 2 && !SL));
  constexpr int V = (VAR == 16 || VAR == 17 || VAR == 20) ? 0 : VAR;
  if constexpr (wide)
    pp_tile_wt<EPI, FMT, VEC, V, SL, two>(A, lda, aps, W, ldw, acc_scale, M, N, ep, m0, n0, kbeg, nk, part, has_part,
                                          st0, sr0);
  else
    // (the q4 prefetch, TVR_PP_PF, not in the stream-K form or the statistics epilogue: their extra VGPRs
    // there spilled 4 / 8)
    pp_tile<EPI, FMT, VEC, V, SL, WX, !SKM && EPI != EPI_STATS>(A, lda, aps, W, ldw, wps, acc_scale, M, N, ep, m0, n0,
                                                                kbeg, nk, part, has_part, st0, sr0);
}

// K must be a multiple of BK (host-checked); any M, N.
// VAR (diagnostic builds, tools/gemm_split_probe): 1 no staging in the loop
// (stale LDS: timing only), 2 no s_setprio, 13 s_setprio 1 once for waves 4-7, 14 the cluster flips in the
// sliced form too, 3 no group offset, 4 no vmcnt
// waits in the loop (racy: timing only), 6 per-block stamps (start, loop
// start, loop end, end) of wave 0 to ep.stamps[4 block + i], 7 the register
// epilogue (no LDS pass), 8 the stamps of 6 with the epilogue's global stores
// skipped (timing only), 12 every k-tile staged from k-tile 0 (L2-hot operands,
// same instruction stream: timing only), 16 / 17 the one-plane wide / narrow wave tile.  SKM: the stream-K form (sk_blocks
// blocks; EPI_BIAS partial tiles only).  SL: x2f16 sliced accumulation (above).  WX: x2f16 activations
// against weights exact in fp16 (one plane staged, two products; pp_tile).
template <int EPI, int FMT, bool VEC = true, int VAR = 0, bool SKM = false, bool SL = false, bool WX = false>
__global__ void __launch_bounds__(PP_THREADS, 1)
gemm_pingpong_kernel(const uint16_t* __restrict__ A, int lda, size_t aps, const uint16_t* __restrict__ W, int ldw,
                     size_t wps, float acc_scale, int M, int N, int K, GemmEpi ep) {
  const unsigned long long st0 = ep.stamps ? __builtin_amdgcn_s_memtime() : 0;  // clock diagnostics
  const unsigned long long sr0 = ep.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
  const int nbm = (M + 255) >> 8, nbn = (N + 255) >> 8;
  const int nk_all = K / PlanarFmt<FMT>::BK;
  const int gm = ep.group_m > 0 ? ep.group_m : GEMM_GROUP_M;
  // XCD-aware bijective remap: the blocks of one XCD (b = x mod 8) take a
  // contiguous range of logical indices, so neighbouring tiles (and a
  // stream-K tile's consecutive contributors) share that XCD's L2
  auto remap = [](int bid, int nwg) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  };
  const int count = ep.tile_count > 0 ? ep.tile_count : nbm * nbn;
  if constexpr (SKM) {
    // stream-K: block g takes the k-iterations [g I / G, (g + 1) I / G) of
    // the launch's tiles, at most two segments (G >= tiles).  A template of its
    // own: the segment loop around the K loop costs VGPRs the plain launches
    // (one segment, no loop) must not pay.
    const int G = ep.sk_blocks;
    const int g = remap(blockIdx.x, G);
    const long long I = (long long)count * nk_all;
    long long it = (long long)g * I / G;
    const long long it1 = (long long)(g + 1) * I / G;
    // the (at most) two segments as straight-line code: a loop around the
    // K loop kept its state live across iterations (68-83 VGPRs spilled)
    auto segment = [&](int seg) {
      const int lt = (int)(it / nk_all);
      const int kbeg = (int)(it - (long long)lt * nk_all);
      const int nk = (int)min((long long)(nk_all - kbeg), it1 - it);
      int m0, n0;
      pp_tile_coords(ep.tile_base + lt, nbm, nbn, m0, n0, gm);
      pp_tile_any<EPI, FMT, VEC, VAR, SL, WX, SKM>(A, lda, aps, W, ldw, wps, acc_scale, M, N, ep, m0, n0, kbeg, nk,
                                  ep.out0 + ((size_t)2 * g + seg) * PP_TILE_ELEMS, 1, st0, sr0);
      it += nk;
    };
    segment(0);
    if (it < it1) segment(1);
  } else {
    // this launch: tiles [tile_base, tile_base + count) of the grouped raster,
    // each split over S k-ranges (block = (tile, split))
    const int S = ep.k_split > 1 ? ep.k_split : 1;
    const int wgs = remap(blockIdx.x, count * S);
    const int lt = wgs / S, split = wgs - lt * S;
    int m0, n0;
    pp_tile_coords(ep.tile_base + lt, nbm, nbn, m0, n0, gm);
    const int kbeg = (int)((long long)split * nk_all / S);
    const int nk = (int)((long long)(split + 1) * nk_all / S) - kbeg;  // this block's k-tiles
    pp_tile_any<EPI, FMT, VEC, VAR, SL, WX, SKM>(A, lda, aps, W, ldw, wps, acc_scale, M, N, ep, m0, n0, kbeg, nk,
                                ep.out0 + ((size_t)split * count + lt) * PP_TILE_ELEMS, S > 1, st0, sr0);
  }
}

// Sum of the k_split partial tiles [S][count][256][256] (fixed order:
// deterministic) + bias, then the launch's real epilogue on four consecutive
// columns per thread (N, ld0 and the epilogue strides multiples of 4:
// host-checked).  Tiles [tile_base, tile_base + count) of the raster.
template <int EPI, int FMT>
__global__ void __launch_bounds__(256)
splitk_reduce_kernel(const float* __restrict__ part, int S, int tile_base, int count, int M, int N, GemmEpi ep) {
  const int nbm = (M + 255) >> 8, nbn = (N + 255) >> 8;
  const size_t total = (size_t)count * (PP_TILE_ELEMS / 4);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int lt = (int)(i / (PP_TILE_ELEMS / 4)), e = (int)(i % (PP_TILE_ELEMS / 4)) * 4;
    int m0, n0;
    pp_tile_coords(tile_base + lt, nbm, nbn, m0, n0, ep.group_m > 0 ? ep.group_m : GEMM_GROUP_M);
    const int m = m0 + (e >> 8), c = n0 + (e & 255);
    if (m >= M || c >= N) continue;
    const float* p = part + (size_t)lt * PP_TILE_ELEMS + e;
    f32x4 v = *(const f32x4*)p;
    for (int s = 1; s < S; ++s) v += *(const f32x4*)(p + (size_t)s * count * PP_TILE_ELEMS);
    if (ep.bias) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += ep.bias[c + r];
    }
    const size_t orow = ep.out_rows ? (size_t)ep.out_rows[m] : (size_t)m;
    epi_store4<EPI, FMT>(ep, orow, c, v);
  }
}

// Stream-K fix-up: tile lt's k-iterations [lt KT, (lt + 1) KT) were covered by
// the blocks g = b0 .. b1 (block g holds [floor(g I / G), floor((g + 1) I / G)),
// so the block holding iteration x is floor(((x + 1) G - 1) / I)); each left
// its share in slot 1 if it began in an earlier tile, else slot 0.  Summed in
// block (= k) order: deterministic.  Then bias + the launch's epilogue, four
// consecutive columns per thread (host-checked as splitk_reduce_kernel).
template <int EPI, int FMT>
__global__ void __launch_bounds__(256)
splitk_sk_reduce_kernel(const float* __restrict__ part, int G, int KT, int tile_base, int count, int M, int N,
                        GemmEpi ep) {
  const int nbm = (M + 255) >> 8, nbn = (N + 255) >> 8;
  const long long I = (long long)count * KT;
  const size_t total = (size_t)count * (PP_TILE_ELEMS / 4);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int lt = (int)(i / (PP_TILE_ELEMS / 4)), e = (int)(i % (PP_TILE_ELEMS / 4)) * 4;
    int m0, n0;
    pp_tile_coords(tile_base + lt, nbm, nbn, m0, n0, ep.group_m > 0 ? ep.group_m : GEMM_GROUP_M);
    const int m = m0 + (e >> 8), c = n0 + (e & 255);
    if (m >= M || c >= N) continue;
    const long long x0 = (long long)lt * KT, x1 = x0 + KT - 1;
    const int b0 = (int)(((x0 + 1) * G - 1) / I), b1 = (int)(((x1 + 1) * G - 1) / I);
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    for (int b = b0; b <= b1; ++b) {
      const int slot = ((long long)b * I / G) < x0 ? 1 : 0;
      v += *(const f32x4*)(part + ((size_t)2 * b + slot) * PP_TILE_ELEMS + e);
    }
    if (ep.bias) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += ep.bias[c + r];
    }
    const size_t orow = ep.out_rows ? (size_t)ep.out_rows[m] : (size_t)m;
    epi_store4<EPI, FMT>(ep, orow, c, v);
  }
}

}  // namespace tvr

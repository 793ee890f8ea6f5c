// attention_mfma.hpp — causal attention of short ragged sequences on the fp32
// matrix cores: one wave per (sequence, head), no LDS, no block barriers.
//
// The patched forwards attend over T <= 128 positions (T = 15 at C3, 33 at
// C5) with d_head <= 128.  Per (sequence, head) and 16-query tile:
//   S^T = K Q^T    v_mfma_f32_16x16x4_f32, D[key][query]: lane l holds the
//                  scores of query l&15 against keys 4(l>>4)+r, r = 0..3
//   causal softmax per query (in-lane over r, then xor-16/32 shuffles)
//   Z^T = V^T P^T  the S^T accumulator IS the B operand: in k step r lane
//                  group g supplies key 4g + r, so V is read in that order;
//                  D[dim][query]: lane l holds 4 consecutive dims of query
//                  l&15 -> one 16-B store (fp32) / 8-B stores (activation
//                  formats).
// K, Q and V fragments are loaded from global memory straight into registers.
// Lane group g owns dims [g DH/4, (g+1) DH/4) of Q and K (contiguous float4
// loads); the rotary pairs (i, i + rd/2) with rd = DH/4 (every Pythia:
// rotary_pct 0.25; the host checks it) stay inside lane group 0, at
// compile-time register indices.  f32-input MFMA is exact fp32
// (a k-ordered fmaf chain per step); the dot products are summed in a permuted
// k order relative to a sequential loop, i.e. within fp32 rounding of the
// TransformerLens attention (oracle/hooked_pythia.py _attn):
// scores q.k / sqrt(d_head), -inf causal mask, fp32 softmax, z = P V.
// (It replaced an LDS-staged block-per-(sequence, head) kernel, 1.21 -> 0.45
// ms per launch at C3: DESIGN.md section 3.3.)
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gemm_planar.hpp"
#include "kernels.hpp"
#include "split.hpp"

namespace tvr {

constexpr int ATTM_WAVES = 4;  // (sequence, head) pairs per block

// E consecutive floats at a 4-B-aligned address as 16-B loads + the rest (global_load_dwordx4 needs only
// dword alignment): a lane's E = 5 dims were five 4-B loads, each instruction touching all 20 lines of the
// wave's 1,280-B span — the kernel ran at the TA's line rate (C2: 30 us per launch at 1,768 rows)
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
template <int E>
__device__ __forceinline__ void load_span(const float* __restrict__ p, float (&x)[E]) {
#pragma unroll
  for (int i = 0; i + 4 <= E; i += 4) {
    const f32x4u v = *(const f32x4u*)(p + i);
    x[i] = v[0];
    x[i + 1] = v[1];
    x[i + 2] = v[2];
    x[i + 3] = v[3];
  }
#pragma unroll
  for (int i = E & ~3; i < E; ++i) x[i] = p[i];
}

// The P V product's dimension order (TVR_ATT_VPERM, default 0).  Output tile dt of Z^T = V^T P^T holds the
// dims d(i, dt) of its 16 rows i: 0 -> d = 16 dt + i (NDT 4-B loads per key row and lane, 64 B per row per
// instruction; a lane's z values are 4-dim groups 16 dt + 4 g, so a store instruction writes 32-B (planes)
// / 64-B (fp32) row runs); 1 -> d = NDT i + dt, so lane (li, g) reads the NDT CONSECUTIVE floats
// V[key][NDT li ..] of a key row (16-B loads) and ends with the DH / 4 consecutive dims [g DH / 4, (g + 1)
// DH / 4) of its query, whose direct stores are 8-B pieces 64 B apart.  Every output element sums the same
// products over the same keys in the same order either way (bit-identical), but 1 measured slower where z is
// stored from registers: 12B (NKT 4, d_head 128) 4,278 vs 3,810 us per launch, 6.9B (STAGE 3) 2,524 vs
// 2,410; C3 (STAGE 2, z through LDS) 701 vs 702 (profiles/r06/attention_vperm_ab_r06s2c.txt)
#ifndef TVR_ATT_VPERM
#define TVR_ATT_VPERM 0
#endif
constexpr bool ATT_VPERM = TVR_ATT_VPERM;
// Unstaged kernels (ZL, TVR_ATT_ZLDS, default 1): z leaves through a per-wave [16][DH] LDS region (8 KB at
// d_head 128) as the staged forms do — whole-row 16-B stores per plane — instead of one 8-B (planes) /
// 16-B (fp32) store per lane and 4-dim group, 32-B row runs per instruction: 12B (NKT 4, d_head 128)
// 3,819 / 3,735 -> 3,449 / 3,451 us per launch, same box (profiles/r06/attention_zlds_ab_r06s2d.txt)
#ifndef TVR_ATT_ZLDS
#define TVR_ATT_ZLDS 1
#endif

// grid = ceil(n_seqs * n_heads / ATTM_WAVES) blocks of 64 * ATTM_WAVES threads;
// NKT = key tiles the launch's longest sequence needs (1, 2, 4 or 8: the
// register arrays are sized by it), or 0 for longer sequences (up to n_ctx):
// the keys then go in chunks of 8 tiles with an online softmax (running max
// and sum per query, the z accumulator rescaled per chunk) and key tiles past
// the query tile's last position are skipped.  Latency-bound (short dependent
// MFMA chains, global loads): as many waves per SIMD as the fragments allow
// without spilling (4 at one key tile, 3 up to four, else 2).
// zf_last: the fp32 hook_z copy only for each sequence's last row, at row s of
// zf (the extraction's capture reads nothing else), instead of every row;
// otherwise rows below zf_rows only (a fused clean + patch sweep traces its
// clean rows, which come first).
// STAGE (NKT == 1 only: T <= 16, the C3 / C1 sweeps): the wave's Q, K and V
// head slices are first copied into LDS by LDS-DMA (global_load_lds_dwordx4),
// lane l moving 16-B chunk l of a packed [16 rows][DH] image, so each
// instruction reads whole 16-B chunks of consecutive rows' slices (DH * 4 B
// contiguous per row) instead of 16 rows x 4 lane-group chunks, and V's
// fragments come from LDS instead of 4-B global loads; the fragments are then
// read from LDS in the MFMA layout.  No block barrier: each wave owns its
// region and waits for its own DMAs (vmcnt).
// STAGE 2: K and V only (Q loaded directly; 2/3 of the LDS, so 3 blocks per CU).
// STAGE 3 (NKT == 2: 16 < T <= 32, the C4 / 6.9B sweeps): V's 32 rows only, as
// one packed [32][DH] image DMA'd before Q and K are loaded; the PV MFMAs read
// it from LDS instead of 4-B global loads issued after the softmax.
template <int FMT, int DH, int NKT, int STAGE = 0>
__global__ void __launch_bounds__(64 * ATTM_WAVES, STAGE == 1 ? 2 : STAGE == 2 ? 3 : (DH <= 80 && NKT == 1) ? 4 : (DH <= 80 && NKT <= 4 && NKT > 0) ? 3 : 2)
attention_mfma_kernel(const float* __restrict__ qkv, int ldq, const float* __restrict__ cache, int ldc,
                      const SeqDesc* __restrict__ seqs, int n_seqs, int n_heads, void* __restrict__ z, int ldz,
                      float* __restrict__ zf, int ldzf, int zf_last, int zf_rows, unsigned* __restrict__ flag,
                      const float* __restrict__ cos_t, const float* __restrict__ sin_t, int d,
                      float inv_attn_scale) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int CH = DH / 4;    // dims per lane group in Q K^T
  constexpr int NDT = DH / 16;  // 16-dim output tiles
  constexpr bool LONG = NKT == 0;
  constexpr int MAXKT = LONG ? 8 : NKT;
  static_assert(DH % 16 == 0 && DH <= 128 && MAXKT * 16 <= ATT_MAX_T, "d_head / key tiles");
  static_assert(STAGE == 0 || (STAGE <= 2 && NKT == 1) || (STAGE == 3 && NKT == 2), "LDS staging: key tiles");
  constexpr int SMAT = 16 * DH;  // floats of one staged [16][DH] matrix
  // staged matrices (STAGE 3: V's two key tiles); K's offset
  constexpr int NMAT = STAGE == 1 ? 3 : 2, KOFF = STAGE == 1 ? SMAT : 0;
  constexpr bool ZL = TVR_ATT_ZLDS && STAGE == 0;  // z through a per-wave [16][DH] region
  __shared__ __attribute__((aligned(16))) float att_lds[STAGE ? ATTM_WAVES * NMAT * SMAT : ZL ? ATTM_WAVES * SMAT : 4];
  const int lane = threadIdx.x & 63;
  const int pair = blockIdx.x * ATTM_WAVES + (threadIdx.x >> 6);
  if (pair >= n_seqs * n_heads) return;  // a whole wave; nothing below synchronises
  const int s = pair / n_heads, h = pair - s * n_heads;
  const SeqDesc sd = seqs[s];
  const int T = sd.p0 + sd.n;
  const int nkt = (T + 15) >> 4;
  const int li = lane & 15, g = lane >> 4;
  constexpr int rd = CH, half = CH / 2;  // rotary_dim = d_head / 4

  // row of absolute position j: the prefix (clean trace, or a shared-prefix
  // leader's rows of this run), or this sequence's own rows
  const float* pfx = sd.prefix_live ? qkv : cache;
  const int ldp = sd.prefix_live ? ldq : ldc;
  auto row_of = [&](int j) -> const float* {
    return j < sd.p0 ? pfx + (size_t)(sd.cache_row + j) * ldp : qkv + (size_t)(sd.row0 + j - sd.p0) * ldq;
  };
  // dims [g CH, g CH + CH) of a Q or K head row (global or staged), rotated for position pos
  auto load_chunk = [&](const float* r, int pos, float (&x)[CH]) {
#pragma unroll
    for (int c = 0; c < CH; c += 4) {
      const f4 v = *(const f4*)(r + g * CH + c);
      x[c] = v[0];
      x[c + 1] = v[1];
      x[c + 2] = v[2];
      x[c + 3] = v[3];
    }
    if (g == 0) {  // TL rotate-half rotary on dims [0, rd)
#pragma unroll
      for (int i = 0; i < half; ++i) {
        const float x0 = x[i], x1 = x[i + half];
        x[i] = x0 * cos_t[pos * rd + i] - x1 * sin_t[pos * rd + i];
        x[i + half] = x1 * cos_t[pos * rd + i + half] + x0 * sin_t[pos * rd + i + half];
      }
    }
  };

  // the lane's NDT A-operand values of the P V product from V row vrow (&V[key][h DH], global or staged)
  auto load_v = [&](const float* vrow, float (&x)[NDT]) {
    if constexpr (ATT_VPERM) {
      load_span<NDT>(vrow + NDT * li, x);
    } else {
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) x[dt] = vrow[16 * dt + li];
    }
  };

  float* stg = att_lds + (STAGE ? (threadIdx.x >> 6) * NMAT * SMAT : ZL ? (threadIdx.x >> 6) * SMAT : 0);
  if constexpr (STAGE == 3) {
    // V's rows 0 .. 31 (clamped to T - 1) as a packed [32][DH] image, issued before Q and K are loaded so
    // its latency hides behind theirs and the QK^T / softmax; waited for (vmcnt) before the first PV MFMA
#pragma unroll
    for (int i = 0; i < DH / 8; ++i) {
      const int id = i * 64 + lane, row = id / CH, c = id - row * CH;
      glds16(row_of(min(row, T - 1)) + 2 * d + h * DH + 4 * c, stg + i * 256);
    }
  } else if constexpr (STAGE != 0) {
    // rows: Q = the query tile's rows (padding repeats the last), K / V = keys 0 .. 15 (clamped to T - 1);
    // instruction i of matrix m moves chunks 64 i + lane = (row, c) of the packed image
#pragma unroll
    for (int mat = STAGE == 1 ? 0 : 1; mat < 3; ++mat) {
#pragma unroll
      for (int i = 0; i < DH / 16; ++i) {
        const int id = i * 64 + lane, row = id / CH, c = id - row * CH;
        const float* src = mat == 0 ? qkv + (size_t)(sd.row0 + min(sd.q0 + row, sd.n - 1)) * ldq
                                    : row_of(min(row, T - 1)) + mat * d;
        glds16(src + h * DH + 4 * c, stg + (mat - (STAGE == 1 ? 0 : 1)) * SMAT + i * 256);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  for (int q0 = sd.q0; q0 < sd.n; q0 += 16) {
    // this lane's query column: relative row q0 + li (padding reuses the last row)
    const int qi = min(q0 + li, sd.n - 1);
    float qf[CH];
    if constexpr (STAGE == 1)
      load_chunk(stg + li * DH, sd.p0 + qi, qf);  // T <= 16: one query tile, staged from q0
    else
      load_chunk(qkv + (size_t)(sd.row0 + qi) * ldq + h * DH, sd.p0 + qi, qf);
    f4 zt[NDT];
    if constexpr (LONG) {
      const int qpos = sd.p0 + q0 + li;  // this lane's query (absolute position)
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) zt[dt] = f4{0.f, 0.f, 0.f, 0.f};
      // running max / sum of this lane's query over the chunks of keys so far
      float m_run = -INFINITY, l_run = 0.f;
      // key tiles this query tile sees (causal): through its last row's position
      const int kt_end = min(nkt, (sd.p0 + min(q0 + 15, sd.n - 1)) / 16 + 1);
      for (int kb = 0; kb < kt_end; kb += MAXKT) {
        f4 st[MAXKT];
#pragma unroll
        for (int kt = 0; kt < MAXKT; ++kt) {
          st[kt] = f4{0.f, 0.f, 0.f, 0.f};
          if (kb + kt < kt_end) {
            const int kj = min(16 * (kb + kt) + li, T - 1);
            float kf[CH];
            load_chunk(row_of(kj) + d + h * DH, kj, kf);
            f4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < CH; c += 2) {
              a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[c], qf[c], a0, 0, 0, 0);
              a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[c + 1], qf[c + 1], a1, 0, 0, 0);
            }
            st[kt] = a0 + a1;
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        float mx = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < MAXKT; ++kt) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = 16 * (kb + kt) + 4 * g + r;
            const float v = (kb + kt < kt_end && key <= qpos && key < T) ? st[kt][r] * inv_attn_scale : -INFINITY;
            st[kt][r] = v;
            mx = fmaxf(mx, v);
          }
        }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        // online softmax: rescale what the earlier chunks accumulated (key 0 is in
        // the first chunk of every query, so m_new is finite from there on)
        const float m_new = fmaxf(m_run, mx);
        const float scale = m_run == -INFINITY ? 0.f : expf(m_run - m_new);
        m_run = m_new;
        float sum = 0.f;
#pragma unroll
        for (int kt = 0; kt < MAXKT; ++kt) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = st[kt][r] == -INFINITY ? 0.f : expf(st[kt][r] - m_new);
            st[kt][r] = e;
            sum += e;
          }
        }
        sum += __shfl_xor(sum, 16, 64);
        sum += __shfl_xor(sum, 32, 64);
        l_run = l_run * scale + sum;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) zt[dt] *= scale;
#pragma unroll
        for (int kt = 0; kt < MAXKT; ++kt) {
          if (kb + kt < kt_end) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float vf[NDT];
              load_v(row_of(min(16 * (kb + kt) + 4 * g + r, T - 1)) + 2 * d + h * DH, vf);
#pragma unroll
              for (int dt = 0; dt < NDT; ++dt)
                zt[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf[dt], st[kt][r], zt[dt], 0, 0, 0);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      // zt[dt]: dims of query li (D[dim][query li]); l_run is that query's softmax sum
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) zt[dt] /= l_run;
    } else {
      // one key tile (T <= 16, the C3 sweeps): V's fragments are loaded with Q and
      // K, so the wave pays one global-memory latency instead of two
      constexpr int VP = NKT == 1 ? 4 : 1, VPD = NKT == 1 ? NDT : 1;
      float vpre[VP][VPD];
      if constexpr (NKT == 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          load_v(STAGE ? stg + KOFF + SMAT + (4 * g + r) * DH : row_of(min(4 * g + r, T - 1)) + 2 * d + h * DH,
                 vpre[r]);
        }
      }

      // causal key tiles of this query tile: through its last row's position.  A tile past it is masked for
      // every query of the tile (exp(-inf) = 0 in the softmax, P V adds exact zeros), so skipping its QK^T
      // and PV products leaves every result bit-identical (the LONG path's kt_end): at T = 33 (C5) the three
      // query tiles need 1 / 2 / 3 key tiles, 6 of the 9 products; at T = 23 (C4) 3 of 4
      const int nkq = min(nkt, (sd.p0 + min(q0 + 15, sd.n - 1)) / 16 + 1);
      f4 st[MAXKT];
#pragma unroll
      for (int kt = 0; kt < MAXKT; ++kt) {
        st[kt] = f4{0.f, 0.f, 0.f, 0.f};
        if (kt < nkq) {
          const int kj = min(16 * kt + li, T - 1);
          float kf[CH];
          if constexpr (STAGE == 1 || STAGE == 2)
            load_chunk(stg + KOFF + li * DH, kj, kf);  // staged row li = key min(li, T - 1)
          else
            load_chunk(row_of(kj) + d + h * DH, kj, kf);
          // two accumulation chains (16x16x4 f32: 32-cycle issue, 40-cycle dependent latency)
          f4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int c = 0; c < CH; c += 2) {
            a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[c], qf[c], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[c + 1], qf[c + 1], a1, 0, 0, 0);
          }
          st[kt] = a0 + a1;
        }
        // one key tile's fragments live at a time (hoisting every tile's loads spills)
        __builtin_amdgcn_sched_barrier(0);
      }
      // causal softmax over keys 16kt + 4g + r for the query at absolute position qpos
      const int qpos = sd.p0 + q0 + li;
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < MAXKT; ++kt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = 16 * kt + 4 * g + r;
          const float v = (kt < nkq && key <= qpos && key < T) ? st[kt][r] * inv_attn_scale : -INFINITY;
          st[kt][r] = v;
          mx = fmaxf(mx, v);
        }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      float sum = 0.f;
#pragma unroll
      for (int kt = 0; kt < MAXKT; ++kt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = st[kt][r] == -INFINITY ? 0.f : expf(st[kt][r] - mx);
          st[kt][r] = e;
          sum += e;
        }
      }
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
#pragma unroll
      for (int kt = 0; kt < MAXKT; ++kt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) st[kt][r] = st[kt][r] / sum;
      }

      if constexpr (STAGE == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // V's image has landed
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) zt[dt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < MAXKT; ++kt) {
        if (kt < nkq) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if constexpr (NKT == 1) {
#pragma unroll
              for (int dt = 0; dt < NDT; ++dt)
                zt[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(vpre[r][dt], st[kt][r], zt[dt], 0, 0, 0);
            } else if constexpr (STAGE == 3) {
              float vf[NDT];
              load_v(stg + (16 * kt + 4 * g + r) * DH, vf);  // staged row = key min(., T - 1)
#pragma unroll
              for (int dt = 0; dt < NDT; ++dt)
                zt[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf[dt], st[kt][r], zt[dt], 0, 0, 0);
            } else {
              float vf[NDT];
              load_v(row_of(min(16 * kt + 4 * g + r, T - 1)) + 2 * d + h * DH, vf);  // P = 0 past T
#pragma unroll
              for (int dt = 0; dt < NDT; ++dt)
                zt[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf[dt], st[kt][r], zt[dt], 0, 0, 0);
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // the lane's output in 4-dim groups c: VPERM dims g DH / 4 + 4 c .. + 3 (zt[dt][r] is dim NDT (4 g + r) + dt),
    // else dims 16 c + 4 g .. + 3 (zt[c])
    auto zgroup = [&](int c) -> f4 {
      if constexpr (ATT_VPERM) {
        f4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = zt[(4 * c + e) % NDT][(4 * c + e) / NDT];
        return v;
      } else {
        return zt[c];
      }
    };
    auto zcol = [&](int c) { return ATT_VPERM ? g * (DH / 4) + 4 * c : 16 * c + 4 * g; };
    if constexpr (STAGE == 1 || STAGE == 2 || ZL) {
      // z through the wave's first staged region (Q or K: read above; ZL its own): then each lane stores 8 consecutive
      // dims of one row (one 16-B store per plane), so a row's DH dims leave as one contiguous run per plane
      if constexpr (ZL) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous query tile's z reads
#pragma unroll
      for (int c = 0; c < NDT; ++c) *(f4*)(stg + li * DH + zcol(c)) = zgroup(c);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      constexpr int C8 = DH / 8;  // 8-dim chunks per row
      for (int id = lane; id < 16 * C8; id += 64) {
        const int r = id / C8, c = id - r * C8;
        if (q0 + r >= sd.n) continue;
        const float* src = stg + r * DH + 8 * c;
        const f4 a = *(const f4*)src, b = *(const f4*)(src + 4);
        const size_t zrow = (size_t)(sd.row0 + q0 + r);
        const int col = h * DH + 8 * c;
        if constexpr (FMT != ACT_F32) {
          const float v8[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
          store_act8<FMT>((uint16_t*)z + zrow * 2 * ldz + col, ldz, v8, flag);
        } else {
          *(f4*)((float*)z + zrow * ldz + col) = a;
          *(f4*)((float*)z + zrow * ldz + col + 4) = b;
        }
        float* zd = nullptr;
        if (zf && !zf_last && zrow < (size_t)zf_rows) zd = zf + zrow * ldzf + col;
        if (zf && zf_last && q0 + r == sd.n - 1) zd = zf + (size_t)s * ldzf + col;
        if (zd) {
          *(f4*)zd = a;
          *(f4*)(zd + 4) = b;
        }
      }
    } else if (q0 + li < sd.n) {
      const size_t zrow = (size_t)(sd.row0 + q0 + li);
#pragma unroll
      for (int c = 0; c < NDT; ++c) {
        const int col = h * DH + zcol(c);
        const f4 v = zgroup(c);
        if constexpr (FMT != ACT_F32)
          store_act4<FMT>((uint16_t*)z + zrow * 2 * ldz + col, ldz, v[0], v[1], v[2], v[3], flag);
        else
          *(f4*)((float*)z + zrow * ldz + col) = v;
        if (zf && !zf_last && zrow < (size_t)zf_rows) *(f4*)(zf + zrow * ldzf + col) = v;
        if (zf && zf_last && q0 + li == sd.n - 1) *(f4*)(zf + (size_t)s * ldzf + col) = v;
      }
    }
  }
}

}  // namespace tvr

namespace tvr {

// Single-query attention (the patched forwards of last-position sites:
// ADD_ATTN_OUT_LASTPOS / NONE, one computed row per sequence, q0 = n - 1 —
// the C2 layer sweeps, FV evaluations and head-count grid): a 16-query MFMA
// tile per (sequence, head) wastes 15 of its 16 rows there.  Here ONE wave
// serves HG heads of one sequence: lane l holds E = HG DH / 64 consecutive
// dims (head l / (DH / E), chunk l mod (DH / E)), so the query / key / value
// slices of the wave's heads are one contiguous, coalesced load per row; the
// head's q.k is a butterfly over its DH / E lanes, the softmax is online over
// the keys (fp32, the same -inf-free form: every key <= the query), and z goes
// out as one contiguous span per wave.  Rotary (TL rotate-half on dims
// [0, DH / 4)): the partner of dim i (i +- rd / 2) sits in lane l ^ (rd / 2 / E)
// at the same element (E divides rd / 2 for every Pythia head size).
template <int DH>
struct RowAttnShape {
  static constexpr int HG = DH == 128 ? 2 : 4;  // heads per wave
  static constexpr int E = HG * DH / 64;        // dims per lane (16: 1, 64: 4, 80: 5, 128: 4)
  static constexpr int LPH = DH / E;            // lanes per head
};

template <int FMT, int DH>
__global__ void __launch_bounds__(256)
attention_row_kernel(const float* __restrict__ qkv, int ldq, const float* __restrict__ cache, int ldc,
                     const SeqDesc* __restrict__ seqs, int s_begin, int n_seqs, int n_heads, void* __restrict__ z,
                     int ldz, float* __restrict__ zf, int ldzf, int zf_last, int zf_rows, unsigned* __restrict__ flag,
                     const float* __restrict__ cos_t, const float* __restrict__ sin_t, int d, float inv_attn_scale) {
  using S = RowAttnShape<DH>;
  constexpr int E = S::E, LPH = S::LPH, HG = S::HG;
  constexpr int rd = DH / 4, half = rd / 2, OFF = half / E;  // partner lane distance (xor)
  static_assert(half % E == 0 && (OFF & (OFF - 1)) == 0, "rotary pairs must map onto lane pairs");
  const int lane = threadIdx.x & 63;
  const int groups = n_heads / HG;
  const int wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wid >= n_seqs * groups) return;  // a whole wave
  const int s = s_begin + wid / groups, h0 = (wid % groups) * HG;
  const SeqDesc sd = seqs[s];
  const int T = sd.p0 + sd.n, qpos = T - 1;
  const int e = lane % LPH;                 // chunk of the head
  const int col = h0 * DH + lane * E;       // this lane's first column within a Q / K / V block
  const float* pfx = sd.prefix_live ? qkv : cache;
  const int ldp = sd.prefix_live ? ldq : ldc;
  auto row_of = [&](int j) -> const float* {
    return j < sd.p0 ? pfx + (size_t)(sd.cache_row + j) * ldp : qkv + (size_t)(sd.row0 + j - sd.p0) * ldq;
  };
  auto rotate = [&](float (&x)[E], int pos) {
    float p[E];
#pragma unroll
    for (int i = 0; i < E; ++i) p[i] = __shfl_xor(x[i], OFF, 64);  // every lane, before any divergence
    if (e < 2 * OFF) {
      const float sg = (e & OFF) == 0 ? -1.f : 1.f;  // x0 cos - x1 sin | x1 cos + x0 sin
      float cs[E], sn[E];
      load_span<E>(cos_t + pos * rd + e * E, cs);
      load_span<E>(sin_t + pos * rd + e * E, sn);
#pragma unroll
      for (int i = 0; i < E; ++i) x[i] = x[i] * cs[i] + sg * p[i] * sn[i];
    }
  };
  float q[E];
  {
    load_span<E>(row_of(qpos) + col, q);
    rotate(q, qpos);
  }
  float m_run = -INFINITY, l_run = 0.f, acc[E];
#pragma unroll
  for (int i = 0; i < E; ++i) acc[i] = 0.f;
  constexpr int KB = 4;  // keys per batch: their loads in flight together
  for (int j0 = 0; j0 < T; j0 += KB) {
    float kv[KB][E], vv[KB][E];
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int j = min(j0 + u, T - 1);
      const float* r = row_of(j);
      load_span<E>(r + d + col, kv[u]);
      load_span<E>(r + 2 * d + col, vv[u]);
    }
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int j = j0 + u;
      rotate(kv[u], min(j, T - 1));
      float sc = 0.f;
#pragma unroll
      for (int i = 0; i < E; ++i) sc = fmaf(q[i], kv[u][i], sc);
#pragma unroll
      for (int o = LPH / 2; o > 0; o >>= 1) sc += __shfl_xor(sc, o, 64);
      if (j >= T) continue;  // wave-uniform (T is the sequence's)
      sc *= inv_attn_scale;
      const float m_new = fmaxf(m_run, sc);
      const float scale = m_run == -INFINITY ? 0.f : expf(m_run - m_new);
      const float p = expf(sc - m_new);
      l_run = l_run * scale + p;
#pragma unroll
      for (int i = 0; i < E; ++i) acc[i] = fmaf(p, vv[u][i], acc[i] * scale);
      m_run = m_new;
    }
  }
  const size_t zrow = (size_t)(sd.row0 + sd.n - 1);
  const float inv = 1.0f / l_run;
  // z through a per-wave LDS row: lane l's E dims at 4 l E B would go out as E 2-B (planes) or 4-B stores
  // per lane, each instruction touching the whole span's lines; re-read as 4 consecutive dims per lane
  // they go out as 8-B plane / 16-B fp32 stores
  __shared__ __attribute__((aligned(16))) float zs[4][HG * DH];
  float* zw = zs[(threadIdx.x >> 6) & 3];
#pragma unroll
  for (int i = 0; i < E; ++i) zw[lane * E + i] = acc[i] * inv;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int c0 = h0 * DH;
  for (int c = 4 * lane; c < HG * DH; c += 256) {
    const f32x4 v = *(const f32x4*)(zw + c);
    if constexpr (FMT != ACT_F32)
      store_act4<FMT>((uint16_t*)z + zrow * 2 * ldz + c0 + c, ldz, v[0], v[1], v[2], v[3], flag);
    else
      *(f32x4u*)((float*)z + zrow * ldz + c0 + c) = v;
    if (zf && zf_last) *(f32x4u*)(zf + (size_t)s * ldzf + c0 + c) = v;  // the capture's compact last-row copy
    else if (zf && zrow < (size_t)zf_rows) *(f32x4u*)(zf + zrow * ldzf + c0 + c) = v;
  }
}

}  // namespace tvr

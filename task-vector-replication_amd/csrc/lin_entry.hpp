// lin_entry.hpp — the first layer after a head-replacement patch, linearised.
//
// A REPLACE_HEAD_ALLPOS site (layer l-1, head h, vector v) enters the
// staircase at layer l with, at every position,
//     r = r_c + v - z_h W_O[h]            (entry_kernel; r_c the clean row)
// and layer l's QKV + MLP-in GEMM reads LNPre(r) = (r - mu) / sigma, so
//     y = LNPre(r) W1^T = (r W1^T - mu c1) / sigma,      c1[n] = sum_j W1[n][j]
// Every term of r W1^T is already known or cheap:
//     r_c W1^T = sigma_c y_c + mu_c c1     (y_c: the clean row's own GEMM output
//                                           at layer l, computed in the same sweep)
//     v W1^T   = G[v]                      (one [n_vectors] x d GEMM per layer)
//     z_h W_O[h] W1^T = z_h Wsc[h]         (Wsc = W1[l] W_O[l-1]: [D1][H dh],
//                                           a model constant, K = d_head)
// so the entering rows' K = d_model GEMM (2 d D1 FLOP per row) becomes a
// K = d_head one (2 d_head D1): 32x less work at 2.8B, the same fp32-accurate
// arithmetic (x2f16 split, 3 products; the sums above are exact algebra, each
// term carries fp32-level rounding).  Only the QKV + MLP-in GEMM of the ENTRY
// layer is linear in the patch: attention and GELU are not, so layers > l run
// in full.  The reference computes every such row with a full batch-1
// forward (scratch2.py:181-194).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gemm_planar.hpp"

namespace tvr {

// One block's rows: entering rows [row0, row0 + rows) of the layer's row list
// (rows <= 64), all of head `head`.
struct LinMB {
  int row0, rows, head, pad;
};
// One entering row: its activation row, its clean row (trace row of the same
// prompt position: y_c, z_h and the clean LN statistics) and its vector's row of G.
struct LinRow {
  int out_row, clean_row, vrow, pad;
};

constexpr int LIN_THREADS = 256;  // 4 waves, each 64 rows x 64 columns of a 64 x 256 tile

// out[n][j] = in[j * ldi + n] for n, j < d (the W_O block of w2, transposed: load time)
__global__ void transpose_kernel(const float* __restrict__ in, int ldi, float* __restrict__ out, int d) {
  __shared__ float t[32][33];
  const int j0 = blockIdx.y * 32, n0 = blockIdx.x * 32;
  for (int r = threadIdx.y; r < 32; r += blockDim.y)
    if (j0 + r < d && n0 + threadIdx.x < d) t[r][threadIdx.x] = in[(size_t)(j0 + r) * ldi + n0 + threadIdx.x];
  __syncthreads();
  for (int r = threadIdx.y; r < 32; r += blockDim.y)
    if (n0 + r < d && j0 + threadIdx.x < d) out[(size_t)(n0 + r) * d + j0 + threadIdx.x] = t[threadIdx.x][r];
}

// c1[n] = sum_j w[n][j] (fp64 accumulation, one wave per row: load time)
__global__ void rowsum_kernel(const float* __restrict__ w, int n_rows, int k, float* __restrict__ c1) {
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  double s = 0.0;
  for (int j = lane; j < k; j += 64) s += (double)w[(size_t)row * k + j];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) c1[row] = (float)s;
}

// Wsc fp32 [N][H dh] -> planes [NPL][H][N][KP] (head-major, k zero-padded to
// KP): X2F16 two fp16 planes of w * scale (as the model's weight planes),
// BF16 one plane: bf16, except the attention-score rows n < n_qk (Q, K), which
// are fp16 of w * scale (the bf16 mode runs those projections on fp16
// operands, as launch_w1 does for the full entry GEMM).
template <int FMT>
__global__ void lin_planes_kernel(const float* __restrict__ s, int N, int H, int dh, int KP, float scale,
                                  uint16_t* __restrict__ out, int n_qk = 0) {
  const size_t n_out = (size_t)H * N * KP;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_out; i += (size_t)gridDim.x * blockDim.x) {
    const int k = (int)(i % KP);
    const size_t hn = i / KP;
    const int n = (int)(hn % N), h = (int)(hn / N);
    const float w = k < dh ? s[(size_t)n * H * dh + h * dh + k] : 0.0f;
    if constexpr (FMT == ACT_X2F16) {
      const float x = w * scale;
      const _Float16 h0 = (_Float16)x;
      out[i] = __builtin_bit_cast(uint16_t, h0);
      out[n_out + i] = __builtin_bit_cast(uint16_t, (_Float16)(x - (float)h0));
    } else {
      out[i] = n < n_qk ? __builtin_bit_cast(uint16_t, (_Float16)(w * scale)) : bf16_bits(w);
    }
  }
}

// The entering rows' QKV + MLP-in outputs (see the file comment).  Block
// (m-block b, column tile c): rows of mbs[b] x columns [256 c, 256 c + 256);
// wave w takes columns 64 w .. 64 w + 63 as 4 x 4 accumulators of 16 x 16,
// D = Wsc z^T on v_mfma_f32_16x16x32_{f16,bf16} (lane l ends with four
// consecutive columns of row l & 15, as gemm_planar.hpp).  z (fp32, the clean
// run's hook_z at layer l-1) is split in registers: 16 z = z0 + z1 (X2F16),
// products z0 w0 + z0 w1 + z1 w0.  The tile then goes through LDS so that the
// combine reads y_c and stores its outputs as whole 1-KB rows (4 consecutive
// columns per thread): per element
//     y = (sigma_c (y_c - b1) + (mu_c - mu) c1 + G[v] - z_h Wsc[h]) / sigma + b1
// (each row's sigma_c / sigma, (mu_c - mu) / sigma and 1 / sigma staged in LDS first)
// (y_c = the clean row's qkv, or its pre-GELU MLP-in value raw_h), stored as
// the QKV + MLP-in epilogue does: Q|K|V fp32 to qkv, GELU(h) in the
// activation format to the a2 columns after z.
constexpr int LIN_LDR = 260;  // floats per LDS row (conflict-free 16-B writes of the 16 x 16 fragments)
// Occupancy (round 6): the block was held to 2 per CU by both its LDS tile (66 KB) and its registers (221),
// i.e. 8 waves per CU for a latency-bound kernel.  Now the tile goes through LDS in two 128-column passes
// (TVR_LIN_HALVES 2: 35 KB), the product's z / Wsc loads are single-buffered (TVR_LIN_SB 1) and the combine
// issues the loads of 4 rows at a time (TVR_LIN_RB), so the kernel fits 168 VGPRs without spills: 3 waves per
// SIMD (TVR_LIN_WAVES).  C3 341.5 / 341.8 -> 327.6 / 328.2 us per launch (0.43 -> 0.45 of HBM), 12B 1,128 ->
// 1,072, same box; the halves alone (2 waves / SIMD, one more barrier) 465 us
// (profiles/r06/lin_entry_occupancy_ab_r06s2l.txt).  A/B: -DTVR_LIN_HALVES=1 -DTVR_LIN_SB=0 -DTVR_LIN_WAVES=0
// -DTVR_LIN_RB=8 (round 5's form)
#ifndef TVR_LIN_HALVES
#define TVR_LIN_HALVES 2
#endif
#ifndef TVR_LIN_SB
#define TVR_LIN_SB 1
#endif
#ifndef TVR_LIN_WAVES
#define TVR_LIN_WAVES 3
#endif
#ifndef TVR_LIN_RB
#define TVR_LIN_RB 4  // rows per combine batch (their y_c / G loads issued together)
#endif
constexpr int LIN_HALVES = TVR_LIN_HALVES;
// NK = KP / 32 k-steps, fully unrolled with the next step's z / Wsc loads
// issued before this step's MFMAs.  1-D grid of n_mb x column tiles with the
// XCD-aware bijective remap (gemm_pingpong.hpp): the m-blocks that share a
// head's Wsc tile are consecutive work items, so they run on one XCD together
// and read that tile from one L2.
template <int FMT, int NK>
__global__ void
#if TVR_LIN_WAVES > 0
__launch_bounds__(LIN_THREADS, TVR_LIN_WAVES)
#else
__launch_bounds__(LIN_THREADS)
#endif
lin_entry_kernel(const LinMB* __restrict__ mbs, int n_mb, const LinRow* __restrict__ rows,
                 const uint16_t* __restrict__ wp, size_t wps, float acc_scale, const float* __restrict__ z, int d,
                 int dh, const float2* __restrict__ stats, float* __restrict__ qkv, const float* __restrict__ raw_h,
                 int d_mlp, const float* __restrict__ G, const float* __restrict__ c1, const float* __restrict__ b1,
                 int N, uint16_t* __restrict__ out1h, int ld1h, int ps1h, unsigned* __restrict__ range_flag,
                 int ct_base = 0) {
  using frag = typename PlanarFmt<FMT>::frag;
  constexpr int KP = 32 * NK;
  constexpr int CW = 256 / LIN_HALVES, LDR = LIN_HALVES == 1 ? LIN_LDR : CW + 4;  // columns per LDS pass, row stride
  __shared__ __attribute__((aligned(16))) float tile[64 * LDR];
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int work = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int mbi = work % n_mb, ct = work / n_mb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col0 = (ct_base + ct) * 256, nb = col0 + wave * 64;
  const LinMB mb = mbs[mbi];
  const int r16 = lane & 15, g = lane >> 4;
  // per-row combine coefficients, staged while the product runs:
  // y = A (y_c - b1) + B c1 + I (G[v] - z Wsc) + b1,  A = sigma_c / sigma, B = (mu_c - mu) / sigma, I = 1 / sigma
  __shared__ f32x4 rcoef[64];
  __shared__ int4 rrow[64];
  if (threadIdx.x < mb.rows) {
    const LinRow q = rows[mb.row0 + threadIdx.x];
    const float2 st = stats[q.out_row], sc = stats[q.clean_row];
    const float inv = 1.0f / st.y;
    rcoef[threadIdx.x] = f32x4{sc.y * inv, (sc.x - st.x) * inv, inv, 0.f};
    rrow[threadIdx.x] = make_int4(q.out_row, q.clean_row, q.vrow, 0);
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};
  if (nb < N) {  // (a wave past N skips the product but joins the barriers)
    const float* zr[4];
    bool live[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      live[i] = 16 * i + r16 < mb.rows;
      zr[i] = z + (size_t)rows[mb.row0 + (live[i] ? 16 * i + r16 : 0)].clean_row * d + mb.head * dh + 8 * g;
    }
    const uint16_t* wr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) wr[j] = wp + ((size_t)mb.head * N + min(nb + 16 * j + r16, N - 1)) * KP + 8 * g;
    // raw loads of k-step s (lane: 8 k values at 32 s + 8 g; dh % 16 == 0: a chunk is wholly in or out)
    constexpr int NB = TVR_LIN_SB ? 1 : 2;  // load buffers
    f32x4 zx[NB][4], zy[NB][4];
    frag w0[NB][4], w1[NB][4];
    auto load = [&](int s, int b) {
      const bool kin = 32 * s + 8 * g < dh;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        zx[b][i] = f32x4{};
        zy[b][i] = f32x4{};
        if (live[i] && kin) {
          zx[b][i] = *(const f32x4*)(zr[i] + 32 * s);
          zy[b][i] = *(const f32x4*)(zr[i] + 32 * s + 4);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        w0[b][j] = *(const frag*)(wr[j] + 32 * s);
        if constexpr (FMT == ACT_X2F16) w1[b][j] = *(const frag*)(wr[j] + 32 * s + wps);
      }
    };
    if (NB == 2) load(0, 0);
#pragma unroll
    for (int s = 0; s < NK; ++s) {
      const int b = NB == 2 ? s & 1 : 0;
      if (NB == 1)
        load(s, 0);
      else if (s + 1 < NK)
        load(s + 1, b ^ 1);
      frag a0[4], a1[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v[8] = {zx[b][i][0], zx[b][i][1], zx[b][i][2], zx[b][i][3],
                            zy[b][i][0], zy[b][i][1], zy[b][i][2], zy[b][i][3]};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if constexpr (FMT == ACT_X2F16) {
            const float s16 = v[e] * X2_ASCALE;
            const _Float16 h0 = (_Float16)s16;
            a0[i][e] = h0;
            a1[i][e] = (_Float16)(s16 - (float)h0);
          } else if constexpr (FMT == ACT_F16) {  // the bf16 mode's Q / K columns
            a0[i][e] = (_Float16)v[e];
          } else {
            a0[i][e] = (__bf16)v[e];
          }
        }
      }  // (z's X2F16 range was checked by its producer, the attention kernel)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x4 c = acc[i][j];
          if constexpr (FMT == ACT_X2F16) {
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0[b][j], a1[i], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[b][j], a0[i], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0[b][j], a0[i], c, 0, 0, 0);
          } else if constexpr (FMT == ACT_F16) {
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0[b][j], a0[i], c, 0, 0, 0);
          } else {
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[b][j], a0[i], c, 0, 0, 0);
          }
          acc[i][j] = c;
        }
    }
  }
  // combine + store: thread t takes columns col0 + 4 (t & 63) .. +3 of rows t >> 6, + 4, ...
  // in batches of 8 rows whose y_c / G loads are all issued before the batch's
  // stores (qkv is read at clean rows and written at entering rows, so the
  // compiler may not move a load past a store; one load after a store would
  // make it wait for that store to reach memory: s_waitcnt vmcnt counts both).
  // (LIN_HALVES 2: the same per column pass; the waves whose 64 columns lie in the pass write them first)
  constexpr int TPR = CW / 4, RS = LIN_THREADS / TPR, RB = TVR_LIN_RB;  // threads per row, rows per step, rows per batch
  const int cl = 4 * (threadIdx.x % TPR), n3 = 3 * d;
  for (int hf = 0; hf < LIN_HALVES; ++hf) {
  if (hf > 0) __syncthreads();  // the previous pass's tile reads are done
  if (nb < N && (wave * 64) / CW == hf) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *(f32x4*)(tile + (16 * i + r16) * LDR + (wave * 64) % CW + 16 * j + 4 * g) = acc[i][j] * acc_scale;
  }
  __syncthreads();
  const int n0 = col0 + hf * CW + cl;
  if (n0 >= N) continue;
  const f32x4 b = *(const f32x4*)(b1 + n0), c = *(const f32x4*)(c1 + n0);
  for (int r0 = threadIdx.x / TPR; r0 < mb.rows; r0 += RS * RB) {
    int4 q[RB];
    f32x4 yc[RB], gv[RB];
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      q[i] = rrow[min(r0 + RS * i, mb.rows - 1)];
      yc[i] = n0 < n3 ? *(const f32x4*)(qkv + (size_t)q[i].y * n3 + n0)
                      : *(const f32x4*)(raw_h + (size_t)q[i].y * d_mlp + (n0 - n3));
      gv[i] = *(const f32x4*)(G + (size_t)q[i].z * N + n0);
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int r = r0 + RS * i;
      if (r >= mb.rows) break;
      const f32x4 k = rcoef[r];
      const f32x4 v = *(const f32x4*)(tile + r * LDR + cl);
      f32x4 y;
#pragma unroll
      for (int e = 0; e < 4; ++e) y[e] = k[0] * (yc[i][e] - b[e]) + k[1] * c[e] + k[2] * (gv[i][e] - v[e]) + b[e];
      if (n0 < n3) {
        *(f32x4*)(qkv + (size_t)q[i].x * n3 + n0) = y;
      } else {
        const f32x2 g01 = gelu_erf2(f32x2{y[0], y[1]}), g23 = gelu_erf2(f32x2{y[2], y[3]});
        store_act4<FMT>(out1h + (size_t)q[i].x * ld1h + (n0 - n3), ps1h, g01.x, g01.y, g23.x, g23.y, range_flag);
      }
    }
  }
  }
}


// The rows of G on the exact-fp16 weights (tvr_model_set_exact16): the processed W1' = fold_ln(W1) has
// W1'[n][k] = W1[n][k] gamma_k - m_n, so for ANY vector v
//     v W1'^T = ((v - mean(v)) o gamma) W1^T
// (sum_k (v_k - mean) gamma_k W1[n][k] = sum_k v_k gamma_k W1[n][k] - m_n sum_k v_k), with gamma1 for the
// Q | K | V columns and gamma2 for the MLP-in ones: row r of out1 / out2 (x2f16 activation format, [rows][2][d]
// halves) is vector vids[r] centred and scaled, for the one-plane GEMM against the raw W1.  One wave per row.
__global__ void __launch_bounds__(256) lin_gamma_rows_kernel(const float* __restrict__ v, int d,
                                                            const int32_t* __restrict__ vids,
                                                            const float* __restrict__ g1, const float* __restrict__ g2,
                                                            uint16_t* __restrict__ out1, uint16_t* __restrict__ out2,
                                                            int rows, unsigned* flag) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x >> 6) + wave;
  if (r >= rows) return;
  const float* x = v + (size_t)vids[r] * d;
  float s = 0.f;
  for (int c = 4 * lane; c < d; c += 256) {
    const f32x4 q = *(const f32x4*)(x + c);
    s += (q[0] + q[1]) + (q[2] + q[3]);
  }
  const float mean = wave_sum(s) / (float)d;
  for (int c = 4 * lane; c < d; c += 256) {
    const f32x4 q = *(const f32x4*)(x + c) - mean;
    const f32x4 a = *(const f32x4*)(g1 + c) * q, b = *(const f32x4*)(g2 + c) * q;
    store_act4<ACT_X2F16>(out1 + (size_t)r * 2 * d + c, d, a[0], a[1], a[2], a[3], flag);
    store_act4<ACT_X2F16>(out2 + (size_t)r * 2 * d + c, d, b[0], b[1], b[2], b[3], flag);
  }
}

}  // namespace tvr

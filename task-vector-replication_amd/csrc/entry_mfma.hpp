// entry_mfma.hpp — the REPLACE_HEAD site entry on the fp32 matrix cores.
//
// A head-replacement site (layer e-1, head h, vector v) enters layer e with
//     resid[i][c] = snap[p0 + i][c] + v[c] - sum_k z[p0 + i][h dh + k] W_O[c][h dh + k]
// at every position i (kernels.hpp entry_kernel, parallel residual, SURVEY §7,
// scratch2.py:188).  entry_kernel does the z . W_O product on the VALU (one
// FMA per (position, column, k) and thread: 1.2 G FMAs per C3 entry layer);
// here it is a [16 positions x dh] x [dh x 64 columns] tile per wave on
// v_mfma_f32_16x16x4_f32 (exact fp32 products, as the attention kernel).
// Grid = (groups, ceil(d / ENTRY_COLS)), 4 waves of 16 ENTRY_NT columns each; a group is up to
// ENTRY_GROUP sites of one head (the host groups a layer's REPLACE_HEAD entries),
// whose W_O[h] columns the wave reads once into registers: the launch was bound
// by re-reading the 80 KB W_O slice of a 256-column block for every site.  But
// a group's sites run one after another in its block, so a few large groups
// leave the chip latency-bound: at C3 (a layer's 12 prompts x 32 heads: 12
// sites per head) groups of 12 / 8+4 / 4+4+4 ran 76 / 88 / 63 us per launch
// (r04m, same box); the host splits a head's sites into ceil(n / ENTRY_GROUP)
// groups of balanced size (the re-reads of W_O[h] come from L2).  (Software-
// pipelining a group's tiles — the next z tile loaded to registers during this
// tile's MFMAs, double-buffered LDS, one barrier per tile — ran 78 us against
// 64 us, same box r04p: not kept.)  The
// MFMA's k index is a permutation applied to both operands: lane group g
// supplies k = g CH + j at k-step j (CH = dh / 4), so a lane's A operand is CH
// consecutive floats of one W_O row (float4 loads) and its B operand CH
// consecutive floats of one z row, read from the z tile in LDS.  With W_O as
// the A operand the product is D[column][position]: each lane ends with four
// consecutive columns of one position, so the clean rows, the vector and the
// patched rows move as 16-B accesses (64 B of a row per lane group).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gemm_f32.hpp"
#include "kernels.hpp"

namespace tvr {

#ifndef TVR_ENTRY_GROUP
#define TVR_ENTRY_GROUP 4
#endif
constexpr int ENTRY_GROUP = TVR_ENTRY_GROUP;  // sites of one head per block: W_O[h] read once for them
// 16-column tiles per wave: 1 (a wave's W_O[h] columns in 20 VGPRs at d_head 80, so more waves per SIMD
// hide the dependent load chains): 54 / 61 / 66 us per C3 entry launch at 1 / 2 / 4 (r04w, same box)
#ifndef TVR_ENTRY_NT
#define TVR_ENTRY_NT 1
#endif
constexpr int ENTRY_NT = TVR_ENTRY_NT;
constexpr int ENTRY_COLS = (ENTRY_THREADS / 64) * 16 * ENTRY_NT;   // columns per block

template <int DH>
__global__ void __launch_bounds__(ENTRY_THREADS)
entry_replace_mfma_kernel(const EntryDesc* __restrict__ ents, const int32_t* __restrict__ gidx,
                          const int2* __restrict__ groups, const float* __restrict__ snap,
                          const float* __restrict__ zsnap, const float* __restrict__ w2, int ldw2,
                          const float* __restrict__ vectors, float* __restrict__ resid, int d) {
  constexpr int CH = DH / 4;  // k values per lane group
  static_assert(DH % 16 == 0, "d_head");
  __shared__ __attribute__((aligned(16))) float zt[16 * (DH + 4)];  // 16 positions x DH (+4: conflict-free rows)
  constexpr int LDZ = DH + 4;
  const int2 grp = groups[blockIdx.x];  // entries gidx[grp.x .. + grp.y): REPLACE_HEAD sites of one head
  const int head = ents[gidx[grp.x]].head;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int li = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.y * ENTRY_COLS + wave * 16 * ENTRY_NT;  // this wave's first column

  // B operands: W_O row (column c = n0 + 16 nt + li), k = g CH .. g CH + CH - 1
  float wb[ENTRY_NT][CH];
#pragma unroll
  for (int nt = 0; nt < ENTRY_NT; ++nt) {
    const int c = min(n0 + 16 * nt + li, d - 1);
    const float* wr = w2 + (size_t)c * ldw2 + head * DH + g * CH;
#pragma unroll
    for (int q = 0; q < CH; q += 4) {
      const float4 v4 = *(const float4*)(wr + q);
      wb[nt][q] = v4.x; wb[nt][q + 1] = v4.y; wb[nt][q + 2] = v4.z; wb[nt][q + 3] = v4.w;
    }
  }
  for (int gi = 0; gi < grp.y; ++gi) {
    const EntryDesc e = ents[gidx[grp.x + gi]];
    for (int t0 = 0; t0 < e.n; t0 += 16) {
      const int tn = min(16, e.n - t0);
      __syncthreads();  // the previous tile's reads are done
      for (int x = threadIdx.x; x < 16 * (DH / 4); x += ENTRY_THREADS) {
        const int r = x / (DH / 4), q = (x - r * (DH / 4)) * 4;
        const float4 v4 = *(const float4*)(zsnap + (size_t)(e.src_row + e.p0 + t0 + min(r, tn - 1)) * d +
                                           e.head * DH + q);
        *(float4*)(zt + r * LDZ + q) = v4;
      }
      __syncthreads();
      if (n0 >= d) continue;  // (a wave past d joins the barriers only)
      // the clean rows' values and the vector first (no load between the stores below); lane (li, g) owns
      // position li and columns n0 + 16 nt + 4 g .. + 3
      const int pr = min(li, tn - 1);
      f32x4 sv[ENTRY_NT], vc[ENTRY_NT];
#pragma unroll
      for (int nt = 0; nt < ENTRY_NT; ++nt) {
        const int c = min(n0 + 16 * nt + 4 * g, d - 4);
        vc[nt] = *(const f32x4*)(vectors + (size_t)e.vec * d + c);
        sv[nt] = *(const f32x4*)(snap + (size_t)(e.src_row + e.p0 + t0 + pr) * d + c);
      }
      float za[CH];  // B operand: z row li, k = g CH ..
#pragma unroll
      for (int q = 0; q < CH; q += 4) {
        const f32x4 v4 = *(const f32x4*)(zt + li * LDZ + g * CH + q);
        za[q] = v4[0]; za[q + 1] = v4[1]; za[q + 2] = v4[2]; za[q + 3] = v4[3];
      }
      f32x4 acc[ENTRY_NT];
#pragma unroll
      for (int nt = 0; nt < ENTRY_NT; ++nt) {
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};  // two chains (dependent-issue latency)
#pragma unroll
        for (int j = 0; j < CH; j += 2) {
          a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[nt][j], za[j], a0, 0, 0, 0);
          a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[nt][j + 1], za[j + 1], a1, 0, 0, 0);
        }
        acc[nt] = a0 + a1;  // D[column 16 nt + 4 g + r][position li]
      }
      if (li < tn) {
#pragma unroll
        for (int nt = 0; nt < ENTRY_NT; ++nt) {
          const int c = n0 + 16 * nt + 4 * g;
          if (c < d) *(f32x4*)(resid + (size_t)(e.row0 + t0 + li) * d + c) = sv[nt] + (vc[nt] - acc[nt]);
        }
      }
    }
  }
}

}  // namespace tvr

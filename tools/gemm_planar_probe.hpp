// tools/gemm_planar_probe.hpp — the previous engine GEMM for the planar
// activation formats (one barrier per K step, both waves of a SIMD reading LDS
// and issuing MFMAs together), kept OUT of the product for the A/B variants
// of tools/gemm_split_probe.hip only.  The engine runs gemm_pingpong_kernel
// (task-vector-replication_amd/csrc/gemm_pingpong.hpp), which shares this
// kernel's operand formats, LDS image and epilogues.
#pragma once
#include "../task-vector-replication_amd/csrc/gemm_planar.hpp"

namespace tvr {

template <int BM_, int BN_, int WM_, int WN_>
struct PlanarTile {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
  static constexpr int THREADS = WM * WN * 64;
  static constexpr int TM = BM / WM / 16, TN = BN / WN / 16;  // 16x16 accumulators per wave
  static_assert(BM == BN, "one LDS plane size for A and W");
};
using PlanarLarge = PlanarTile<256, 256, 2, 4>;  // 8 waves of 128x64, 1 block per CU (128 KB LDS)
using PlanarSmall = PlanarTile<128, 128, 2, 2>;  // 4 waves of 64x64

template <class TL>
inline int gemm_planar_grid(int M, int N) {
  return ((M + TL::BM - 1) / TL::BM) * ((N + TL::BN - 1) / TL::BN);
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

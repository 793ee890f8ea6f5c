// kernels.hpp — the non-GEMM kernels of the patched Pythia forward.
//
// All of them are HBM/L2-bound byte movers or tiny contractions; the FLOPs
// live in gemm_f32.hpp.  Semantics follow TransformerLens as the reference
// uses it: LayerNormPre after fold_ln, NeoX rotate-half
// rotary on the first rotary_dim dims, causal softmax in fp32, per-head
// result = z @ W_O[h] (hook_result, scratch2.py:98,188).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "split.hpp"

namespace tvr {

// ---------------------------------------------------------------------------
// Descriptors built by the host planner (engine.hip).

// One sequence as seen by attention at a layer: its computed rows are the
// positions [p0, p0+n); positions [0, p0) come from the clean trace's K/V.
struct SeqDesc {
  int32_t row0;       // first computed row in the activation buffers
  int32_t n;          // number of computed rows
  int32_t p0;         // absolute position of row0
  int32_t cache_row;  // row of position 0 for the K/V prefix (positions < p0), -1: none
  int32_t q0;         // first computed row that is a query (n-1: last row only)
  int32_t prefix_live;  // 0: the prefix is in the clean trace (cache); 1: in this run's qkv rows
                        // (a shared-prefix follower reads its leader's rows: tvr_patch_sweep)
};

// How a patch site's residual is materialised at its entry layer e
// (resid_pre[e] rows [p0, p0+n)), from the clean trace.
struct EntryDesc {
  int32_t kind;       // tvr_site_kind
  int32_t row0;       // destination row (activation buffer)
  int32_t n;          // rows
  int32_t p0;         // first position
  int32_t src_row;    // trace row of position 0 of `seq`
  int32_t src2_row;   // SET_RESID: trace row supplying the patched position
  int32_t patch_pos;  // SET_RESID: absolute patched position
  int32_t head;       // REPLACE_HEAD
  int32_t vec;        // vector row
  int32_t pad;
};

// ---------------------------------------------------------------------------
// wave_sum / wave_max: split.hpp

// ---------------------------------------------------------------------------
// hook_embed: resid[r] = W_E[tokens[r]]   (one float4 per thread)
__global__ void embed_kernel(const int32_t* __restrict__ tokens,
                             const float* __restrict__ W_E, float* __restrict__ out,
                             int rows, int d) {
  const int d4 = d >> 2;
  const size_t total = (size_t)rows * d4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / d4), c = (int)(i % d4);
    const int tok = tokens[r];
    ((float4*)out)[i] = ((const float4*)(W_E + (size_t)tok * d))[c];
  }
}

// dst[r] = src[r] - mean(src[r]) (one wave per row, d % 4 == 0): the exact-fp16 weight path's residual
// stream carries one extra constant per row (engine.hip tvr_model, x16), which the TL residual lacks
// V4: src and dst 16-B aligned, d % 4 == 0 (float4 accesses); else element-wise (a caller's offset view).
// src == dst allowed (each lane reads an element before it writes it, in both passes)
template <bool V4>
__global__ void center_rows_kernel(const float* src, float* dst, int rows, int d) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x >> 6) + wave;
  if (r >= rows) return;
  float s = 0.f;
  if constexpr (V4) {
    const float4* x = (const float4*)(src + (size_t)r * d);
    float4* y = (float4*)(dst + (size_t)r * d);
    for (int c = lane; c < d / 4; c += 64) {
      const float4 v = x[c];
      s += (v.x + v.y) + (v.z + v.w);
    }
    const float mean = wave_sum(s) / (float)d;
    for (int c = lane; c < d / 4; c += 64) {
      const float4 v = x[c];
      y[c] = make_float4(v.x - mean, v.y - mean, v.z - mean, v.w - mean);
    }
  } else {
    const float* x = src + (size_t)r * d;
    float* y = dst + (size_t)r * d;
    for (int c = lane; c < d; c += 64) s += x[c];
    const float mean = wave_sum(s) / (float)d;
    for (int c = lane; c < d; c += 64) y[c] = x[c] - mean;
  }
}

// ---------------------------------------------------------------------------
// LayerNormPre (TL, after fold_ln): x -= mean(x); x /= sqrt(mean(x^2) + eps).
// One wave per row; rows optionally gathered through `row_idx`.  FMT: y is
// fp32 (ACT_F32) or a planar activation format (split.hpp; ldy counts logical
// elements); the outputs are bounded by sqrt(d), so no range check.
// NV: float4 per lane held in registers (10: d <= 2560, 20: d <= 5120, Pythia-12B; d % 256 == 0), else the
// three-pass loop; LN_G_F4 gamma float4 per lane per group (x2f16 gamma-scaled rows)
constexpr int LN_G_F4 = 10;
// g1 (x2f16, engine.hip's exact-fp16 weights): y = LNPre(x) * g1 and, with y2, y2 = LNPre(x) * g2 instead
// (LN1's and LN2's gamma, or the final LN's alone: the read-in weights' fold_ln scale moved onto the rows),
// range-checked into flag.
template <int FMT, int NV>
__global__ void __launch_bounds__(256) lnpre_kernel(const float* __restrict__ x, int ldx,
                             const int32_t* __restrict__ row_idx,
                             void* __restrict__ y, int ldy, int rows, int d,
                             float eps, float2* __restrict__ stats, float* __restrict__ copy = nullptr,
                             int copy_rows = 0, const float* __restrict__ g1 = nullptr,
                             const float* __restrict__ g2 = nullptr, void* __restrict__ y2 = nullptr,
                             unsigned* __restrict__ flag = nullptr) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x >> 6) + wave;
  if (r >= rows) return;
  const int src = row_idx ? row_idx[r] : r;
  const float4* xr = (const float4*)(x + (size_t)src * ldx);
  const int d4 = d >> 2;
  constexpr int LN_REG_F4 = NV;
  if (NV > 0 && d4 % 64 == 0 && d4 <= 64 * LN_REG_F4) {  // the row in registers: one global read
    const int nv = d4 >> 6;
    float4 v[NV > 0 ? NV : 1];
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < LN_REG_F4; ++u)
      if (u < nv) v[u] = xr[lane + 64 * u];
    // the gammas of the x2f16 rows, LN_G_F4 float4 per lane at a time: loaded here, with the row, and not
    // between the row's stores — vmcnt counts stores too, so a load issued after a store waits for that
    // store to reach memory, and round 5's per-float4 gamma loads serialised the row into 10 store round
    // trips (14 us per launch at any row count in the C2 sweeps, profiles/r06/c2_trace_r06h.txt)
    constexpr int G = NV < LN_G_F4 ? NV : LN_G_F4;
    [[maybe_unused]] float4 ga[G > 0 ? G : 1], gb[G > 0 ? G : 1];
    if constexpr (FMT == ACT_X2F16) {
      if (g1) {
#pragma unroll
        for (int u = 0; u < G; ++u)
          if (u < nv) {
            ga[u] = ((const float4*)g1)[lane + 64 * u];
            if (y2) gb[u] = ((const float4*)g2)[lane + 64 * u];
          }
      }
    }
    if (copy && r < copy_rows) {  // the input row itself (a fused sweep's clean rows -> the trace)
      float4* cr = (float4*)(copy + (size_t)r * ldx);
#pragma unroll
      for (int u = 0; u < LN_REG_F4; ++u)
        if (u < nv) cr[lane + 64 * u] = v[u];
    }
#pragma unroll
    for (int u = 0; u < LN_REG_F4; ++u)
      if (u < nv) s += (v[u].x + v[u].y) + (v[u].z + v[u].w);
    const float mean = wave_sum(s) / (float)d;
    float ss = 0.f;
#pragma unroll
    for (int u = 0; u < LN_REG_F4; ++u) {
      if (u < nv) {
        v[u].x -= mean; v[u].y -= mean; v[u].z -= mean; v[u].w -= mean;
        ss += (v[u].x * v[u].x + v[u].y * v[u].y) + (v[u].z * v[u].z + v[u].w * v[u].w);
      }
    }
    const float scale = sqrtf(wave_sum(ss) / (float)d + eps);
    if (stats && lane == 0) stats[r] = make_float2(mean, scale);
    if constexpr (FMT == ACT_X2F16) {
      if (g1) {  // the gamma-scaled row(s): y = x g1 (and y2 = x g2 when y2 is given)
        float mx = 0.f;
#pragma unroll
        for (int g0 = 0; g0 < LN_REG_F4; g0 += G) {
          if (g0 > 0) {  // the next group's gammas (d > 64 G * 4: one wait for the stores so far)
#pragma unroll
            for (int u = 0; u < G; ++u)
              if (g0 + u < nv) {
                ga[u] = ((const float4*)g1)[lane + 64 * (g0 + u)];
                if (y2) gb[u] = ((const float4*)g2)[lane + 64 * (g0 + u)];
              }
          }
#pragma unroll
          for (int u = 0; u < G; ++u) {
            if (g0 + u < nv) {
              const int c = lane + 64 * (g0 + u);
              const float4 w = v[g0 + u];
              const float4 o = make_float4(w.x / scale, w.y / scale, w.z / scale, w.w / scale);
              const float4 a = ga[u];
              const float4 p = make_float4(o.x * a.x, o.y * a.y, o.z * a.z, o.w * a.w);
              store_ln4<FMT>((uint16_t*)y + (size_t)r * 2 * ldy + 4 * c, ldy, p.x, p.y, p.z, p.w);
              mx = fmaxf(mx, fmaxf(fmaxf(fabsf(p.x), fabsf(p.y)), fmaxf(fabsf(p.z), fabsf(p.w))));
              if (y2) {
                const float4 b = gb[u];
                const float4 q = make_float4(o.x * b.x, o.y * b.y, o.z * b.z, o.w * b.w);
                store_ln4<FMT>((uint16_t*)y2 + (size_t)r * 2 * ldy + 4 * c, ldy, q.x, q.y, q.z, q.w);
                mx = fmaxf(mx, fmaxf(fmaxf(fabsf(q.x), fabsf(q.y)), fmaxf(fabsf(q.z), fabsf(q.w))));
              }
            }
          }
        }
        if (mx * X2_ASCALE >= X2_FP16_OVERFLOW && flag) atomicOr(flag, 1u);
        return;
      }
    }
#pragma unroll
    for (int u = 0; u < LN_REG_F4; ++u) {
      if (u < nv) {
        const int c = lane + 64 * u;
        const float4 o = make_float4(v[u].x / scale, v[u].y / scale, v[u].z / scale, v[u].w / scale);
        if constexpr (FMT != ACT_F32) {
          store_ln4<FMT>((uint16_t*)y + (size_t)r * 2 * ldy + 4 * c, ldy, o.x, o.y, o.z, o.w);
        } else {
          ((float4*)((float*)y + (size_t)r * ldy))[c] = o;
        }
      }
    }
    return;
  }
  float s = 0.f;
  for (int c = lane; c < d4; c += 64) {
    const float4 v = xr[c];
    s += (v.x + v.y) + (v.z + v.w);
    if (copy && r < copy_rows) ((float4*)(copy + (size_t)r * ldx))[c] = v;
  }
  const float mean = wave_sum(s) / (float)d;
  float ss = 0.f;
  for (int c = lane; c < d4; c += 64) {
    float4 v = xr[c];
    v.x -= mean; v.y -= mean; v.z -= mean; v.w -= mean;
    ss += (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w);
  }
  const float scale = sqrtf(wave_sum(ss) / (float)d + eps);
  if (stats && lane == 0) stats[r] = make_float2(mean, scale);
  float mx = 0.f;
  for (int c = lane; c < d4; c += 64) {
    float4 v = xr[c];
    v.x = (v.x - mean) / scale; v.y = (v.y - mean) / scale;
    v.z = (v.z - mean) / scale; v.w = (v.w - mean) / scale;
    if constexpr (FMT == ACT_X2F16) {
      if (g1) {
        const float4 a = ((const float4*)g1)[c];
        const float4 p = make_float4(v.x * a.x, v.y * a.y, v.z * a.z, v.w * a.w);
        store_ln4<FMT>((uint16_t*)y + (size_t)r * 2 * ldy + 4 * c, ldy, p.x, p.y, p.z, p.w);
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(p.x), fabsf(p.y)), fmaxf(fabsf(p.z), fabsf(p.w))));
        if (y2) {
          const float4 b = ((const float4*)g2)[c];
          const float4 q = make_float4(v.x * b.x, v.y * b.y, v.z * b.z, v.w * b.w);
          store_ln4<FMT>((uint16_t*)y2 + (size_t)r * 2 * ldy + 4 * c, ldy, q.x, q.y, q.z, q.w);
          mx = fmaxf(mx, fmaxf(fmaxf(fabsf(q.x), fabsf(q.y)), fmaxf(fabsf(q.z), fabsf(q.w))));
        }
        continue;
      }
    }
    if constexpr (FMT != ACT_F32) {
      store_ln4<FMT>((uint16_t*)y + (size_t)r * 2 * ldy + 4 * c, ldy, v.x, v.y, v.z, v.w);
    } else {
      ((float4*)((float*)y + (size_t)r * ldy))[c] = v;
    }
  }
  if (mx * X2_ASCALE >= X2_FP16_OVERFLOW && flag) atomicOr(flag, 1u);
}

// ---------------------------------------------------------------------------
// Longest sequence the attention kernel takes (attention_mfma.hpp: up to 8
// key tiles of 16 in registers).
constexpr int ATT_MAX_T = 128;

// ---------------------------------------------------------------------------
// Site entry: materialise resid_pre[e] rows of every site entering at layer e
// from the clean trace.  grid = (n_entries, ceil(d/256)); thread owns column c.
//   snap   trace hook_resid_pre[e]                [tokens][d]
//   zsnap  trace attn.hook_z[e-1]                 [tokens][d]  (REPLACE_HEAD)
//   w2     layer e-1 fused [d][d+d_mlp] (cols h*dh.. = W_O[h]^T)
// REPLACE_HEAD (parallel residual): resid_pre[e] = clean resid_pre[e]
//   + vec - z[e-1][:, h] @ W_O[e-1, h], at every position (scratch2.py:188).
constexpr int ENTRY_THREADS = 256;
constexpr int ENTRY_POS_CHUNK = 16;
constexpr int ENTRY_K_CHUNK = 16;

// dynamic LDS: min(T, ENTRY_LDS_POS) x dh floats (the site's head slice of z,
// staged ENTRY_LDS_POS positions at a time; REPLACE_HEAD only)
constexpr int ENTRY_LDS_POS = 128;
__global__ void __launch_bounds__(ENTRY_THREADS)
entry_kernel(const EntryDesc* __restrict__ ents, const float* __restrict__ snap,
             const float* __restrict__ zsnap, const float* __restrict__ w2, int ldw2,
             const float* __restrict__ vectors, float* __restrict__ resid, int d, int dh, int skip_replace) {
  extern __shared__ __attribute__((aligned(16))) float zs[];
  const EntryDesc e = ents[blockIdx.x];
  const int c = blockIdx.y * ENTRY_THREADS + threadIdx.x;
  if (e.kind == 1) {  // TVR_SITE_REPLACE_HEAD_ALLPOS (unless entry_mfma.hpp takes them)
    if (skip_replace) return;
    const bool col = c < d;  // no early return: every thread joins the barriers
    const float* w = w2 + (size_t)(col ? c : 0) * ldw2 + e.head * dh;
    const float vc = col ? vectors[(size_t)e.vec * d + c] : 0.f;
    for (int s0 = 0; s0 < e.n; s0 += ENTRY_LDS_POS) {
      const int sn = min(ENTRY_LDS_POS, e.n - s0);
      __syncthreads();  // the previous chunk's reads are done
      for (int x = threadIdx.x; x < sn * dh; x += ENTRY_THREADS) {
        const int pos = x / dh, k = x - pos * dh;
        zs[x] = zsnap[(size_t)(e.src_row + e.p0 + s0 + pos) * d + e.head * dh + k];
      }
      __syncthreads();
      if (!col) continue;
      for (int p0 = 0; p0 < sn; p0 += ENTRY_POS_CHUNK) {
        // the clean rows' values first: no load between this chunk's stores (s_waitcnt
        // vmcnt counts loads and stores together, so a load after a store waits for it)
        float sv[ENTRY_POS_CHUNK], acc[ENTRY_POS_CHUNK];
#pragma unroll
        for (int u = 0; u < ENTRY_POS_CHUNK; ++u) {
          acc[u] = 0.f;
          sv[u] = snap[(size_t)(e.src_row + e.p0 + s0 + min(p0 + u, sn - 1)) * d + c];
        }
        for (int k0 = 0; k0 < dh; k0 += ENTRY_K_CHUNK) {
          float wk[ENTRY_K_CHUNK];
#pragma unroll
          for (int q = 0; q < ENTRY_K_CHUNK; q += 4) {
            const float4 v4 = *(const float4*)(w + k0 + q);  // dh % 16 == 0 (checked on the host)
            wk[q] = v4.x; wk[q + 1] = v4.y; wk[q + 2] = v4.z; wk[q + 3] = v4.w;
          }
#pragma unroll
          for (int u = 0; u < ENTRY_POS_CHUNK; ++u) {
            if (p0 + u < sn) {
              const float* zr = zs + (p0 + u) * dh + k0;
#pragma unroll
              for (int q = 0; q < ENTRY_K_CHUNK; ++q) acc[u] += zr[q] * wk[q];
            }
          }
        }
#pragma unroll
        for (int u = 0; u < ENTRY_POS_CHUNK; ++u) {
          if (p0 + u < sn) {
            resid[(size_t)(e.row0 + s0 + p0 + u) * d + c] = sv[u] + (vc - acc[u]);
          }
        }
      }
    }
    return;
  }
  if (c >= d) return;
  // rows in batches of 8 whose loads precede their stores (as above)
  const float add = e.kind == 2 ? vectors[(size_t)e.vec * d + c] : 0.f;  // TVR_SITE_ADD_ATTN_OUT_LASTPOS
  constexpr int B = 8;
  for (int i0 = 0; i0 < e.n; i0 += B) {
    float v[B];
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const int pos = e.p0 + min(i0 + u, e.n - 1);
      // NONE / SET_RESID_PRE_POS copy rows, one of them from another run
      const int srow = (e.kind == 3 && pos == e.patch_pos) ? e.src2_row : e.src_row + pos;
      v[u] = snap[(size_t)srow * d + c];
    }
#pragma unroll
    for (int u = 0; u < B; ++u)
      if (i0 + u < e.n) resid[(size_t)(e.row0 + i0 + u) * d + c] = v[u] + add;
  }
}

// ---------------------------------------------------------------------------
// Capture + mean-over-prompts reduction, z form (mean_p result =
// (mean_p z) @ W_O), for every layer of a forward in ONE pair of launches
// after the layer loop (blockIdx.z = layer; layer l's hook_z rows at
// z + l * zstride).  Deterministic two-pass: partial[l][g][c] = sum over rows
// g, g+G, ...; then zsum[l][c] += sum_g partial[l][g][c].  rows == nullptr:
// row i is z row i (the attention kernel's compact last-row copy).
constexpr int CAP_GROUPS = 128;  // row groups of the partial pass (fixed-order sums: deterministic)
__global__ void capture_partial_kernel(const float* __restrict__ z, int ldz, size_t zstride,
                                       const int32_t* __restrict__ rows, int n,
                                       float* __restrict__ partial, int d) {
  const int c4 = blockIdx.x * blockDim.x + threadIdx.x;  // float4 column
  const int g = blockIdx.y, l = blockIdx.z;
  if (c4 * 4 >= d) return;
  z += (size_t)l * zstride;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  int i = g;
  for (; i + 3 * CAP_GROUPS < n; i += 4 * CAP_GROUPS) {  // four rows' loads in flight, summed in row order
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = i + u * CAP_GROUPS;
      v[u] = ((const float4*)(z + (size_t)(rows ? rows[r] : r) * ldz))[c4];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w;
    }
  }
  for (; i < n; i += CAP_GROUPS) {
    const float4 v = ((const float4*)(z + (size_t)(rows ? rows[i] : i) * ldz))[c4];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  ((float4*)(partial + ((size_t)l * CAP_GROUPS + g) * d))[c4] = s;
}

__global__ void capture_finish_kernel(const float* __restrict__ partial,
                                      float* __restrict__ zsum, int d) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x, l = blockIdx.y;
  if (c >= d) return;
  partial += (size_t)l * CAP_GROUPS * d;
  float s = 0.f;
  for (int g = 0; g < CAP_GROUPS; ++g) s += partial[(size_t)g * d + c];
  zsum[(size_t)l * d + c] += s;
}

// out[l][h][c] = sum_k zsum[l][h*dh + k] * w2_l[c][h*dh + k]
__global__ void project_heads_kernel(const float* __restrict__ zsum,
                                     const float* const* __restrict__ w2s, int ldw2,
                                     float* __restrict__ out, int H, int d, int dh) {
  const int l = blockIdx.z, h = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d) return;
  const float* w = w2s[l] + (size_t)c * ldw2 + h * dh;
  const float* zz = zsum + (size_t)l * d + h * dh;
  float a = 0.f;
  for (int k = 0; k < dh; ++k) a += zz[k] * w[k];
  out[((size_t)l * H + h) * d + c] = a;
}

// ---------------------------------------------------------------------------
// Last-row statistics: softmax(logits)[target], top-k ids (descending value,
// lowest id first on ties: torch.argmax's first-occurrence rule).
constexpr int STATS_THREADS = 256;
constexpr int STATS_MAX_K = 16;

// One pass over the row (float4 loads when the row is 16-B aligned): each
// thread keeps an online (max, sum of exp) pair and its running argmax; the
// block combines them in a fixed order (deterministic).  Top-k rounds after
// the first rescan the row (L2-resident) with the chosen ids excluded.
__device__ __forceinline__ void stats_merge(float& m, float& s, float om, float os) {
  const float nm = fmaxf(m, om);
  s = (m == -INFINITY ? 0.f : s * expf(m - nm)) + (om == -INFINITY ? 0.f : os * expf(om - nm));
  m = nm;
}

__global__ void __launch_bounds__(STATS_THREADS)
row_stats_kernel(const float* __restrict__ logits, int ldl, int V,
                 const int32_t* __restrict__ targets, float* __restrict__ out_prob,
                 int32_t* __restrict__ out_topk, int topk) {
  __shared__ float s_val[STATS_THREADS / 64];
  __shared__ int s_idx[STATS_THREADS / 64];
  __shared__ float s_m[STATS_THREADS / 64], s_s[STATS_THREADS / 64];
  __shared__ int s_sel[STATS_MAX_K];
  const int r = blockIdx.x, t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const float* x = logits + (size_t)r * ldl;

  float m = -INFINITY, se = 0.f, bv = -INFINITY;
  int bi = 0x7fffffff;
  const bool vec = (((uintptr_t)x) & 15) == 0;
  const int V4 = vec ? V >> 2 : 0;
  for (int q = t; q < V4; q += STATS_THREADS) {
    const float4 v = ((const float4*)x)[q];
    const float m4 = fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w));
    if (m4 > m) {
      se = (m == -INFINITY ? 0.f : se * expf(m - m4));
      m = m4;
    }
    se += (expf(v.x - m) + expf(v.y - m)) + (expf(v.z - m) + expf(v.w - m));
    argmax_merge(bv, bi, v.x, 4 * q);
    argmax_merge(bv, bi, v.y, 4 * q + 1);
    argmax_merge(bv, bi, v.z, 4 * q + 2);
    argmax_merge(bv, bi, v.w, 4 * q + 3);
  }
  for (int v = 4 * V4 + t; v < V; v += STATS_THREADS) {  // tail (or the whole row, unaligned)
    const float xv = x[v];
    if (xv > m) {
      se = (m == -INFINITY ? 0.f : se * expf(m - xv));
      m = xv;
    }
    se += expf(xv - m);
    argmax_merge(bv, bi, xv, v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(se, o, 64);
    stats_merge(m, se, om, os);
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    argmax_merge(bv, bi, ov, oi);
  }
  if (lane == 0) {
    s_m[wave] = m;
    s_s[wave] = se;
    s_val[wave] = bv;
    s_idx[wave] = bi;
  }
  __syncthreads();
  if (t == 0) {
    float fm = s_m[0], fs = s_s[0], fv = s_val[0];
    int fi = s_idx[0];
    for (int w = 1; w < STATS_THREADS / 64; ++w) {
      stats_merge(fm, fs, s_m[w], s_s[w]);
      argmax_merge(fv, fi, s_val[w], s_idx[w]);
    }
    if (out_prob) {
      const int tg = targets ? targets[r] : -1;
      out_prob[r] = (tg >= 0 && tg < V) ? expf(x[tg] - fm) / fs : 0.f;
    }
    if (out_topk && topk > 0) {
      s_sel[0] = fi;
      out_topk[(size_t)r * topk] = fi;
    }
  }
  if (!out_topk || topk <= 1) return;
  __syncthreads();
  // top-k rounds 1..k-1: (value desc, index asc) block argmax with exclusion
  for (int j = 1; j < topk; ++j) {
    bv = -INFINITY;
    bi = 0x7fffffff;
    for (int v = t; v < V; v += STATS_THREADS) {
      bool taken = false;
      for (int q = 0; q < j; ++q) taken |= (s_sel[q] == v);
      if (taken) continue;
      argmax_merge(bv, bi, x[v], v);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      argmax_merge(bv, bi, ov, oi);
    }
    if (lane == 0) { s_val[wave] = bv; s_idx[wave] = bi; }
    __syncthreads();
    if (t == 0) {
      float fv = s_val[0];
      int fi = s_idx[0];
      for (int w = 1; w < STATS_THREADS / 64; ++w) argmax_merge(fv, fi, s_val[w], s_idx[w]);
      s_sel[j] = fi;
      out_topk[(size_t)r * topk + j] = fi;
    }
    __syncthreads();
  }
}

// Combine the per-tile records of EPI_STATS (gemm_f32.hpp GemmEpi::stats) into
// each row's target probability and top-k: one wave per row; lane l merges
// tiles l, l + 64, ... in order, then a butterfly (fixed order: deterministic).
// Top-k: topk rounds of (value desc, column asc) argmax over every tile's
// candidates with the chosen columns excluded; each column is a candidate of
// exactly one tile, and a tile's K candidates include every column of it that
// can be in the row's top K.
constexpr int MERGE_WAVES = 4;
__global__ void __launch_bounds__(64 * MERGE_WAVES)
stats_merge_kernel(const float* __restrict__ part, int tiles, int K, const float* __restrict__ tlogit,
                   const int32_t* __restrict__ targets, int n, int V, float* __restrict__ out_prob,
                   int32_t* __restrict__ out_topk, int topk) {
  __shared__ int s_sel[MERGE_WAVES][STATS_MAX_K];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * MERGE_WAVES + wave;
  if (r >= n) return;
  const int rec = 2 + 2 * K;
  const float* base = part + (size_t)r * tiles * rec;
  float m = -INFINITY, s = 0.f;
  for (int t = lane; t < tiles; t += 64) stats_merge(m, s, base[(size_t)t * rec], base[(size_t)t * rec + 1]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    stats_merge(m, s, om, os);
  }
  if (out_prob && lane == 0) {
    const int tg = targets ? targets[r] : -1;
    out_prob[r] = (tg >= 0 && tg < V) ? expf(tlogit[r] - m) / s : 0.f;
  }
  if (!out_topk || topk <= 0) return;
  for (int j = 0; j < topk; ++j) {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int t = lane; t < tiles; t += 64) {
      const float* c = base + (size_t)t * rec + 2;
      for (int q = 0; q < K; ++q) {
        const int id = __float_as_int(c[K + q]);
        bool taken = false;
        for (int u = 0; u < j; ++u) taken |= s_sel[wave][u] == id;
        if (!taken) argmax_merge(bv, bi, c[q], id);
      }
    }
    wave_argmax(bv, bi);
    if (lane == 0) {
      s_sel[wave][j] = bi;
      out_topk[(size_t)r * topk + j] = bi;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // s_sel[wave][j] before the next round's reads
  }
}

}  // namespace tvr

// engine.hip — runtime behind include/tvr.h.
//
// Owns the per-model rotary tables and activation workspace, plans batched
// sweeps (the "staircase": sites sorted by entry layer so the active rows of
// layer l are always a prefix of the activation buffer) and enqueues the
// kernels of kernels.hpp / gemm_f32.hpp on the caller's stream.
//
// Reference loops replaced (see include/tvr.h for the per-entry-point map):
// scratch2.py:81-100 (extraction), :114-150 (layer sweeps), :171-197 (CIE),
// :292-314 (FV eval) and scratch.py:106-147 (residual patch sweep).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "tvr.h"
#include "gemm_f32.hpp"
#include "attention_mfma.hpp"
#include "gemm_pingpong.hpp"
#include "gemm_skinny.hpp"
#include "gemm_planar.hpp"
#include "gemm_x2f16.hpp"
#include "gemm_x3bf16.hpp"
#include "kernels.hpp"
#include "lin_entry.hpp"
#include "entry_mfma.hpp"

using namespace tvr;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define TVR_HIP(expr)                                                           \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess)                                                       \
      return fail(TVR_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

#define TVR_TRY(expr)        \
  do {                       \
    int _rc = (expr);        \
    if (_rc != TVR_OK) return _rc; \
  } while (0)

constexpr size_t kAlign = 256;
inline size_t align_up(size_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

// Bump allocator over one device allocation.
struct Carve {
  size_t off = 0;
  template <class T>
  size_t take(size_t count) {
    const size_t at = off;
    off = align_up(off + count * sizeof(T));
    return at;
  }
};

// Pinned host staging for per-call metadata (descriptors, tokens).  Two
// buffers used alternately; an event guards reuse.
struct Staging {
  void* buf[2] = {nullptr, nullptr};
  size_t cap[2] = {0, 0};
  hipEvent_t done[2] = {nullptr, nullptr};
  bool pending[2] = {false, false};
  int next = 0;
};

// A GEMM weight operand: the fp32 matrix and, in a split mode, its planes
// (plane stride wps elements): TVR_GEMM_X3BF16 three bf16 planes in x;
// the planar modes in h: TVR_GEMM_X2F16 two fp16 planes of w * wscale,
// TVR_GEMM_BF16 one bf16 plane.
struct MatW {
  const float* f = nullptr;
  const uint16_t* x = nullptr;
  const uint16_t* h = nullptr;
  size_t wps = 0;
  float wscale = 1.0f;
  bool x16 = false;  // h is ONE plane holding the weights exactly (fp16 values: tvr_model_set_exact16)
  MatW rows(size_t elems) const {
    return {f ? f + elems : nullptr, x ? x + elems : nullptr, h ? h + elems : nullptr, wps, wscale, x16};
  }
};

// Launch plan of a planar GEMM (plan_pp), cached per (M, N, K, format, GELU epilogue, stream-K switch).
using PlanKey = std::tuple<int, int, int, int, int, int>;
struct PpPlan {
  int ksplit = 1;    // whole launch
  int tail_base = 0; // > 0: tiles [0, tail_base) plain, the rest split tail_split ways
  int tail_split = 1;
  int sk_base = -1;  // >= 0: tiles [0, sk_base) plain, the rest stream-K over sk_blocks blocks
  int sk_blocks = 0;
};
}  // namespace

struct tvr_model {
  tvr_config cfg{};
  int D1 = 0;  // 3d + d_mlp
  int K2 = 0;  // d + d_mlp
  const float* w_embed = nullptr;
  std::vector<tvr_layer_weights> layers;
  const float* w_unembed_t = nullptr;
  const float* b_unembed = nullptr;
  float* rot_cos = nullptr;
  float* rot_sin = nullptr;
  const float** d_w2s = nullptr;
  // GEMM operands (x planes set by tvr_model_set_gemm)
  int gemm_mode = TVR_GEMM_F32;
  uint16_t* planes = nullptr;
  unsigned* range_flag = nullptr;  // device word: X2F16 input out of range since the last status read
  std::vector<MatW> w1, w2;
  // TVR_GEMM_BF16 only: W1's Q / K rows [0, 2d) as one fp16 plane of
  // wscale * W (the attention-score projections run on fp16 operands: launch_w1)
  std::vector<MatW> w1qk;
  MatW wu;
  char* ws = nullptr;
  size_t ws_bytes = 0;
  float* splitk_ws = nullptr;  // split-K partial products (launch_gemm), grown on demand
  size_t splitk_bytes = 0;
  Staging staging;
  // profiling (tvr_profile_enable): event pairs around GEMM launches (kind =
  // GEMM epilogue index 0-2) and the HBM-bound kernels (kind 3 + tvr_hbm_kind)
  bool prof = false;
  struct ProfRec { hipEvent_t a, b; int epi; double flops, bytes; };
  std::vector<ProfRec> prof_recs;
  std::vector<hipEvent_t> prof_pool;
  // Linearised entry layer (lin_entry.hpp), built on the first patch sweep that
  // uses it in a planar mode and dropped on a mode change: for layers
  // l = 1 .. L-2, Wsc = W1[l] W_O[l-1] as weight planes [NPL][H][D1][KP]
  // (head-major, d_head zero-padded to KP) and c1[l] = row sums of W1[l].
  int lin_mode = -1;
  int lin_failed_mode = -1;  // the planes did not fit in this GEMM mode: the sweeps use the full entry GEMM
  int lin_kp = 0;
  uint16_t* lin_planes = nullptr;  // layer l at (l - 1) * NPL * H * D1 * KP halves
  float* lin_c1 = nullptr;         // [L][D1]
  std::vector<float> lin_scale;    // per layer: X2F16 plane scale (1 for BF16)
  std::map<PlanKey, PpPlan> plans;  // plan_pp_cached: GEMM launch plans per shape
  // Exact-fp16 weights (tvr_model_set_exact16; x2f16 mode only): the checkpoint's own W1 rows (Q | K | V |
  // MLP-in, before fold_ln) and W2 (W_O | W_out, before center_writing_weights) as one caller-owned fp16
  // plane each, and LN1 / LN2's gamma.  The QKV + MLP-in GEMM then reads LNPre(x) * gamma1 (Q, K, V
  // columns) / * gamma2 (MLP-in columns) against the raw rows — fold_ln's centring of the read-in weights
  // is a no-op on a centred LNPre row — and the O + MLP-out GEMM the raw W2, whose missing centring adds one
  // constant to every element of a row's residual, which every LayerNorm (and the centred trace export)
  // removes.  Both then run 2 MFMA products per slice instead of 3 (gemm_pingpong.hpp WX).
  bool x16 = false;
  std::vector<MatW> w1x, w2x;
  std::vector<const float*> g1, g2;
  // the unembed's raw W_U [V][d] (one fp16 plane) and the final LN's gamma (tvr_model_set_exact16_unembed): the
  // fused-statistics unembed reads LNPre(x) * gf against it (2 products).  fold_ln's centring is a no-op again,
  // and center_unembed's mean over the vocabulary is one constant per row of logits, which the statistics
  // (softmax probability, top-k) do not see; the logits paths keep the processed W_U.
  MatW wux;
  const float* gf = nullptr;
};

struct tvr_trace {
  tvr_model* model = nullptr;
  int max_seqs = 0, max_tokens = 0;
  float* resid = nullptr;  // [L+1][max_tokens][d]
  float* z = nullptr;      // [L][max_tokens][d]
  float* qkv = nullptr;    // [L][max_tokens][3d]
  std::vector<int> seq_off, seq_len;
  std::vector<int32_t> tokens;  // host copy of the traced ids (shared-prefix detection in patch sweeps)
  int n_seq = 0, n_tokens = 0;
  // A deferred clean forward (tvr_forward_clean_deferred): the metadata above
  // is set, the buffers are not; the next tvr_patch_sweep on this trace runs
  // the clean rows inside its own launches (filling the buffers as
  // tvr_forward_clean would) and writes these outputs; any other use of the
  // trace runs it on its own first (flush_pending).
  bool pending = false;
  bool uncentred = false;  // filled on the exact-fp16 weight path: hook_resid_pre is centred on export
  std::vector<int32_t> p_targets;  // [n_seq] or empty
  float* p_prob = nullptr;
  int32_t* p_topk = nullptr;
  int p_k = 0;
  void* p_stream = nullptr;  // the stream of the deferral (its inputs / outputs are ordered on it)
};

namespace {

constexpr int kFinalChunk = 1024;

int ensure_workspace(tvr_model* m, size_t bytes, hipStream_t st) {
  if (bytes <= m->ws_bytes) return TVR_OK;
  TVR_HIP(hipStreamSynchronize(st));
  if (m->ws) TVR_HIP(hipFree(m->ws));
  m->ws = nullptr;
  m->ws_bytes = 0;
  const size_t want = align_up(bytes + bytes / 8);
  if (hipMalloc(&m->ws, want) != hipSuccess) {
    m->ws = nullptr;
    (void)hipGetLastError();
    return fail(TVR_ERR_NOMEM, "workspace allocation of " + std::to_string(want) + " bytes failed");
  }
  m->ws_bytes = want;
  return TVR_OK;
}

int ensure_splitk(tvr_model* m, size_t bytes, hipStream_t st) {
  if (bytes <= m->splitk_bytes) return TVR_OK;
  TVR_HIP(hipStreamSynchronize(st));
  if (m->splitk_ws) TVR_HIP(hipFree(m->splitk_ws));
  m->splitk_ws = nullptr;
  m->splitk_bytes = 0;
  const size_t want = align_up(bytes);
  if (hipMalloc(&m->splitk_ws, want) != hipSuccess) {
    m->splitk_ws = nullptr;
    (void)hipGetLastError();
    return fail(TVR_ERR_NOMEM, "split-K workspace allocation of " + std::to_string(want) + " bytes failed");
  }
  m->splitk_bytes = want;
  return TVR_OK;
}

// Copy host bytes to device through pinned staging (async on `st`).
int upload(tvr_model* m, hipStream_t st, void* dst, const void* src, size_t bytes) {
  if (bytes == 0) return TVR_OK;
  Staging& s = m->staging;
  const int i = s.next;
  s.next ^= 1;
  if (s.pending[i]) {
    TVR_HIP(hipEventSynchronize(s.done[i]));
    s.pending[i] = false;
  }
  if (s.cap[i] < bytes) {
    if (s.buf[i]) TVR_HIP(hipHostFree(s.buf[i]));
    s.buf[i] = nullptr;
    const size_t want = align_up(std::max(bytes, (size_t)1 << 20));
    TVR_HIP(hipHostMalloc(&s.buf[i], want, hipHostMallocDefault));
    s.cap[i] = want;
  }
  if (!s.done[i]) TVR_HIP(hipEventCreateWithFlags(&s.done[i], hipEventDisableTiming));
  std::memcpy(s.buf[i], src, bytes);
  TVR_HIP(hipMemcpyAsync(dst, s.buf[i], bytes, hipMemcpyHostToDevice, st));
  TVR_HIP(hipEventRecord(s.done[i], st));
  s.pending[i] = true;
  return TVR_OK;
}

// Several host arrays packed into ONE upload (one staging buffer, one copy).
struct UploadBatch {
  std::vector<char> host;
  struct Item { size_t host_off; size_t dev_off; size_t bytes; };
  std::vector<Item> items;
  template <class T>
  void add(size_t dev_off, const std::vector<T>& v) {
    items.push_back({host.size(), dev_off, v.size() * sizeof(T)});
    const char* p = reinterpret_cast<const char*>(v.data());
    host.insert(host.end(), p, p + v.size() * sizeof(T));
  }
};

int flush_uploads(tvr_model* m, hipStream_t st, char* base, const UploadBatch& ub) {
  // Items are carved contiguously in order, so the batch is one span.
  if (ub.items.empty()) return TVR_OK;
  const size_t first = ub.items.front().dev_off;
  std::vector<char> span;
  size_t end = first;
  for (const auto& it : ub.items) end = std::max(end, it.dev_off + it.bytes);
  span.assign(end - first, 0);
  for (const auto& it : ub.items)
    std::memcpy(span.data() + (it.dev_off - first), ub.host.data() + it.host_off, it.bytes);
  return upload(m, st, base + first, span.data(), span.size());
}

hipEvent_t prof_event(tvr_model* m) {
  hipEvent_t e = nullptr;
  if (!m->prof_pool.empty()) {
    e = m->prof_pool.back();
    m->prof_pool.pop_back();
  } else if (hipEventCreate(&e) != hipSuccess) {
    e = nullptr;
  }
  return e;
}

// HIP events around one HBM-bound launch (or a short launch sequence) while
// profiling: done(kind, algorithmic bytes) records the closing event.
struct ProfSpan {
  tvr_model* m;
  hipStream_t st;
  hipEvent_t a = nullptr, b = nullptr;
  ProfSpan(tvr_model* m_, hipStream_t s) : m(m_), st(s) {
    if (m && m->prof) {
      a = prof_event(m);
      b = prof_event(m);
      if (a) (void)hipEventRecord(a, st);
    }
  }
  void done(int kind, double bytes) {
    if (!a || !b) return;
    (void)hipEventRecord(b, st);
    m->prof_recs.push_back({a, b, 3 + kind, 0.0, bytes});
    a = b = nullptr;
  }
  ~ProfSpan() {  // not done (error path): events back to the pool
    if (a) m->prof_pool.push_back(a);
    if (b) m->prof_pool.push_back(b);
  }
};

// TVR_PREFIX_SHARE=0 turns off shared-prefix rows in tvr_forward_clean /
// tvr_patch_sweep (read per call; the tests run both settings and compare).
bool env_flag(const char* name) {
  const char* e = getenv(name);
  return !(e && std::string(e) == "0");
}
bool prefix_share_enabled() { return env_flag("TVR_PREFIX_SHARE"); }
// TVR_LIN_ENTRY=0 runs the entry layer of REPLACE_HEAD sites through the full
// GEMM instead of lin_entry.hpp (the tests compare both).
bool lin_entry_enabled() { return env_flag("TVR_LIN_ENTRY"); }

// Activation format of the model's GEMM inputs (split.hpp).
int act_fmt(const tvr_model* m) {
  return m->gemm_mode == TVR_GEMM_X2F16 ? ACT_X2F16 : m->gemm_mode == TVR_GEMM_BF16 ? ACT_BF16 : ACT_F32;
}

// the exact-fp16 weight path (tvr_model_set_exact16) is on: x2f16 mode with the raw planes attached
bool use_x16(const tvr_model* m) { return m->x16 && m->gemm_mode == TVR_GEMM_X2F16; }

// gemm_pingpong_kernel over tiles [tile_base, tile_base + count) of a planar
// launch's raster (count 0: all), VEC epilogue
// Raster group (m-blocks walked before the next block column): 4, or 2 when
// there are at most 16 block columns (tools/gemm_split_probe x2ppgm<N>: at
// M = 90,000 the qkv shape ran 459 / 451 / 419 TF at 4 / 8 / 16, the
// MLP-out shape (10 columns) 470 / 466 / 458 at 2 / 4 / 8).
// A/B knobs TVR_PP_GM_SMALL / TVR_PP_GM_LARGE (read once) override the two values.
int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && *e ? atoi(e) : dflt;
}
int pp_group_m(int N) {
  static const int small = env_int("TVR_PP_GM_SMALL", 2), large = env_int("TVR_PP_GM_LARGE", 4);
  return (N + 255) / 256 <= 16 ? small : large;
}

void launch_pp(int epi, const uint16_t* Ah, int lda, int a_fmt, const MatW& W, int ldw, int M, int N, int K,
               const GemmEpi& ep0, float acc_scale, int tile_base, int count, bool vec, bool sl, hipStream_t st) {
  GemmEpi ep = ep0;
  ep.tile_base = tile_base;
  ep.tile_count = count;
  ep.group_m = pp_group_m(N);
  const dim3 g(count > 0 ? count : gemm_pingpong_grid(M, N));
  const bool wx = a_fmt == ACT_X2F16 && W.x16;  // one exact fp16 weight plane: 2 products (launch_gemm checks)
#define TVR_PP1(E, F, V, S, X)                                                                                    \
  hipLaunchKernelGGL((gemm_pingpong_kernel<E, F, V, 0, false, S, X>), g, dim3(PP_THREADS), 0, st, Ah, 2 * lda,    \
                     (size_t)lda, W.h, ldw, W.wps, acc_scale, M, N, K, ep)
#define TVR_PP1V(E, F, S, X) \
  if (vec) { TVR_PP1(E, F, true, S, X); } else { TVR_PP1(E, F, false, S, X); }
#define TVR_PP1F(E)                                                                                \
  if (a_fmt == ACT_X2F16) {                                                                        \
    if (wx) {                                                                                      \
      if (sl) { TVR_PP1V(E, ACT_X2F16, true, true); } else { TVR_PP1V(E, ACT_X2F16, false, true); } \
    } else {                                                                                       \
      if (sl) { TVR_PP1V(E, ACT_X2F16, true, false); } else { TVR_PP1V(E, ACT_X2F16, false, false); } \
    }                                                                                              \
  } else {                                                                                         \
    TVR_PP1V(E, ACT_BF16, false, false);                                                           \
  }
  if (a_fmt == ACT_F16) {  // the bf16 mode's Q / K columns: plain fp32 outputs only (launch_gemm checks)
    TVR_PP1V(EPI_BIAS, ACT_F16, false, false);
    return;
  }
  switch (epi) {
    case EPI_BIAS: TVR_PP1F(EPI_BIAS); break;
    case EPI_SPLIT_GELU_ACT: TVR_PP1F(EPI_SPLIT_GELU_ACT); break;
    case EPI_STATS:  // LDS epilogue only (vec: N % 4 == 0, host-checked)
      if (a_fmt != ACT_X2F16) {
        TVR_PP1(EPI_STATS, ACT_BF16, true, false, false);
      } else if (sl) {
        if (wx) { TVR_PP1(EPI_STATS, ACT_X2F16, true, true, true); } else { TVR_PP1(EPI_STATS, ACT_X2F16, true, true, false); }
      } else {
        if (wx) { TVR_PP1(EPI_STATS, ACT_X2F16, true, false, true); } else { TVR_PP1(EPI_STATS, ACT_X2F16, true, false, false); }
      }
      break;
    default: TVR_PP1F(EPI_RESID); break;
  }
#undef TVR_PP1F
#undef TVR_PP1V
#undef TVR_PP1
}

// The same tiles with K split over `ksplit` blocks per tile: fp32 partial
// tiles to the model's split-K workspace, then splitk_reduce_kernel sums them
// in order and applies the epilogue (deterministic).
int launch_pp_splitk(int epi, const uint16_t* Ah, int lda, int a_fmt, const MatW& W, int ldw, int M, int N, int K,
                     const GemmEpi& ep0, float acc_scale, int tile_base, int count, int ksplit, bool sl, tvr_model* m,
                     hipStream_t st) {
  const int rc = ensure_splitk(m, (size_t)ksplit * count * PP_TILE_ELEMS * sizeof(float), st);
  if (rc != TVR_OK) return rc;
  GemmEpi ep = ep0;  // the reduce's epilogue: same raster as the partial launch
  ep.group_m = pp_group_m(N);
  GemmEpi pe{};
  pe.group_m = ep.group_m;
  pe.out0 = m->splitk_ws;
  pe.a_rows = ep.a_rows;
  pe.k_split = ksplit;
  pe.tile_base = tile_base;
  pe.tile_count = count;
  const dim3 g(count * ksplit), rg((unsigned)std::min<long>(4096, ((long)count * (PP_TILE_ELEMS / 4) + 255) / 256));
  pe.a2 = ep.a2;  // the exact-fp16 QKV + MLP-in launch's second A operand (by column)
  pe.a2_col = ep.a2_col;
  const bool wx = a_fmt == ACT_X2F16 && W.x16;
  if (a_fmt == ACT_X2F16 && wx && sl)
    hipLaunchKernelGGL((gemm_pingpong_kernel<EPI_BIAS, ACT_X2F16, true, 0, false, true, true>), g, dim3(PP_THREADS), 0,
                       st, Ah, 2 * lda, (size_t)lda, W.h, ldw, W.wps, acc_scale, M, N, K, pe);
  else if (a_fmt == ACT_X2F16 && wx)
    hipLaunchKernelGGL((gemm_pingpong_kernel<EPI_BIAS, ACT_X2F16, true, 0, false, false, true>), g, dim3(PP_THREADS), 0,
                       st, Ah, 2 * lda, (size_t)lda, W.h, ldw, W.wps, acc_scale, M, N, K, pe);
  else if (a_fmt == ACT_X2F16 && sl)  // sliced accumulation (gemm_pingpong.hpp)
    hipLaunchKernelGGL((gemm_pingpong_kernel<EPI_BIAS, ACT_X2F16, true, 0, false, true>), g, dim3(PP_THREADS), 0, st,
                       Ah, 2 * lda, (size_t)lda, W.h, ldw, W.wps, acc_scale, M, N, K, pe);
  else if (a_fmt == ACT_X2F16)
    hipLaunchKernelGGL((gemm_pingpong_kernel<EPI_BIAS, ACT_X2F16, true>), g, dim3(PP_THREADS), 0, st, Ah, 2 * lda,
                       (size_t)lda, W.h, ldw, W.wps, acc_scale, M, N, K, pe);
  else if (a_fmt == ACT_F16)
    hipLaunchKernelGGL((gemm_pingpong_kernel<EPI_BIAS, ACT_F16, true>), g, dim3(PP_THREADS), 0, st, Ah, 2 * lda,
                       (size_t)lda, W.h, ldw, W.wps, acc_scale, M, N, K, pe);
  else
    hipLaunchKernelGGL((gemm_pingpong_kernel<EPI_BIAS, ACT_BF16, true>), g, dim3(PP_THREADS), 0, st, Ah, 2 * lda,
                       (size_t)lda, W.h, ldw, W.wps, acc_scale, M, N, K, pe);
#define TVR_SK_REDUCE(E, F)                                                                                     \
  hipLaunchKernelGGL((splitk_reduce_kernel<E, F>), rg, dim3(256), 0, st, (const float*)m->splitk_ws, ksplit, \
                     tile_base, count, M, N, ep)
#define TVR_SK_REDUCE_F(E) \
  if (a_fmt == ACT_X2F16) { TVR_SK_REDUCE(E, ACT_X2F16); } else { TVR_SK_REDUCE(E, ACT_BF16); }
  switch (epi) {
    case EPI_BIAS: TVR_SK_REDUCE_F(EPI_BIAS); break;
    case EPI_SPLIT_GELU_ACT: TVR_SK_REDUCE_F(EPI_SPLIT_GELU_ACT); break;
    default: TVR_SK_REDUCE_F(EPI_RESID); break;
  }
#undef TVR_SK_REDUCE_F
#undef TVR_SK_REDUCE
  return TVR_OK;
}

// Stream-K over tiles [tile_base, tile_base + count): G blocks share their
// k-iterations evenly (gemm_pingpong_kernel sk_blocks), fp32 partial tiles to
// the model's split-K workspace, then splitk_sk_reduce_kernel sums each tile's
// partials in k order and applies the epilogue (deterministic).
int launch_pp_sk(int epi, const uint16_t* Ah, int lda, int a_fmt, const MatW& W, int ldw, int M, int N, int K,
                 const GemmEpi& ep0, float acc_scale, int tile_base, int count, int G, bool sl, tvr_model* m,
                 hipStream_t st) {
  const int rc = ensure_splitk(m, (size_t)2 * G * PP_TILE_ELEMS * sizeof(float), st);
  if (rc != TVR_OK) return rc;
  GemmEpi ep = ep0;
  ep.group_m = pp_group_m(N);
  GemmEpi pe{};
  pe.group_m = ep.group_m;
  pe.out0 = m->splitk_ws;
  pe.a_rows = ep.a_rows;
  pe.sk_blocks = G;
  pe.tile_base = tile_base;
  pe.tile_count = count;
  const dim3 g(G), rg((unsigned)std::min<long>(4096, ((long)count * (PP_TILE_ELEMS / 4) + 255) / 256));
  pe.a2 = ep.a2;
  pe.a2_col = ep.a2_col;
  const bool wx = a_fmt == ACT_X2F16 && W.x16;
  if (a_fmt == ACT_X2F16 && wx && sl)
    hipLaunchKernelGGL((gemm_pingpong_kernel<EPI_BIAS, ACT_X2F16, true, 0, true, true, true>), g, dim3(PP_THREADS), 0, st,
                       Ah, 2 * lda, (size_t)lda, W.h, ldw, W.wps, acc_scale, M, N, K, pe);
  else if (a_fmt == ACT_X2F16 && wx)
    hipLaunchKernelGGL((gemm_pingpong_kernel<EPI_BIAS, ACT_X2F16, true, 0, true, false, true>), g, dim3(PP_THREADS), 0,
                       st, Ah, 2 * lda, (size_t)lda, W.h, ldw, W.wps, acc_scale, M, N, K, pe);
  else if (a_fmt == ACT_X2F16 && sl)  // sliced accumulation (gemm_pingpong.hpp)
    hipLaunchKernelGGL((gemm_pingpong_kernel<EPI_BIAS, ACT_X2F16, true, 0, true, true>), g, dim3(PP_THREADS), 0, st,
                       Ah, 2 * lda, (size_t)lda, W.h, ldw, W.wps, acc_scale, M, N, K, pe);
  else if (a_fmt == ACT_X2F16)
    hipLaunchKernelGGL((gemm_pingpong_kernel<EPI_BIAS, ACT_X2F16, true, 0, true>), g, dim3(PP_THREADS), 0, st, Ah, 2 * lda,
                       (size_t)lda, W.h, ldw, W.wps, acc_scale, M, N, K, pe);
  else if (a_fmt == ACT_F16)
    hipLaunchKernelGGL((gemm_pingpong_kernel<EPI_BIAS, ACT_F16, true, 0, true>), g, dim3(PP_THREADS), 0, st, Ah, 2 * lda,
                       (size_t)lda, W.h, ldw, W.wps, acc_scale, M, N, K, pe);
  else
    hipLaunchKernelGGL((gemm_pingpong_kernel<EPI_BIAS, ACT_BF16, true, 0, true>), g, dim3(PP_THREADS), 0, st, Ah, 2 * lda,
                       (size_t)lda, W.h, ldw, W.wps, acc_scale, M, N, K, pe);
  const int KT = K / (a_fmt == ACT_X2F16 ? 32 : 64);
#define TVR_SKR(E, F)                                                                                         \
  hipLaunchKernelGGL((splitk_sk_reduce_kernel<E, F>), rg, dim3(256), 0, st, (const float*)m->splitk_ws, G, KT, \
                     tile_base, count, M, N, ep)
#define TVR_SKR_F(E) \
  if (a_fmt == ACT_X2F16) { TVR_SKR(E, ACT_X2F16); } else { TVR_SKR(E, ACT_BF16); }
  switch (epi) {
    case EPI_BIAS: TVR_SKR_F(EPI_BIAS); break;
    case EPI_SPLIT_GELU_ACT: TVR_SKR_F(EPI_SPLIT_GELU_ACT); break;
    default: TVR_SKR_F(EPI_RESID); break;
  }
#undef TVR_SKR_F
#undef TVR_SKR
  return TVR_OK;
}

// Launch shape of a planar GEMM on 256 CUs (gemm_pingpong_kernel, one block
// per CU): the whole launch plain, the whole launch split over K (fp32
// partials + splitk_reduce_kernel), or its last tiles split (a partly empty
// last round), and — opt-in, TVR_STREAM_K=1 — stream-K for the last round.
// Launches of up to 1,024 tiles (the small-M layer sweeps: C2's M = 156 + 52 l
// rows) are planned by simulating the dispatch (plan_sim): blocks in
// blockIdx order through the kernel's XCD remap onto the first free of 256
// CUs, a block costing its k-tiles at a rate set by its tile's real rows (a
// wave group skips the MFMAs of its padding 16-row slices; the staging
// remains) plus prologue and epilogue, a split plan the reduce's partial round
// trip on top.  Larger launches keep the round heuristic (their full rounds
// dominate).  Costs in us: profiles/r03/c2_sweep_dispatches_r03f.txt (a C2
// sweep per dispatch: 1.5-2.2 us per x2f16 k-tile per block, reduce at ~5 TB/s).
// stream-K is opt-in: on the C2 sweeps it measured slower than the split-K
// plan (O + MLP-out 8.2 vs 5.7 ms per sweep) and equal on C3
// (profiles/r03/c2_stream_k_ab.txt)
// TVR_STREAM_K: "1" every planned launch, "O" the O + MLP-out launches only (EPI_RESID: 10 column tiles at
// 2.8B, so a rank's share of a split sweep ends in partly filled rounds), else off
int sk_mode() {
  const char* e = getenv("TVR_STREAM_K");
  return !e ? 0 : std::string(e) == "1" ? 1 : std::string(e) == "O" ? 2 : 0;
}
bool sk_enabled(int epi = EPI_BIAS) {
  const int md = sk_mode();
  return md == 1 || (md == 2 && epi == EPI_RESID);
}

struct PlanCost {
  double kt_us, pro_us, epi_us, part_us;
};

// Simulated time (us) of tiles [t0, t0 + cnt) of the raster launched with S
// blocks per tile (S = 1: plain epilogue; S > 1: partial tiles, no reduce).
double plan_sim(int M, int N, int nkt, int t0, int cnt, int S, const PlanCost& pc) {
  const int nbm = (M + 255) / 256, nbn = (N + 255) / 256, gm = pp_group_m(N);
  const int nb = cnt * S, P = 256;
  std::vector<double> cu(P, 0.0);  // CU free times (a min-heap)
  auto remap = [](int bid, int nwg) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  };
  double end = 0.0;
  for (int b = 0; b < nb; ++b) {
    const int wgs = remap(b, nb), lt = wgs / S, split = wgs - lt * S;
    int m0, n0;
    pp_tile_coords(t0 + lt, nbm, nbn, m0, n0, gm);
    (void)n0;
    const int rows = std::min(256, M - m0);
    const int s0 = (std::min(rows, 128) + 15) / 16, s1 = (std::max(rows - 128, 0) + 15) / 16;
    const double frac = 0.3 + 0.7 * std::max(s0, s1) / 8.0;
    const int kb = (int)((long long)split * nkt / S), ke = (int)((long long)(split + 1) * nkt / S);
    const double dur = pc.pro_us + (ke - kb) * pc.kt_us * frac + (S > 1 ? pc.part_us : pc.epi_us);
    std::pop_heap(cu.begin(), cu.end(), std::greater<double>());
    cu.back() += dur;
    end = std::max(end, cu.back());
    std::push_heap(cu.begin(), cu.end(), std::greater<double>());
  }
  return end;
}

// the split-K reduce of tiles [t0, t0 + cnt) over S partials: launch + partials read + output written
double plan_reduce_us(int M, int N, int t0, int cnt, int S) {
  const int nbm = (M + 255) / 256, nbn = (N + 255) / 256, gm = pp_group_m(N);
  double rows = 0.0;
  for (int t = t0; t < t0 + cnt; ++t) {
    int m0, n0;
    pp_tile_coords(t, nbm, nbn, m0, n0, gm);
    rows += std::min(256, M - m0) * (double)std::min(256, N - n0);
  }
  return 4.0 + rows * 4.0 * (2.0 * S + 1.0) / 5.0e6;  // partials written (by the GEMM) + read, output written
}

// sliced: the launch runs the x2f16 sliced accumulation (~13 % more per k-tile: gemm_pingpong.hpp); wx: one
// exact weight plane, 2 products (0.72 of the 3-product k-tile, 0.85 sliced: profiles/r05/wx_probe_r05r.jsonl)
PpPlan plan_pp(int M, int N, int K, int a_fmt, int epi, bool sliced = false, bool wx = false) {
  PpPlan p;
  const int tiles = gemm_pingpong_grid(M, N), nkt = K / (a_fmt == ACT_X2F16 ? 32 : 64);
  const double kt_scale = wx ? (sliced ? 0.85 : 0.72) : 1.0;
  const double kt_us = (a_fmt == ACT_X2F16 ? 1.9 : 1.3) * (sliced ? 1.13 : 1.0) * kt_scale, seg_us = 15.0,
               epi_us = 10.0;
  // stream-K of `cnt` tiles over min(256, iterations) blocks vs one plain round
  auto sk_us = [&](int cnt) {
    const int G = (int)std::min<long long>(256, (long long)cnt * nkt);
    return std::ceil((double)cnt * nkt / G) * kt_us + 2.0 * seg_us + (cnt + 2.0 * G) * 0.0655 + 5.0;
  };
  const double round_plain_us = nkt * kt_us + epi_us;
  if (sk_enabled(epi) && (long long)tiles * nkt >= 4LL * 256) {
    const int rounds = (tiles + 255) / 256;
    const int tb = tiles - 256 * (rounds - 1);  // tiles of the last (partly empty) round
    if (tb < 256 && sk_us(tb) + 5.0 < round_plain_us) {
      p.sk_base = tiles - tb;
      p.sk_blocks = (int)std::min<long long>(256, (long long)tb * nkt);
      return p;
    }
  }
  if (tiles <= 1024) {
    const PlanCost pc{kt_us, 3.0, epi == EPI_SPLIT_GELU_ACT ? 15.0 : 10.0, 7.0};
    double best = plan_sim(M, N, nkt, 0, tiles, 1, pc);
    // at most 4,096 partial tiles (1 GiB of split-K workspace, which only grows: ensure_splitk)
    for (int S = 2; S <= 16 && nkt / S >= 8 && tiles * S <= 4096; ++S) {
      const double c = plan_sim(M, N, nkt, 0, tiles, S, pc) + plan_reduce_us(M, N, 0, tiles, S);
      if (c < best * 0.97) {  // a split must win clearly: the model is approximate
        best = c;
        p.ksplit = S;
      }
    }
    if (tiles > 256) {
      const int base = 256 * ((tiles - 1) / 256), cnt = tiles - base;
      const double head = plan_sim(M, N, nkt, 0, base, 1, pc);
      for (int S = 2; S <= 16 && nkt / S >= 8; ++S) {
        const double c = head + plan_sim(M, N, nkt, base, cnt, S, pc) + plan_reduce_us(M, N, base, cnt, S);
        if (c < best * 0.97) {
          best = c;
          p.ksplit = 1;
          p.tail_base = base;
          p.tail_split = S;
        }
      }
    }
    return p;
  }
  const int rounds = (tiles + 255) / 256;
  const int tb = tiles - 256 * (rounds - 1);
  if (tb > 224) return p;
  int best = 1;
  double br = 1.0;
  for (int s = 2; s <= 16 && nkt / s >= 8; ++s) {
    const double r = std::ceil(tb * (double)s / 256.0) / s;
    if (r < br - 1e-9) {
      br = r;
      best = s;
    }
  }
  if (best < 2) return p;
  const double round_us = nkt * 2.5 * kt_scale;  // ~2.3-2.7 us per k-tile per block (profiles/gemm_pingpong_anatomy_r01.jsonl)
  const double saved_us = (1.0 - br) * round_us;
  const double cost_us = (best + 1.0) * tb * (double)PP_TILE_ELEMS * 8.0 / 5.0e6;  // partials written + read, ~5 TB/s
  if (saved_us > 1.5 * cost_us + 10.0) {
    p.tail_base = 256 * (rounds - 1);
    p.tail_split = best;
  }
  return p;
}

// plan_pp, cached per launch shape on the model (the sweeps repeat their
// per-layer shapes: the simulation runs once per shape)
PpPlan plan_pp_cached(tvr_model* m, int M, int N, int K, int a_fmt, int epi, bool wx = false) {
  const PlanKey key{M, N, K, a_fmt + (wx ? 16 : 0), epi == EPI_SPLIT_GELU_ACT ? 1 : epi == EPI_RESID ? 2 : 0, sk_mode()};
  auto it = m->plans.find(key);
  if (it != m->plans.end()) return it->second;
  const PpPlan p = plan_pp(M, N, K, a_fmt, epi, a_fmt == ACT_X2F16 && (K >= PP_SLICE_MIN_K || m->K2 >= PP_SLICE_MIN_K),
                           wx);
  if (m->plans.size() > 4096) m->plans.clear();
  m->plans.emplace(key, p);
  return p;
}

// C = A @ W^T with epilogue `epi`.  A is fp32 [M][lda] (a_fmt ACT_F32:
// gemm_f32_nt_kernel, or the in-GEMM splits of the primitive ABI entry points
// when W carries x3bf16 / x2f16 planes) or a planar activation format
// (split.hpp: lda logical elements per row) with the same format's weight
// planes (W.h): gemm_pingpong_kernel, split-K below 192 tiles and a split last
// round when it pays (plan_pp; not for EPI_STATS, whose statistics exist only
// in the whole-K LDS epilogue).
int launch_gemm(int epi, const void* A, int lda, int a_fmt, const MatW& W, int ldw, int M, int N,
                int K, const GemmEpi& ep, hipStream_t st, tvr_model* m = nullptr,
                unsigned* range_flag = nullptr) {
  if (M <= 0 || N <= 0) return TVR_OK;
  const bool planar = a_fmt != ACT_F32;
  if (planar && !W.h) return fail(TVR_ERR_INVALID, "gemm: planar activations need the planar weight planes");
  if (epi == EPI_SPLIT_GELU_ACT && !planar)
    return fail(TVR_ERR_INVALID, "gemm: the activation-format GELU epilogue belongs to the planar paths");
  if (epi == EPI_SPLIT_GELU && planar)
    return fail(TVR_ERR_INVALID, "gemm: planar paths write GELU columns in their activation format");
  if (epi == EPI_STATS && (!planar || N % 4 != 0 || !ep.stats))
    return fail(TVR_ERR_INVALID, "gemm: the fused statistics epilogue needs a planar format, N % 4 == 0 and a "
                                 "statistics buffer");
  if (a_fmt == ACT_F16 && epi != EPI_BIAS)
    return fail(TVR_ERR_INVALID, "gemm: the fp16 operand format has the plain (bias) epilogue only");
  if (W.x16 && a_fmt != ACT_X2F16)
    return fail(TVR_ERR_INVALID, "gemm: one-plane exact fp16 weights take x2f16 activations");
  if (ep.a2 && (a_fmt == ACT_F32 || ep.a2_col % 256 != 0))
    return fail(TVR_ERR_INVALID, "gemm: a second A operand needs a planar format and a 256-column boundary");
  if (K % GEMM_BK != 0 || lda % 4 != 0 || ldw % 4 != 0 || ((W.x || W.h) && ldw % 8 != 0) ||
      ((a_fmt == ACT_BF16 || a_fmt == ACT_F16) && K % 64 != 0))
    return fail(TVR_ERR_UNSUPPORTED, "gemm: K, lda, ldw must be multiples of 32/4/4 (8 for planes, K of 64 for "
                                     "bf16; K=" + std::to_string(K) + ")");
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  if (m && m->prof) {
    ev0 = prof_event(m);
    ev1 = prof_event(m);
    if (ev0) TVR_HIP(hipEventRecord(ev0, st));
  }
  // X2F16: both operands scaled (W by wscale, A by 16); F16: W only; BF16: neither
  const float acc_scale = a_fmt == ACT_BF16 ? 1.0f : a_fmt == ACT_F16 ? 1.0f / W.wscale : 1.0f / (W.wscale * X2_ASCALE);
  if (planar) {
    const uint16_t* Ah = static_cast<const uint16_t*>(A);
    const bool vec = planar_epilogue_vec(epi, ep, N);
    // x2f16 sliced accumulation (gemm_pingpong.hpp) on every GEMM of a model whose O + MLP-out K reaches
    // PP_SLICE_MIN_K (6.9B, 12B), or on any launch of that K
    // (one-plane weights, A/B of the precision it costs: TVR_WX_SLICE=0 runs them unsliced, 2 slices the
    // O + MLP-out launches only)
    static const int wx_slice = env_int("TVR_WX_SLICE", 1);
    const bool sl = a_fmt == ACT_X2F16 && (K >= PP_SLICE_MIN_K || (m && m->K2 >= PP_SLICE_MIN_K)) &&
                    (!W.x16 || wx_slice == 1 || (wx_slice == 2 && epi == EPI_RESID));
    if (ep.skinny && epi == EPI_BIAS && M <= SK_USE_M && !ep.out_rows && ep.k_split <= 1 && vec &&
        a_fmt != ACT_F16 && !W.x16 && !ep.a2) {
      // a few rows (the linearised entry's G on a rank of a head split): gemm_skinny.hpp
      const dim3 g(gemm_skinny_grid(N));
#define TVR_SK(F, MT)                                                                                  \
  hipLaunchKernelGGL((gemm_skinny_kernel<F, MT>), g, dim3(SK_THREADS), 0, st, Ah, 2 * lda, (size_t)lda, W.h, \
                     ldw, W.wps, acc_scale, M, N, K, ep)
#define TVR_SK_F(F)                     \
  switch ((M + 15) / 16) {              \
    case 1: TVR_SK(F, 1); break;        \
    case 2: TVR_SK(F, 2); break;        \
    case 3: TVR_SK(F, 3); break;        \
    default: TVR_SK(F, 4); break;       \
  }
      if (a_fmt == ACT_X2F16) { TVR_SK_F(ACT_X2F16); } else { TVR_SK_F(ACT_BF16); }
#undef TVR_SK_F
#undef TVR_SK
    } else {
      PpPlan plan;
      if (m && vec && epi != EPI_STATS) plan = plan_pp_cached(m, M, N, K, a_fmt, epi, a_fmt == ACT_X2F16 && W.x16);
      if (plan.sk_base >= 0) {
        if (plan.sk_base > 0)
          launch_pp(epi, Ah, lda, a_fmt, W, ldw, M, N, K, ep, acc_scale, 0, plan.sk_base, true, sl, st);
        TVR_TRY(launch_pp_sk(epi, Ah, lda, a_fmt, W, ldw, M, N, K, ep, acc_scale, plan.sk_base,
                             gemm_pingpong_grid(M, N) - plan.sk_base, plan.sk_blocks, sl, m, st));
      } else if (plan.ksplit > 1) {
        TVR_TRY(launch_pp_splitk(epi, Ah, lda, a_fmt, W, ldw, M, N, K, ep, acc_scale, 0, gemm_pingpong_grid(M, N),
                                 plan.ksplit, sl, m, st));
      } else if (plan.tail_base > 0) {
        launch_pp(epi, Ah, lda, a_fmt, W, ldw, M, N, K, ep, acc_scale, 0, plan.tail_base, true, sl, st);
        TVR_TRY(launch_pp_splitk(epi, Ah, lda, a_fmt, W, ldw, M, N, K, ep, acc_scale, plan.tail_base,
                                 gemm_pingpong_grid(M, N) - plan.tail_base, plan.tail_split, sl, m, st));
      } else {
        launch_pp(epi, Ah, lda, a_fmt, W, ldw, M, N, K, ep, acc_scale, 0, 0, vec, sl, st);
      }
    }
  } else {
    const float* Af = static_cast<const float*>(A);
    unsigned* flag = m ? m->range_flag : range_flag;
    // exact-product fp32 GEMMs of a model whose O + MLP-out K reaches PP_SLICE_MIN_K (6.9B, 12B), or any launch
    // of that K: the sliced accumulation (gemm_f32.hpp SLICE_KT; the small tile holds the second accumulator set)
    const bool f32_sliced = !W.h && !W.x && (K >= PP_SLICE_MIN_K || (m && m->K2 >= PP_SLICE_MIN_K));
    const bool large = gemm_use_large(M, N) && !f32_sliced;
#define TVR_GEMM_LAUNCH(E, TL)                                                                                    \
  do {                                                                                                            \
    if (f32_sliced)                                                                                               \
      hipLaunchKernelGGL((gemm_f32_nt_kernel<E, TileSmall, F32_SLICE_KT>), dim3(gemm_grid<TileSmall>(M, N)),      \
                         dim3(TileSmall::THREADS), 0, st, Af, lda, W.f, ldw, M, N, K, ep);                        \
    else                                                                                                          \
      hipLaunchKernelGGL((gemm_f32_nt_kernel<E, TL>), dim3(gemm_grid<TL>(M, N)), dim3(TL::THREADS), 0,             \
                         st, Af, lda, W.f, ldw, M, N, K, ep);                                                     \
  } while (0)
#define TVR_X3_LAUNCH(E, TL)                                                                      \
  hipLaunchKernelGGL((gemm_x3bf16_nt_kernel<E, TL>), dim3(gemm_x3_grid<TL>(M, N)), dim3(TL::THREADS), \
                     0, st, Af, lda, W.x, ldw, W.wps, M, N, K, ep)
#define TVR_X2_LAUNCH(E, TL)                                                                         \
  hipLaunchKernelGGL((gemm_x2f16_nt_kernel<E, TL>), dim3(gemm_x2_grid<TL>(M, N)), dim3(TL::THREADS), 0, \
                     st, Af, lda, W.h, ldw, W.wps, acc_scale, flag, M, N, K, ep)
#define TVR_GEMM_PICK(E)                                                          \
  if (W.h) {                                                                      \
    if (large) TVR_X2_LAUNCH(E, X2Large); else TVR_X2_LAUNCH(E, X2Small);         \
  } else if (W.x) {                                                               \
    if (large) TVR_X3_LAUNCH(E, X3Large); else TVR_X3_LAUNCH(E, X3Small);         \
  } else {                                                                        \
    if (large) TVR_GEMM_LAUNCH(E, TileLarge); else TVR_GEMM_LAUNCH(E, TileSmall); \
  }
    switch (epi) {
      case EPI_BIAS: TVR_GEMM_PICK(EPI_BIAS); break;
      case EPI_SPLIT_GELU: TVR_GEMM_PICK(EPI_SPLIT_GELU); break;
      default: TVR_GEMM_PICK(EPI_RESID); break;
    }
#undef TVR_GEMM_PICK
#undef TVR_X2_LAUNCH
#undef TVR_X3_LAUNCH
#undef TVR_GEMM_LAUNCH
  }
  TVR_HIP(hipGetLastError());
  if (ev0 && ev1) {
    TVR_HIP(hipEventRecord(ev1, st));
    // minimal operand bytes: W read once (fp32 4, 3 bf16 planes 6, 2 fp16 planes 4, bf16 2 B per element),
    // A once in its format (fp32 / x2f16 4, bf16 2), C once as fp32
    // (EPI_STATS: the per-tile statistics records instead of C)
    const double wbytes = W.x ? 6.0 : (a_fmt == ACT_BF16 || a_fmt == ACT_F16 ? 2.0 : 4.0);
    const double abytes = a_fmt == ACT_BF16 || a_fmt == ACT_F16 ? 2.0 : 4.0;
    const double cbytes = epi == EPI_STATS ? 4.0 * M * (double)ep.stats_tiles * (2 + 2 * ep.stats_k)
                                           : 4.0 * M * (double)N;
    const int kind = epi == EPI_SPLIT_GELU_ACT ? (int)EPI_SPLIT_GELU : epi == EPI_STATS ? (int)EPI_BIAS : epi;
    m->prof_recs.push_back({ev0, ev1, kind, 2.0 * M * N * (double)K,
                            abytes * M * (double)K + cbytes + wbytes * N * (double)K});
  }
  return TVR_OK;
}

// TVR_GEMM_BF16: the attention-score columns [0, 2d) of the linearised entry
// run on fp16 operands when they are whole 256-column tiles (else 0: bf16)
int lin_qk_cols(const tvr_config& c) { return (2 * c.d_model) % 256 == 0 ? 2 * c.d_model : 0; }

// The linearised entry layer's model constants (lin_entry.hpp) for the
// current planar mode: per layer l = 1 .. L-2, Wsc = W1[l] W_O[l-1] on the
// exact-product fp32 MFMA GEMM, its planes (X2F16: per-layer power-of-two
// scale, as the weights), and c1[l] = row sums of W1[l] in fp64.
int ensure_lin(tvr_model* m, hipStream_t st) {
  const int fmt = act_fmt(m);
  if (fmt == ACT_F32) return fail(TVR_ERR_INVALID, "lin entry: needs a planar GEMM mode");
  if (m->lin_planes && m->lin_mode == m->gemm_mode) return TVR_OK;
  if (m->lin_failed_mode == m->gemm_mode)  // remembered: no sync, no allocation attempt per sweep
    return fail(TVR_ERR_NOMEM, "lin entry: the W1 W_O planes do not fit (earlier attempt)");
  const tvr_config& c = m->cfg;
  const int L = c.n_layers, d = c.d_model, H = c.n_heads, dh = c.d_head, N = m->D1;
  if (L < 3) return fail(TVR_ERR_INVALID, "lin entry: needs >= 3 layers");
  TVR_HIP(hipStreamSynchronize(st));
  if (m->lin_planes) TVR_HIP(hipFree(m->lin_planes));
  if (m->lin_c1) TVR_HIP(hipFree(m->lin_c1));
  m->lin_planes = nullptr;
  m->lin_c1 = nullptr;
  const int KP = (dh + 31) / 32 * 32, npl = fmt == ACT_X2F16 ? 2 : 1;
  const size_t per = (size_t)H * N * KP;
  float *wt = nullptr, *sc = nullptr;
  unsigned* d_max = nullptr;
  auto cleanup = [&]() {
    if (wt) (void)hipFree(wt);
    if (sc) (void)hipFree(sc);
    if (d_max) (void)hipFree(d_max);
  };
  // The split-K partials workspace is released for a second attempt; the
  // planes are kept only if that workspace can be re-reserved at its former
  // size afterwards (the sweep's split-K launches need it back: otherwise they
  // would fail with NOMEM where the full-GEMM entry succeeds).
  const size_t splitk_had = m->splitk_bytes;
  for (int attempt = 0;; ++attempt) {
    bool ok = hipMalloc(&m->lin_planes, (size_t)(L - 2) * npl * per * sizeof(uint16_t)) == hipSuccess &&
              hipMalloc(&m->lin_c1, (size_t)L * N * sizeof(float)) == hipSuccess &&
              hipMalloc(&wt, (size_t)d * d * sizeof(float)) == hipSuccess &&
              hipMalloc(&sc, (size_t)N * d * sizeof(float)) == hipSuccess &&
              hipMalloc(&d_max, sizeof(unsigned)) == hipSuccess;
    if (ok && attempt > 0 && splitk_had > 0) {
      (void)hipGetLastError();
      ok = hipMalloc(&m->splitk_ws, splitk_had) == hipSuccess;
      if (ok) {
        m->splitk_bytes = splitk_had;
      } else {
        m->splitk_ws = nullptr;
      }
    }
    if (ok) break;
    (void)hipGetLastError();
    cleanup();
    wt = sc = nullptr;
    d_max = nullptr;
    if (m->lin_planes) (void)hipFree(m->lin_planes);
    if (m->lin_c1) (void)hipFree(m->lin_c1);
    m->lin_planes = nullptr;
    m->lin_c1 = nullptr;
    if (attempt == 0 && m->splitk_ws) {
      (void)hipFree(m->splitk_ws);
      m->splitk_ws = nullptr;
      m->splitk_bytes = 0;
      continue;
    }
    m->lin_failed_mode = m->gemm_mode;
    return fail(TVR_ERR_NOMEM, "lin entry: the W1 W_O planes do not fit");
  }
  m->lin_scale.assign(L, 1.0f);
  int rc = TVR_OK;
  for (int l = 1; l <= L - 2 && rc == TVR_OK; ++l) {
    hipLaunchKernelGGL(transpose_kernel, dim3((d + 31) / 32, (d + 31) / 32), dim3(32, 8), 0, st,
                       m->layers[l - 1].w2, m->K2, wt, d);
    GemmEpi e{};
    e.out0 = sc;
    e.ld0 = d;
    rc = launch_gemm(EPI_BIAS, m->layers[l].w1, d, ACT_F32, MatW{wt}, d, N, d, d, e, st);
    if (rc != TVR_OK) break;
    float scale = 1.0f;
    {  // X2F16: one power-of-two scale from max |Wsc|; BF16: from max |Wsc| over the Q / K rows (fp16 there)
      unsigned hm = 0;
      hipError_t e2 = hipMemsetAsync(d_max, 0, sizeof(unsigned), st);
      if (e2 == hipSuccess) {
        const size_t n_abs = fmt == ACT_X2F16 ? (size_t)N * d : (size_t)2 * d * d;
        hipLaunchKernelGGL(absmax_kernel, dim3(1024), dim3(256), 0, st, sc, n_abs, d_max);
        e2 = hipGetLastError();
      }
      if (e2 == hipSuccess) e2 = hipMemcpyAsync(&hm, d_max, sizeof(unsigned), hipMemcpyDeviceToHost, st);
      if (e2 == hipSuccess) e2 = hipStreamSynchronize(st);
      if (e2 != hipSuccess) {
        rc = fail(TVR_ERR_HIP, std::string("lin entry: ") + hipGetErrorString(e2));
        break;
      }
      float v;
      std::memcpy(&v, &hm, sizeof(v));
      scale = x2_weight_scale(v);
    }
    if (fmt == ACT_X2F16) {
      hipLaunchKernelGGL(lin_planes_kernel<ACT_X2F16>, dim3(4096), dim3(256), 0, st, sc, N, H, dh, KP, scale,
                         m->lin_planes + (size_t)(l - 1) * npl * per, 0);
    } else {  // fp16 Q / K rows when they fill whole 256-column tiles of lin_entry_kernel (every Pythia but tiny)
      const int n_qk = lin_qk_cols(c);
      if (n_qk == 0) scale = 1.0f;
      hipLaunchKernelGGL(lin_planes_kernel<ACT_BF16>, dim3(4096), dim3(256), 0, st, sc, N, H, dh, KP, scale,
                         m->lin_planes + (size_t)(l - 1) * npl * per, n_qk);
    }
    m->lin_scale[l] = scale;
    hipLaunchKernelGGL(rowsum_kernel, dim3((N + 3) / 4), dim3(256), 0, st, m->layers[l].w1, N, d,
                       m->lin_c1 + (size_t)l * N);
    if (hipGetLastError() != hipSuccess) rc = fail(TVR_ERR_HIP, "lin entry: plane build launch failed");
  }
  if (rc == TVR_OK && hipStreamSynchronize(st) != hipSuccess) rc = fail(TVR_ERR_HIP, "lin entry: build failed");
  cleanup();
  if (rc != TVR_OK) {
    (void)hipFree(m->lin_planes);
    (void)hipFree(m->lin_c1);
    m->lin_planes = nullptr;
    m->lin_c1 = nullptr;
    return rc;
  }
  m->lin_kp = KP;
  m->lin_mode = m->gemm_mode;
  return TVR_OK;
}

// y: fp32 [rows][ldy] (ACT_F32) or a planar activation format
// copy: rows < copy_rows of x also go there unchanged (same stride; a fused
// sweep's clean rows into the trace's hook_resid_pre)
// g1 / g2 / y2 (x2f16, exact-fp16 weights): y = LNPre(x) * g1 and y2 = LNPre(x) * g2 (range-checked)
int launch_lnpre(const float* x, int ldx, const int32_t* idx, void* y, int ldy, int rows,
                 int d, float eps, int fmt, hipStream_t st, tvr_model* m = nullptr, float2* stats = nullptr,
                 float* copy = nullptr, int copy_rows = 0, const float* g1 = nullptr, const float* g2 = nullptr,
                 void* y2 = nullptr) {
  if (rows <= 0) return TVR_OK;
  ProfSpan ps(m, st);
  if (d % 4 != 0 || ldx % 4 != 0 || ldy % 4 != 0)
    return fail(TVR_ERR_UNSUPPORTED, "lnpre: d and strides must be multiples of 4");
  if (g1 && (fmt != ACT_X2F16 || (y2 && !g2) || !m))
    return fail(TVR_ERR_INTERNAL, "lnpre: the gamma-scaled rows are an x2f16 model path");
  const int rows_per_block = 4;
  const dim3 grid((rows + rows_per_block - 1) / rows_per_block), block(64 * rows_per_block);
  // the row in registers: 10 float4 per lane up to d = 2560, 20 up to 5120 (d % 256 == 0), else three passes
  const int nv = d % 256 != 0 ? 0 : d <= 2560 ? 10 : d <= 5120 ? 20 : 0;
#define TVR_LNPRE(F, NV, ...) \
  hipLaunchKernelGGL((lnpre_kernel<F, NV>), grid, block, 0, st, x, ldx, idx, y, ldy, rows, d, eps, stats, copy, copy_rows, __VA_ARGS__)
#define TVR_LNPRE_NV(F, ...)                 \
  if (nv == 10) {                            \
    TVR_LNPRE(F, 10, __VA_ARGS__);           \
  } else if (nv == 20) {                     \
    TVR_LNPRE(F, 20, __VA_ARGS__);           \
  } else {                                   \
    TVR_LNPRE(F, 0, __VA_ARGS__);            \
  }
  if (fmt == ACT_X2F16) {
    TVR_LNPRE_NV(ACT_X2F16, g1, g2, y2, m ? m->range_flag : nullptr);
  } else if (fmt == ACT_BF16) {
    TVR_LNPRE_NV(ACT_BF16, nullptr, nullptr, nullptr, nullptr);
  } else {
    TVR_LNPRE_NV(ACT_F32, nullptr, nullptr, nullptr, nullptr);
  }
#undef TVR_LNPRE_NV
#undef TVR_LNPRE
  TVR_HIP(hipGetLastError());
  // fp32 rows in, rows out in the activation format (x2f16 / fp32 4 B; bf16 2 + the fp16 plane 2 B per element;
  // the gamma-scaled pair two x2f16 rows)
  ps.done(TVR_HBM_LNPRE, (double)rows * d * (y2 ? 12.0 : 8.0) +
                             (copy ? (double)std::min(rows, copy_rows) * d * 4.0 : 0.0));
  return TVR_OK;
}

// Activation buffers of one launch sequence.  In the planar modes xn and a2
// hold the model's activation format `fmt` (split.hpp) in the same bytes.
struct Acts {
  float* resid;   // [R][d]
  float* xn;      // [R][d]
  float* qkv;     // [R][3d]
  float* a2;      // [R][K2]  (z | gelu(mlp-in))
  int fmt;
  // exact-fp16 weights (use_x16): xn holds LNPre(resid) * gamma1 and xn2 [R][d] LNPre(resid) * gamma2
  float* xn2 = nullptr;
  // a fused clean + patch sweep: rows < mirror_rows (the clean rows) of the
  // layer's resid_pre (LayerNorm's input) and qkv (the QKV epilogue's fp32
  // columns) are also written to the trace by the kernels producing them
  float* resid_mirror = nullptr;
  float* qkv_mirror = nullptr;
  int mirror_rows = 0;
};

// z: the z columns of a2 (fp32 or activation format fmt); zf: optional fp32 copy [rows][d].
// attention_mfma_kernel (one wave per (sequence, head), fp32 MFMA, no LDS) for
// the Pythia head sizes d_head 16 (tiny), 64, 80, 128 with rotary_dim =
// d_head / 4 (every Pythia: rotary_pct 0.25); check_config rejects the rest.
// row_from: sequences [row_from, n_seqs) have exactly one query row (their
// last: q0 = n - 1) and go to attention_row_kernel (HG heads per wave).
bool row_attention_ok(const tvr_config& c) {
  const int hg = c.d_head == 128 ? 2 : 4;
  return c.n_heads % hg == 0 && (c.d_head == 16 || c.d_head == 64 || c.d_head == 80 || c.d_head == 128);
}

int launch_attention(tvr_model* m, const float* qkv, const float* cache_qkv, const SeqDesc* d_seqs,
                     int n_seqs, int maxT, void* z, int fmt, float* zf, hipStream_t st, bool zf_last = false,
                     int zf_rows = INT_MAX, int row_from = INT_MAX) {
  if (n_seqs <= 0) return TVR_OK;
  const tvr_config& c = m->cfg;
  const int d = c.d_model;
  const float inv_scale = 1.0f / std::sqrt((float)c.d_head);
  const int dh = c.d_head;
  if (row_from < n_seqs && row_attention_ok(c) && env_flag("TVR_ROW_ATTN")) {  // TVR_ROW_ATTN=0: A/B, tests
    const int nr = n_seqs - row_from, hg = dh == 128 ? 2 : 4;
    const dim3 rg((nr * (c.n_heads / hg) + 3) / 4), rb(256);
#define TVR_ATTR(F, DHV)                                                                                         \
  hipLaunchKernelGGL((attention_row_kernel<F, DHV>), rg, rb, 0, st, qkv, 3 * d, cache_qkv, 3 * d, d_seqs, row_from, \
                     nr, c.n_heads, z, m->K2, zf, d, zf_last ? 1 : 0, zf_rows, m->range_flag, m->rot_cos, m->rot_sin, \
                     d, inv_scale)
#define TVR_ATTR_DH(F)                                                                         \
  if (dh == 16) { TVR_ATTR(F, 16); } else if (dh == 64) { TVR_ATTR(F, 64); }                   \
  else if (dh == 80) { TVR_ATTR(F, 80); } else { TVR_ATTR(F, 128); }
    if (fmt == ACT_X2F16) {
      TVR_ATTR_DH(ACT_X2F16);
    } else if (fmt == ACT_BF16) {
      TVR_ATTR_DH(ACT_BF16);
    } else {
      TVR_ATTR_DH(ACT_F32);
    }
#undef TVR_ATTR_DH
#undef TVR_ATTR
    TVR_HIP(hipGetLastError());
    n_seqs = row_from;  // the MFMA kernel takes the rest (below)
    if (n_seqs <= 0) return TVR_OK;
  }
  const int pairs = n_seqs * c.n_heads;
  const dim3 grid((pairs + ATTM_WAVES - 1) / ATTM_WAVES), block(64 * ATTM_WAVES);
  // key tiles in registers: 1 / 2 / 4 / 8, or 0 = longer than 128 (chunked online softmax)
  const int kt = (maxT + 15) / 16, nkt = kt <= 1 ? 1 : kt <= 2 ? 2 : kt <= 4 ? 4 : kt <= 8 ? 8 : 0;
  // one key tile: K / V slices staged through LDS by LDS-DMA (default, 2); TVR_ATT_STAGE=1 stages Q as
  // well, 0 loads directly (A/B: profiles/r03/attention_stage_ab.txt)
  const char* se = getenv("TVR_ATT_STAGE");
  const int stage = se && std::string(se) == "0" ? 0 : se && std::string(se) == "1" ? 1 : 2;
  // two key tiles: V staged through LDS (STAGE 3); TVR_ATT_VSTAGE=0 loads it directly (A/B)
  const bool vstage = env_flag("TVR_ATT_VSTAGE");  // read per launch, as TVR_ATT_STAGE (in-process A/B tests)
#define TVR_ATTM(F, DHV, NK, ...)                                                                                   \
  hipLaunchKernelGGL((attention_mfma_kernel<F, DHV, NK __VA_OPT__(,) __VA_ARGS__>), grid, block, 0, st, qkv, 3 * d, cache_qkv, 3 * d, d_seqs, \
                     n_seqs, c.n_heads, z, m->K2, zf, d, zf_last ? 1 : 0, zf_rows, m->range_flag, m->rot_cos, m->rot_sin, d, \
                     inv_scale)
#define TVR_ATTM_NK(F, DHV)                                                                     \
  if (nkt == 1 && stage == 1) TVR_ATTM(F, DHV, 1, (DHV <= 80 ? 1 : 0)); /* d_head 128: 98 KB, not staged */ \
  else if (nkt == 1 && stage == 2) TVR_ATTM(F, DHV, 1, (DHV <= 80 ? 2 : 0));                  \
  else if (nkt == 1) TVR_ATTM(F, DHV, 1);                                                       \
  else if (nkt == 2 && vstage) TVR_ATTM(F, DHV, 2, 3);                                          \
  else if (nkt == 2) TVR_ATTM(F, DHV, 2);                                                       \
  else if (nkt == 4) TVR_ATTM(F, DHV, 4);                                                       \
  else if (nkt == 8) TVR_ATTM(F, DHV, 8);                                                       \
  else TVR_ATTM(F, DHV, 0)
#define TVR_ATTM_DH(F)                                                                          \
  if (dh == 16) { TVR_ATTM_NK(F, 16); } else if (dh == 64) { TVR_ATTM_NK(F, 64); }              \
  else if (dh == 80) { TVR_ATTM_NK(F, 80); } else { TVR_ATTM_NK(F, 128); }
  if (fmt == ACT_X2F16) {
    TVR_ATTM_DH(ACT_X2F16);
  } else if (fmt == ACT_BF16) {
    TVR_ATTM_DH(ACT_BF16);
  } else {
    TVR_ATTM_DH(ACT_F32);
  }
#undef TVR_ATTM_DH
#undef TVR_ATTM_NK
#undef TVR_ATTM
  TVR_HIP(hipGetLastError());
  return TVR_OK;
}

// One transformer block over the first R rows (Pythia parallel residual):
//   x = LNPre(resid); [qkv | h] = x @ W1^T + b1; z = attn(qkv); resid += [z|gelu h] @ W2^T + b2
// (run_block computes up to z; run_block_out the second projection.)
// The QKV+MLP-in epilogue: Q|K|V fp32 to qkv (row stride 3d), GELU(h) into
// the a2 columns after z (fp32, or the activation format).
GemmEpi epi_qkv_mlpin(tvr_model* m, const float* b1, float* qkv, const Acts& a) {
  const bool planar = a.fmt != ACT_F32;
  const int d = m->cfg.d_model;
  GemmEpi e{};
  e.bias = b1;
  e.out0 = qkv;
  e.ld0 = 3 * d;
  e.n_split = 3 * d;
  e.out0m = a.qkv_mirror;
  e.mirror_rows = a.mirror_rows;
  if (planar) {
    e.out1h = reinterpret_cast<uint16_t*>(a.a2) + d;
    e.ld1h = 2 * m->K2;
    e.ps1h = m->K2;
    e.range_flag = m->range_flag;
  } else {
    e.out1 = a.a2 + d;
    e.ld1 = m->K2;
  }
  return e;
}

// Algorithmic bytes of one attention launch: Q of the queried rows and K, V of
// every row of the launch (fp32 qkv), z out in the activation format, plus the
// fp32 hook_z copy when one is written (trace / capture).  The shared prefix
// rows read from the trace or a leader are not counted.
double attention_bytes(int d, int q_rows, int kv_rows, int fmt, int zf_rows) {
  return ((double)q_rows * d + 2.0 * kv_rows * d) * 4.0 + (double)q_rows * d * (fmt == ACT_BF16 ? 2.0 : 4.0) +
         (double)zf_rows * d * 4.0;
}

// W1 GEMM over LayerNorm outputs xn (a.fmt), columns [c0, c0 + N) of W1, with
// an epilogue ep already addressed to column c0 (EPI_SPLIT_GELU_ACT planar /
// EPI_SPLIT_GELU fp32).  TVR_GEMM_BF16 runs the attention-score columns
// (Q, K: [0, 2d)) on the fp16 operands instead (W1's fp16 Q / K plane, xn's
// fp16 plane 1: store_ln4) with plain fp32 stores, the rest on bf16.
// xn2 (use_x16): xn / xn2 are LNPre rows scaled by gamma1 / gamma2, and the GEMM runs on the raw W1 rows
// (one exact fp16 plane): the Q | K | V columns [0, 3d) read xn, the MLP-in columns xn2 — per tile in one
// launch when the boundary falls on a 256-column tile edge of the launch, else as two launches.
int launch_w1(tvr_model* m, int l, const void* xn, int M, int c0, int N, const GemmEpi& ep, hipStream_t st,
              const void* xn2 = nullptr) {
  const int d = m->cfg.d_model;
  const int fmt = act_fmt(m);
  const int epi = fmt != ACT_F32 ? EPI_SPLIT_GELU_ACT : EPI_SPLIT_GELU;
  if (xn2) {
    if (!use_x16(m) || fmt != ACT_X2F16) return fail(TVR_ERR_INTERNAL, "launch_w1: gamma-scaled rows off the x16 path");
    const MatW W = m->w1x[l].rows((size_t)c0 * d);
    const int qkv_end = 3 * d - c0;  // first column of the launch that reads xn2
    if (qkv_end <= 0)
      return launch_gemm(epi, xn2, d, fmt, W, d, M, N, d, ep, st, m);
    if (qkv_end >= N)
      return launch_gemm(epi, xn, d, fmt, W, d, M, N, d, ep, st, m);
    if (qkv_end % 256 == 0) {
      GemmEpi e = ep;
      e.a2 = static_cast<const uint16_t*>(xn2);
      e.a2_col = qkv_end;
      return launch_gemm(epi, xn, d, fmt, W, d, M, N, d, e, st, m);
    }
    // two launches: columns [c0, 3d) below the GELU split, then the MLP-in columns (their GELU outputs and raw
    // pre-activations are indexed from n_split, which becomes 0)
    GemmEpi e1 = ep;
    e1.n_split = std::min(ep.n_split, qkv_end);
    TVR_TRY(launch_gemm(epi, xn, d, fmt, W, d, M, qkv_end, d, e1, st, m));
    GemmEpi e2 = ep;
    e2.bias = ep.bias ? ep.bias + qkv_end : nullptr;
    e2.out0 = ep.out0 ? ep.out0 + qkv_end : nullptr;
    if (ep.out0m) e2.out0m = ep.out0m + qkv_end;
    e2.n_split = ep.n_split - qkv_end;
    if (e2.n_split < 0) return fail(TVR_ERR_INTERNAL, "launch_w1: MLP-in columns below the GELU split");
    return launch_gemm(epi, xn2, d, fmt, W.rows((size_t)qkv_end * d), d, M, N - qkv_end, d, e2, st, m);
  }
  const int nqk = fmt == ACT_BF16 && !m->w1qk.empty() ? std::min(std::max(2 * d - c0, 0), N) : 0;
  if (nqk > 0) {
    GemmEpi e{};
    e.bias = ep.bias;
    e.out0 = ep.out0;
    e.ld0 = ep.ld0;
    e.a_rows = ep.a_rows;
    e.out_rows = ep.out_rows;
    e.out0m = ep.out0m;
    e.mirror_rows = ep.mirror_rows;
    TVR_TRY(launch_gemm(EPI_BIAS, static_cast<const uint16_t*>(xn) + d, d, ACT_F16,
                        m->w1qk[l].rows((size_t)c0 * d), d, M, nqk, d, e, st, m));
    if (nqk == N) return TVR_OK;
  }
  GemmEpi e = ep;
  if (nqk > 0) {
    e.bias = ep.bias ? ep.bias + nqk : nullptr;
    e.out0 = ep.out0 + nqk;
    if (ep.out0m) e.out0m = ep.out0m + nqk;
    e.n_split = ep.n_split - nqk;
  }
  return launch_gemm(epi, xn, d, fmt, m->w1[l].rows((size_t)(c0 + nqk) * d), d, M, N - nqk, d, e, st, m);
}

// zf_last: the fp32 hook_z copy of each sequence's last row only, at row s of zf
int run_block(tvr_model* m, int l, int R, const SeqDesc* d_seqs, int n_seqs, int maxT,
              Acts& a, float* qkv_out, const float* cache_qkv, float* zf, hipStream_t st, bool zf_last = false,
              int zf_rows = INT_MAX, int row_from = INT_MAX) {
  const tvr_config& c = m->cfg;
  const int d = c.d_model;
  const tvr_layer_weights& w = m->layers[l];
  TVR_TRY(launch_lnpre(a.resid, d, nullptr, a.xn, d, R, d, c.ln_eps, a.fmt, st, m, nullptr, a.resid_mirror,
                       a.mirror_rows, a.xn2 ? m->g1[l] : nullptr, a.xn2 ? m->g2[l] : nullptr, a.xn2));
  const GemmEpi e1 = epi_qkv_mlpin(m, w.b1, qkv_out, a);
  TVR_TRY(launch_w1(m, l, a.xn, R, 0, m->D1, e1, st, a.xn2));
  ProfSpan ps(m, st);
  TVR_TRY(launch_attention(m, qkv_out, cache_qkv, d_seqs, n_seqs, maxT, a.a2, a.fmt, zf, st, zf_last, zf_rows,
                           row_from));
  ps.done(TVR_HBM_ATTENTION, attention_bytes(d, R, R, a.fmt, zf ? (zf_last ? n_seqs : std::min(R, zf_rows)) : 0));
  return TVR_OK;
}

// The last layer when only each sequence's LAST row is read afterwards (patch
// sweeps, extraction): every row still needs K and V (they are attended to),
// but Q, the MLP, attention output and the second projection are computed for
// the n_last rows listed in d_last only (~5% of a CIE sweep's FLOPs saved).
// d_seqs must carry q0 = n - 1.  write_out = false skips the second projection
// (nothing downstream reads the final residual).
// row_from: the sequences [row_from, n_seqs) query their last row only (the
// single-query kernel); the ones before it (a fused sweep's clean sequences,
// whose every row the trace keeps: q0 = 0) go to the MFMA kernel.
int run_block_last_rows(tvr_model* m, int l, int R, const SeqDesc* d_seqs, int n_seqs, int maxT, Acts& a,
                        const float* cache_qkv, const int32_t* d_last, int n_last, bool write_out,
                        float* zf, hipStream_t st, bool zf_last = false, int zf_rows = INT_MAX, int row_from = 0) {
  const tvr_config& c = m->cfg;
  const int d = c.d_model;
  const tvr_layer_weights& w = m->layers[l];
  TVR_TRY(launch_lnpre(a.resid, d, nullptr, a.xn, d, R, d, c.ln_eps, a.fmt, st, m, nullptr, a.resid_mirror,
                       a.mirror_rows, a.xn2 ? m->g1[l] : nullptr, a.xn2 ? m->g2[l] : nullptr, a.xn2));
  GemmEpi kv{};  // K | V columns (w1 rows [d, 3d)) for every row (all below n_split: no GELU)
  kv.bias = w.b1 + d;
  kv.out0 = a.qkv + d;
  kv.ld0 = 3 * d;
  kv.n_split = 2 * d;
  TVR_TRY(launch_w1(m, l, a.xn, R, d, 2 * d, kv, st, a.xn2));
  GemmEpi e1 = epi_qkv_mlpin(m, w.b1, a.qkv, a);  // all columns for the last rows, gathered and scattered in place
  e1.a_rows = d_last;
  e1.out_rows = d_last;
  TVR_TRY(launch_w1(m, l, a.xn, n_last, 0, m->D1, e1, st, a.xn2));
  ProfSpan ps(m, st);
  TVR_TRY(launch_attention(m, a.qkv, cache_qkv, d_seqs, n_seqs, maxT, a.a2, a.fmt, zf, st, zf_last, zf_rows,
                           row_from));
  ps.done(TVR_HBM_ATTENTION, attention_bytes(d, n_last, R, a.fmt, zf ? std::min(n_last, zf_rows) : 0));
  if (!write_out) return TVR_OK;
  GemmEpi e2{};
  e2.bias = w.b2;
  e2.out0 = a.resid;
  e2.ld0 = d;
  e2.resid = a.resid;
  e2.ldr = d;
  e2.a_rows = d_last;
  e2.out_rows = d_last;
  return launch_gemm(EPI_RESID, a.a2, m->K2, a.fmt, use_x16(m) ? m->w2x[l] : m->w2[l], m->K2, n_last, d, m->K2, e2,
                     st, m);
}

int run_block_out(tvr_model* m, int l, int R, Acts& a, hipStream_t st) {
  const int d = m->cfg.d_model;
  const tvr_layer_weights& w = m->layers[l];
  GemmEpi e2{};
  e2.bias = w.b2;
  e2.out0 = a.resid;
  e2.ld0 = d;
  e2.resid = a.resid;
  e2.ldr = d;
  return launch_gemm(EPI_RESID, a.a2, m->K2, a.fmt, use_x16(m) ? m->w2x[l] : m->w2[l], m->K2, R, d, m->K2, e2, st, m);
}

// Final LN + unembed of selected rows + softmax target prob + top-k, chunked.
// Planar modes without requested logits: the unembed GEMM's fused statistics
// epilogue (EPI_STATS: per-tile max / sum exp / top-k candidates / target
// logit, no [rows][V] logits in HBM) + stats_merge_kernel.  Otherwise the
// logits are written (to out_logits, or the scratch) and row_stats_kernel
// reads them back.
bool final_fused(const tvr_model* m, int fmt, const float* out_logits) {
  return fmt != ACT_F32 && !out_logits && m->cfg.d_vocab % 4 == 0;
}
// rows per unembed launch: the fused statistics keep ~200 records per row (no
// [rows][V] logits), so a whole sweep's sites go in one launch (one partly
// empty last round instead of one per 1,024 rows: 37 rounds instead of 52 at
// C3); the logits paths keep 1,024-row chunks of [rows][V] scratch.
int final_chunk(const tvr_model* m, int fmt, const float* out_logits) {
  return final_fused(m, fmt, out_logits) ? 16384 : kFinalChunk;
}
// floats of run_final's scratch for chunks of fc rows
size_t final_scratch_floats(const tvr_model* m, int fmt, int fc, int topk, const float* out_logits) {
  const int V = m->cfg.d_vocab;
  if (final_fused(m, fmt, out_logits)) return (size_t)fc * ((V + 255) / 256) * (2 + 2 * topk) + fc;
  return out_logits ? 0 : (size_t)fc * V;
}

int run_final(tvr_model* m, const float* resid, const int32_t* d_rows, const int32_t* d_targets,
              int n, float* xf, float* scratch, float* out_prob, int32_t* out_topk, int topk,
              float* out_logits, int fmt, hipStream_t st) {
  const tvr_config& c = m->cfg;
  const int d = c.d_model, V = c.d_vocab;
  const bool fused = final_fused(m, fmt, out_logits);
  const int tiles = (V + 255) / 256, chunk = final_chunk(m, fmt, out_logits);
  for (int s = 0; s < n; s += chunk) {
    const int cn = std::min(chunk, n - s);
    // the exact-fp16 unembed: LNPre(x) o gamma_f against the raw W_U (the statistics are invariant to the
    // per-row constant this leaves in the logits; the logits path removes it below)
    const bool xu = use_x16(m) && m->wux.h;
    TVR_TRY(launch_lnpre(resid, d, d_rows + s, xf, d, cn, d, c.ln_eps, fmt, st, m, nullptr, nullptr, 0,
                         xu ? m->gf : nullptr));
    if (fused) {
      float* part = scratch;
      float* tlogit = scratch + (size_t)cn * tiles * (2 + 2 * topk);
      GemmEpi e{};
      e.bias = m->b_unembed;
      e.stats = part;
      e.stats_k = topk;
      e.stats_tiles = tiles;
      e.targets = d_targets ? d_targets + s : nullptr;
      e.tlogit = tlogit;
      TVR_TRY(launch_gemm(EPI_STATS, xf, d, fmt, xu ? m->wux : m->wu, d, cn, V, d, e, st, m));
      ProfSpan ps(m, st);
      hipLaunchKernelGGL(stats_merge_kernel, dim3((cn + MERGE_WAVES - 1) / MERGE_WAVES), dim3(64 * MERGE_WAVES), 0,
                         st, part, tiles, topk, tlogit, d_targets ? d_targets + s : nullptr, cn, V,
                         out_prob ? out_prob + s : nullptr, out_topk ? out_topk + (size_t)s * topk : nullptr, topk);
      TVR_HIP(hipGetLastError());
      ps.done(TVR_HBM_ROW_STATS, (double)cn * (tiles * (2.0 + 2.0 * topk) + 1.0) * 4.0);  // the records + target logit
      continue;
    }
    float* lg = out_logits ? out_logits + (size_t)s * V : scratch;
    GemmEpi e{};
    e.bias = m->b_unembed;
    e.out0 = lg;
    e.ld0 = V;
    TVR_TRY(launch_gemm(EPI_BIAS, xf, d, fmt, xu ? m->wux : m->wu, d, cn, V, d, e, st, m));
    if (xu) {
      // TL's W_U' = center_unembed(fold_ln(W_U)): (LNPre(x) o gamma_f) W_U^T + b_U' differs from TL's logits by
      // -LNPre(x) . (the vocab mean of the d-centred rows), one constant per row, and TL's logits have mean 0 over
      // the vocabulary (W_U' and b_U' are centred over it): subtract each row's mean
      const bool v4 = ((uintptr_t)lg & 15) == 0 && V % 4 == 0;
      if (v4)
        hipLaunchKernelGGL(center_rows_kernel<true>, dim3((cn + 3) / 4), dim3(256), 0, st, lg, lg, cn, V);
      else
        hipLaunchKernelGGL(center_rows_kernel<false>, dim3((cn + 3) / 4), dim3(256), 0, st, lg, lg, cn, V);
      TVR_HIP(hipGetLastError());
    }
    ProfSpan ps(m, st);
    hipLaunchKernelGGL(row_stats_kernel, dim3(cn), dim3(STATS_THREADS), 0, st, lg, V, V,
                       d_targets ? d_targets + s : nullptr, out_prob ? out_prob + s : nullptr,
                       out_topk ? out_topk + (size_t)s * topk : nullptr, topk);
    TVR_HIP(hipGetLastError());
    ps.done(TVR_HBM_ROW_STATS, (double)cn * V * 4.0);  // one fp32 logit row per site
  }
  return TVR_OK;
}

int check_config(const tvr_config& c) {
  if (c.n_layers <= 0 || c.d_model <= 0 || c.n_heads <= 0 || c.d_head <= 0 || c.d_mlp <= 0 ||
      c.d_vocab <= 0 || c.n_ctx <= 0)
    return fail(TVR_ERR_INVALID, "config: all sizes must be positive");
  if (c.n_heads * c.d_head != c.d_model)
    return fail(TVR_ERR_INVALID, "config: n_heads * d_head must equal d_model");
  if (c.rotary_dim < 0 || c.rotary_dim > c.d_head || (c.rotary_dim & 1))
    return fail(TVR_ERR_INVALID, "config: rotary_dim must be even and <= d_head");
  if (c.d_model % GEMM_BK != 0 || (c.d_model + c.d_mlp) % GEMM_BK != 0)
    return fail(TVR_ERR_UNSUPPORTED, "config: d_model and d_model + d_mlp must be multiples of 32");
  if (!(c.d_head == 16 || c.d_head == 64 || c.d_head == 80 || c.d_head == 128) || c.rotary_dim * 4 != c.d_head)
    return fail(TVR_ERR_UNSUPPORTED, "config: the attention kernel covers the Pythia heads: d_head 16 / 64 / 80 / "
                                     "128 with rotary_dim = d_head / 4");
  return TVR_OK;
}

}  // namespace

// ===========================================================================
namespace {
int flush_pending(tvr_trace* t, void* stream);
}  // namespace

extern "C" {

const char* tvr_version(void) {
  return "tvr-mi355x 0.5.0 (gfx950, fp32 MFMA | fp32-accurate 3-plane bf16 / 2-plane fp16 split MFMA | bf16 MFMA)";
}
int32_t tvr_abi_version(void) { return TVR_ABI_VERSION; }
const char* tvr_last_error(void) { return g_last_error.c_str(); }

int tvr_model_create(const tvr_config* cfg, const float* w_embed, const tvr_layer_weights* layers,
                     const float* w_unembed_t, const float* b_unembed, tvr_model** out) {
  if (!cfg || !w_embed || !layers || !w_unembed_t || !out)
    return fail(TVR_ERR_INVALID, "tvr_model_create: null argument");
  TVR_TRY(check_config(*cfg));
  for (int l = 0; l < cfg->n_layers; ++l)
    if (!layers[l].w1 || !layers[l].b1 || !layers[l].w2 || !layers[l].b2)
      return fail(TVR_ERR_INVALID, "tvr_model_create: null weight in layer " + std::to_string(l));
  auto* m = new tvr_model();
  m->cfg = *cfg;
  m->D1 = 3 * cfg->d_model + cfg->d_mlp;
  m->K2 = cfg->d_model + cfg->d_mlp;
  m->w_embed = w_embed;
  m->layers.assign(layers, layers + cfg->n_layers);
  m->w_unembed_t = w_unembed_t;
  m->b_unembed = b_unembed;
  for (int l = 0; l < cfg->n_layers; ++l) {
    m->w1.push_back(MatW{layers[l].w1});
    m->w2.push_back(MatW{layers[l].w2});
  }
  m->wu = MatW{w_unembed_t};
  // TL calculate_sin_cos_rotary: freq = base^(i / (rd/2)), repeated "(2 d)",
  // angle = pos / freq, all in fp32.
  const int rd = std::max(cfg->rotary_dim, 2), n_ctx = cfg->n_ctx;
  std::vector<float> hc((size_t)n_ctx * rd), hs((size_t)n_ctx * rd);
  const int half = rd / 2;
  for (int p = 0; p < n_ctx; ++p)
    for (int i = 0; i < rd; ++i) {
      const float dim = (float)(i % half);
      const float freq = std::pow(cfg->rotary_base, dim / (float)half);
      const float ang = (float)p / freq;
      hc[(size_t)p * rd + i] = std::cos(ang);
      hs[(size_t)p * rd + i] = std::sin(ang);
    }
  std::vector<const float*> w2s(cfg->n_layers);
  for (int l = 0; l < cfg->n_layers; ++l) w2s[l] = layers[l].w2;
  hipError_t e = hipMalloc(&m->rot_cos, hc.size() * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&m->rot_sin, hs.size() * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&m->d_w2s, w2s.size() * sizeof(float*));
  if (e == hipSuccess) e = hipMalloc(&m->range_flag, sizeof(unsigned));
  if (e == hipSuccess) e = hipMemset(m->range_flag, 0, sizeof(unsigned));
  if (e == hipSuccess) e = hipMemcpy(m->rot_cos, hc.data(), hc.size() * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(m->rot_sin, hs.data(), hs.size() * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(m->d_w2s, w2s.data(), w2s.size() * sizeof(float*), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    tvr_model_destroy(m);
    return fail(TVR_ERR_HIP, std::string("tvr_model_create: ") + hipGetErrorString(e));
  }
  *out = m;
  return TVR_OK;
}

int tvr_model_destroy(tvr_model* m) {
  if (!m) return TVR_OK;
  (void)hipDeviceSynchronize();
  if (m->rot_cos) (void)hipFree(m->rot_cos);
  if (m->rot_sin) (void)hipFree(m->rot_sin);
  if (m->d_w2s) (void)hipFree(m->d_w2s);
  if (m->planes) (void)hipFree(m->planes);
  if (m->lin_planes) (void)hipFree(m->lin_planes);
  if (m->lin_c1) (void)hipFree(m->lin_c1);
  if (m->range_flag) (void)hipFree(m->range_flag);
  if (m->ws) (void)hipFree(m->ws);
  if (m->splitk_ws) (void)hipFree(m->splitk_ws);
  for (auto& r : m->prof_recs) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  for (auto e : m->prof_pool) (void)hipEventDestroy(e);
  for (int i = 0; i < 2; ++i) {
    if (m->staging.buf[i]) (void)hipHostFree(m->staging.buf[i]);
    if (m->staging.done[i]) (void)hipEventDestroy(m->staging.done[i]);
  }
  delete m;
  return TVR_OK;
}

size_t tvr_workspace_bytes(const tvr_model* m) { return m ? m->ws_bytes : 0; }

int32_t tvr_model_get_gemm(const tvr_model* m) { return m ? m->gemm_mode : -1; }

// X2F16 mode: the weight planes again for the current exact-fp16 binding (with / without the w2 planes),
// on the null stream
static int replan_x2f16(tvr_model* m) {
  if (m->gemm_mode != TVR_GEMM_X2F16) return TVR_OK;
  TVR_HIP(hipDeviceSynchronize());  // no launch on any stream may still read the planes about to be freed
  TVR_TRY(tvr_model_set_gemm(m, TVR_GEMM_F32, nullptr));
  return tvr_model_set_gemm(m, TVR_GEMM_X2F16, nullptr);
}

int tvr_model_set_exact16_unembed(tvr_model* m, const uint16_t* wu, const float* gf) {
  if (!m) return fail(TVR_ERR_INVALID, "tvr_model_set_exact16_unembed: null model");
  if (!wu != !gf) return fail(TVR_ERR_INVALID, "tvr_model_set_exact16_unembed: give both arrays or neither");
  m->wux = wu ? MatW{nullptr, nullptr, wu, 0, 1.0f, true} : MatW{};
  m->gf = gf;
  return TVR_OK;
}

int tvr_model_set_exact16(tvr_model* m, const tvr_exact16_layer* layers) {
  if (!m) return fail(TVR_ERR_INVALID, "tvr_model_set_exact16: null model");
  const tvr_config& c = m->cfg;
  if (!layers) {
    const bool was = m->x16;
    m->x16 = false;
    m->w1x.clear();
    m->w2x.clear();
    m->g1.clear();
    m->g2.clear();
    return was ? replan_x2f16(m) : TVR_OK;
  }
  for (int l = 0; l < c.n_layers; ++l)
    if (!layers[l].w1 || !layers[l].w2 || !layers[l].g1 || !layers[l].g2)
      return fail(TVR_ERR_INVALID, "tvr_model_set_exact16: null array in layer " + std::to_string(l));
  // the one-plane kernel's staging reads rows of 8-halve chunks and d of 4-float groups (launch_gemm's K / ld
  // checks cover the rest)
  if (c.d_model % 32 != 0 || m->K2 % 32 != 0)
    return fail(TVR_ERR_UNSUPPORTED, "tvr_model_set_exact16: d_model and d_model + d_mlp must be multiples of 32");
  m->w1x.clear();
  m->w2x.clear();
  m->g1.clear();
  m->g2.clear();
  for (int l = 0; l < c.n_layers; ++l) {
    // one plane of the raw values themselves: weight scale 1 (fp16 subnormals reach the matrix cores as
    // they are: tools/denorm_probe.py), no second plane (wps 0 is never read: WX kernels only)
    m->w1x.push_back(MatW{nullptr, nullptr, layers[l].w1, 0, 1.0f, true});
    m->w2x.push_back(MatW{nullptr, nullptr, layers[l].w2, 0, 1.0f, true});
    m->g1.push_back(layers[l].g1);
    m->g2.push_back(layers[l].g2);
  }
  m->x16 = true;
  return replan_x2f16(m);
}

int tvr_model_set_gemm(tvr_model* m, int32_t mode, void* stream) {
  if (!m) return fail(TVR_ERR_INVALID, "tvr_model_set_gemm: null model");
  if (mode != TVR_GEMM_F32 && mode != TVR_GEMM_X3BF16 && mode != TVR_GEMM_X2F16 && mode != TVR_GEMM_BF16)
    return fail(TVR_ERR_INVALID, "tvr_model_set_gemm: unknown mode " + std::to_string(mode));
  if (mode == m->gemm_mode) return TVR_OK;
  if (mode == TVR_GEMM_BF16 && (m->cfg.d_model % 64 != 0 || m->K2 % 64 != 0))
    return fail(TVR_ERR_UNSUPPORTED, "tvr_model_set_gemm: bf16 needs d_model and d_model + d_mlp multiples of 64");
  const hipStream_t st = (hipStream_t)stream;
  TVR_HIP(hipStreamSynchronize(st));
  // back to plain fp32 operands first (frees the previous mode's planes)
  for (auto& w : m->w1) w = MatW{w.f};
  for (auto& w : m->w2) w = MatW{w.f};
  m->w1qk.clear();
  m->wu = MatW{m->wu.f};
  if (m->planes) TVR_HIP(hipFree(m->planes));
  m->planes = nullptr;
  if (m->lin_planes) TVR_HIP(hipFree(m->lin_planes));
  if (m->lin_c1) TVR_HIP(hipFree(m->lin_c1));
  m->lin_planes = nullptr;
  m->lin_c1 = nullptr;
  m->lin_mode = -1;
  m->lin_failed_mode = -1;
  m->gemm_mode = TVR_GEMM_F32;
  if (mode == TVR_GEMM_F32) return TVR_OK;

  const tvr_config& c = m->cfg;
  const int L = c.n_layers;
  const size_t n1 = (size_t)m->D1 * c.d_model, n2 = (size_t)c.d_model * m->K2;
  const size_t nu = (size_t)c.d_vocab * c.d_model;
  const int np = mode == TVR_GEMM_X3BF16 ? 3 : mode == TVR_GEMM_X2F16 ? 2 : 1;
  const size_t nqk = (size_t)2 * c.d_model * c.d_model;  // BF16: W1's Q / K rows as an fp16 plane
  // diagnostic knobs, read per call, for the bf16 bars' negative controls (tests/test_gpu_full_depth.py
  // test_bf16_bars_reject_a_wrong_bf16_path) — never set in production: TVR_DEBUG_BF16_QK=0 drops the fp16
  // Q / K operands (the Q / K columns run on bf16 like the rest), TVR_DEBUG_BF16_TRUNC=1 builds the bf16
  // weight planes by truncation instead of round-to-nearest-even
  const bool bf16_qk16 = env_int("TVR_DEBUG_BF16_QK", 1) != 0;
  const bool bf16_trunc = env_int("TVR_DEBUG_BF16_TRUNC", 0) != 0;
  const size_t total = np * ((mode == TVR_GEMM_X2F16 && m->x16 ? 0 : n1 + n2) * L + nu) +
                       (mode == TVR_GEMM_BF16 && bf16_qk16 ? nqk * L : 0);
  if (hipMalloc(&m->planes, total * sizeof(uint16_t)) != hipSuccess) {
    m->planes = nullptr;
    (void)hipGetLastError();
    return fail(TVR_ERR_NOMEM, "tvr_model_set_gemm: weight planes (" + std::to_string(total * 2) +
                                   " bytes) do not fit");
  }
  // every GEMM weight matrix in order: w1[0], w2[0], ..., w1[L-1], w2[L-1], wu — in X2F16 with exact-fp16
  // weights bound (tvr_model_set_exact16) without the w1 / w2 planes: every QKV + MLP-in, O + MLP-out and
  // linearised-entry G GEMM reads the raw fp16 rows (2.8B: 5.9 + 4.2 GB, 12B: 26 + 19 GB not allocated)
  const bool skip_x16 = mode == TVR_GEMM_X2F16 && m->x16;
  std::vector<MatW*> mats;
  std::vector<size_t> sizes;
  for (int l = 0; l < L && !skip_x16; ++l) {
    mats.push_back(&m->w1[l]);
    sizes.push_back(n1);
    mats.push_back(&m->w2[l]);
    sizes.push_back(n2);
  }
  mats.push_back(&m->wu); sizes.push_back(nu);
  if (mode == TVR_GEMM_BF16 && bf16_qk16) {  // the fp16 Q / K planes: one scale per layer from max |W_QK|
    for (int l = 0; l < L; ++l) {
      mats.push_back(nullptr);
      sizes.push_back(nqk);
    }
  }
  std::vector<float> scale(mats.size(), 1.0f);  // sized after the Q / K entries: one per matrix
  // the planes of every matrix exactly fill the allocation: checked BEFORE any conversion kernel writes
  // (a fp16 Q / K entry is one plane, every other matrix np planes)
  size_t planned = 0;
  for (size_t i = 0; i < mats.size(); ++i) planned += (mats[i] ? (size_t)np : 1) * sizes[i];
  auto drop_planes = [&]() {
    (void)hipFree(m->planes);
    m->planes = nullptr;
    for (auto& w : m->w1) w = MatW{w.f};
    for (auto& w : m->w2) w = MatW{w.f};
    m->w1qk.clear();
    m->wu = MatW{m->wu.f};
  };
  if (planned != total) {
    drop_planes();
    return fail(TVR_ERR_INTERNAL, "tvr_model_set_gemm: planes planned " + std::to_string(planned) +
                                      " != allocated " + std::to_string(total));
  }
  if (mode == TVR_GEMM_X2F16 || mode == TVR_GEMM_BF16) {
    // one power-of-two scale per matrix from its largest magnitude
    unsigned* d_max = nullptr;
    TVR_HIP(hipMalloc(&d_max, mats.size() * sizeof(unsigned)));
    std::vector<unsigned> h_max(mats.size(), 0);
    hipError_t e = hipMemsetAsync(d_max, 0, mats.size() * sizeof(unsigned), st);
    for (size_t i = 0; i < mats.size() && e == hipSuccess; ++i) {
      const float* src = mats[i] ? mats[i]->f : m->w1[i - (mats.size() - L)].f;  // null: layer's Q / K rows
      if (mode == TVR_GEMM_BF16 && mats[i]) continue;
      hipLaunchKernelGGL(absmax_kernel, dim3(1024), dim3(256), 0, st, src, sizes[i], d_max + i);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h_max.data(), d_max, mats.size() * sizeof(unsigned),
                                            hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(d_max);
    if (e != hipSuccess) return fail(TVR_ERR_HIP, std::string("tvr_model_set_gemm: ") + hipGetErrorString(e));
    for (size_t i = 0; i < mats.size(); ++i) {
      float v;
      std::memcpy(&v, &h_max[i], sizeof(v));
      scale[i] = x2_weight_scale(v);
    }
  }
  uint16_t* p = m->planes;
  for (size_t i = 0; i < mats.size(); ++i) {
    const size_t n = sizes[i];
    if (!mats[i]) {  // BF16: layer l's fp16 Q / K plane (the first 2d rows of W1, row stride d)
      const int l = (int)(i - (mats.size() - L));
      const float* f = m->w1[l].f;
      hipLaunchKernelGGL(f16_plane_kernel, dim3(2048), dim3(256), 0, st, f, scale[i], p, n);
      TVR_HIP(hipGetLastError());
      m->w1qk.push_back(MatW{f, nullptr, p, n, scale[i]});
      p += n;
      continue;
    }
    MatW& w = *mats[i];
    if (mode == TVR_GEMM_X3BF16) {
      hipLaunchKernelGGL(split_planes_kernel, dim3(2048), dim3(256), 0, st, w.f, p, n);
      w = MatW{w.f, p, nullptr, n, 1.0f};
    } else if (mode == TVR_GEMM_BF16) {
      hipLaunchKernelGGL(bf16_plane_kernel, dim3(2048), dim3(256), 0, st, w.f, p, n, (int)bf16_trunc);
      w = MatW{w.f, nullptr, p, n, 1.0f};
    } else {
      hipLaunchKernelGGL(split_planes_f16_kernel, dim3(2048), dim3(256), 0, st, w.f, scale[i], p, n);
      w = MatW{w.f, nullptr, p, n, scale[i]};
    }
    TVR_HIP(hipGetLastError());
    p += np * n;
  }
  if ((size_t)(p - m->planes) != total) {
    (void)hipStreamSynchronize(st);
    const size_t written = (size_t)(p - m->planes);
    drop_planes();
    return fail(TVR_ERR_INTERNAL, "tvr_model_set_gemm: planes written " + std::to_string(written) +
                                      " != allocated " + std::to_string(total));
  }
  TVR_HIP(hipMemsetAsync(m->range_flag, 0, sizeof(unsigned), st));
  TVR_HIP(hipStreamSynchronize(st));
  m->gemm_mode = mode;
  return TVR_OK;
}

int tvr_model_range_status(tvr_model* m, void* stream) {
  if (!m) return fail(TVR_ERR_INVALID, "tvr_model_range_status: null model");
  const hipStream_t st = (hipStream_t)stream;
  unsigned h = 0;
  TVR_HIP(hipMemcpyAsync(&h, m->range_flag, sizeof(unsigned), hipMemcpyDeviceToHost, st));
  TVR_HIP(hipStreamSynchronize(st));
  if (h == 0) return TVR_OK;
  TVR_HIP(hipMemsetAsync(m->range_flag, 0, sizeof(unsigned), st));
  TVR_HIP(hipStreamSynchronize(st));
  return fail(TVR_ERR_RANGE, "a GEMM input reached |a| >= " + std::to_string((int)(X2_FP16_OVERFLOW / X2_ASCALE)) +
                                 ", outside the fp16-split (X2F16) range; results since the last check are not "
                                 "fp32-accurate: use gemm mode x3bf16 or f32");
}

int tvr_profile_enable(tvr_model* m, int32_t on) {
  if (!m) return fail(TVR_ERR_INVALID, "tvr_profile_enable: null model");
  TVR_HIP(hipDeviceSynchronize());
  for (auto& r : m->prof_recs) {
    m->prof_pool.push_back(r.a);
    m->prof_pool.push_back(r.b);
  }
  m->prof_recs.clear();
  m->prof = on != 0;
  return TVR_OK;
}

int tvr_profile_read(tvr_model* m, tvr_kernel_stats* out) {
  if (!m || !out) return fail(TVR_ERR_INVALID, "tvr_profile_read: null argument");
  tvr_kernel_stats s{};
  for (auto& r : m->prof_recs) {
    if (r.epi >= 3) continue;  // HBM-bound kernels: tvr_profile_read_hbm
    TVR_HIP(hipEventSynchronize(r.b));
    float ms = 0.f;
    TVR_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    s.gemm_launches[r.epi] += 1;
    s.gemm_flops[r.epi] += r.flops;
    s.gemm_bytes[r.epi] += r.bytes;
    s.gemm_ms[r.epi] += ms;
  }
  *out = s;
  return TVR_OK;
}

int tvr_profile_read_hbm(tvr_model* m, tvr_hbm_stats* out) {
  if (!m || !out) return fail(TVR_ERR_INVALID, "tvr_profile_read_hbm: null argument");
  tvr_hbm_stats s{};
  for (auto& r : m->prof_recs) {
    if (r.epi < 3) continue;
    TVR_HIP(hipEventSynchronize(r.b));
    float ms = 0.f;
    TVR_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    const int k = r.epi - 3;
    s.launches[k] += 1;
    s.ms[k] += ms;
    s.bytes[k] += r.bytes;
  }
  *out = s;
  return TVR_OK;
}

int tvr_trace_create(tvr_model* m, int32_t max_seqs, int32_t max_tokens, tvr_trace** out) {
  if (!m || !out || max_seqs <= 0 || max_tokens <= 0)
    return fail(TVR_ERR_INVALID, "tvr_trace_create: bad argument");
  const tvr_config& c = m->cfg;
  auto* t = new tvr_trace();
  t->model = m;
  t->max_seqs = max_seqs;
  t->max_tokens = max_tokens;
  const size_t per = (size_t)max_tokens * c.d_model * sizeof(float);
  hipError_t e = hipMalloc(&t->resid, per * (c.n_layers + 1));
  if (e == hipSuccess) e = hipMalloc(&t->z, per * c.n_layers);
  if (e == hipSuccess) e = hipMalloc(&t->qkv, per * 3 * c.n_layers);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    tvr_trace_destroy(t);
    return fail(TVR_ERR_NOMEM, "tvr_trace_create: device allocation failed");
  }
  *out = t;
  return TVR_OK;
}

int tvr_trace_destroy(tvr_trace* t) {
  if (!t) return TVR_OK;
  // a deferred clean forward still owes its outputs to the caller: run it once
  // everything already queued on any stream (work sharing the model's
  // workspace included) has finished, on the null stream — the deferral's
  // stream may already have been destroyed by a C caller
  int rc = TVR_OK;
  if (t->pending) {
    (void)hipDeviceSynchronize();
    rc = flush_pending(t, nullptr);
  }
  (void)hipDeviceSynchronize();
  if (t->resid) (void)hipFree(t->resid);
  if (t->z) (void)hipFree(t->z);
  if (t->qkv) (void)hipFree(t->qkv);
  delete t;
  return rc;
}

int tvr_trace_flush(tvr_trace* t, void* stream) {
  if (!t) return fail(TVR_ERR_INVALID, "tvr_trace_flush: null trace");
  return flush_pending(t, stream);
}

int tvr_trace_read(const tvr_trace* t, int32_t what, int32_t layer, float* dst, void* stream) {
  if (!t || !dst) return fail(TVR_ERR_INVALID, "tvr_trace_read: null argument");
  TVR_TRY(flush_pending(const_cast<tvr_trace*>(t), stream));  // a deferred clean forward runs now
  const int L = t->model->cfg.n_layers, d = t->model->cfg.d_model;
  const size_t stride = (size_t)t->max_tokens * d;
  const float* src = nullptr;
  if (what == TVR_TRACE_RESID_PRE && layer >= 0 && layer <= L) src = t->resid + layer * stride;
  if (what == TVR_TRACE_Z && layer >= 0 && layer < L) src = t->z + layer * stride;
  if (!src) return fail(TVR_ERR_INVALID, "tvr_trace_read: bad hook/layer");
  if (what == TVR_TRACE_RESID_PRE && t->uncentred && t->n_tokens > 0) {
    // TL's residual stream is centred (every write to it is: W_E, W_O, W_out, their biases); the x16 path's
    // differs from it by one constant per row
    // (a caller's dst may be any float*, e.g. an offset view: the float4 form only where it is 16-B aligned)
    const bool v4 = ((uintptr_t)dst & 15) == 0 && ((uintptr_t)src & 15) == 0 && d % 4 == 0;
    if (v4)
      hipLaunchKernelGGL(center_rows_kernel<true>, dim3((t->n_tokens + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                         src, dst, t->n_tokens, d);
    else
      hipLaunchKernelGGL(center_rows_kernel<false>, dim3((t->n_tokens + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                         src, dst, t->n_tokens, d);
    TVR_HIP(hipGetLastError());
    return TVR_OK;
  }
  TVR_HIP(hipMemcpyAsync(dst, src, (size_t)t->n_tokens * d * sizeof(float), hipMemcpyDeviceToDevice,
                         (hipStream_t)stream));
  return TVR_OK;
}

int32_t tvr_trace_num_tokens(const tvr_trace* t) { return t ? t->n_tokens : 0; }

}  // extern "C"

namespace {
// The batched clean forward behind tvr_forward_clean / tvr_forward_logits.
//   tokens     host ids (embedded), or nullptr with resid_in: device [R][d]
//              hook_resid_pre of start_layer (TL forward(resid, start_at_layer=))
//   all_rows   logits of EVERY row to out_logits [R][V] (TL forward's [1, T, V]);
//              otherwise each sequence's last row (out_prob / out_topk / out_logits [n][V])
int forward_impl(tvr_model* m, tvr_trace* trace, const int32_t* tokens, const float* resid_in, int start_layer,
                 const int32_t* seq_lens, int32_t n_seq, const int32_t* targets, float* out_prob,
                 int32_t* out_topk, int32_t topk, float* out_logits, bool all_rows, float* capture_zsum,
                 void* stream) {
  if (!m || (!tokens && !resid_in) || !seq_lens || n_seq <= 0)
    return fail(TVR_ERR_INVALID, "tvr_forward_clean: bad argument");
  if (start_layer < 0 || start_layer >= m->cfg.n_layers || (tokens && start_layer != 0) || (resid_in && trace))
    return fail(TVR_ERR_INVALID, "forward: start_layer needs a residual input and no trace");
  if (topk < 0 || topk > STATS_MAX_K) return fail(TVR_ERR_INVALID, "topk must be in [0, 16]");
  if (topk > 0 && !out_topk) return fail(TVR_ERR_INVALID, "topk > 0 needs out_topk");
  hipStream_t st = (hipStream_t)stream;
  const tvr_config& c = m->cfg;
  const int d = c.d_model, L = c.n_layers;
  std::vector<int32_t> off(n_seq), last(n_seq);
  int R = 0, maxT = 0;
  for (int s = 0; s < n_seq; ++s) {
    const int T = seq_lens[s];
    if (T <= 0) return fail(TVR_ERR_INVALID, "sequence " + std::to_string(s) + " is empty");
    if (T > c.n_ctx)
      return fail(TVR_ERR_UNSUPPORTED, "sequence length " + std::to_string(T) + " exceeds n_ctx " +
                                           std::to_string(c.n_ctx));
    off[s] = R;
    last[s] = R + T - 1;
    R += T;
    maxT = std::max(maxT, T);
  }
  for (int r = 0; tokens && r < R; ++r)
    if (tokens[r] < 0 || tokens[r] >= c.d_vocab)
      return fail(TVR_ERR_INVALID, "token id " + std::to_string(tokens[r]) + " out of range");
  if (trace && (n_seq > trace->max_seqs || R > trace->max_tokens))
    return fail(TVR_ERR_INVALID, "trace capacity exceeded");
  if (trace) trace->uncentred = use_x16(m);

  std::vector<SeqDesc> seqs(n_seq);
  for (int s = 0; s < n_seq; ++s) seqs[s] = {off[s], seq_lens[s], 0, -1, 0, 0};
  std::vector<int32_t> tok = tokens ? std::vector<int32_t>(tokens, tokens + R) : std::vector<int32_t>();
  // Shared prefixes without a trace (only each prompt's last row is read
  // afterwards): a prompt whose leading tokens equal those of the first prompt
  // with its first token computes only the rows after the common prefix and
  // reads the prefix K/V from that prompt's rows (SeqDesc.prefix_live); every
  // extraction prompt starts with BOS.  With a trace every row is kept (patch
  // sweeps read any position of it).
  if (!trace && tokens && !all_rows && prefix_share_enabled()) {
    std::map<int, int> first;  // first token -> first prompt starting with it
    std::vector<int32_t> ctok;
    ctok.reserve(R);
    int Rc = 0;
    for (int s = 0; s < n_seq; ++s) {
      const int T = seq_lens[s];
      const int32_t* tk = tokens + off[s];
      int P = 0, ld = -1;
      const auto it = first.find(tk[0]);
      if (it == first.end()) {
        first.emplace(tk[0], s);
      } else {
        ld = it->second;
        const int32_t* tl = tokens + off[ld];
        const int cap = std::min(T - 1, seq_lens[ld]);
        while (P < cap && tk[P] == tl[P]) ++P;
      }
      seqs[s] = P > 0 ? SeqDesc{Rc, T - P, P, seqs[ld].row0, 0, 1} : SeqDesc{Rc, T, 0, -1, 0, 0};
      ctok.insert(ctok.end(), tk + P, tk + T);
      last[s] = Rc + T - P - 1;
      Rc += T - P;
    }
    tok.swap(ctok);
    R = Rc;
  }
  // without a trace only each prompt's last row is read after the last layer
  const bool trim = trace == nullptr && !all_rows;
  std::vector<SeqDesc> seqs_last(seqs);
  for (auto& q : seqs_last) q.q0 = q.n - 1;
  std::vector<int32_t> tg(n_seq, -1);
  if (targets) std::copy(targets, targets + n_seq, tg.begin());

  const int n_out = all_rows ? R : n_seq;  // rows of the final LN + unembed
  std::vector<int32_t> out_rows;
  if (all_rows) {
    out_rows.resize(R);
    for (int r = 0; r < R; ++r) out_rows[r] = r;
  }
  const int FC = std::min(final_chunk(m, act_fmt(m), out_logits), n_out);
  Carve cv;
  const size_t o_seqs = cv.take<SeqDesc>(n_seq);
  const size_t o_seqs_last = cv.take<SeqDesc>(n_seq);
  const size_t o_tok = cv.take<int32_t>(R);
  const size_t o_last = cv.take<int32_t>(n_seq);
  const size_t o_rows = all_rows ? cv.take<int32_t>(R) : 0;
  const size_t o_tg = cv.take<int32_t>(n_seq);
  const size_t o_resid = cv.take<float>((size_t)R * d);
  const size_t o_xn = cv.take<float>((size_t)R * d);
  const size_t o_xn2 = use_x16(m) ? cv.take<float>((size_t)R * d) : 0;
  const size_t o_qkv = trace ? 0 : cv.take<float>((size_t)R * 3 * d);
  const size_t o_a2 = cv.take<float>((size_t)R * m->K2);
  const size_t o_xf = cv.take<float>((size_t)FC * d);
  const size_t o_lg = cv.take<float>(final_scratch_floats(m, act_fmt(m), FC, topk, out_logits));
  const int n_cap = capture_zsum ? L - start_layer : 0;  // layers captured (one reduction after the loop)
  const size_t o_cap = capture_zsum ? cv.take<float>((size_t)n_cap * CAP_GROUPS * d) : 0;
  // fp32 hook_z of each prompt's last row, every layer, for the capture when no
  // trace slot receives it (the attention kernel writes that row only, at row s
  // of the layer's slab)
  const bool zf_last = capture_zsum && !trace;
  const size_t o_zf = zf_last ? cv.take<float>((size_t)n_cap * n_seq * d) : 0;
  TVR_TRY(ensure_workspace(m, cv.off, st));
  char* base = m->ws;
  UploadBatch ub;
  ub.add(o_seqs, seqs);
  ub.add(o_seqs_last, seqs_last);
  ub.add(o_tok, tok);
  ub.add(o_last, last);
  if (all_rows) ub.add(o_rows, out_rows);
  ub.add(o_tg, tg);
  TVR_TRY(flush_uploads(m, st, base, ub));

  const int fmt = act_fmt(m);
  Acts a{(float*)(base + o_resid), (float*)(base + o_xn), trace ? nullptr : (float*)(base + o_qkv),
         (float*)(base + o_a2), fmt};
  if (use_x16(m)) a.xn2 = (float*)(base + o_xn2);
  const SeqDesc* d_seqs = (const SeqDesc*)(base + o_seqs);
  const int32_t* d_last = (const int32_t*)(base + o_last);
  const size_t tstride = trace ? (size_t)trace->max_tokens * d : 0;

  if (tokens) {
    const size_t total = (size_t)R * (d / 4);
    const int blocks = (int)std::min<size_t>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(embed_kernel, dim3(blocks), dim3(256), 0, st, (const int32_t*)(base + o_tok),
                       m->w_embed, a.resid, R, d);
    TVR_HIP(hipGetLastError());
  } else {
    TVR_HIP(hipMemcpyAsync(a.resid, resid_in, (size_t)R * d * sizeof(float), hipMemcpyDeviceToDevice, st));
  }
  for (int l = start_layer; l < L; ++l) {
    if (trace)
      TVR_HIP(hipMemcpyAsync(trace->resid + l * tstride, a.resid, (size_t)R * d * sizeof(float),
                             hipMemcpyDeviceToDevice, st));
    float* qkv = trace ? trace->qkv + (size_t)l * 3 * tstride : a.qkv;
    // attention writes the fp32 hook_z straight into the trace (or the capture buffer)
    float* zf = trace ? trace->z + l * tstride
                      : (capture_zsum ? (float*)(base + o_zf) + (size_t)(l - start_layer) * n_seq * d : nullptr);
    const bool want_out = out_prob || out_topk || out_logits;
    if (trim && l == L - 1) {
      TVR_TRY(run_block_last_rows(m, l, R, (const SeqDesc*)(base + o_seqs_last), n_seq, maxT, a, nullptr,
                                  d_last, n_seq, want_out, zf, st, zf_last));
    } else {
      TVR_TRY(run_block(m, l, R, d_seqs, n_seq, maxT, a, qkv, nullptr, zf, st, zf_last));
    }
    if (!(trim && l == L - 1)) TVR_TRY(run_block_out(m, l, R, a, st));
  }
  if (capture_zsum) {  // every layer's Σ over prompts of hook_z at the last row: one launch pair
    float* part = (float*)(base + o_cap);
    const float* z0 = trace ? trace->z + start_layer * tstride : (const float*)(base + o_zf);
    ProfSpan ps(m, st);
    hipLaunchKernelGGL(capture_partial_kernel, dim3((d / 4 + 63) / 64, CAP_GROUPS, n_cap), dim3(64), 0, st,
                       z0, d, trace ? tstride : (size_t)n_seq * d, zf_last ? nullptr : d_last, n_seq, part, d);
    hipLaunchKernelGGL(capture_finish_kernel, dim3((d + 255) / 256, n_cap), dim3(256), 0, st, part,
                       capture_zsum + (size_t)start_layer * d, d);
    TVR_HIP(hipGetLastError());
    ps.done(TVR_HBM_CAPTURE, (double)n_cap * ((double)n_seq + 1.0) * d * 4.0);  // hook_z at every last row in, [L][d] out
  }
  if (trace) {
    TVR_HIP(hipMemcpyAsync(trace->resid + L * tstride, a.resid, (size_t)R * d * sizeof(float),
                           hipMemcpyDeviceToDevice, st));
    trace->seq_off.assign(off.begin(), off.end());
    trace->seq_len.assign(seq_lens, seq_lens + n_seq);
    trace->tokens.assign(tokens, tokens + R);  // trace => tokens (checked above)
    trace->n_seq = n_seq;
    trace->n_tokens = R;
  }
  if (all_rows)
    TVR_TRY(run_final(m, a.resid, (const int32_t*)(base + o_rows), nullptr, R, (float*)(base + o_xf),
                      (float*)(base + o_lg), nullptr, nullptr, 0, out_logits, fmt, st));
  else if (out_prob || out_topk || out_logits)
    TVR_TRY(run_final(m, a.resid, d_last, (const int32_t*)(base + o_tg), n_seq, (float*)(base + o_xf),
                      (float*)(base + o_lg), out_prob, out_topk, topk, out_logits, fmt, st));
  return TVR_OK;
}
// Run a deferred clean forward on its own (the trace is used other than by a
// patch sweep).
int flush_pending(tvr_trace* t, void* stream) {
  if (!t->pending) return TVR_OK;
  t->pending = false;
  const std::vector<int32_t> tok(t->tokens), lens(t->seq_len), tg(t->p_targets);
  return forward_impl(t->model, t, tok.data(), nullptr, 0, lens.data(), (int32_t)lens.size(),
                      tg.empty() ? nullptr : tg.data(), t->p_prob, t->p_topk, t->p_k, nullptr, false, nullptr, stream);
}
}  // namespace

extern "C" {

int tvr_forward_clean(tvr_model* m, tvr_trace* trace, const int32_t* tokens, const int32_t* seq_lens,
                      int32_t n_seq, const int32_t* targets, float* out_prob, int32_t* out_topk,
                      int32_t topk, float* out_logits, float* capture_zsum, void* stream) {
  if (!tokens) return fail(TVR_ERR_INVALID, "tvr_forward_clean: bad argument");
  if (trace) TVR_TRY(flush_pending(trace, stream));  // its outputs are owed to the caller
  return forward_impl(m, trace, tokens, nullptr, 0, seq_lens, n_seq, targets, out_prob, out_topk, topk, out_logits,
                      false, capture_zsum, stream);
}

int tvr_forward_clean_deferred(tvr_model* m, tvr_trace* trace, const int32_t* tokens, const int32_t* seq_lens,
                               int32_t n_seq, const int32_t* targets, float* out_prob, int32_t* out_topk,
                               int32_t topk, void* stream) {
  if (!m || !trace || !tokens || !seq_lens || n_seq <= 0)
    return fail(TVR_ERR_INVALID, "tvr_forward_clean_deferred: bad argument");
  if (trace->model != m) return fail(TVR_ERR_INVALID, "trace belongs to another model");
  if (topk < 0 || topk > STATS_MAX_K) return fail(TVR_ERR_INVALID, "topk must be in [0, 16]");
  if (topk > 0 && !out_topk) return fail(TVR_ERR_INVALID, "topk > 0 needs out_topk");
  TVR_TRY(flush_pending(trace, stream));
  const tvr_config& c = m->cfg;
  std::vector<int> off(n_seq);
  int R = 0;
  for (int s = 0; s < n_seq; ++s) {
    const int T = seq_lens[s];
    if (T <= 0) return fail(TVR_ERR_INVALID, "sequence " + std::to_string(s) + " is empty");
    if (T > c.n_ctx)
      return fail(TVR_ERR_UNSUPPORTED, "sequence length " + std::to_string(T) + " exceeds n_ctx " +
                                           std::to_string(c.n_ctx));
    off[s] = R;
    R += T;
  }
  for (int r = 0; r < R; ++r)
    if (tokens[r] < 0 || tokens[r] >= c.d_vocab)
      return fail(TVR_ERR_INVALID, "token id " + std::to_string(tokens[r]) + " out of range");
  if (n_seq > trace->max_seqs || R > trace->max_tokens) return fail(TVR_ERR_INVALID, "trace capacity exceeded");
  trace->seq_off = off;
  trace->seq_len.assign(seq_lens, seq_lens + n_seq);
  trace->tokens.assign(tokens, tokens + R);
  trace->n_seq = n_seq;
  trace->n_tokens = R;
  trace->p_targets = targets ? std::vector<int32_t>(targets, targets + n_seq) : std::vector<int32_t>();
  trace->p_prob = out_prob;
  trace->p_topk = out_topk;
  trace->p_k = topk;
  trace->p_stream = stream;
  trace->pending = true;
  return TVR_OK;
}

int tvr_forward_logits(tvr_model* m, const int32_t* tokens, const float* resid_in, int32_t start_layer,
                       const int32_t* seq_lens, int32_t n_seq, float* out_logits, void* stream) {
  if (!out_logits || (tokens == nullptr) == (resid_in == nullptr))
    return fail(TVR_ERR_INVALID, "tvr_forward_logits: give exactly one of tokens / resid_in, and out_logits");
  return forward_impl(m, nullptr, tokens, resid_in, start_layer, seq_lens, n_seq, nullptr, nullptr, nullptr, 0,
                      out_logits, true, nullptr, stream);
}



int tvr_patch_sweep(tvr_model* m, tvr_trace* trace, const tvr_site* sites, int32_t n_sites,
                    const float* vectors, int32_t n_vectors, float* out_prob, int32_t* out_topk,
                    int32_t topk, float* out_logits, void* stream) {
  if (!m || !trace || !sites || n_sites <= 0)
    return fail(TVR_ERR_INVALID, "tvr_patch_sweep: bad argument");
  if (trace->model != m) return fail(TVR_ERR_INVALID, "trace belongs to another model");
  if (trace->n_seq <= 0) return fail(TVR_ERR_INVALID, "trace is empty: run tvr_forward_clean first");
  if (topk < 0 || topk > STATS_MAX_K) return fail(TVR_ERR_INVALID, "topk must be in [0, 16]");
  if (topk > 0 && !out_topk) return fail(TVR_ERR_INVALID, "topk > 0 needs out_topk");
  hipStream_t st = (hipStream_t)stream;
  const tvr_config& c = m->cfg;
  const int d = c.d_model, L = c.n_layers;
  // Fused clean forward (a deferred tvr_forward_clean on this trace): the
  // clean rows [0, Rc) (trace row layout) run in the same launches as the
  // site rows, which follow them; the sites read the clean K/V from the live
  // buffer, and the trace is filled as the layers go.  This removes the clean
  // forward's own small-M launches (52 prompts x 3 tokens).
  const bool fused = trace->pending;
  if (fused) trace->uncentred = use_x16(m);  // this sweep fills the trace's clean rows
  const int Rc = fused ? trace->n_tokens : 0, nc = fused ? trace->n_seq : 0;

  // --- plan -----------------------------------------------------------------
  std::vector<int> entry(n_sites), p0(n_sites), nrow(n_sites);
  int maxT = 0;
  for (int s = 0; s < nc; ++s) maxT = std::max(maxT, trace->seq_len[s]);
  for (int i = 0; i < n_sites; ++i) {
    const tvr_site& s = sites[i];
    if (s.seq < 0 || s.seq >= trace->n_seq)
      return fail(TVR_ERR_INVALID, "site " + std::to_string(i) + ": seq out of range");
    const int T = trace->seq_len[s.seq];
    maxT = std::max(maxT, T);
    switch (s.kind) {
      case TVR_SITE_NONE:
        entry[i] = L; p0[i] = T - 1; nrow[i] = 1;
        break;
      case TVR_SITE_REPLACE_HEAD_ALLPOS:
        if (s.layer < 0 || s.layer >= L || s.head < 0 || s.head >= c.n_heads)
          return fail(TVR_ERR_INVALID, "site " + std::to_string(i) + ": layer/head out of range");
        if (!vectors || s.vec < 0 || s.vec >= n_vectors)
          return fail(TVR_ERR_INVALID, "site " + std::to_string(i) + ": vector out of range");
        entry[i] = s.layer + 1; p0[i] = 0; nrow[i] = T;
        break;
      case TVR_SITE_ADD_ATTN_OUT_LASTPOS:
        if (s.layer < 0 || s.layer >= L)
          return fail(TVR_ERR_INVALID, "site " + std::to_string(i) + ": layer out of range");
        if (!vectors || s.vec < 0 || s.vec >= n_vectors)
          return fail(TVR_ERR_INVALID, "site " + std::to_string(i) + ": vector out of range");
        entry[i] = s.layer + 1; p0[i] = T - 1; nrow[i] = 1;
        break;
      case TVR_SITE_SET_RESID_PRE_POS:
        if (s.layer < 0 || s.layer >= L || s.pos < 0 || s.pos >= T || s.src_seq < 0 ||
            s.src_seq >= trace->n_seq || s.src_pos < 0 || s.src_pos >= trace->seq_len[s.src_seq])
          return fail(TVR_ERR_INVALID, "site " + std::to_string(i) + ": resid patch out of range");
        entry[i] = s.layer; p0[i] = s.pos; nrow[i] = T - s.pos;
        break;
      default:
        return fail(TVR_ERR_INVALID, "site " + std::to_string(i) + ": unknown kind");
    }
  }
  // every site computes one row (its last position: ADD_ATTN_OUT_LASTPOS,
  // NONE, a SET_RESID_PRE_POS of the last position): the site sequences go to
  // the single-query attention kernel
  bool single_rows = true;
  for (int i = 0; i < n_sites; ++i) single_rows = single_rows && nrow[i] == 1;
  // Shared prefixes (REPLACE_HEAD_ALLPOS): sites with the same (layer, head,
  // vector) whose sequences start with the same tokens compute identical rows
  // over that common prefix (position j attends to positions <= j only, and
  // the patch is the same at every position).  The first such site (the
  // leader) computes them; a follower starts at its common-prefix length P
  // and reads positions < P's K/V from the leader's rows of this run
  // (SeqDesc.prefix_live).  A CIE sweep's prompts all start with BOS, so
  // (n_prompts - 1) / n_prompts of the position-0 rows — 1/T of the sweep's
  // rows — are not recomputed.  The reference's batch-1 forwards compute that
  // row identically for every prompt (scratch2.py:181-194).
  std::vector<int> leader(n_sites, -1);
  if (prefix_share_enabled() && (int)trace->tokens.size() >= trace->n_tokens) {
    std::map<std::tuple<int, int, int, int>, int> first;
    for (int i = 0; i < n_sites; ++i) {
      const tvr_site& s = sites[i];
      if (s.kind != TVR_SITE_REPLACE_HEAD_ALLPOS) continue;
      const int32_t* tk = trace->tokens.data() + trace->seq_off[s.seq];
      const auto key = std::make_tuple(s.layer, s.head, s.vec, (int)tk[0]);
      const auto it = first.find(key);
      if (it == first.end()) {
        first.emplace(key, i);
        continue;
      }
      const int ld = it->second;
      const int32_t* tl = trace->tokens.data() + trace->seq_off[sites[ld].seq];
      const int T = trace->seq_len[s.seq];
      const int cap = std::min(T - 1, trace->seq_len[sites[ld].seq]);  // the last row stays the site's own
      int P = 0;
      while (P < cap && tk[P] == tl[P]) ++P;
      if (P == 0) continue;
      leader[i] = ld;
      p0[i] = P;
      nrow[i] = T - P;
    }
  }
  std::vector<int> order(n_sites);
  for (int i = 0; i < n_sites; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return entry[a] < entry[b]; });
  std::vector<int> row0(n_sites);
  std::vector<int> cnt_le(L + 1, 0), rows_le(L + 1, 0);  // sites / rows with entry <= l
  int R = 0;
  for (int k = 0; k < n_sites; ++k) {
    const int i = order[k];
    row0[i] = R;
    R += nrow[i];
  }
  {
    int k = 0, rows = 0;
    for (int l = 0; l <= L; ++l) {
      while (k < n_sites && entry[order[k]] <= l) { rows += nrow[order[k]]; ++k; }
      cnt_le[l] = k;
      rows_le[l] = rows;
    }
  }
  // sequence descriptors: the fused clean sequences first, then the sites in entry order
  std::vector<SeqDesc> seqs(nc + n_sites);
  for (int s = 0; s < nc; ++s) seqs[s] = SeqDesc{trace->seq_off[s], trace->seq_len[s], 0, -1, 0, 0};
  std::vector<EntryDesc> ents(n_sites);
  for (int k = 0; k < n_sites; ++k) {
    const int i = order[k];
    const tvr_site& s = sites[i];
    const int srow = trace->seq_off[s.seq];
    seqs[nc + k] = leader[i] >= 0 ? SeqDesc{Rc + row0[i], nrow[i], p0[i], Rc + row0[leader[i]], 0, 1}
                                  : SeqDesc{Rc + row0[i], nrow[i], p0[i], srow, 0, 0};
    EntryDesc e{};
    e.kind = s.kind;
    e.row0 = Rc + row0[i];
    e.n = nrow[i];
    e.p0 = p0[i];
    e.src_row = srow;
    e.src2_row = (s.kind == TVR_SITE_SET_RESID_PRE_POS) ? trace->seq_off[s.src_seq] + s.src_pos : 0;
    e.patch_pos = s.pos;
    e.head = s.head;
    e.vec = s.vec;
    ents[k] = e;
  }
  // entry layers' head-replacement sites grouped by head, at most ENTRY_GROUP per
  // group, groups of one head balanced (entry_mfma.hpp); ent_other: the layer has sites of other kinds (entry_kernel)
  std::vector<char> ent_other(L + 1, 0);
  std::vector<int32_t> egidx;
  std::vector<int2> egroups;
  std::vector<int> eg_beg(L + 1, 0), eg_cnt(L + 1, 0);
  for (int l = 0; l <= L; ++l) {
    eg_beg[l] = (int)egroups.size();
    std::map<int, std::vector<int>> byhead;
    for (int k = l > 0 ? cnt_le[l - 1] : 0; k < cnt_le[l]; ++k) {
      if (ents[k].kind == TVR_SITE_REPLACE_HEAD_ALLPOS)
        byhead[ents[k].head].push_back(k);
      else
        ent_other[l] = 1;
    }
    for (const auto& hv : byhead) {  // ceil(n / ENTRY_GROUP) groups of balanced size (the launch ends with its
      const size_t n = hv.second.size(), ng = (n + ENTRY_GROUP - 1) / ENTRY_GROUP;  // largest group)
      for (size_t gi = 0; gi < ng; ++gi) {
        const size_t a = gi * n / ng, b = (gi + 1) * n / ng;
        egroups.push_back(make_int2((int)egidx.size(), (int)(b - a)));
        egidx.insert(egidx.end(), hv.second.begin() + a, hv.second.begin() + b);
      }
    }
    eg_cnt[l] = (int)egroups.size() - eg_beg[l];
  }
  // algorithmic bytes of each layer's entry launch (profiling): the clean rows
  // read and the patched rows written, the vector, and for REPLACE_HEAD the
  // head's z rows plus its W_O slice once per distinct head
  std::vector<double> entry_bytes(L + 1, 0.0);  // entry layers 0..L (L: the final norm's input)
  for (int l = 0; l <= L; ++l) {
    std::vector<char> seen(c.n_heads, 0);
    for (int k = l > 0 ? cnt_le[l - 1] : 0; k < cnt_le[l]; ++k) {
      const EntryDesc& e = ents[k];
      double b = (2.0 * e.n * d + d) * 4.0;
      if (e.kind == TVR_SITE_REPLACE_HEAD_ALLPOS) {
        b += (double)e.n * c.d_head * 4.0;
        if (!seen[e.head]) b += (double)d * c.d_head * 4.0;
        seen[e.head] = 1;
      }
      entry_bytes[l] += b;
    }
  }
  std::vector<int32_t> last(n_sites), tg(n_sites);
  for (int i = 0; i < n_sites; ++i) {
    last[i] = Rc + row0[i] + nrow[i] - 1;
    tg[i] = sites[i].target;
  }
  // the last layer computes every clean row (the trace keeps them) and each site's last row
  std::vector<SeqDesc> seqs_last(seqs);
  std::vector<int32_t> last_sorted(Rc + n_sites);
  for (int r = 0; r < Rc; ++r) last_sorted[r] = r;
  for (int k = 0; k < n_sites; ++k) {
    seqs_last[nc + k].q0 = seqs_last[nc + k].n - 1;
    last_sorted[Rc + k] = last[order[k]];
  }
  std::vector<int32_t> clean_last(nc), clean_tg(nc, -1);
  for (int s = 0; s < nc; ++s) clean_last[s] = trace->seq_off[s] + trace->seq_len[s] - 1;
  if (fused && !trace->p_targets.empty()) clean_tg = trace->p_targets;
  const int ktop = std::max(topk, fused ? trace->p_k : 0);

  // Linearised entry layers (lin_entry.hpp): layer l in [1, L-2] of a fused
  // sweep whose entering sites are all REPLACE_HEAD computes its entering
  // rows' QKV + MLP-in outputs from the clean rows' (this sweep's rows
  // [0, Rc)) and a K = d_head GEMM.  Tables per such layer: the distinct
  // vectors (rows of G), the entering rows grouped by head, m-blocks of <= 64
  // rows of one head.
  const int fmt0 = act_fmt(m);
  std::vector<char> use_lin(L, 0);
  std::vector<int32_t> lin_vids;
  std::vector<LinRow> lin_rows;
  std::vector<LinMB> lin_mbs;
  std::vector<int> lin_vid_off(L, 0), lin_nv(L, 0), lin_mb_off(L, 0), lin_nmb(L, 0), lin_nrows(L, 0);
  int lin_max_nv = 0;
  if (fused && fmt0 != ACT_F32 && L >= 3 && lin_entry_enabled()) {
    for (int l = 1; l <= L - 2; ++l) {
      const int k0 = cnt_le[l - 1], k1 = cnt_le[l];
      bool ok = k1 > k0;
      for (int k = k0; k < k1 && ok; ++k) ok = sites[order[k]].kind == TVR_SITE_REPLACE_HEAD_ALLPOS;
      if (!ok) continue;
      use_lin[l] = 1;
      std::map<int, int> vrow;
      lin_vid_off[l] = (int)lin_vids.size();
      for (int k = k0; k < k1; ++k)
        if (vrow.emplace(sites[order[k]].vec, (int)vrow.size()).second) lin_vids.push_back(sites[order[k]].vec);
      lin_nv[l] = (int)vrow.size();
      lin_max_nv = std::max(lin_max_nv, lin_nv[l]);
      lin_mb_off[l] = (int)lin_mbs.size();
      const int r_first = (int)lin_rows.size();
      for (int h = 0; h < c.n_heads; ++h) {
        const int g0 = (int)lin_rows.size();
        for (int k = k0; k < k1; ++k) {
          const int i = order[k];
          const tvr_site& s = sites[i];
          if (s.head != h) continue;
          for (int q = 0; q < nrow[i]; ++q)
            lin_rows.push_back(LinRow{Rc + row0[i] + q, trace->seq_off[s.seq] + p0[i] + q, vrow[s.vec], 0});
        }
        for (int r = g0; r < (int)lin_rows.size(); r += 64)
          lin_mbs.push_back(LinMB{r, std::min(64, (int)lin_rows.size() - r), h, 0});
      }
      lin_nmb[l] = (int)lin_mbs.size() - lin_mb_off[l];
      lin_nrows[l] = (int)lin_rows.size() - r_first;
    }
  }
  bool any_lin = !lin_mbs.empty();
  if (any_lin) {
    const int rc = ensure_lin(m, st);
    if (rc == TVR_ERR_NOMEM) {  // the W1 W_O planes do not fit: the full-GEMM entry (TVR_LIN_ENTRY=0) instead
      any_lin = false;
      std::fill(use_lin.begin(), use_lin.end(), 0);
      lin_vids.clear();
      lin_rows.clear();
      lin_mbs.clear();
      lin_max_nv = 0;
    } else {
      TVR_TRY(rc);
    }
  }

  const int RA = Rc + R;  // rows of the activation buffers
  // run_final chunks: the sites' (logits requested or not) and the fused clean rows' (never logits)
  const int FCs = std::min(final_chunk(m, fmt0, out_logits), n_sites), FCc = std::min(final_chunk(m, fmt0, nullptr), nc);
  Carve cv;
  const size_t o_seqs = cv.take<SeqDesc>(nc + n_sites);
  const size_t o_seqs_last = cv.take<SeqDesc>(nc + n_sites);
  const size_t o_last_sorted = cv.take<int32_t>(Rc + n_sites);
  const size_t o_ents = cv.take<EntryDesc>(n_sites);
  const size_t o_last = cv.take<int32_t>(n_sites);
  const size_t o_tg = cv.take<int32_t>(n_sites);
  const size_t o_clast = cv.take<int32_t>(nc);
  const size_t o_ctg = cv.take<int32_t>(nc);
  const size_t o_ctok = cv.take<int32_t>(Rc);
  // (uploaded tables first: flush_uploads sends one span from the first to the last)
  const size_t o_lin_rows = cv.take<LinRow>(lin_rows.size());
  const size_t o_lin_mbs = cv.take<LinMB>(lin_mbs.size());
  const size_t o_lin_vids = cv.take<int32_t>(lin_vids.size());
  const size_t o_egidx = cv.take<int32_t>(egidx.size());
  const size_t o_egroups = cv.take<int2>(egroups.size());
  const size_t o_resid = cv.take<float>((size_t)RA * d);
  const size_t o_xn = cv.take<float>((size_t)RA * d);
  const size_t o_xn2 = use_x16(m) ? cv.take<float>((size_t)RA * d) : 0;
  const size_t o_qkv = cv.take<float>((size_t)RA * 3 * d);
  const size_t o_a2 = cv.take<float>((size_t)RA * m->K2);
  const size_t o_xf = cv.take<float>((size_t)std::max(FCs, FCc) * d);
  const size_t o_lg = cv.take<float>(std::max(final_scratch_floats(m, fmt0, FCs, ktop, out_logits),
                                              final_scratch_floats(m, fmt0, FCc, ktop, nullptr)));
  const size_t o_lnstats = cv.take<float2>(any_lin ? RA : 0);
  const size_t o_raw = cv.take<float>(any_lin ? (size_t)Rc * c.d_mlp : 0);
  const size_t o_vact = cv.take<float>(any_lin ? (size_t)n_vectors * d : 0);  // vectors in the activation format
  const size_t o_g = cv.take<float>((size_t)lin_max_nv * m->D1);
  // exact-fp16 weights: one layer's G rows (centred vectors x LN1 / LN2 gamma, activation format)
  const bool lin_x16 = any_lin && use_x16(m);
  const size_t o_vg = cv.take<float>(lin_x16 ? (size_t)2 * lin_max_nv * d : 0);
  TVR_TRY(ensure_workspace(m, cv.off, st));
  char* base = m->ws;
  UploadBatch ub;
  ub.add(o_seqs, seqs);
  ub.add(o_seqs_last, seqs_last);
  ub.add(o_last_sorted, last_sorted);
  ub.add(o_ents, ents);
  ub.add(o_last, last);
  ub.add(o_tg, tg);
  if (fused) {
    ub.add(o_clast, clean_last);
    ub.add(o_ctg, clean_tg);
    ub.add(o_ctok, std::vector<int32_t>(trace->tokens.begin(), trace->tokens.begin() + Rc));
  }
  if (any_lin) {
    ub.add(o_lin_rows, lin_rows);
    ub.add(o_lin_mbs, lin_mbs);
    ub.add(o_lin_vids, lin_vids);
  }
  ub.add(o_egidx, egidx);
  ub.add(o_egroups, egroups);
  TVR_TRY(flush_uploads(m, st, base, ub));

  const int fmt = act_fmt(m);
  Acts a{(float*)(base + o_resid), (float*)(base + o_xn), (float*)(base + o_qkv),
         (float*)(base + o_a2), fmt};
  if (use_x16(m)) a.xn2 = (float*)(base + o_xn2);
  const SeqDesc* d_seqs = (const SeqDesc*)(base + o_seqs);
  const EntryDesc* d_ents = (const EntryDesc*)(base + o_ents);
  const size_t tstride = (size_t)trace->max_tokens * d;
  const size_t rbytes = (size_t)Rc * d * sizeof(float);  // the clean rows of one [rows][d] buffer
  if (fused) {
    const size_t total = (size_t)Rc * (d / 4);
    hipLaunchKernelGGL(embed_kernel, dim3((int)std::min<size_t>((total + 255) / 256, 8192)), dim3(256), 0, st,
                       (const int32_t*)(base + o_ctok), m->w_embed, a.resid, Rc, d);
    TVR_HIP(hipGetLastError());
  }

  auto enter = [&](int l) -> int {
    const int k0 = l > 0 ? cnt_le[l - 1] : 0, k1 = cnt_le[l];
    if (k1 <= k0) return TVR_OK;
    // the clean rows' hook_resid_pre: the live rows [0, Rc) in a fused sweep (the trace's copy is written by
    // this layer's LayerNorm, after the entry), else the trace
    const float* snap = fused ? a.resid : trace->resid + (size_t)l * tstride;
    const float* zsnap = l > 0 ? trace->z + (size_t)(l - 1) * tstride : nullptr;
    const float* w2 = l > 0 ? m->layers[l - 1].w2 : nullptr;
    const dim3 eg(k1 - k0, (d + ENTRY_THREADS - 1) / ENTRY_THREADS);
    ProfSpan ps(m, st);
    const bool mf = eg_cnt[l] > 0 && (c.d_head == 16 || c.d_head == 64 || c.d_head == 80 || c.d_head == 128);
    if (mf) {
      const dim3 gg(eg_cnt[l], (d + ENTRY_COLS - 1) / ENTRY_COLS);
      const int32_t* gidx = (const int32_t*)(base + o_egidx);
      const int2* grps = (const int2*)(base + o_egroups) + eg_beg[l];
#define TVR_ENTRY_MF(DH)                                                                                   \
  hipLaunchKernelGGL(entry_replace_mfma_kernel<DH>, gg, dim3(ENTRY_THREADS), 0, st, d_ents, gidx, grps, snap, \
                     zsnap, w2, m->K2, vectors, a.resid, d)
      switch (c.d_head) {
        case 16: TVR_ENTRY_MF(16); break;
        case 64: TVR_ENTRY_MF(64); break;
        case 80: TVR_ENTRY_MF(80); break;
        default: TVR_ENTRY_MF(128); break;
      }
#undef TVR_ENTRY_MF
      TVR_HIP(hipGetLastError());
    }
    if (ent_other[l] || !mf) {
      const size_t zbytes = mf ? 0 : (size_t)std::min(maxT, ENTRY_LDS_POS) * c.d_head * sizeof(float);
      if (zbytes > 64 * 1024)
        TVR_HIP(hipFuncSetAttribute((const void*)entry_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)zbytes));
      hipLaunchKernelGGL(entry_kernel, eg, dim3(ENTRY_THREADS), zbytes, st, d_ents + k0, snap, zsnap, w2, m->K2,
                         vectors, a.resid, d, c.d_head, mf ? 1 : 0);
      TVR_HIP(hipGetLastError());
    }
    ps.done(TVR_HBM_ENTRY, entry_bytes[l]);
    return TVR_OK;
  };

  float2* lnstats = (float2*)(base + o_lnstats);
  float* raw_h = (float*)(base + o_raw);
  uint16_t* vact = (uint16_t*)(base + o_vact);
  if (any_lin) {
    const size_t n = (size_t)n_vectors * d;
    const dim3 g((unsigned)std::min<size_t>((n + 255) / 256, 8192));
    if (fmt == ACT_X2F16)
      hipLaunchKernelGGL(act_rows_kernel<ACT_X2F16>, g, dim3(256), 0, st, vectors, d, vact, n_vectors, d,
                         m->range_flag);
    else  // bf16 plane + the fp16 plane the Q / K columns of G read (as LayerNorm's store_ln4)
      hipLaunchKernelGGL(act_rows_bf16_f16_kernel, g, dim3(256), 0, st, vectors, d, vact, n_vectors, d);
    TVR_HIP(hipGetLastError());
  }
  // layer l's block with the linearised entry rows [Rp, Rl) (use_lin[l])
  auto run_block_lin = [&](int l, int Rl, const float* cache, float* zf) -> int {
    const tvr_layer_weights& w = m->layers[l];
    const int Rp = Rc + rows_le[l - 1], D1 = m->D1;
    TVR_TRY(launch_lnpre(a.resid, d, nullptr, a.xn, d, Rl, d, c.ln_eps, fmt, st, m, lnstats, a.resid_mirror,
                         a.mirror_rows, a.xn2 ? m->g1[l] : nullptr, a.xn2 ? m->g2[l] : nullptr, a.xn2));
    GemmEpi e1 = epi_qkv_mlpin(m, w.b1, a.qkv, a);
    e1.raw = raw_h;
    e1.raw_rows = Rc;
    e1.ld_raw = c.d_mlp;
    TVR_TRY(launch_w1(m, l, a.xn, Rp, 0, D1, e1, st, a.xn2));
    ProfSpan ps(m, st);
    const bool prof = m->prof;
    m->prof = false;  // G and the entry rows are timed as one HBM-kind span, not as GEMM-family launches
    GemmEpi eg{};
    eg.out0 = (float*)(base + o_g);
    eg.ld0 = D1;
    eg.a_rows = (const int32_t*)(base + o_lin_vids) + lin_vid_off[l];
    eg.skinny = 1;
    int rc = TVR_OK;
    const int nqk = fmt == ACT_BF16 && !m->w1qk.empty() ? 2 * d : 0;  // bf16: Q / K columns on fp16 operands
    if (lin_x16) {
      // G = v W1'^T on the raw fp16 W1 (one plane, 2 products): rows ((v - mean) o gamma1 | gamma2), lin_entry.hpp
      uint16_t* vg1 = (uint16_t*)(base + o_vg);
      uint16_t* vg2 = vg1 + (size_t)2 * lin_nv[l] * d;
      hipLaunchKernelGGL(lin_gamma_rows_kernel, dim3((lin_nv[l] + 3) / 4), dim3(256), 0, st, vectors, d,
                         (const int32_t*)(base + o_lin_vids) + lin_vid_off[l], m->g1[l], m->g2[l], vg1, vg2,
                         lin_nv[l], m->range_flag);
      rc = hipGetLastError() == hipSuccess ? TVR_OK : fail(TVR_ERR_HIP, "lin_gamma_rows_kernel launch");
      GemmEpi ex = eg;
      ex.a_rows = nullptr;  // the rows are the layer's vectors in order
      const int q = 3 * d;  // first MLP-in column: it and the columns after it read the gamma2 rows
      if (rc == TVR_OK && q % 256 == 0) {
        ex.a2 = vg2;
        ex.a2_col = q;
        rc = launch_gemm(EPI_BIAS, vg1, d, fmt, m->w1x[l], d, lin_nv[l], D1, d, ex, st, m);
      } else if (rc == TVR_OK) {  // two launches (d % 256 != 0: the tiny test model)
        rc = launch_gemm(EPI_BIAS, vg1, d, fmt, m->w1x[l], d, lin_nv[l], q, d, ex, st, m);
        GemmEpi e2 = ex;
        e2.out0 = ex.out0 + q;
        if (rc == TVR_OK)
          rc = launch_gemm(EPI_BIAS, vg2, d, fmt, m->w1x[l].rows((size_t)q * d), d, lin_nv[l], D1 - q, d, e2, st, m);
      }
    } else if (nqk > 0) {
      rc = launch_gemm(EPI_BIAS, vact + d, d, ACT_F16, m->w1qk[l], d, lin_nv[l], nqk, d, eg, st, m);
      GemmEpi e2 = eg;
      e2.out0 = eg.out0 + nqk;
      if (rc == TVR_OK)
        rc = launch_gemm(EPI_BIAS, vact, d, fmt, m->w1[l].rows((size_t)nqk * d), d, lin_nv[l], D1 - nqk, d, e2, st,
                         m);
    } else {
      rc = launch_gemm(EPI_BIAS, vact, d, fmt, m->w1[l], d, lin_nv[l], D1, d, eg, st, m);
    }
    m->prof = prof;
    TVR_TRY(rc);
    const int npl = fmt == ACT_X2F16 ? 2 : 1, KP = m->lin_kp;
    const size_t per = (size_t)c.n_heads * D1 * KP;
    const uint16_t* wp = m->lin_planes + (size_t)(l - 1) * npl * per;
    // X2F16: every column tile in one launch; BF16: the Q / K column tiles [0, 2d) on the fp16 rows of the
    // planes (scale lin_scale[l]), the rest on bf16
    const int n_ct = (D1 + 255) / 256, ct_qk = fmt == ACT_BF16 ? lin_qk_cols(c) / 256 : 0;
    float acc_scale = fmt == ACT_X2F16 ? 1.0f / (m->lin_scale[l] * X2_ASCALE) : 1.0f;
    dim3 g;
    int ct_base = 0;
#define TVR_LIN(F, NK)                                                                                             \
  hipLaunchKernelGGL((lin_entry_kernel<F, NK>), g, dim3(LIN_THREADS), 0, st,                                       \
                     (const LinMB*)(base + o_lin_mbs) + lin_mb_off[l], lin_nmb[l], (const LinRow*)(base + o_lin_rows), \
                     wp, per, acc_scale, trace->z + (size_t)(l - 1) * tstride, d, c.d_head, lnstats, a.qkv, raw_h,     \
                     c.d_mlp, (const float*)(base + o_g), m->lin_c1 + (size_t)l * D1, w.b1, D1,                         \
                     reinterpret_cast<uint16_t*>(a.a2) + d, 2 * m->K2, m->K2, m->range_flag, ct_base)
#define TVR_LIN_K(F)                                                      \
  if (KP == 32) TVR_LIN(F, 1);                                            \
  else if (KP == 64) TVR_LIN(F, 2);                                       \
  else if (KP == 96) TVR_LIN(F, 3);                                       \
  else TVR_LIN(F, 4)
    if (fmt == ACT_X2F16) {
      g = dim3(lin_nmb[l] * n_ct);
      TVR_LIN_K(ACT_X2F16);
    } else {
      if (ct_qk > 0) {
        g = dim3(lin_nmb[l] * ct_qk);
        acc_scale = 1.0f / m->lin_scale[l];
        TVR_LIN_K(ACT_F16);
      }
      g = dim3(lin_nmb[l] * (n_ct - ct_qk));
      acc_scale = 1.0f;
      ct_base = ct_qk;
      TVR_LIN_K(ACT_BF16);
    }
#undef TVR_LIN_K
#undef TVR_LIN
    TVR_HIP(hipGetLastError());
    // algorithmic bytes: the entering rows' outputs written and their clean rows' y_c read (4 B per
    // column each), z slices, the layer's Wsc planes once, G written + read, the vectors' planes
    const double nr = lin_nrows[l];
    ps.done(TVR_HBM_LIN_ENTRY, nr * (8.0 * D1 + 4.0 * c.d_head) + 2.0 * npl * per +
                                   lin_nv[l] * (8.0 * D1 + 4.0 * d) + 2.0 * npl * (double)D1 * d);
    ProfSpan pa(m, st);
    TVR_TRY(launch_attention(m, a.qkv, cache, d_seqs, nc + cnt_le[l], maxT, a.a2, a.fmt, zf, st, false, Rc));
    pa.done(TVR_HBM_ATTENTION, attention_bytes(d, Rl, Rl, a.fmt, zf ? std::min(Rl, Rc) : 0));
    return run_block_out(m, l, Rl, a, st);
  };

  for (int l = 0; l < L; ++l) {
    const int Rl = Rc + rows_le[l];
    float* tqkv = trace->qkv + (size_t)l * 3 * tstride;
    if (fused) {  // the clean rows' hook_resid_pre / K,V cache go to the trace from the kernels writing them
      a.resid_mirror = trace->resid + l * tstride;
      a.qkv_mirror = tqkv;
      a.mirror_rows = Rc;
    }
    TVR_TRY(enter(l));
    if (Rl == 0) continue;
    const float* cache = fused ? a.qkv : tqkv;
    float* zf = fused ? trace->z + l * tstride : nullptr;  // the clean rows' hook_z (rows < Rc)
    if (use_lin[l]) {
      TVR_TRY(run_block_lin(l, Rl, cache, zf));
    } else if (l == L - 1 && Rc + cnt_le[l] < Rl) {  // (every row a last row, e.g. C2's: the plain block)
      TVR_TRY(run_block_last_rows(m, l, Rl, (const SeqDesc*)(base + o_seqs_last), nc + cnt_le[l], maxT, a, cache,
                                  (const int32_t*)(base + o_last_sorted), Rc + cnt_le[l], true, zf, st, false, Rc,
                                  nc));
    } else {
      TVR_TRY(run_block(m, l, Rl, d_seqs, nc + cnt_le[l], maxT, a, a.qkv, cache, zf, st, false, Rc,
                        single_rows ? nc : INT_MAX));
      TVR_TRY(run_block_out(m, l, Rl, a, st));
    }
  }
  a.resid_mirror = a.qkv_mirror = nullptr;
  a.mirror_rows = 0;
  if (fused) {
    TVR_HIP(hipMemcpyAsync(trace->resid + L * tstride, a.resid, rbytes, hipMemcpyDeviceToDevice, st));
    trace->pending = false;
  }
  TVR_TRY(enter(L));
  TVR_TRY(run_final(m, a.resid, (const int32_t*)(base + o_last), (const int32_t*)(base + o_tg), n_sites,
                    (float*)(base + o_xf), (float*)(base + o_lg), out_prob, out_topk, topk, out_logits, fmt, st));
  if (fused && (trace->p_prob || trace->p_topk))
    TVR_TRY(run_final(m, a.resid, (const int32_t*)(base + o_clast), (const int32_t*)(base + o_ctg), nc,
                      (float*)(base + o_xf), (float*)(base + o_lg), trace->p_prob, trace->p_topk, trace->p_k,
                      nullptr, fmt, st));
  return TVR_OK;
}

int tvr_gemm_plan(int32_t M, int32_t N, int32_t K, int32_t gemm_mode, int32_t flags, int32_t* out) {
  if (M <= 0 || N <= 0 || K <= 0 || !out || (gemm_mode != TVR_GEMM_X2F16 && gemm_mode != TVR_GEMM_BF16) ||
      (flags & ~(TVR_PLAN_GELU | TVR_PLAN_MODEL_SLICED | TVR_PLAN_EXACT16)))
    return fail(TVR_ERR_INVALID, "tvr_gemm_plan: bad argument");
  const int fmt = gemm_mode == TVR_GEMM_X2F16 ? ACT_X2F16 : ACT_BF16;
  if (K % (fmt == ACT_X2F16 ? 32 : 64) != 0) return fail(TVR_ERR_UNSUPPORTED, "tvr_gemm_plan: K not a k-tile multiple");
  // the same sliced rule as plan_pp_cached / launch_gemm
  const bool sliced = fmt == ACT_X2F16 && (K >= PP_SLICE_MIN_K || (flags & TVR_PLAN_MODEL_SLICED));
  const PpPlan p = plan_pp(M, N, K, fmt, (flags & TVR_PLAN_GELU) ? EPI_SPLIT_GELU_ACT : EPI_RESID, sliced,
                           fmt == ACT_X2F16 && (flags & TVR_PLAN_EXACT16));
  out[0] = p.ksplit;
  out[1] = p.tail_base;
  out[2] = p.tail_split;
  out[3] = p.sk_base;
  out[4] = p.sk_blocks;
  return TVR_OK;
}

int tvr_project_heads(tvr_model* m, const float* zsum, float* out, void* stream) {
  if (!m || !zsum || !out) return fail(TVR_ERR_INVALID, "tvr_project_heads: null argument");
  const tvr_config& c = m->cfg;
  hipLaunchKernelGGL(project_heads_kernel, dim3((c.d_model + 255) / 256, c.n_heads, c.n_layers),
                     dim3(256), 0, (hipStream_t)stream, zsum, m->d_w2s, m->K2, out, c.n_heads,
                     c.d_model, c.d_head);
  TVR_HIP(hipGetLastError());
  return TVR_OK;
}

int tvr_gemm_f32(const float* A, int32_t lda, const float* W, int32_t ldw, const float* bias, float* C,
                 int32_t ldc, int32_t M, int32_t N, int32_t K, void* stream) {
  if (!A || !W || !C || M < 0 || N < 0 || K <= 0) return fail(TVR_ERR_INVALID, "tvr_gemm_f32: bad argument");
  GemmEpi e{};
  e.bias = bias;
  e.out0 = C;
  e.ld0 = ldc;
  return launch_gemm(EPI_BIAS, A, lda, ACT_F32, MatW{W}, ldw, M, N, K, e, (hipStream_t)stream);
}

int tvr_split_planes(const float* w, uint16_t* out, size_t n, void* stream) {
  if (!w || !out) return fail(TVR_ERR_INVALID, "tvr_split_planes: null argument");
  if (n == 0) return TVR_OK;
  hipLaunchKernelGGL(split_planes_kernel, dim3(2048), dim3(256), 0, (hipStream_t)stream, w, out, n);
  TVR_HIP(hipGetLastError());
  return TVR_OK;
}

int tvr_gemm_x3bf16(const float* A, int32_t lda, const uint16_t* W, int32_t ldw, size_t wps,
                    const float* bias, float* C, int32_t ldc, int32_t M, int32_t N, int32_t K, void* stream) {
  if (!A || !W || !C || M < 0 || N < 0 || K <= 0 || wps < (size_t)ldw * (N > 0 ? N - 1 : 0) + K)
    return fail(TVR_ERR_INVALID, "tvr_gemm_x3bf16: bad argument");
  GemmEpi e{};
  e.bias = bias;
  e.out0 = C;
  e.ld0 = ldc;
  return launch_gemm(EPI_BIAS, A, lda, ACT_F32, MatW{nullptr, W, nullptr, wps, 1.0f}, ldw, M, N, K, e,
                     (hipStream_t)stream);
}

int tvr_weight_planes(int32_t fmt, const float* w, float scale, uint16_t* out, size_t n, void* stream) {
  if (!w || !out || (fmt != TVR_GEMM_X2F16 && fmt != TVR_GEMM_BF16))
    return fail(TVR_ERR_INVALID, "tvr_weight_planes: bad argument");
  if (n == 0) return TVR_OK;
  if (fmt == TVR_GEMM_X2F16)
    hipLaunchKernelGGL(split_planes_f16_kernel, dim3(2048), dim3(256), 0, (hipStream_t)stream, w, scale, out, n);
  else
    hipLaunchKernelGGL(bf16_plane_kernel, dim3(2048), dim3(256), 0, (hipStream_t)stream, w, out, n, 0);
  TVR_HIP(hipGetLastError());
  return TVR_OK;
}

int tvr_gemm_x2f16(const float* A, int32_t lda, const uint16_t* W, int32_t ldw, size_t wps, float w_scale,
                   const float* bias, float* C, int32_t ldc, int32_t M, int32_t N, int32_t K,
                   uint32_t* range_flag, void* stream) {
  if (!A || !W || !C || M < 0 || N < 0 || K <= 0 || !(w_scale > 0.0f) ||
      wps < (size_t)ldw * (N > 0 ? N - 1 : 0) + K)
    return fail(TVR_ERR_INVALID, "tvr_gemm_x2f16: bad argument");
  GemmEpi e{};
  e.bias = bias;
  e.out0 = C;
  e.ld0 = ldc;
  return launch_gemm(EPI_BIAS, A, lda, ACT_F32, MatW{nullptr, nullptr, W, wps, w_scale}, ldw, M, N, K, e,
                     (hipStream_t)stream, nullptr, range_flag);
}

int tvr_act_rows(int32_t fmt, const float* a, int32_t lda, uint16_t* out, int32_t rows, int32_t K,
                 uint32_t* range_flag, void* stream) {
  if (!a || !out || rows < 0 || K <= 0 || lda < K || (fmt != TVR_GEMM_X2F16 && fmt != TVR_GEMM_BF16))
    return fail(TVR_ERR_INVALID, "tvr_act_rows: bad argument");
  const size_t n = (size_t)rows * K;
  if (n == 0) return TVR_OK;
  const dim3 grid((unsigned)std::min<size_t>((n + 255) / 256, 8192)), block(256);
  if (fmt == TVR_GEMM_X2F16)
    hipLaunchKernelGGL(act_rows_kernel<ACT_X2F16>, grid, block, 0, (hipStream_t)stream, a, lda, out, rows, K, range_flag);
  else
    hipLaunchKernelGGL(act_rows_kernel<ACT_BF16>, grid, block, 0, (hipStream_t)stream, a, lda, out, rows, K, range_flag);
  TVR_HIP(hipGetLastError());
  return TVR_OK;
}

int tvr_gemm_planar(int32_t fmt, const uint16_t* A, int32_t lda, const uint16_t* W, int32_t ldw, size_t wps,
                    float w_scale, const float* bias, float* C, int32_t ldc, int32_t M, int32_t N, int32_t K,
                    void* stream) {
  if (!A || !W || !C || M < 0 || N < 0 || K <= 0 || lda < K || !(w_scale > 0.0f) ||
      (fmt != TVR_GEMM_X2F16 && fmt != TVR_GEMM_BF16) || wps < (size_t)ldw * (N > 0 ? N - 1 : 0) + K)
    return fail(TVR_ERR_INVALID, "tvr_gemm_planar: bad argument");
  GemmEpi e{};
  e.bias = bias;
  e.out0 = C;
  e.ld0 = ldc;
  return launch_gemm(EPI_BIAS, A, lda, fmt == TVR_GEMM_X2F16 ? ACT_X2F16 : ACT_BF16,
                     MatW{nullptr, nullptr, W, wps, w_scale}, ldw, M, N, K, e, (hipStream_t)stream);
}

int tvr_lnpre_f32(const float* x, int32_t ldx, float* y, int32_t ldy, int32_t rows, int32_t d, float eps,
                  void* stream) {
  if (!x || !y || rows < 0 || d <= 0) return fail(TVR_ERR_INVALID, "tvr_lnpre_f32: bad argument");
  return launch_lnpre(x, ldx, nullptr, y, ldy, rows, d, eps, ACT_F32, (hipStream_t)stream);
}

}  // extern "C"

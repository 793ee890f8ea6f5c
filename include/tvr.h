/*
 * tvr.h — C ABI of the MI355X-native task-vector / function-vector engine.
 *
 * The reference (IMMachinations/Task-Vector-Replication) drives every patched
 * forward through TransformerLens from Python loops:
 *   - extraction   scratch2.py:81-100   (run_with_cache + hook_result[0,-1])
 *   - layer sweeps scratch2.py:107-150  (run_with_hooks, hook_attn_out[0,-1] += v)
 *   - CIE sweep    scratch2.py:171-197  (run_with_hooks, hook_result[0,:,h] = mean)
 *   - FV eval      scratch2.py:292-314  (run_with_hooks + top-k)
 *   - resid patch  scratch.py:106-147   (cache surgery + forward(start_at_layer=L))
 * There is no native FFI in the reference: its Python façade binds these
 * entry points through ctypes.  Every entry point below
 * replaces one of those loops with ONE batched launch sequence whose batch
 * dimension enumerates patch sites.
 *
 * Conventions
 *   - Host arrays: token ids, sequence lengths, targets and site records.
 *   - Device arrays: weights, vectors and all outputs; owned by the caller
 *     (PyTorch) and preallocated.  Traces and the activation workspace are
 *     owned by the engine (allocated outside timed regions, reused).
 *   - `stream` is a hipStream_t passed as void*; everything is enqueued on it
 *     and nothing synchronises the host except tvr_*_create / destroy.
 *   - Every function returns TVR_OK (0) or a negative error code; no C++
 *     exception crosses the ABI.  tvr_last_error() explains the last failure
 *     on the calling thread.
 *   - Numerics: LayerNorm, attention, the residual stream, the injections and
 *     the softmax are fp32 (the reference's TransformerLens default dtype).
 *     The GEMMs run on the matrix-core path chosen by tvr_model_set_gemm:
 *     TVR_GEMM_F32 at tvr_model_create; the Python façade selects
 *     TVR_GEMM_X2F16, an fp32-accurate emulation (each fp32 operand as two
 *     fp16 planes, three fp16 MFMA products, fp32 accumulation), by default.
 */
#ifndef TVR_H_
#define TVR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TVR_ABI_VERSION 11

enum tvr_status {
  TVR_OK = 0,
  TVR_ERR_INVALID = -1,     /* bad argument / shape (reference: ValueError) */
  TVR_ERR_HIP = -2,         /* HIP runtime failure */
  TVR_ERR_NOMEM = -3,       /* device allocation failed */
  TVR_ERR_UNSUPPORTED = -4, /* shape outside what the kernels handle */
  TVR_ERR_RANGE = -5,       /* a GEMM input exceeded the TVR_GEMM_X2F16 range */
  TVR_ERR_INTERNAL = -6     /* an engine invariant failed (a bug: report it) */
};

/* Patch-site kinds: the declarative replacement for TransformerLens hooks. */
enum tvr_site_kind {
  /* No patch: re-evaluate the clean last-position distribution. */
  TVR_SITE_NONE = 0,
  /* blocks.{layer}.attn.hook_result[0,:,head,:] = vectors[vec] at every
   * position (scratch2.py:167-169, 187-189). */
  TVR_SITE_REPLACE_HEAD_ALLPOS = 1,
  /* blocks.{layer}.hook_attn_out[0,-1,:] += vectors[vec]
   * (scratch2.py:107-109). */
  TVR_SITE_ADD_ATTN_OUT_LASTPOS = 2,
  /* blocks.{layer}.hook_resid_pre of sequence `seq` with row `pos` replaced by
   * the same hook's row `src_pos` of sequence `src_seq`, then
   * forward(start_at_layer=layer) (scratch.py:140-143, 201-209). */
  TVR_SITE_SET_RESID_PRE_POS = 3
};

typedef struct tvr_config {
  int32_t n_layers;
  int32_t d_model;
  int32_t n_heads;
  int32_t d_head;
  int32_t d_mlp;
  int32_t d_vocab;
  int32_t rotary_dim;
  int32_t n_ctx;       /* rotary table length */
  float ln_eps;
  float rotary_base;
} tvr_config;

/* Per-layer weights after TransformerLens processing (fold_ln,
 * center_writing_weights, fold_value_biases), in the engine's fused layout.
 *   w1 [3*d_model + d_mlp][d_model]  rows: Q(head,d_head) | K | V | MLP-in
 *   b1 [3*d_model + d_mlp]           (V part is zero after fold_value_biases)
 *   w2 [d_model][d_model + d_mlp]    cols: O(head,d_head) | MLP-out
 *   b2 [d_model]                     b_O (with folded value bias) + b_out   */
typedef struct tvr_layer_weights {
  const float* w1;
  const float* b1;
  const float* w2;
  const float* b2;
} tvr_layer_weights;

/* One patched forward = one (prompt, patch site) pair = one unit of the
 * metric "patched-forward prompts/sec". */
typedef struct tvr_site {
  int32_t seq;      /* clean sequence (prompt) index in the trace */
  int32_t kind;     /* enum tvr_site_kind */
  int32_t layer;    /* hook layer */
  int32_t head;     /* REPLACE_HEAD_ALLPOS */
  int32_t pos;      /* SET_RESID_PRE_POS: patched position in `seq` (>= 0) */
  int32_t src_seq;  /* SET_RESID_PRE_POS: sequence supplying the row */
  int32_t src_pos;  /* SET_RESID_PRE_POS: position supplying the row */
  int32_t vec;      /* row of `vectors` (REPLACE / ADD) */
  int32_t target;   /* token whose probability is reported, -1: none */
} tvr_site;

typedef struct tvr_model tvr_model;
typedef struct tvr_trace tvr_trace;

const char* tvr_version(void);
int32_t tvr_abi_version(void);
const char* tvr_last_error(void);

/* Replaces HookedTransformer.from_pretrained(...) (scratch.py:26,
 * scratch2.py:26): binds processed device weights (caller keeps them alive). */
int tvr_model_create(const tvr_config* cfg, const float* w_embed /*[V][d]*/,
                     const tvr_layer_weights* layers /*[n_layers] host*/,
                     const float* w_unembed_t /*[V][d]*/,
                     const float* b_unembed /*[V]*/, tvr_model** out);
int tvr_model_destroy(tvr_model* model);

/* Matrix-core path of the model's GEMMs (every other op is fp32 regardless).
 *   TVR_GEMM_F32     v_mfma_f32_32x32x2_f32 on the fp32 weights
 *   TVR_GEMM_X3BF16  fp32-accurate 3-plane bf16 split on v_mfma_f32_32x32x16_bf16:
 *                    each operand x = x0+x1+x2 (bf16 planes, 24 significand bits),
 *                    six cross products accumulated in fp32; weight planes 6 B/param
 *   TVR_GEMM_X2F16   fp32-accurate 2-plane fp16 split on v_mfma_f32_16x16x32_f16
 *                    (the fp16 form of 3xTF32): x = x0+x1 (2 x 11 significand
 *                    bits, power-of-two scaled into fp16 range), three cross
 *                    products accumulated in fp32; weight planes 4 B/param.
 *                    GEMM inputs must satisfy |a| < 4095 (LayerNorm outputs,
 *                    attention mixes and GELU outputs of any Pythia do); a
 *                    launch that sees a larger one is reported by
 *                    tvr_model_range_status.
 *   TVR_GEMM_BF16    bf16 weights and GEMM inputs on v_mfma_f32_16x16x32_bf16,
 *                    fp32 accumulation (the north star's bf16 configuration,
 *                    tolerance 2e-2; NOT fp32-accurate); weights 2 B/param.
 * Measured errors of both split modes against fp64 are at or below the fp32
 * MFMA GEMM's.  TransformerLens runs its matmuls in fp32
 * (scratch2.py:26 loads the default dtype); F32, X3BF16 and X2F16 meet that.
 * Everything outside the GEMMs (LayerNorm, attention, residual stream,
 * softmax) is fp32 in every mode.  The planes are built on the device once.
 * Synchronises `stream`. */
enum tvr_gemm_mode { TVR_GEMM_F32 = 0, TVR_GEMM_X3BF16 = 1, TVR_GEMM_X2F16 = 2, TVR_GEMM_BF16 = 3 };
int tvr_model_set_gemm(tvr_model* model, int32_t mode, void* stream);
int32_t tvr_model_get_gemm(const tvr_model* model);
/* TVR_OK, or TVR_ERR_RANGE if an X2F16 GEMM enqueued since the last call saw
 * an input outside its range (its results are then not fp32-accurate and must
 * be discarded).  Synchronises `stream`; clears the flag. */
int tvr_model_range_status(tvr_model* model, void* stream);

/* Exact-fp16 weights (the checkpoint dtype of every Pythia), for TVR_GEMM_X2F16.
 * Per layer, caller-owned device arrays, kept alive by the caller:
 *   w1  fp16 [3d + d_mlp][d]  the checkpoint's Q | K | V rows (engine order, as
 *                             tvr_layer_weights.w1) and MLP-in rows BEFORE fold_ln
 *   w2  fp16 [d][d + d_mlp]   W_O | W_out BEFORE center_writing_weights
 *   g1, g2 fp32 [d]           LN1 / LN2 gamma (ln_1.w, ln_2.w)
 * They must be the raw tensors the model's processed w1 / w2 were made from
 * (tvr_layer_weights: fold_ln, centring and fold_value_biases applied to them).
 * In X2F16 mode the QKV + MLP-in GEMM then reads LNPre(x) * gamma1 (Q, K, V
 * columns) and * gamma2 (MLP-in columns) against w1 — fold_ln's centring of the
 * read-in weights is a no-op on a centred LNPre row — and the O + MLP-out GEMM
 * reads w2 uncentred: the residual stream then carries one constant per row,
 * which every LayerNorm removes and tvr_trace_read's hook_resid_pre export
 * subtracts.  Weights exact in fp16 need 2 matrix products per 32-deep slice
 * instead of 3.  Results equal the processed-weight path's to fp32 rounding.
 * Pass layers == NULL to detach.  Other modes ignore the binding. */
typedef struct {
  const uint16_t* w1;
  const uint16_t* w2;
  const float* g1;
  const float* g2;
} tvr_exact16_layer;
int tvr_model_set_exact16(tvr_model* model, const tvr_exact16_layer* layers /*[n_layers] host, or NULL*/);
/* The unembed's part of the exact-fp16 binding (X2F16 mode, with the layers
 * bound): wu fp16 [d_vocab][d_model] = the checkpoint's embed_out.weight
 * BEFORE fold_ln / center_unembed, gf fp32 [d_model] = the final LN's gamma.
 * The patch sweeps' fused-statistics unembed then reads LNPre(x) * gf against
 * wu (2 products); the omitted centring over the vocabulary is one constant per
 * row of logits, which softmax probabilities and top-k do not see.  Paths that
 * return logits keep the processed W_U.  NULL, NULL detaches. */
int tvr_model_set_exact16_unembed(tvr_model* model, const uint16_t* wu, const float* gf);

/* Clean-run trace: every layer's hook_resid_pre, attn.hook_z and the K/V
 * inputs, the state run_with_cache keeps (scratch2.py:96, scratch.py:132,137). */
int tvr_trace_create(tvr_model* model, int32_t max_seqs, int32_t max_tokens,
                     tvr_trace** out);
/* Destroying a trace with a deferred clean forward pending runs it first (on
 * the null stream) so the caller's out_prob / out_topk are written. */
int tvr_trace_destroy(tvr_trace* trace);
/* Run a pending deferred clean forward now (tvr_forward_clean_deferred) on
 * `stream`; no-op otherwise. */
int tvr_trace_flush(tvr_trace* trace, void* stream);
/* Copy a traced hook into a caller device buffer [n_tokens][d] (async on
 * `stream`): what = TVR_TRACE_RESID_PRE gives blocks.{layer}.hook_resid_pre
 * (layer == n_layers: the final residual), TVR_TRACE_Z blocks.{layer}.attn.hook_z.
 * dst needs only float alignment (4 B). */
enum tvr_trace_hook { TVR_TRACE_RESID_PRE = 0, TVR_TRACE_Z = 1 };
int tvr_trace_read(const tvr_trace* trace, int32_t what, int32_t layer, float* dst,
                   void* stream);
int32_t tvr_trace_num_tokens(const tvr_trace* trace);

/* Batched clean forward of n_seq prompts (ragged lengths, packed tokens).
 * Replaces the per-prompt model.forward / run_with_cache calls
 * (scratch2.py:96,143,183,297; scratch.py:127,132,137).
 *   trace        may be NULL (no snapshots kept)
 *   targets      host [n_seq] token ids or NULL; out_prob [n_seq] gets
 *                softmax(logits[-1])[target]
 *   out_topk     device [n_seq][topk] int32 (descending, lowest id on ties)
 *   out_logits   device [n_seq][V] last-position logits, or NULL
 *   capture_zsum device [n_layers][d] fp32: += hook_z at each prompt's last
 *                position (the reduction of scratch2.py:97-98), or NULL   */
int tvr_forward_clean(tvr_model* model, tvr_trace* trace, const int32_t* tokens,
                      const int32_t* seq_lens, int32_t n_seq,
                      const int32_t* targets, float* out_prob,
                      int32_t* out_topk, int32_t topk, float* out_logits,
                      float* capture_zsum, void* stream);

/* tvr_forward_clean (no logits, no capture) deferred into the next
 * tvr_patch_sweep on `trace`: that sweep runs the clean rows in its own
 * launches (one staircase instead of a clean forward + a staircase), fills the
 * trace exactly as tvr_forward_clean would, and writes out_prob / out_topk
 * (stream-ordered: read them after that sweep).  Any other use of the trace
 * first (tvr_trace_read, tvr_forward_clean, another deferral) runs the clean
 * forward on its own.  Same checks and errors as tvr_forward_clean; no GPU
 * work is enqueued by this call.  The reference's pattern it serves: a clean
 * forward and the patched forwards of the same prompts (scratch2.py:143-148,
 * 183-192). */
int tvr_forward_clean_deferred(tvr_model* model, tvr_trace* trace, const int32_t* tokens,
                               const int32_t* seq_lens, int32_t n_seq,
                               const int32_t* targets, float* out_prob,
                               int32_t* out_topk, int32_t topk, void* stream);

/* Logits of EVERY position, out_logits device [sum(seq_lens)][V]: the
 * TransformerLens forward's [1, T, V] (scratch2.py:143,183,297;
 * scratch.py:127,143).  Exactly one input:
 *   tokens   host ids (packed, seq_lens per sequence), start_layer 0, or
 *   resid_in device [sum(seq_lens)][d] = blocks.{start_layer}.hook_resid_pre,
 *            continued from that block (forward(resid, start_at_layer=L),
 *            scratch.py:143,206,209).
 * Sequences up to n_ctx tokens (beyond 128 the attention runs its chunked
 * online-softmax form). */
int tvr_forward_logits(tvr_model* model, const int32_t* tokens, const float* resid_in,
                       int32_t start_layer, const int32_t* seq_lens, int32_t n_seq,
                       float* out_logits, void* stream);

/* Batched patch sweep over sites against a clean trace (the staircase: a site
 * at layer l reuses the clean run's layers <= l and K/V prefix).  Replaces the
 * per-site run_with_hooks loops (scratch2.py:122-125,145-148,185-194,301,311;
 * scratch.py:140-145).
 *   vectors  device [n_vectors][d]
 *   out_prob device [n_sites], out_topk device [n_sites][topk],
 *   out_logits device [n_sites][V] or NULL                                  */
int tvr_patch_sweep(tvr_model* model, tvr_trace* trace,
                    const tvr_site* sites, int32_t n_sites,
                    const float* vectors, int32_t n_vectors, float* out_prob,
                    int32_t* out_topk, int32_t topk, float* out_logits,
                    void* stream);

/* out[l][h][:] = zsum[l][h*d_head:(h+1)*d_head] @ W_O[l,h]: turns the z-form
 * capture into the hook_result form of scratch2.py:98 (sum over prompts). */
int tvr_project_heads(tvr_model* model, const float* zsum /*[L][d]*/,
                      float* out /*[L][H][d]*/, void* stream);

/* Primitive kernels, exported for unit tests and tools. */
/* C[M][N] = A[M][K] (row stride lda) @ W[N][K]^T (row stride ldw) + bias */
int tvr_gemm_f32(const float* A, int32_t lda, const float* W, int32_t ldw,
                 const float* bias, float* C, int32_t ldc, int32_t M,
                 int32_t N, int32_t K, void* stream);
/* Split W [n] fp32 into 3 bf16 planes out [3][n] (uint16 storage). */
int tvr_split_planes(const float* w, uint16_t* out, size_t n, void* stream);
/* tvr_gemm_f32 on the 3-plane operand: W planes [3][.][ldw] with plane
 * stride wps elements (as tvr_split_planes writes them, wps = n). */
int tvr_gemm_x3bf16(const float* A, int32_t lda, const uint16_t* W, int32_t ldw,
                    size_t wps, const float* bias, float* C, int32_t ldc,
                    int32_t M, int32_t N, int32_t K, void* stream);
/* Weight planes of a planar mode (fmt = TVR_GEMM_X2F16 or TVR_GEMM_BF16):
 * X2F16 two fp16 planes out [2][n] of w * scale (scale a power of two; the
 * engine uses 2^(15 - ceil log2 max|W|)), BF16 one bf16 plane out [n]. */
int tvr_weight_planes(int32_t fmt, const float* w, float scale, uint16_t* out, size_t n,
                      void* stream);
/* tvr_gemm_f32 with the split happening inside the GEMM: A fp32, W planes
 * [2][.][ldw] (plane stride wps) from tvr_weight_planes(TVR_GEMM_X2F16, ..,
 * w_scale, ..).  *range_flag (device, may be NULL) is or-ed with 1 if |A|
 * reaches the split's range limit. */
int tvr_gemm_x2f16(const float* A, int32_t lda, const uint16_t* W, int32_t ldw,
                   size_t wps, float w_scale, const float* bias, float* C,
                   int32_t ldc, int32_t M, int32_t N, int32_t K,
                   uint32_t* range_flag, void* stream);
/* The activation format the engine's producers write for every GEMM input in
 * a planar mode: logical [rows][K] -> halves [rows][2][K]; X2F16: plane 0 =
 * fp16(16 a), plane 1 = fp16(16 a - plane 0), *range_flag (may be NULL) |= 1
 * if |a| >= 4095; BF16: plane 0 = bf16(a). */
int tvr_act_rows(int32_t fmt, const float* a, int32_t lda, uint16_t* out, int32_t rows,
                 int32_t K, uint32_t* range_flag, void* stream);
/* The engine's planar GEMM: A in the activation format above (lda logical
 * elements per row, >= K), W planes from tvr_weight_planes (w_scale: the
 * X2F16 scale, 1 for BF16). */
int tvr_gemm_planar(int32_t fmt, const uint16_t* A, int32_t lda, const uint16_t* W,
                    int32_t ldw, size_t wps, float w_scale, const float* bias,
                    float* C, int32_t ldc, int32_t M, int32_t N, int32_t K,
                    void* stream);
/* TransformerLens LayerNormPre over rows: (x - mean) / sqrt(var + eps) */
int tvr_lnpre_f32(const float* x, int32_t ldx, float* y, int32_t ldy,
                  int32_t rows, int32_t d, float eps, void* stream);

/* Kernel timing (HIP events recorded on the launch stream around every GEMM
 * launch while enabled).  tvr_profile_read synchronises the recorded events
 * and returns totals since the last enable; used by bench.py for the
 * roofline's achieved TFLOP/s of the dominant kernel. */
typedef struct tvr_kernel_stats {
  /* index = GEMM epilogue: 0 unembed (bias), 1 QKV+MLP-in (split + GELU),
   * 2 O+MLP-out (bias + parallel residual) */
  int64_t gemm_launches[3];
  double gemm_flops[3];   /* algorithmic 2*M*N*K summed over launches */
  double gemm_ms[3];      /* summed launch durations */
  double gemm_bytes[3];   /* minimal operand bytes (A + W + C) summed */
} tvr_kernel_stats;
int tvr_profile_enable(tvr_model* model, int32_t on);
int tvr_profile_read(tvr_model* model, tvr_kernel_stats* out);

/* The HBM-bound kernels, timed the same way (HIP events around each launch
 * while profiling is enabled) with their algorithmic bytes: achieved GB/s =
 * bytes / ms.  Index = enum tvr_hbm_kind. */
enum tvr_hbm_kind {
  TVR_HBM_ENTRY = 0,      /* patch injection at the entry layer (REPLACE_HEAD / ADD / SET_RESID):
                           * clean rows in, patched rows out, z rows + W_O slice per head */
  TVR_HBM_CAPTURE = 1,    /* extraction: sum of hook_z at every prompt's last row -> [d] per layer */
  TVR_HBM_LNPRE = 2,      /* LayerNormPre rows -> GEMM input format */
  TVR_HBM_ATTENTION = 3,  /* attention: fp32 Q/K/V rows in, z out (activation format [+ fp32 hook_z]) */
  TVR_HBM_ROW_STATS = 4,  /* softmax target probability / top-k over one logit row per site */
  TVR_HBM_LIN_ENTRY = 5,  /* linearised entry layer of REPLACE_HEAD sites (the vectors' W1 product G and
                           * the K = d_head entry-row GEMM with its combine epilogue): entering rows' outputs
                           * written + their clean rows' outputs read, z slices, W1 W_O planes once */
  TVR_HBM_KINDS = 6
};
typedef struct tvr_hbm_stats {
  int64_t launches[6];
  double ms[6];     /* summed launch durations */
  double bytes[6];  /* algorithmic bytes summed */
} tvr_hbm_stats;
int tvr_profile_read_hbm(tvr_model* model, tvr_hbm_stats* out);

/* The launch plan the engine uses for one planar GEMM of M x N x K
 * (gemm_pingpong_kernel, 256 x 256 tiles; engine.hip plan_pp): out[0] k-split
 * of the whole launch, out[1] first tile of a split tail (0: none), out[2] the
 * tail's split, out[3] first stream-K tile (-1: none), out[4] stream-K blocks.
 * gemm_mode: TVR_GEMM_X2F16 or TVR_GEMM_BF16; flags bit 0 (TVR_PLAN_GELU):
 * the QKV + MLP-in launch (GELU epilogue); bit 1 (TVR_PLAN_MODEL_SLICED): the
 * launch belongs to a model whose O + MLP-out K reaches the sliced-accumulation
 * threshold (6.9B, 12B: every x2f16 GEMM of such a model runs sliced, as does
 * any launch with K >= that threshold); bit 2 (TVR_PLAN_EXACT16): one exact
 * fp16 weight plane (tvr_model_set_exact16: 2 products, cheaper k-tiles).
 * Host-only, no device call (diagnostics, CPU tests).  (ABI 10; flag bits 1
 * and 2 from round 5) */
enum { TVR_PLAN_GELU = 1, TVR_PLAN_MODEL_SLICED = 2, TVR_PLAN_EXACT16 = 4 };
int tvr_gemm_plan(int32_t M, int32_t N, int32_t K, int32_t gemm_mode, int32_t flags, int32_t* out);

/* Bytes of engine workspace currently held by the model (diagnostics);
 * the weight planes of the split / bf16 modes are not included (X3BF16 6 B,
 * X2F16 4 B, BF16 2 B per GEMM weight). */
size_t tvr_workspace_bytes(const tvr_model* model);

#ifdef __cplusplus
}
#endif

#endif /* TVR_H_ */

// torch_ops.cpp — the engine's entry points as torch.library operators
// (namespace ``tvr``), a thin layer over the C ABI of include/tvr.h
// (libtvr.so).  SURVEY.md §8(b): the façade calls ``torch.ops.tvr.*`` so the
// engine composes with torch's streams, allocator and graphs instead of
// taking raw pointers from Python.
//
//   tvr::forward_clean   tvr_forward_clean / _deferred   (scratch2.py:96,143,183)
//   tvr::patch_sweep     tvr_patch_sweep                 (scratch2.py:122-125,185-194)
//   tvr::project_heads   tvr_project_heads               (scratch2.py:97-98)
//   tvr::forward_logits  tvr_forward_logits              (scratch.py:143,206,209)
//
// Every op enqueues on torch's CURRENT stream of the output device and
// allocates its outputs through torch's caching allocator; host arrays
// (token ids, lengths, targets, site records) are CPU int32 tensors, the
// handles the int64 values of the tvr_model* / tvr_trace* the façade created.
// Status codes become exceptions with the engine's message: TVR_ERR_INVALID
// raises ValueError (the reference's shape errors, scratch2.py:172-175),
// everything else RuntimeError.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <string>
#include <tuple>

#include "tvr.h"

namespace {

void check(int rc, const char* what) {
  if (rc == TVR_OK) return;
  const std::string msg = std::string(what) + ": " + tvr_last_error();
  TORCH_CHECK_VALUE(rc != TVR_ERR_INVALID, msg);
  TORCH_CHECK(false, msg, " (status ", rc, ")");
}

tvr_model* as_model(int64_t h) {
  TORCH_CHECK_VALUE(h != 0, "tvr: null model handle");
  return reinterpret_cast<tvr_model*>(static_cast<intptr_t>(h));
}

// torch's ROCm build presents HIP devices as DeviceType::CUDA: its guard and
// current-stream accessors are the "masquerading" ones
using DeviceGuard = c10::hip::HIPGuardMasqueradingAsCUDA;

void* cur_stream(const c10::Device& dev) { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(dev.index()).stream(); }

void need_gpu(const c10::Device& dev) {
  TORCH_CHECK(dev.is_cuda(), "the HIP engine needs a GPU device (no CPU fallback): got device ", dev);
}

const int32_t* host_i32(const at::Tensor& t, const char* name) {
  TORCH_CHECK_VALUE(t.device().is_cpu() && t.scalar_type() == at::kInt && t.is_contiguous(), "tvr: ", name,
                    " must be a contiguous CPU int32 tensor");
  return t.data_ptr<int32_t>();
}

const int32_t* opt_host_i32(const std::optional<at::Tensor>& t, const char* name) {
  return t.has_value() ? host_i32(*t, name) : nullptr;
}

const float* in_f32(const std::optional<at::Tensor>& t, const c10::Device& dev, const char* name) {
  if (!t.has_value()) return nullptr;
  TORCH_CHECK_VALUE(t->device() == dev && t->scalar_type() == at::kFloat && t->is_contiguous(), "tvr: ", name,
                    " must be a contiguous fp32 tensor on ", dev);
  return t->data_ptr<float>();
}

at::TensorOptions f32(const c10::Device& dev) { return at::TensorOptions().dtype(at::kFloat).device(dev); }

// (prob [n], topk [n, k] int32, logits [n, V], zsum [L, d]); outputs not
// requested are empty tensors.  defer: tvr_forward_clean_deferred (the next
// patch_sweep on the trace writes prob / topk).
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> forward_clean(
    int64_t model, int64_t trace, const at::Tensor& tokens, const at::Tensor& seq_lens,
    const std::optional<at::Tensor>& targets, int64_t topk, bool want_logits, bool capture, bool defer,
    int64_t n_layers, int64_t d_model, int64_t d_vocab, c10::Device device) {
  const int64_t n = seq_lens.numel();
  TORCH_CHECK_VALUE(n > 0, "tvr: no prompts");
  need_gpu(device);
  DeviceGuard guard(device);
  const int32_t* tg = opt_host_i32(targets, "targets");
  TORCH_CHECK_VALUE(!targets.has_value() || targets->numel() == n, "targets must have one entry per prompt");
  auto prob = tg ? at::empty({n}, f32(device)) : at::empty({0}, f32(device));
  auto top = at::empty({topk ? n : 0, topk}, at::TensorOptions().dtype(at::kInt).device(device));
  auto logits = want_logits ? at::empty({n, d_vocab}, f32(device)) : at::empty({0}, f32(device));
  auto zsum = capture ? at::zeros({n_layers, d_model}, f32(device)) : at::empty({0}, f32(device));
  auto* tr = reinterpret_cast<tvr_trace*>(static_cast<intptr_t>(trace));
  void* st = cur_stream(device);
  if (defer) {
    TORCH_CHECK_VALUE(tr && !want_logits && !capture, "defer needs a trace and no logits / capture");
    check(tvr_forward_clean_deferred(as_model(model), tr, host_i32(tokens, "tokens"), host_i32(seq_lens, "seq_lens"),
                                     (int32_t)n, tg, tg ? prob.data_ptr<float>() : nullptr,
                                     topk ? top.data_ptr<int32_t>() : nullptr, (int32_t)topk, st),
          "tvr_forward_clean_deferred");
  } else {
    check(tvr_forward_clean(as_model(model), tr, host_i32(tokens, "tokens"), host_i32(seq_lens, "seq_lens"),
                            (int32_t)n, tg, tg ? prob.data_ptr<float>() : nullptr,
                            topk ? top.data_ptr<int32_t>() : nullptr, (int32_t)topk,
                            want_logits ? logits.data_ptr<float>() : nullptr,
                            capture ? zsum.data_ptr<float>() : nullptr, st),
          "tvr_forward_clean");
  }
  return {prob, top, logits, zsum};
}

// sites: CPU int32 [n_sites, 9] in tvr_site field order
std::tuple<at::Tensor, at::Tensor, at::Tensor> patch_sweep(int64_t model, int64_t trace, const at::Tensor& sites,
                                                           const std::optional<at::Tensor>& vectors, int64_t topk,
                                                           bool want_prob, bool want_logits, int64_t d_vocab,
                                                           c10::Device device) {
  static_assert(sizeof(tvr_site) == 9 * sizeof(int32_t), "tvr_site is 9 int32 fields");
  TORCH_CHECK_VALUE(sites.dim() == 2 && sites.size(1) == 9, "tvr: sites must be [n_sites, 9] int32");
  const int64_t n = sites.size(0);
  TORCH_CHECK_VALUE(n > 0, "tvr: no patch sites");
  TORCH_CHECK_VALUE(trace != 0, "tvr: patch_sweep needs a trace");
  need_gpu(device);
  DeviceGuard guard(device);
  const float* vec = in_f32(vectors, device, "vectors");
  const int32_t nvec = vectors.has_value() ? (int32_t)(vectors->numel() / std::max<int64_t>(vectors->size(-1), 1)) : 0;
  auto prob = want_prob ? at::empty({n}, f32(device)) : at::empty({0}, f32(device));
  auto top = at::empty({topk ? n : 0, topk}, at::TensorOptions().dtype(at::kInt).device(device));
  auto logits = want_logits ? at::empty({n, d_vocab}, f32(device)) : at::empty({0}, f32(device));
  check(tvr_patch_sweep(as_model(model), reinterpret_cast<tvr_trace*>(static_cast<intptr_t>(trace)),
                        reinterpret_cast<const tvr_site*>(host_i32(sites, "sites")), (int32_t)n, vec, nvec,
                        want_prob ? prob.data_ptr<float>() : nullptr, topk ? top.data_ptr<int32_t>() : nullptr,
                        (int32_t)topk, want_logits ? logits.data_ptr<float>() : nullptr, cur_stream(device)),
        "tvr_patch_sweep");
  return {prob, top, logits};
}

// zsum [L, d] -> [L, H, d]
at::Tensor project_heads(int64_t model, const at::Tensor& zsum, int64_t n_heads) {
  TORCH_CHECK_VALUE(zsum.dim() == 2, "tvr: zsum must be [n_layers, d_model]");
  const c10::Device dev = zsum.device();
  need_gpu(dev);
  DeviceGuard guard(dev);
  const float* z = in_f32(zsum, dev, "zsum");
  auto out = at::empty({zsum.size(0), n_heads, zsum.size(1)}, f32(dev));
  check(tvr_project_heads(as_model(model), z, out.data_ptr<float>(), cur_stream(dev)), "tvr_project_heads");
  return out;
}

// logits of every position [sum(seq_lens), V]; exactly one of tokens (host ids)
// and resid (device [sum(seq_lens), d] entering block start_layer)
at::Tensor forward_logits(int64_t model, const std::optional<at::Tensor>& tokens,
                          const std::optional<at::Tensor>& resid, int64_t start_layer, const at::Tensor& seq_lens,
                          int64_t d_vocab, c10::Device device) {
  need_gpu(device);
  DeviceGuard guard(device);
  const int32_t* lens = host_i32(seq_lens, "seq_lens");
  int64_t rows = 0;
  for (int64_t i = 0; i < seq_lens.numel(); ++i) rows += lens[i];
  auto out = at::empty({rows, d_vocab}, f32(device));
  check(tvr_forward_logits(as_model(model), opt_host_i32(tokens, "tokens"), in_f32(resid, device, "resid"),
                           (int32_t)start_layer, lens, (int32_t)seq_lens.numel(), out.data_ptr<float>(),
                           cur_stream(device)),
        "tvr_forward_logits");
  return out;
}

}  // namespace

TORCH_LIBRARY(tvr, m) {
  m.def("forward_clean(int model, int trace, Tensor tokens, Tensor seq_lens, Tensor? targets, int topk, "
        "bool want_logits, bool capture, bool defer, int n_layers, int d_model, int d_vocab, Device device) "
        "-> (Tensor, Tensor, Tensor, Tensor)");
  m.def("patch_sweep(int model, int trace, Tensor sites, Tensor? vectors, int topk, bool want_prob, "
        "bool want_logits, int d_vocab, Device device) -> (Tensor, Tensor, Tensor)");
  m.def("project_heads(int model, Tensor zsum, int n_heads) -> Tensor");
  m.def("forward_logits(int model, Tensor? tokens, Tensor? resid, int start_layer, Tensor seq_lens, int d_vocab, "
        "Device device) -> Tensor");
}

// Mixed host / device tensor arguments: one implementation for every backend key.
TORCH_LIBRARY_IMPL(tvr, CompositeExplicitAutograd, m) {
  m.impl("forward_clean", &forward_clean);
  m.impl("patch_sweep", &patch_sweep);
  m.impl("project_heads", &project_heads);
  m.impl("forward_logits", &forward_logits);
}

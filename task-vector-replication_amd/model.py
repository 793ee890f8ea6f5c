"""``Model``: the handle the façade passes where the reference passes a
TransformerLens ``HookedTransformer`` (scratch2.py:26 and every ``model=``
argument).  It owns the processed device weights, exposes ``cfg`` and the
token helpers, and drives the engine's batched entry points:

* ``forward_clean``  — many prompts in one launch sequence (replaces the
  per-prompt ``forward`` / ``run_with_cache`` calls);
* ``patch_sweep``    — many (prompt, patch site) pairs in one staircase
  launch sequence (replaces the per-site ``run_with_hooks`` loops);
* ``project_heads``  — z-form capture → ``hook_result`` form.

The compute entry points run as torch.library operators (``torch.ops.tvr.*``,
csrc/torch_ops.cpp over the C ABI) on torch's current stream, with outputs
from torch's allocator; nothing here has a CPU fallback (the engine refuses to
run without a GPU).

The x2f16 range check (include/tvr.h ``tvr_model_range_status``) reads a
device-side sticky flag and synchronises: a direct call checks after itself,
an experiment function (``range_checked``) once at its end, so its sweeps
enqueue back to back.
"""
from __future__ import annotations

import contextlib
import ctypes
import functools
import inspect
import random
import warnings
import weakref
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .config import CConfig, PythiaConfig, get_config
from .tokenizer import HFTokenizer, SyntheticTokenizer, TokenizerMixin
from .weights import (EngineWeights, config_from_hf_json, load_hf_safetensors, process_to_engine,
                      synth_engine_weights)

SITE_DTYPE = np.dtype([(f, np.int32) for f in _lib.SITE_FIELDS])


def range_checked(fn):
    """Run ``fn`` (an experiment function taking ``model``) inside the model's
    range scope: the x2f16 range flag is read once when the outermost scope
    ends instead of after every engine call.

    If that check fails (``_lib.RangeError``: a GEMM input reached the fp16
    split's limit, so the call's results are not fp32-accurate), the model
    moves to the next path without that limit (``Model.range_fallback``:
    the processed-weight GEMMs when the exact-fp16 ones were bound — their A
    operand is LNPre(x)·γ — else gemm ``"x3bf16"``), warns, records it in
    ``model.range_fallbacks``, restores the global ``random`` state the call
    started from and runs the call again: same process, same prompts (the
    functions shuffle private copies of their inputs; substitute_task's
    in-place sort is idempotent)."""
    sig = inspect.signature(fn)

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        try:
            model = sig.bind_partial(*args, **kwargs).arguments.get("model")
        except TypeError:  # a bad call: let fn raise its own error
            model = None
        if not isinstance(model, Model):
            return fn(*args, **kwargs)
        if model._range_depth > 0 or not model.range_fallback:  # the outermost call retries
            with model.range_scope(fn.__name__):
                return fn(*args, **kwargs)
        state = random.getstate()
        while True:
            try:
                with model.range_scope(fn.__name__):
                    return fn(*args, **kwargs)
            except _lib.RangeError as e:
                if not model._fall_back(fn.__name__, e):
                    raise
                random.setstate(state)
    return wrapper


def make_sites(n: int) -> np.ndarray:
    """Zeroed site records (layout of ``tvr_site``), target = -1."""
    s = np.zeros(n, dtype=SITE_DTYPE)
    s["target"] = -1
    return s


class Trace:
    """Engine-owned clean-run snapshots (resid_pre per layer, z, K/V).

    A caller's trace keeps its model alive; the experiment functions' scratch
    trace (``weak``) does not, so ``del model`` frees the model's device memory
    at once (no model <-> trace reference cycle waiting for the collector).
    The model closes every live trace before it destroys itself."""

    def __init__(self, model: "Model", max_seqs: int, max_tokens: int, weak: bool = False):
        self._lib = model._lib
        self._h = None
        h = ctypes.c_void_p()
        _lib.check(self._lib.tvr_trace_create(model._h, max_seqs, max_tokens, ctypes.byref(h)),
                   "tvr_trace_create")
        self._h = h
        self._model_strong = None if weak else model
        self._model_ref = weakref.ref(model)
        model._traces.add(self)
        self.max_seqs = max_seqs
        self.max_tokens = max_tokens
        self.seq_lens: List[int] = []
        self.seq_offsets: List[int] = []
        # output tensors of a deferred clean forward, kept alive until the
        # engine has written them (the next patch sweep or trace read)
        self._pending_out = None

    @property
    def model(self) -> "Model":
        m = self._model_strong if self._model_strong is not None else self._model_ref()
        if m is None:
            raise _lib.EngineError("the trace's model has been destroyed")
        return m

    def resid_pre(self, layer: int) -> torch.Tensor:
        """``blocks.{layer}.hook_resid_pre`` of every traced token ([tokens, d]);
        layer == n_layers gives the final residual."""
        return self._read(_lib.TRACE_RESID_PRE, layer)

    def z(self, layer: int) -> torch.Tensor:
        """``blocks.{layer}.attn.hook_z`` flattened over heads ([tokens, d])."""
        return self._read(_lib.TRACE_Z, layer)

    def _read(self, what: int, layer: int) -> torch.Tensor:
        m = self.model
        buf = torch.empty(sum(self.seq_lens), m.cfg.d_model, device=m.device)
        _lib.check(self._lib.tvr_trace_read(self._h, what, layer, buf.data_ptr(), m._stream()),
                   "tvr_trace_read")
        self._pending_out = None
        return buf

    def flush(self) -> None:
        """Run a pending deferred clean forward now (its prob / top-k tensors
        are written; include/tvr.h tvr_trace_flush)."""
        if self._pending_out is not None:
            _lib.check(self._lib.tvr_trace_flush(self._h, self.model._stream()), "tvr_trace_flush")
            self._pending_out = None

    def close(self) -> None:
        """Run a pending deferred forward (its outputs are owed to the caller)
        and free the trace; idempotent.  Model.__del__ calls it on every live
        trace of the model first, so no trace outlives its engine model."""
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                if getattr(self, "_pending_out", None) is not None:
                    self.flush()  # (tvr_trace_destroy would also run it)
            finally:  # the device buffers are released even if the flush raised
                self._h = None
                self._lib.tvr_trace_destroy(h)

    def __del__(self):
        self.close()


# Matrix-core path of the GEMMs (Model.set_gemm): the fp32-accurate 2-plane
# fp16 split is the fastest path whose error is at or below the fp32 MFMA's.
DEFAULT_GEMM = "x2f16"


class Model(TokenizerMixin):
    def __init__(self, cfg: PythiaConfig, weights: EngineWeights, tokenizer=None,
                 device: Optional[torch.device] = None, gemm: str = DEFAULT_GEMM):
        self._h = None
        self._traces = weakref.WeakSet()  # live traces of this model (closed before the model is destroyed)
        self._range_depth = 0
        self._lib = _lib.load()
        self._ops = _lib.load_ops()
        dev = torch.device(device) if device is not None else weights.w_embed.device
        if dev.type != "cuda" or not torch.cuda.is_available():
            raise _lib.EngineError("the HIP engine needs a GPU device (no CPU fallback): "
                                   f"got device {dev}")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.cfg = cfg
        self.device = dev
        self.weights = weights
        self.tokenizer = tokenizer if tokenizer is not None else SyntheticTokenizer(cfg.d_vocab)
        for t in weights.tensors():
            if t.device != dev or t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError("engine weights must be contiguous fp32 tensors on the model device")
        self._cfg_c = CConfig.from_config(cfg)
        self._layers_c = (_lib.CLayerWeights * cfg.n_layers)(
            *[_lib.CLayerWeights(L.w1.data_ptr(), L.b1.data_ptr(), L.w2.data_ptr(), L.b2.data_ptr())
              for L in weights.layers])
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            _lib.check(self._lib.tvr_model_create(
                ctypes.byref(self._cfg_c), weights.w_embed.data_ptr(), self._layers_c,
                weights.w_unembed_t.data_ptr(), weights.b_unembed.data_ptr(), ctypes.byref(h)),
                "tvr_model_create")
        self._h = h
        self._trace_cache: Optional[Trace] = None
        self.exact16 = False
        self._x16_c = None
        self.gemm = "f32"
        # what an experiment function does when the x2f16 range check fails (range_checked): retry on the
        # next path without the limit (True), or raise (False); the fallbacks taken, as (function, path)
        self.range_fallback = True
        self.range_fallbacks: List[tuple] = []
        if weights.raw16 is not None:  # bound first: the x2f16 planes are then built without W2's
            self.set_exact16(True)
        self.set_gemm(gemm)

    # ------------------------------------------------------------------ build
    @classmethod
    def from_pretrained(cls, name: str, device="cuda", seed: int = 0, checkpoint: Optional[str] = None,
                        tokenizer_path: Optional[str] = None, std: float = 0.02, ln_std: float = 0.1,
                        cfg: Optional[PythiaConfig] = None, gemm: str = DEFAULT_GEMM,
                        fp16_weights: bool = False) -> "Model":
        """``HookedTransformer.from_pretrained`` without a network: the named
        Pythia shape with seeded synthetic weights (generated on the device), or
        a local HF-layout safetensors ``checkpoint`` (file, or directory with
        model.safetensors / sharded index; its config.json, when present,
        supplies the shape for names this module does not know).  ``gemm``
        picks the matrix-core path (see :meth:`set_gemm`).  ``fp16_weights``:
        the synthetic parameters are fp16-valued, as the released checkpoints
        are; with fp16-valued weights (synthetic or a checkpoint's) the
        exact-fp16 GEMMs are bound (:meth:`set_exact16`)."""
        import os
        if cfg is None:
            try:
                cfg = get_config(name)
            except ValueError:
                if not (checkpoint and os.path.isdir(checkpoint)):
                    raise
                cfg = config_from_hf_json(checkpoint)
        dev = torch.device(device)
        if checkpoint:
            w = process_to_engine(cfg, load_hf_safetensors(checkpoint, cfg), device=dev, free_source=True)
        else:
            w = synth_engine_weights(cfg, seed=seed, device=dev, std=std, ln_std=ln_std, fp16=fp16_weights)
        tok = HFTokenizer(tokenizer_path) if tokenizer_path else None
        if dev.type == "cuda":
            torch.cuda.empty_cache()  # the generation's temporaries: the engine's own allocations come next
        return cls(cfg, w, tokenizer=tok, device=dev, gemm=gemm)

    @classmethod
    def from_hf_state_dict(cls, cfg: PythiaConfig, sd, device="cuda", tokenizer=None,
                           gemm: str = DEFAULT_GEMM) -> "Model":
        return cls(cfg, process_to_engine(cfg, sd, device=torch.device(device)), tokenizer, device, gemm)

    def set_gemm(self, mode: str) -> None:
        """Matrix-core path of every GEMM (include/tvr.h ``tvr_model_set_gemm``):
        ``"x2f16"`` (default) — fp32-accurate two-plane fp16 split (the fp16 form
        of 3xTF32: three products on the fp16 MFMA, 4 B per weight for the
        planes; inputs must stay below 4095 in magnitude, checked on the device
        after every engine call); ``"x3bf16"`` — fp32-accurate three-plane bf16
        split (six products, 6 B per weight, no range limit); ``"f32"`` —
        ``v_mfma_f32_32x32x2_f32`` on the fp32 weights; ``"bf16"`` — bf16
        weights and GEMM inputs, fp32 accumulation (NOT fp32-accurate: the
        north star's bf16 configuration, 2e-2 tolerance).  Both splits measure
        at or below the fp32 MFMA GEMM's error against fp64 (DESIGN.md
        section 3).  Everything outside the GEMMs is fp32 in all four."""
        if mode not in _lib.GEMM_MODES:
            raise ValueError(f"gemm mode must be one of {sorted(_lib.GEMM_MODES)}, got {mode!r}")
        with torch.cuda.device(self.device):
            try:
                _lib.check(self._lib.tvr_model_set_gemm(self._h, _lib.GEMM_MODES[mode], self._stream()),
                           "tvr_model_set_gemm")
            finally:  # a failed switch leaves the engine in the fp32 mode: mirror it
                self.gemm = _lib.GEMM_NAMES.get(self._lib.tvr_model_get_gemm(self._h), mode)

    def set_exact16(self, on: bool) -> None:
        """Bind (or detach) the checkpoint's own fp16 GEMM weights
        (``EngineWeights.raw16``; include/tvr.h ``tvr_model_set_exact16``): in
        x2f16 mode the QKV + MLP-in and O + MLP-out GEMMs then run 2 matrix
        products per slice instead of 3 on those exact operands, with LN's
        gamma applied to the rows.  On by default whenever the weights are
        fp16-valued (every released Pythia checkpoint).  Results equal the
        processed-weight path's to fp32 rounding."""
        raw = self.weights.raw16
        if on and raw is None:
            raise ValueError("set_exact16: the weights are not exact in fp16 (EngineWeights.raw16 is None)")
        if on:
            for r in raw:
                for t, dt in ((r.w1, torch.float16), (r.w2, torch.float16), (r.g1, torch.float32),
                              (r.g2, torch.float32)):
                    if t.device != self.device or t.dtype != dt or not t.is_contiguous():
                        raise ValueError("raw16 tensors must be contiguous fp16 (w1, w2) / fp32 (g1, g2) on the "
                                         "model device")
            ru = self.weights.raw16_unembed
            if ru is not None:
                wu, gf = ru
                if wu.device != self.device or wu.dtype != torch.float16 or not wu.is_contiguous() or \
                        gf.device != self.device or gf.dtype != torch.float32:
                    raise ValueError("raw16_unembed must be (fp16 [V, d], fp32 [d]) contiguous on the model device")
            arr = (_lib.CExact16Layer * self.cfg.n_layers)(
                *[_lib.CExact16Layer(r.w1.data_ptr(), r.w2.data_ptr(), r.g1.data_ptr(), r.g2.data_ptr())
                  for r in raw])
        # the engine re-plans the x2f16 weight planes on a (de)tach: hipMalloc / the conversion kernels run on
        # the current device, which must be the model's
        with torch.cuda.device(self.device):
            try:
                if on:
                    self._x16_c = arr  # the engine keeps the binding from here on, even if the re-plan fails
                    _lib.check(self._lib.tvr_model_set_exact16(self._h, arr), "tvr_model_set_exact16")
                    if ru is not None:
                        _lib.check(self._lib.tvr_model_set_exact16_unembed(self._h, wu.data_ptr(), gf.data_ptr()),
                                   "tvr_model_set_exact16_unembed")
                else:
                    _lib.check(self._lib.tvr_model_set_exact16_unembed(self._h, None, None),
                               "tvr_model_set_exact16_unembed")
                    _lib.check(self._lib.tvr_model_set_exact16(self._h, None), "tvr_model_set_exact16")
                    self._x16_c = None
            finally:
                # the engine records the binding before it re-plans, and a failed re-plan (e.g. the planes do
                # not fit) leaves it in the fp32 mode: mirror what the engine holds, error or not
                self.exact16 = bool(on)
                self.gemm = _lib.GEMM_NAMES.get(self._lib.tvr_model_get_gemm(self._h), self.gemm)

    def _fall_back(self, what: str, err: Exception) -> bool:
        """Move to the next GEMM path without the x2f16 range limit after a
        failed range check: exact-fp16 → processed weights (x2f16, 3 products:
        LayerNorm's output, bounded by sqrt(d_model), is the A operand again),
        x2f16 → x3bf16 (no range limit).  False when there is none left."""
        if self.gemm != "x2f16":
            return False
        if self.exact16:
            self.set_exact16(False)  # the engine re-plans the x2f16 planes on the processed weights
            path = "x2f16 (processed weights)"
        else:
            self.set_gemm("x3bf16")
            path = "x3bf16"
        self.range_fallbacks.append((what, path))
        warnings.warn(f"{what}: {err} -- retrying on {path}", RuntimeWarning, stacklevel=3)
        return True

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            for t in list(getattr(self, "_traces", ())):
                t.close()  # before the engine model they point into is freed
            self._trace_cache = None
            self._h = None
            self._lib.tvr_model_destroy(h)

    # ------------------------------------------------------------- internals
    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def _check_range(self, what: str, force: bool = False) -> None:
        """x2f16 only: fail loudly if a GEMM input left the fp16 split's range
        since the last check (synchronises the stream).  Inside a
        ``range_scope`` the check waits for the scope's end."""
        if self.gemm == "x2f16" and (force or self._range_depth == 0):
            _lib.check(self._lib.tvr_model_range_status(self._h, self._stream()), what)

    @contextlib.contextmanager
    def range_scope(self, what: str):
        """Defer the per-call range checks of the engine calls inside to ONE
        check when the outermost scope exits normally (the flag is sticky on
        the device, so nothing is missed; an exception propagates unchecked)."""
        self._range_depth += 1
        try:
            yield self
        except BaseException:
            self._range_depth -= 1
            raise
        self._range_depth -= 1
        self._check_range(what)

    def _op(self, name: str, *args):
        """torch.ops.tvr.<name>: engine errors as EngineError (invalid
        arguments stay ValueError, the reference's error type)."""
        try:
            return getattr(self._ops, name)(*args)
        except ValueError:
            raise
        except RuntimeError as e:
            raise _lib.EngineError(str(e)) from e

    def trace(self, n_seqs: int, n_tokens: int) -> Trace:
        """A new trace with this capacity, owned by the caller (the experiment
        functions use a private one, so they never overwrite it)."""
        return Trace(self, max(n_seqs, 1), max(n_tokens, 1))

    def _sweep_trace(self, n_seqs: int, n_tokens: int) -> Trace:
        """The experiment functions' scratch trace (grown on demand, reused)."""
        t = self._trace_cache
        if t is None or t.max_seqs < n_seqs or t.max_tokens < n_tokens:
            if t is not None:
                t.flush()  # a deferral on the old trace still owes its outputs
            self._trace_cache = None
            t = Trace(self, max(n_seqs, 1), max(n_tokens, 1), weak=True)
            self._trace_cache = t
        return t

    @staticmethod
    def _pack(seqs: Sequence[Sequence[int]]):
        lens = np.asarray([len(s) for s in seqs], dtype=np.int32)
        toks = np.asarray([int(x) for s in seqs for x in s], dtype=np.int32)
        return toks, lens

    # ---------------------------------------------------------- entry points
    def forward_clean(self, seqs: Sequence[Sequence[int]], targets: Optional[Sequence[int]] = None,
                      topk: int = 0, return_logits: bool = False, capture: bool = False,
                      trace: Optional[Trace] = None, defer: bool = False) -> Dict[str, torch.Tensor]:
        """Batched clean forward of ragged prompts (token-id lists).
        Returns ``prob`` [n] (softmax(logits[-1])[target]), ``topk`` [n, k],
        ``logits`` [n, V] (last position), ``zsum`` [L, d] (sum over prompts of
        hook_z at the last position) as requested.
        ``defer`` (with a trace; no logits / capture): the clean rows run inside
        the next ``patch_sweep`` on that trace (tvr_forward_clean_deferred) and
        the returned tensors are written by it — read them after that sweep."""
        n = len(seqs)
        if n == 0:
            raise ValueError("no prompts")
        toks, lens = self._pack(seqs)
        tg = None
        if targets is not None:
            tg = np.asarray([-1 if t is None else int(t) for t in targets], dtype=np.int32)
            if tg.shape[0] != n:
                raise ValueError("targets must have one entry per prompt")
        if trace is not None and (trace.max_seqs < n or trace.max_tokens < int(lens.sum())):
            raise ValueError("trace too small for this batch")
        if defer and (trace is None or return_logits or capture):
            raise ValueError("defer needs a trace and no logits / capture")
        cfg = self.cfg
        prob, top, logits, zsum = self._op(
            "forward_clean", self._h.value, trace._h.value if trace is not None else 0, torch.from_numpy(toks),
            torch.from_numpy(lens), torch.from_numpy(tg) if tg is not None else None, topk, return_logits, capture,
            defer, cfg.n_layers, cfg.d_model, cfg.d_vocab, self.device)
        out = {}
        if tg is not None:
            out["prob"] = prob
        if topk:
            out["topk"] = top
        if return_logits:
            out["logits"] = logits
        if capture:
            out["zsum"] = zsum
        if trace is not None:
            trace.seq_lens = lens.tolist()
            trace.seq_offsets = np.concatenate([[0], np.cumsum(lens)[:-1]]).tolist()
            # a deferred forward's outputs are written by the next sweep on the trace: keep them alive
            trace._pending_out = (prob, top) if defer else None
        if not defer:
            self._check_range("tvr_forward_clean")
        return out

    def patch_sweep(self, trace: Trace, sites: np.ndarray, vectors: Optional[torch.Tensor] = None,
                    topk: int = 0, want_prob: bool = True, return_logits: bool = False
                    ) -> Dict[str, torch.Tensor]:
        """Evaluate every site (records of ``make_sites``) against ``trace``."""
        sites = np.ascontiguousarray(sites, dtype=SITE_DTYPE)
        n = int(sites.shape[0])
        if n == 0:
            raise ValueError("no patch sites")
        if vectors is not None:
            if vectors.device != self.device or vectors.dtype != torch.float32:
                raise ValueError("vectors must be fp32 on the model device")
            vectors = vectors.reshape(-1, self.cfg.d_model).contiguous()
        rows = torch.from_numpy(sites.view(np.int32).reshape(n, len(_lib.SITE_FIELDS)))
        prob, top, logits = self._op("patch_sweep", self._h.value, trace._h.value, rows, vectors, topk, want_prob,
                                     return_logits, self.cfg.d_vocab, self.device)
        self._check_range("tvr_patch_sweep")
        trace._pending_out = None
        out = {}
        if want_prob:
            out["prob"] = prob
        if topk:
            out["topk"] = top
        if return_logits:
            out["logits"] = logits
        return out

    def project_heads(self, zsum: torch.Tensor) -> torch.Tensor:
        """[L, d] z-sums → [L, H, d] hook_result sums."""
        if tuple(zsum.shape) != (self.cfg.n_layers, self.cfg.d_model):
            raise ValueError("zsum must be [n_layers, d_model]")
        return self._op("project_heads", self._h.value, zsum.to(self.device, torch.float32).contiguous(),
                        self.cfg.n_heads)

    # ------------------------------------------------------------ profiling
    def profile(self, on: bool) -> None:
        """Enable/disable HIP-event timing of every GEMM and HBM-bound kernel launch (resets totals)."""
        _lib.check(self._lib.tvr_profile_enable(self._h, 1 if on else 0), "tvr_profile_enable")

    def profile_stats(self) -> dict:
        st = _lib.CKernelStats()
        _lib.check(self._lib.tvr_profile_read(self._h, ctypes.byref(st)), "tvr_profile_read")
        per = {name: {"launches": st.gemm_launches[i], "flops": st.gemm_flops[i], "ms": st.gemm_ms[i],
                      "bytes": st.gemm_bytes[i]} for i, name in enumerate(_lib.GEMM_VARIANTS)}
        per["all"] = {k: sum(v[k] for v in per.values()) for k in ("launches", "flops", "ms", "bytes")}
        return per

    def profile_hbm_stats(self) -> dict:
        """The HBM-bound kernels timed since ``profile(True)``: launches, summed
        ms, algorithmic bytes and achieved GB/s per kind (include/tvr.h
        tvr_hbm_kind)."""
        st = _lib.CHbmStats()
        _lib.check(self._lib.tvr_profile_read_hbm(self._h, ctypes.byref(st)), "tvr_profile_read_hbm")
        return {name: {"launches": st.launches[i], "ms": st.ms[i], "bytes": st.bytes[i],
                       "gbps": st.bytes[i] / (st.ms[i] * 1e-3) / 1e9 if st.ms[i] > 0 else None}
                for i, name in enumerate(_lib.HBM_KINDS)}

    # ------------------------------------------------- TL-style conveniences
    def _as_ids(self, tokens) -> List[int]:
        if isinstance(tokens, str):
            tokens = self.to_tokens(tokens)
        if isinstance(tokens, torch.Tensor):
            if tokens.dim() == 2:
                if tokens.shape[0] != 1:
                    raise ValueError("batch size must be 1")
                tokens = tokens[0]
            return [int(x) for x in tokens.tolist()]
        return [int(x) for x in tokens]

    def forward(self, tokens, start_at_layer: Optional[int] = None, last_only: bool = False) -> torch.Tensor:
        """TransformerLens ``HookedTransformer.forward`` (scratch2.py:143,183,297;
        scratch.py:127,143,206,209) for batch 1: ``tokens`` (a string, ids [T]
        or [1, T]) -> logits [1, T, V] of every position; with
        ``start_at_layer=L``, ``tokens`` is the residual ``hook_resid_pre`` of
        block L ([1, T, d] or [T, d]) and the forward continues from there.
        ``last_only`` returns [1, 1, V] (the only row the reference reads)
        without the other rows' unembedding.  Up to n_ctx tokens."""
        dev, V = self.device, self.cfg.d_vocab
        if start_at_layer is None:
            ids = self._as_ids(tokens)
            if last_only:
                return self.forward_clean([ids], return_logits=True)["logits"].view(1, 1, -1)
            toks, lens = self._pack([ids])
            out = self._op("forward_logits", self._h.value, torch.from_numpy(toks), None, 0, torch.from_numpy(lens),
                           V, dev)
        else:
            resid = torch.as_tensor(tokens).to(dev, torch.float32)
            if resid.dim() == 3:
                if resid.shape[0] != 1:
                    raise ValueError("batch size must be 1")
                resid = resid[0]
            if resid.dim() != 2 or resid.shape[1] != self.cfg.d_model:
                raise ValueError("start_at_layer needs a residual of shape [1, T, d_model]")
            resid = resid.contiguous()
            lens = np.asarray([resid.shape[0]], dtype=np.int32)
            out = self._op("forward_logits", self._h.value, None, resid, int(start_at_layer), torch.from_numpy(lens),
                           V, dev)
        self._check_range("tvr_forward_logits")
        if last_only:
            out = out[-1:]
        return out.view(1, out.shape[0], V)

    __call__ = forward

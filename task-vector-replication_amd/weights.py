"""Weights: seeded synthetic Pythia checkpoints and TransformerLens processing.

``HookedTransformer.from_pretrained`` (scratch.py:26, scratch2.py:26) fetches a
checkpoint by name and, with its defaults, processes it with ``fold_ln``,
``center_writing_weights``, ``center_unembed`` and ``fold_value_biases``.  Those
steps define the numerical value of every hook the reference reads
(``hook_result`` excludes b_O and the folded value bias; residuals and logits
are mean-centred), so the engine applies the same processing once at load and
lays the result out for its fused GEMMs:

* ``w1`` [3d + d_mlp, d]: Q | K | V | MLP-in rows (LN1/LN2 folded, read-in
  weights centred over d_model).  LN1 and LN2 both read ``resid_pre`` in a
  parallel block and are identical LayerNormPre after folding, so one
  normalisation feeds one GEMM.
* ``w2`` [d, d + d_mlp]: O | MLP-out columns (write-out weights centred).
* ``b2`` = b_O (+ folded value bias) + b_out.

No network: weights are either generated from a seed (shapes of a named
Pythia) or loaded from a local HF-layout safetensors file.
"""
from __future__ import annotations

import zlib
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from .config import PythiaConfig

HFStateDict = Dict[str, torch.Tensor]


def _seed_for(seed: int, name: str) -> int:
    return (int(seed) * 0x9E3779B1 + zlib.crc32(name.encode())) & 0x7FFF_FFFF_FFFF


def hf_param_shapes(cfg: PythiaConfig) -> Dict[str, tuple]:
    """Parameter names/shapes of ``transformers.GPTNeoXForCausalLM``."""
    d, m, V = cfg.d_model, cfg.d_mlp, cfg.d_vocab
    shapes = {"gpt_neox.embed_in.weight": (V, d)}
    for l in range(cfg.n_layers):
        p = f"gpt_neox.layers.{l}."
        shapes.update({
            p + "input_layernorm.weight": (d,),
            p + "input_layernorm.bias": (d,),
            p + "post_attention_layernorm.weight": (d,),
            p + "post_attention_layernorm.bias": (d,),
            p + "attention.query_key_value.weight": (3 * d, d),
            p + "attention.query_key_value.bias": (3 * d,),
            p + "attention.dense.weight": (d, d),
            p + "attention.dense.bias": (d,),
            p + "mlp.dense_h_to_4h.weight": (m, d),
            p + "mlp.dense_h_to_4h.bias": (m,),
            p + "mlp.dense_4h_to_h.weight": (d, m),
            p + "mlp.dense_4h_to_h.bias": (d,),
        })
    shapes["gpt_neox.final_layer_norm.weight"] = (d,)
    shapes["gpt_neox.final_layer_norm.bias"] = (d,)
    shapes["embed_out.weight"] = (V, d)
    return shapes


def synth_param(cfg: PythiaConfig, name: str, shape: tuple, seed: int = 0,
                device="cpu", std: float = 0.02, ln_std: float = 0.1, fp16: bool = False) -> torch.Tensor:
    """One seeded synthetic parameter (SURVEY.md §8d value distributions):
    weights N(0, std), LayerNorm weights 1 + N(0, ln_std), biases N(0, std).
    ``fp16``: rounded to fp16 values (held in fp32), as every tensor of the
    released Pythia checkpoints is stored (their dtype is float16)."""
    g = torch.Generator(device=device)
    g.manual_seed(_seed_for(seed, name))
    x = torch.randn(shape, generator=g, device=device, dtype=torch.float32)
    if "layernorm" in name or "layer_norm" in name:
        x = (1.0 + ln_std * x) if name.endswith("weight") else x.mul_(std)
    else:
        x = x.mul_(std)
    return x.half().float() if fp16 else x


def synth_hf_state_dict(cfg: PythiaConfig, seed: int = 0, device="cpu", std: float = 0.02,
                        ln_std: float = 0.1, fp16: bool = False) -> HFStateDict:
    """A full seeded synthetic HF-layout state dict (biases and LN params
    non-trivial so fold_ln / fold_value_biases are exercised); ``fp16`` as
    :func:`synth_param`."""
    return {n: synth_param(cfg, n, s, seed, device, std, ln_std, fp16)
            for n, s in hf_param_shapes(cfg).items()}


# Non-parameter entries real GPT-NeoX checkpoints carry per layer (buffers the
# engine recomputes: causal mask, its fill value, rotary inverse frequencies).
HF_BUFFER_SUFFIXES = ("attention.bias", "attention.masked_bias", "attention.rotary_emb.inv_freq")
HF_ALIASES = {"lm_head.weight": "embed_out.weight"}


def _checkpoint_files(path) -> List[str]:
    """A .safetensors file, or a directory holding model.safetensors or the
    shards listed by model.safetensors.index.json."""
    import json
    import os
    if os.path.isdir(path):
        index = os.path.join(path, "model.safetensors.index.json")
        if os.path.exists(index):
            with open(index) as f:
                shards = sorted(set(json.load(f)["weight_map"].values()))
            return [os.path.join(path, s) for s in shards]
        single = os.path.join(path, "model.safetensors")
        if os.path.exists(single):
            return [single]
        raise FileNotFoundError(f"{path}: no model.safetensors or model.safetensors.index.json")
    return [str(path)]


def load_hf_safetensors(path, cfg: Optional[PythiaConfig] = None, device="cpu") -> HFStateDict:
    """Load a local HF GPT-NeoX checkpoint (``GPTNeoXForCausalLM`` layout,
    safetensors only: no code execution), the offline replacement of the
    by-name fetch at scratch.py:26 / scratch2.py:26.  ``path`` is a file or a
    directory (single file or sharded with an index).  Buffers are dropped
    (``attention.bias`` / ``masked_bias`` / ``rotary_emb.inv_freq``), the
    ``lm_head.weight`` alias is mapped to ``embed_out.weight``, fp16 / bf16
    tensors become fp32.  With ``cfg`` the key set and every shape are checked
    against ``hf_param_shapes(cfg)`` (ValueError naming what is missing,
    unexpected or mis-shaped)."""
    from safetensors.torch import load_file
    sd: HFStateDict = {}
    for f in _checkpoint_files(path):
        for k, v in load_file(f, device=str(device)).items():
            if k.endswith(HF_BUFFER_SUFFIXES):
                continue
            sd[HF_ALIASES.get(k, k)] = v.float()
    if cfg is not None:
        want = hf_param_shapes(cfg)
        missing = sorted(set(want) - set(sd))
        extra = sorted(set(sd) - set(want))
        bad = sorted(k for k in set(want) & set(sd) if tuple(sd[k].shape) != tuple(want[k]))
        if missing or extra or bad:
            raise ValueError(f"{path}: checkpoint does not match {cfg.name} "
                             f"(missing {missing[:6]}{'...' if len(missing) > 6 else ''}, "
                             f"unexpected {extra[:6]}, wrong shape {bad[:6]})")
    return sd


def config_from_hf_json(path) -> PythiaConfig:
    """A ``PythiaConfig`` from an HF GPT-NeoX ``config.json`` (a checkpoint
    directory or the file).  The engine implements Pythia's block only:
    parallel residual, rotary, exact-erf GELU."""
    import json
    import os
    f = os.path.join(path, "config.json") if os.path.isdir(path) else str(path)
    with open(f) as fh:
        c = json.load(fh)
    if c.get("model_type", "gpt_neox") != "gpt_neox" or not c.get("use_parallel_residual", True):
        raise ValueError(f"{f}: only GPT-NeoX with the parallel residual (Pythia) is supported")
    if c.get("hidden_act", "gelu") != "gelu":
        raise ValueError(f"{f}: hidden_act {c.get('hidden_act')!r} (Pythia uses exact-erf gelu)")
    return PythiaConfig(n_layers=c["num_hidden_layers"], d_model=c["hidden_size"], n_heads=c["num_attention_heads"],
                        d_mlp=c["intermediate_size"], d_vocab=c["vocab_size"], rotary_pct=c.get("rotary_pct", 0.25),
                        n_ctx=c.get("max_position_embeddings", 2048), ln_eps=c.get("layer_norm_eps", 1e-5),
                        rotary_base=float(c.get("rotary_emb_base", 10000)), name=c.get("_name_or_path", "checkpoint"))


@dataclass
class EngineLayer:
    w1: torch.Tensor
    b1: torch.Tensor
    w2: torch.Tensor
    b2: torch.Tensor


@dataclass
class RawLayer16:
    """One layer's checkpoint tensors for the exact-fp16 GEMMs (include/tvr.h
    ``tvr_model_set_exact16``): W1 rows (Q | K | V in the engine order, then
    MLP-in) and W2 = W_O | W_out BEFORE fold_ln / centring, as fp16 (exact:
    built only from fp16-valued tensors), and LN1 / LN2 gamma (fp32)."""
    w1: torch.Tensor   # fp16 [3d + d_mlp, d]
    w2: torch.Tensor   # fp16 [d, d + d_mlp]
    g1: torch.Tensor   # fp32 [d]
    g2: torch.Tensor   # fp32 [d]


@dataclass
class EngineWeights:
    """Processed weights in the engine layout (all fp32, contiguous)."""
    w_embed: torch.Tensor          # [V, d]
    layers: List[EngineLayer]
    w_unembed_t: torch.Tensor      # [V, d]  (TL W_U transposed)
    b_unembed: torch.Tensor        # [V]
    raw16: Optional[List[RawLayer16]] = None  # the exact-fp16 GEMM operands, when the checkpoint is fp16
    # the unembed's: the checkpoint's embed_out.weight (fp16 [V, d]) and the final LN gamma (fp32 [d])
    raw16_unembed: Optional[tuple] = None

    def tensors(self) -> List[torch.Tensor]:
        out = [self.w_embed, self.w_unembed_t, self.b_unembed]
        for L in self.layers:
            out += [L.w1, L.b1, L.w2, L.b2]
        return out


def _exact16(*ts: torch.Tensor) -> bool:
    """Every value of every tensor is an fp16 value (finite)."""
    for t in ts:
        h = t.half()
        if not bool(torch.isfinite(h).all()) or not bool((h.float() == t).all()):
            return False
    return True


def _process_layer(cfg: PythiaConfig, get, raw: Optional[list] = None) -> EngineLayer:
    """One layer's TL processing.  ``raw`` (a list): the layer's RawLayer16 is
    appended when its GEMM weights are exact in fp16, else None."""
    d, H, dh = cfg.d_model, cfg.n_heads, cfg.d_head
    ln1_w, ln1_b = get("input_layernorm.weight"), get("input_layernorm.bias")
    ln2_w, ln2_b = get("post_attention_layernorm.weight"), get("post_attention_layernorm.bias")
    # HF fuses Q, K, V per head: rows (head, {q,k,v}, d_head).  Engine order: Q | K | V,
    # each (head, d_head).
    wqkv = get("attention.query_key_value.weight").view(H, 3, dh, d).transpose(0, 1).reshape(3 * d, d)
    bqkv = get("attention.query_key_value.bias").view(H, 3, dh).transpose(0, 1).reshape(3 * d)
    w_in, b_in = get("mlp.dense_h_to_4h.weight"), get("mlp.dense_h_to_4h.bias")
    if raw is not None:
        w_o_raw, w_out_raw = get("attention.dense.weight"), get("mlp.dense_4h_to_h.weight")
        if _exact16(wqkv, w_in, w_o_raw, w_out_raw):
            raw.append(RawLayer16(w1=torch.cat([wqkv, w_in], 0).half().contiguous(),
                                  w2=torch.cat([w_o_raw, w_out_raw], 1).half().contiguous(),
                                  g1=ln1_w.float().contiguous().clone(), g2=ln2_w.float().contiguous().clone()))
        else:
            raw.append(None)
    # fold_ln: biases first (they read the unscaled weights), then scale, then centre
    # the read-in weights over d_model.
    bqkv = bqkv + wqkv @ ln1_b
    b_in = b_in + w_in @ ln2_b
    wqkv = wqkv * ln1_w
    w_in = w_in * ln2_w
    wqkv = wqkv - wqkv.mean(dim=1, keepdim=True)
    w_in = w_in - w_in.mean(dim=1, keepdim=True)
    # center_writing_weights: W_O, b_O, W_out, b_out centred over the d_model output.
    w_o, b_o = get("attention.dense.weight"), get("attention.dense.bias")
    w_out, b_out = get("mlp.dense_4h_to_h.weight"), get("mlp.dense_4h_to_h.bias")
    w_o = w_o - w_o.mean(dim=0, keepdim=True)
    w_out = w_out - w_out.mean(dim=0, keepdim=True)
    b_o = b_o - b_o.mean()
    b_out = b_out - b_out.mean()
    # fold_value_biases: b_O += sum_h b_V[h] @ W_O[h]; b_V = 0.
    b_v = bqkv[2 * d:].clone()
    b_o = b_o + w_o @ b_v
    bqkv = torch.cat([bqkv[: 2 * d], torch.zeros_like(b_v)])
    return EngineLayer(
        w1=torch.cat([wqkv, w_in], 0).contiguous(),
        b1=torch.cat([bqkv, b_in]).contiguous(),
        w2=torch.cat([w_o, w_out], 1).contiguous(),
        b2=(b_o + b_out).contiguous(),
    )


def _process_unembed(w_u: torch.Tensor, lnf_w: torch.Tensor, lnf_b: torch.Tensor):
    """ln_final folded into W_U (HF embed_out.weight [V, d] = TL W_U^T), then
    center_unembed.  Pythia has no unembed bias, so b_U starts at 0."""
    b_u = w_u @ lnf_b
    w_u = w_u * lnf_w
    w_u = w_u - w_u.mean(dim=1, keepdim=True)            # fold_ln centring over d_model
    w_u = w_u - w_u.mean(dim=0, keepdim=True)            # center_unembed over vocab
    b_u = b_u - b_u.mean()
    return w_u.contiguous(), b_u.contiguous()


# tensors _process_layer reads twice when raw16 is on (the raw copy and the processing)
_RAW_NAMES = ("attention.query_key_value.weight", "mlp.dense_h_to_4h.weight", "attention.dense.weight",
              "mlp.dense_4h_to_h.weight", "input_layernorm.weight", "post_attention_layernorm.weight")


def _take_keep(sd, name, dev, dtype):
    return sd[name].to(dev, dtype)


def _raw_unembed(wu: torch.Tensor, gf: torch.Tensor) -> Optional[tuple]:
    """(embed_out.weight as fp16, final LN gamma) when the unembed is exact in fp16, else None."""
    return (wu.half().contiguous(), gf.float().contiguous().clone()) if _exact16(wu) else None


def _raw_or_none(raw: Optional[list]) -> Optional[List[RawLayer16]]:
    """The raw16 list when EVERY layer is exact in fp16, else None."""
    if not raw or any(r is None for r in raw):
        return None
    return raw


@torch.no_grad()
def process_to_engine(cfg: PythiaConfig, sd: HFStateDict, device=None,
                      free_source: bool = False, dtype=torch.float32, raw16: bool = True) -> EngineWeights:
    """TransformerLens ``process_weights_`` (fold_ln → center_writing_weights →
    center_unembed → fold_value_biases) straight into the engine layout.
    ``free_source`` pops tensors from ``sd`` as it goes (bounds peak memory).
    ``raw16``: also keep the checkpoint's own GEMM weights as fp16 when every
    one of them is exact in fp16 (released Pythia checkpoints are float16):
    ``EngineWeights.raw16``, the operands of the exact-fp16 GEMMs."""
    dev = device if device is not None else sd["gpt_neox.embed_in.weight"].device

    def take(name):
        t = sd.pop(name) if free_source else sd[name]
        return t.to(dev, dtype)

    w_e = take("gpt_neox.embed_in.weight")
    w_e = (w_e - w_e.mean(dim=1, keepdim=True)).contiguous()
    layers, raw = [], ([] if raw16 else None)
    for l in range(cfg.n_layers):
        p = f"gpt_neox.layers.{l}."
        # with raw16 the raw tensors are read twice (the raw copy, then the processing): kept in sd until the
        # layer is done, then popped (free_source)
        keep = free_source and raw is not None
        layers.append(_process_layer(cfg, lambda n, p=p: _take_keep(sd, p + n, dev, dtype)
                                     if keep and n in _RAW_NAMES else take(p + n), raw))
        if keep:
            for n in _RAW_NAMES:
                sd.pop(p + n, None)
    wu_raw, gf = take("embed_out.weight"), take("gpt_neox.final_layer_norm.weight")
    raw_u = _raw_unembed(wu_raw, gf) if raw16 else None
    w_u, b_u = _process_unembed(wu_raw, gf, take("gpt_neox.final_layer_norm.bias"))
    raw = _raw_or_none(raw)
    return EngineWeights(w_e, layers, w_u, b_u, raw, raw_u if raw is not None else None)


@torch.no_grad()
def synth_engine_weights(cfg: PythiaConfig, seed: int = 0, device="cpu", std: float = 0.02,
                         ln_std: float = 0.1, fp16: bool = False) -> EngineWeights:
    """Generate + process layer by layer (peak memory ~1 layer of raw weights),
    the path used for the multi-GB configs on the GPU.  ``fp16``: every
    parameter fp16-valued, as in the released checkpoints; the raw GEMM
    weights are then kept too (``EngineWeights.raw16``)."""
    shapes = hf_param_shapes(cfg)

    def gen(name):
        return synth_param(cfg, name, shapes[name], seed, device, std, ln_std, fp16)

    w_e = gen("gpt_neox.embed_in.weight")
    w_e = (w_e - w_e.mean(dim=1, keepdim=True)).contiguous()
    layers, raw = [], ([] if fp16 else None)
    for l in range(cfg.n_layers):
        p = f"gpt_neox.layers.{l}."
        layers.append(_process_layer(cfg, lambda n, p=p: gen(p + n), raw))
    wu_raw, gf = gen("embed_out.weight"), gen("gpt_neox.final_layer_norm.weight")
    raw_u = _raw_unembed(wu_raw, gf) if fp16 else None
    w_u, b_u = _process_unembed(wu_raw, gf, gen("gpt_neox.final_layer_norm.bias"))
    raw = _raw_or_none(raw)
    return EngineWeights(w_e, layers, w_u, b_u, raw, raw_u if raw is not None else None)

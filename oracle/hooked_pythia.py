"""ORACLE (test infrastructure only) — TransformerLens HookedTransformer
semantics for Pythia on the CPU.

Follows the TL behaviour the reference depends on:
* ``from_pretrained`` defaults (scratch.py:26, scratch2.py:26): fold_ln,
  center_writing_weights, center_unembed, fold_value_biases;
* Pythia block: parallel residual, LayerNormPre, rotary (rotate-half) on the
  first rotary_dim dims of q/k, causal softmax, ``hook_result`` per head when
  ``cfg.use_attn_result`` (scratch2.py:85-86,176-177);
* hook points ``hook_embed``, ``blocks.{l}.hook_resid_pre``,
  ``blocks.{l}.attn.hook_z``, ``blocks.{l}.attn.hook_result``,
  ``blocks.{l}.hook_attn_out``, ``blocks.{l}.hook_mlp_out``,
  ``blocks.{l}.hook_resid_post``, ``ln_final.hook_normalized``;
* ``run_with_cache`` (scratch2.py:96, scratch.py:132,137), ``run_with_hooks``
  (scratch2.py:123,146,191,301,311), ``forward(resid, start_at_layer=L)``
  (scratch.py:143,206,209).
Weights are kept in TL's layout (W_Q [H, d, dh], W_O [H, dh, d], W_in [d, m],
W_U [d, V]) and processed here from the raw HF GPT-NeoX state dict, separately
from the product's fused layout.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch


@dataclass
class OracleConfig:
    n_layers: int
    d_model: int
    n_heads: int
    d_mlp: int
    d_vocab: int
    rotary_dim: int
    n_ctx: int = 2048
    eps: float = 1e-5
    rotary_base: float = 10000.0
    use_attn_result: bool = False

    @property
    def d_head(self) -> int:
        return self.d_model // self.n_heads


def tl_process_block(g: Callable[[str], torch.Tensor], cfg: OracleConfig) -> Dict[str, torch.Tensor]:
    """One block of TL process_weights_ (every step is per block):
    fold_ln (biases first, then weights, then centre the read-in weights over
    d_model) → center_writing_weights → fold_value_biases.  ``g(name)`` gives
    the block's HF parameter ``name`` (without the ``gpt_neox.layers.{l}.``
    prefix) as a fresh tensor in the working dtype."""
    d, H, dh = cfg.d_model, cfg.n_heads, cfg.d_head
    qkv = g("attention.query_key_value.weight").view(H, 3, dh, d)
    qkv_b = g("attention.query_key_value.bias").view(H, 3, dh)
    b = {
        "W_Q": qkv[:, 0].transpose(1, 2).contiguous(),  # [H, d, dh]
        "W_K": qkv[:, 1].transpose(1, 2).contiguous(),
        "W_V": qkv[:, 2].transpose(1, 2).contiguous(),
        "b_Q": qkv_b[:, 0].clone(), "b_K": qkv_b[:, 1].clone(), "b_V": qkv_b[:, 2].clone(),
        "W_O": g("attention.dense.weight").T.reshape(H, dh, d).contiguous(),
        "b_O": g("attention.dense.bias"),
        "W_in": g("mlp.dense_h_to_4h.weight").T.contiguous(),   # [d, m]
        "b_in": g("mlp.dense_h_to_4h.bias"),
        "W_out": g("mlp.dense_4h_to_h.weight").T.contiguous(),  # [m, d]
        "b_out": g("mlp.dense_4h_to_h.bias"),
    }
    ln1_w, ln1_b = g("input_layernorm.weight"), g("input_layernorm.bias")
    ln2_w, ln2_b = g("post_attention_layernorm.weight"), g("post_attention_layernorm.bias")
    # --- fold_ln ---
    for n in "QKV":
        b["b_" + n] = b["b_" + n] + (b["W_" + n] * ln1_b[None, :, None]).sum(-2)
        b["W_" + n] = b["W_" + n] * ln1_w[None, :, None]
        b["W_" + n] = b["W_" + n] - b["W_" + n].mean(-2, keepdim=True)
    b["b_in"] = b["b_in"] + (b["W_in"] * ln2_b[:, None]).sum(-2)
    b["W_in"] = b["W_in"] * ln2_w[:, None]
    b["W_in"] = b["W_in"] - b["W_in"].mean(-2, keepdim=True)
    # --- center_writing_weights ---
    b["W_O"] = b["W_O"] - b["W_O"].mean(-1, keepdim=True)
    b["b_O"] = b["b_O"] - b["b_O"].mean()
    b["W_out"] = b["W_out"] - b["W_out"].mean(-1, keepdim=True)
    b["b_out"] = b["b_out"] - b["b_out"].mean()
    # --- fold_value_biases ---
    b["b_O"] = b["b_O"] + (b["b_V"][:, :, None] * b["W_O"]).sum([0, 1])
    b["b_V"] = torch.zeros_like(b["b_V"])
    return b


def tl_process_embed(w_e: torch.Tensor) -> torch.Tensor:
    """center_writing_weights on W_E [V, d]."""
    return w_e - w_e.mean(-1, keepdim=True)


def tl_process_unembed(embed_out: torch.Tensor, lnf_w: torch.Tensor, lnf_b: torch.Tensor):
    """HF ``embed_out.weight`` [V, d] → TL (W_U [d, V], b_U [V]): fold_ln of
    ln_final, then center_unembed.  Pythia has no unembed bias (b_U = 0)."""
    w_u = embed_out.T.contiguous()
    b_u = torch.zeros(w_u.shape[1], dtype=w_u.dtype, device=w_u.device)
    b_u = b_u + (w_u * lnf_b[:, None]).sum(-2)
    w_u = w_u * lnf_w[:, None]
    w_u = w_u - w_u.mean(-2, keepdim=True)
    # --- center_unembed ---
    w_u = w_u - w_u.mean(-1, keepdim=True)
    b_u = b_u - b_u.mean()
    return w_u, b_u


def tl_process_weights(sd: Dict[str, torch.Tensor], cfg: OracleConfig, dtype=torch.float32):
    """HF GPT-NeoX state dict → TL state dict, then TL process_weights_:
    fold_ln → center_writing_weights → center_unembed → fold_value_biases
    (each step acts per block or on the embed / unembed alone)."""
    g = lambda k: sd[k].to(dtype).clone()  # noqa: E731
    blocks = [tl_process_block(lambda n, p=f"gpt_neox.layers.{l}.": g(p + n), cfg) for l in range(cfg.n_layers)]
    w_u, b_u = tl_process_unembed(g("embed_out.weight"), g("gpt_neox.final_layer_norm.weight"),
                                  g("gpt_neox.final_layer_norm.bias"))
    return {"W_E": tl_process_embed(g("gpt_neox.embed_in.weight")), "blocks": blocks, "W_U": w_u, "b_U": b_u}


def _cpu(x):
    if isinstance(x, dict):
        return {k: _cpu(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_cpu(v) for v in x]
    return x.cpu() if isinstance(x, torch.Tensor) else x


HookFn = Callable[[torch.Tensor, "HookPoint"], Optional[torch.Tensor]]


class HookPoint:
    def __init__(self, name: str):
        self.name = name


class ActivationCache(dict):
    pass


class HookedPythiaOracle:
    """Batch-1-oriented CPU model with TL hook semantics (works for any batch)."""

    def __init__(self, cfg: OracleConfig, hf_state_dict: Dict[str, torch.Tensor],
                 dtype=torch.float32, tokenizer=None, rotary_table_dtype=None):
        self.cfg = cfg
        self.dtype = dtype
        # TL computes sin / cos in fp32, or fp64 for an fp64 model; ``rotary_table_dtype=torch.float32``
        # evaluates the fp32 reference's tables in this (e.g. fp64) model (oracle/streamed_pythia.py)
        self._table_dtype = rotary_table_dtype
        # processed where the state dict lives (a GPU-resident one processes in
        # seconds), then kept on the CPU: the oracle always runs on the CPU
        self.w = _cpu(tl_process_weights(hf_state_dict, cfg, dtype))
        self.tokenizer = tokenizer
        self._hooks: Dict[str, List[HookFn]] = {}
        self._cache: Optional[ActivationCache] = None
        self._sin, self._cos = self._rotary_tables(cfg.rotary_dim, cfg.n_ctx, cfg.rotary_base)

    # --- TL calculate_sin_cos_rotary (non-adjacent pairs: repeat "(2 d)") ---
    def _rotary_tables(self, rd: int, n_ctx: int, base: float):
        hp = self._table_dtype or (torch.float64 if self.dtype == torch.float64 else torch.float32)
        pos = torch.arange(n_ctx, dtype=hp)
        dim = torch.arange(rd // 2, dtype=hp)
        freq = base ** (dim / (rd / 2))
        freq = torch.cat([freq, freq])
        angles = pos[:, None] / freq[None, :]
        return torch.sin(angles).to(self.dtype), torch.cos(angles).to(self.dtype)

    # ------------------------------------------------------------------ hooks
    def _hook(self, name: str, x: torch.Tensor) -> torch.Tensor:
        for fn in self._hooks.get(name, []):
            r = fn(x, HookPoint(name))
            if r is not None:
                x = r
        if self._cache is not None:
            self._cache[name] = x.detach().clone()
        return x

    # ------------------------------------------------------------- the model
    def _ln_pre(self, x: torch.Tensor) -> torch.Tensor:
        x = x - x.mean(-1, keepdim=True)
        scale = (x.pow(2).mean(-1, keepdim=True) + self.cfg.eps).sqrt()
        return x / scale

    def _rotate(self, x: torch.Tensor) -> torch.Tensor:
        # x [b, pos, head, dh]; TL apply_rotary (rotate_every_two, non-adjacent)
        rd = self.cfg.rotary_dim
        if rd == 0:
            return x
        T = x.shape[1]
        x_rot, x_pass = x[..., :rd], x[..., rd:]
        n = rd // 2
        flip = torch.cat([-x_rot[..., n:], x_rot[..., :n]], dim=-1)
        cos = self._cos[:T][None, :, None, :]
        sin = self._sin[:T][None, :, None, :]
        return torch.cat([x_rot * cos + flip * sin, x_pass], dim=-1)

    def _attn(self, l: int, x: torch.Tensor) -> torch.Tensor:
        b = self.w["blocks"][l]
        q = torch.einsum("bpd,hde->bphe", x, b["W_Q"]) + b["b_Q"]
        k = torch.einsum("bpd,hde->bphe", x, b["W_K"]) + b["b_K"]
        v = torch.einsum("bpd,hde->bphe", x, b["W_V"]) + b["b_V"]
        q, k = self._rotate(q), self._rotate(k)
        scores = torch.einsum("bqhe,bkhe->bhqk", q, k) / math.sqrt(self.cfg.d_head)
        T = x.shape[1]
        mask = torch.triu(torch.ones(T, T, dtype=torch.bool), diagonal=1)
        scores = scores.masked_fill(mask, float("-inf"))
        pattern = torch.softmax(scores, dim=-1)
        z = torch.einsum("bkhe,bhqk->bqhe", v, pattern)
        z = self._hook(f"blocks.{l}.attn.hook_z", z)
        if self.cfg.use_attn_result:
            result = torch.einsum("bqhe,hed->bqhd", z, b["W_O"])
            result = self._hook(f"blocks.{l}.attn.hook_result", result)
            return result.sum(-2) + b["b_O"]
        zf = z.reshape(z.shape[0], z.shape[1], -1)
        return zf @ b["W_O"].reshape(-1, self.cfg.d_model) + b["b_O"]

    def _block(self, l: int, resid: torch.Tensor) -> torch.Tensor:
        b = self.w["blocks"][l]
        resid = self._hook(f"blocks.{l}.hook_resid_pre", resid)
        attn_out = self._hook(f"blocks.{l}.hook_attn_out", self._attn(l, self._ln_pre(resid)))
        h = self._ln_pre(resid) @ b["W_in"] + b["b_in"]
        mlp_out = torch.nn.functional.gelu(h) @ b["W_out"] + b["b_out"]
        mlp_out = self._hook(f"blocks.{l}.hook_mlp_out", mlp_out)
        return self._hook(f"blocks.{l}.hook_resid_post", resid + attn_out + mlp_out)

    def to_tokens(self, text: str, prepend_bos: bool = True) -> torch.Tensor:
        ids = ([0] if prepend_bos else []) + self.tokenizer.encode(text)
        return torch.tensor([ids], dtype=torch.long)

    def to_single_token(self, text: str) -> int:
        ids = self.tokenizer.encode(text)
        assert len(ids) == 1, f"Input string: {text} is not a single token!"
        return ids[0]

    def to_string(self, tokens) -> str:
        if isinstance(tokens, torch.Tensor):
            tokens = tokens.tolist()
        if isinstance(tokens, int):
            return self.tokenizer.decode_one(tokens)
        return self.tokenizer.decode(tokens)

    @torch.no_grad()
    def forward(self, inp, start_at_layer: Optional[int] = None) -> torch.Tensor:
        """tokens [b, T] / [T] / str → logits [b, T, V]; or, with
        ``start_at_layer``, a residual [b, T, d] entering that block."""
        if start_at_layer is None:
            if isinstance(inp, str):
                inp = self.to_tokens(inp)
            if inp.dim() == 1:
                inp = inp[None]
            resid = self._hook("hook_embed", self.w["W_E"][inp])
            start = 0
        else:
            resid = inp.to(self.dtype)
            start = start_at_layer
        for l in range(start, self.cfg.n_layers):
            resid = self._block(l, resid)
        x = self._hook("ln_final.hook_normalized", self._ln_pre(resid))
        return x @ self.w["W_U"] + self.w["b_U"]

    __call__ = forward

    def run_with_cache(self, tokens) -> Tuple[torch.Tensor, ActivationCache]:
        self._cache = ActivationCache()
        try:
            logits = self.forward(tokens)
            return logits, self._cache
        finally:
            self._cache = None

    def run_with_hooks(self, tokens, fwd_hooks: Sequence[Tuple[str, HookFn]] = ()) -> torch.Tensor:
        for name, fn in fwd_hooks:
            self._hooks.setdefault(name, []).append(fn)
        try:
            return self.forward(tokens)
        finally:
            self._hooks.clear()

"""Pythia (GPT-NeoX) shapes and the engine configuration.

The reference loads models by name through TransformerLens
(``HookedTransformer.from_pretrained("pythia-410m")``, scratch.py:26;
``"gpt2-small"``, scratch2.py:26).  TransformerLens' Pythia config is
parallel-residual, rotary (rotate-half, ``rotary_pct`` 0.25), exact-erf GELU,
LN eps 1e-5.  This module names the shapes of the
Pythia family so a model can be built by name without a
network fetch.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field, replace


@dataclass
class PythiaConfig:
    n_layers: int
    d_model: int
    n_heads: int
    d_mlp: int
    d_vocab: int = 50304
    rotary_pct: float = 0.25
    n_ctx: int = 2048
    ln_eps: float = 1e-5
    rotary_base: float = 10000.0
    name: str = "custom"
    # TransformerLens compatibility flag toggled by the reference
    # (scratch2.py:85-86,176-177).  The engine always exposes per-head
    # results, so it has no effect here.
    use_attn_result: bool = field(default=False, compare=False)

    @property
    def d_head(self) -> int:
        return self.d_model // self.n_heads

    @property
    def rotary_dim(self) -> int:
        # TL / HF: int(d_head * rotary_pct)
        return int(self.d_head * self.rotary_pct)

    @property
    def n_params(self) -> int:
        d, m, L, V = self.d_model, self.d_mlp, self.n_layers, self.d_vocab
        per_layer = 4 * d * d + 4 * d + 2 * d * m + m + d + 4 * d
        return 2 * V * d + L * per_layer + 2 * d

    def flops_per_row_layer(self) -> int:
        """Matmul FLOPs of one residual row through one block (2 * P_l)."""
        d, m = self.d_model, self.d_mlp
        return 2 * (4 * d * d + 2 * d * m)

    def with_(self, **kw) -> "PythiaConfig":
        return replace(self, **kw)


PYTHIA_CONFIGS = {
    # name: (layers, d_model, heads, d_mlp, vocab)
    "pythia-70m": PythiaConfig(6, 512, 8, 2048, 50304, name="pythia-70m"),
    "pythia-160m": PythiaConfig(12, 768, 12, 3072, 50304, name="pythia-160m"),
    "pythia-410m": PythiaConfig(24, 1024, 16, 4096, 50304, name="pythia-410m"),
    "pythia-1b": PythiaConfig(16, 2048, 8, 8192, 50304, name="pythia-1b"),
    "pythia-1.4b": PythiaConfig(24, 2048, 16, 8192, 50304, name="pythia-1.4b"),
    "pythia-2.8b": PythiaConfig(32, 2560, 32, 10240, 50304, name="pythia-2.8b"),
    "pythia-6.9b": PythiaConfig(32, 4096, 32, 16384, 50432, name="pythia-6.9b"),
    "pythia-12b": PythiaConfig(36, 5120, 40, 20480, 50688, name="pythia-12b"),
    # test shape (2 layers, d 64, 4 heads, d_head 16, rotary 4)
    "tiny": PythiaConfig(2, 64, 4, 256, 512, n_ctx=256, name="tiny"),
}


def get_config(name: str) -> PythiaConfig:
    key = name.lower().replace("eleutherai/", "")
    if key.endswith("-deduped"):
        key = key[: -len("-deduped")]
    if key not in PYTHIA_CONFIGS:
        raise ValueError(f"unknown model {name!r}; known: {sorted(PYTHIA_CONFIGS)}")
    return replace(PYTHIA_CONFIGS[key])  # a private copy: callers toggle flags on it


class CConfig(ctypes.Structure):
    """Mirror of ``tvr_config`` (include/tvr.h)."""

    _fields_ = [
        ("n_layers", ctypes.c_int32),
        ("d_model", ctypes.c_int32),
        ("n_heads", ctypes.c_int32),
        ("d_head", ctypes.c_int32),
        ("d_mlp", ctypes.c_int32),
        ("d_vocab", ctypes.c_int32),
        ("rotary_dim", ctypes.c_int32),
        ("n_ctx", ctypes.c_int32),
        ("ln_eps", ctypes.c_float),
        ("rotary_base", ctypes.c_float),
    ]

    @classmethod
    def from_config(cls, cfg: PythiaConfig) -> "CConfig":
        return cls(cfg.n_layers, cfg.d_model, cfg.n_heads, cfg.d_head, cfg.d_mlp, cfg.d_vocab,
                   cfg.rotary_dim, cfg.n_ctx, cfg.ln_eps, cfg.rotary_base)

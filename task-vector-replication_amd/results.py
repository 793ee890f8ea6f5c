"""Checkpoint / resume of experiment stages.

The reference keeps ``mean_head_activations`` (scratch2.py:156) and
``causal_indirect_effect`` (scratch2.py:230) in notebook memory and reuses
them from later cells.  Here a stage's tensors are written to one
safetensors file (no pickle: loading executes nothing from the file) with a
small string metadata dict, so extraction, the CIE sweep and the FV
evaluation can rerun independently:

    save_results("letter_to_caps.safetensors", {"mean": mean, "cie": cie},
                 model="pythia-2.8b", n_contexts=2048)
    tensors, meta = load_results("letter_to_caps.safetensors", device="cuda")
"""
from __future__ import annotations

import json
from typing import Dict, Optional, Tuple

import torch
from safetensors.torch import load_file, save_file


def save_results(path: str, tensors: Dict[str, torch.Tensor], **meta) -> None:
    """Write ``tensors`` (any device; stored contiguous on the CPU) and
    JSON-serialisable ``meta`` to ``path``."""
    if not tensors:
        raise ValueError("nothing to save")
    cpu = {k: v.detach().to("cpu").contiguous() for k, v in tensors.items()}
    save_file(cpu, path, metadata={"tvr_meta": json.dumps(meta, sort_keys=True)})


def load_results(path: str, device: Optional[str] = None) -> Tuple[Dict[str, torch.Tensor], dict]:
    """(tensors, meta) as written by :func:`save_results`."""
    from safetensors import safe_open

    with safe_open(path, framework="pt") as f:
        raw = (f.metadata() or {}).get("tvr_meta", "{}")
    tensors = load_file(path, device=device or "cpu")
    return tensors, json.loads(raw)

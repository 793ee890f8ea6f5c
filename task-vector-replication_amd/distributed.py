"""Multi-GPU sharding (one process per GPU, torch.distributed; backend
"nccl" is RCCL over xGMI on ROCm, "gloo" for CPU tests).

The reference is single-device (scratch2.py:23).  The sweeps shard with no
data-path communication:
* CIE: every rank recomputes the clean run of its prompts and owns the sites
  with head ≡ rank (mod world) in every layer — this balances the staircase
  exactly, since each layer keeps H/world heads per rank — then one SUM
  all-reduce of the [L, H] fp32 partial sums (4-6 KB).
* Extraction: prompts split contiguously, local Σ z at the last position,
  one SUM all-reduce of [L, d] fp32 (z form: 0.33 MB for 2.8B), divide by the
  global count, project to the hook_result form.
* Weak-scaling bench: each rank sweeps its own prompts (prompts ≡ rank).
The compute step is injected (``local_fn``) so the partition + reduction logic
is testable on CPU ranks without a GPU.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def contiguous_shard(n: int, rank: int, size: int) -> Tuple[int, int]:
    """[start, stop) of rank's contiguous share of n items (sizes differ by ≤1)."""
    base, extra = divmod(n, size)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def strided_shard(n: int, rank: int, size: int) -> List[int]:
    """Items ≡ rank (mod size): the head split of the CIE sweep."""
    return list(range(rank, n, size))


def all_reduce_sum(t: torch.Tensor, group=None) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def sharded_cie(n_layers: int, n_heads: int, n_prompts: int,
                local_fn: Callable[[Sequence[int]], torch.Tensor], group=None) -> torch.Tensor:
    """CIE averaged over ``n_prompts`` with heads sharded round-robin.
    ``local_fn(heads)`` returns Σ_prompts Δp as [L, H] with zeros outside
    ``heads``."""
    rank, size = (dist.get_rank(group), dist.get_world_size(group)) if dist.is_initialized() else (0, 1)
    heads = strided_shard(n_heads, rank, size)
    part = local_fn(heads) if heads else None
    if part is None:
        raise ValueError("every rank needs at least one head (world size > n_heads)")
    return all_reduce_sum(part.clone(), group) / n_prompts


def sharded_mean_activation(prompts: Sequence[Sequence[int]],
                            local_fn: Callable[[Sequence[Sequence[int]]], torch.Tensor],
                            project: Callable[[torch.Tensor], torch.Tensor], group=None) -> torch.Tensor:
    """Mean hook_result over prompts, prompts split contiguously over ranks.
    ``local_fn(prompts)`` → Σ z [L, d]; ``project`` → [L, H, d]."""
    rank, size = (dist.get_rank(group), dist.get_world_size(group)) if dist.is_initialized() else (0, 1)
    a, b = contiguous_shard(len(prompts), rank, size)
    zsum = local_fn(prompts[a:b]).clone()
    zsum = all_reduce_sum(zsum, group)
    return project(zsum) / len(prompts)


def cie_heads_sharded(mean_head_activations, prompts, answers, model, group=None) -> torch.Tensor:
    """``calculate_average_causal_indirect_effect`` over token-id prompts on
    this rank's GPU with heads sharded across the process group."""
    from .experiments import causal_indirect_effect_sums
    return sharded_cie(model.cfg.n_layers, model.cfg.n_heads, len(prompts),
                       lambda heads: causal_indirect_effect_sums(mean_head_activations, prompts, answers,
                                                                 model, heads=heads), group)


def mean_activation_sharded(prompts, model, group=None) -> torch.Tensor:
    """``generate_mean_activation`` over pre-built prompts, prompt-sharded."""
    from .experiments import sum_last_z
    return sharded_mean_activation(prompts, lambda ps: sum_last_z(model, ps), model.project_heads, group)

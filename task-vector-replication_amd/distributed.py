"""Multi-GPU sharding (one process per GPU, torch.distributed; backend
"nccl" is RCCL over xGMI on ROCm, "gloo" for CPU tests).

The reference is single-device (scratch2.py:23).  Every sweep shards with no
data-path communication and ONE collective at the end; the
model is replicated per GPU (2.8B fp32 11 GB, 12B 47 GB << 288 GB):

* CIE (scratch2.py:181-194): every rank recomputes the clean run of the
  prompts and owns a balanced block of (layer, head) sites
  (``balanced_site_shard``): the staircase work of a site at layer l is the
  L - 1 - l blocks after it, so the layer pairs (l, L-1-l) all weigh the same;
  whole pairs are dealt round-robin and the pairs left over (and the middle
  layer of an odd L) are split by head (h = rank mod world).  Exact balance
  whenever world divides H, and each rank's sites fill whole layers, so its
  staircase GEMMs keep the single-GPU row counts (large M, whole 256-row
  tiles) instead of 1/world of them at every layer — then one SUM all-reduce
  of the [L, H] partial sums (4-6 KB).
* Extraction (scratch2.py:87-98): prompts split contiguously, local Σ z at
  the last position, one SUM all-reduce of [L, d] fp32 (z form: 0.33 MB for
  2.8B), divide by the global count, project to the hook_result form.
* Injection sweeps (layer sweeps scratch2.py:118-125,141-148; FV evaluation
  :295-313 and the head-count grid :420-424): the (prompt, layer / vector)
  sites round-robin over ranks (site i on rank i mod world), then one
  all_gather of the per-site outputs (probability, top-k ids), so every rank
  holds every site in global order and finishes the reduction identically.
The compute step is injected (``local_fn``) in the generic helpers so the
partition + collective logic is testable on CPU ranks without a GPU.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def world(group=None) -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def contiguous_shard(n: int, rank: int, size: int) -> Tuple[int, int]:
    """[start, stop) of rank's contiguous share of n items (sizes differ by ≤1)."""
    base, extra = divmod(n, size)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def strided_shard(n: int, rank: int, size: int) -> List[int]:
    """Items ≡ rank (mod size): the head split of the CIE sweep and the site
    split of the injection sweeps."""
    return list(range(rank, n, size))


def all_reduce_sum(t: torch.Tensor, group=None) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def gather_strided(part: torch.Tensor, n: int, group=None) -> torch.Tensor:
    """Inverse of ``strided_shard``: every rank passes its items' rows
    (``part`` [len(strided_shard(n, rank, size)), ...]) and gets all n rows in
    global order.  One all_gather of equal-size (padded) buffers."""
    rank, size = world(group)
    if size == 1:
        return part
    cap = -(-n // size)
    buf = part.new_zeros((cap,) + tuple(part.shape[1:]))
    buf[: part.shape[0]] = part
    parts = [torch.empty_like(buf) for _ in range(size)]
    dist.all_gather(parts, buf, group=group)
    out = part.new_empty((n,) + tuple(part.shape[1:]))
    for r, p in enumerate(parts):
        ids = strided_shard(n, r, size)
        if ids:
            out[torch.as_tensor(ids, device=out.device)] = p[: len(ids)]
    return out


class SiteShard:
    """Round-robin site partition of one sweep (site i on rank i mod world)
    plus the all_gather that reassembles the per-site outputs; passed as
    ``shard=`` to the injection-sweep helpers of experiments.py."""

    def __init__(self, group=None):
        self.group = group
        self.rank, self.size = world(group)

    def select(self, n_sites: int) -> List[int]:
        return strided_shard(n_sites, self.rank, self.size)

    def gather(self, part: torch.Tensor, n_sites: int) -> torch.Tensor:
        return gather_strided(part, n_sites, self.group)


def sharded_site_outputs(n_sites: int, local_fn: Callable[[Sequence[int]], torch.Tensor], group=None) -> torch.Tensor:
    """Per-site outputs of a sweep with sites round-robin over ranks:
    ``local_fn(site_ids)`` → [len(site_ids), ...] (an empty list gives an
    empty tensor of the same trailing shape); returns [n_sites, ...]."""
    shard = SiteShard(group)
    return shard.gather(local_fn(shard.select(n_sites)), n_sites)


def balanced_site_shard(n_layers: int, n_heads: int, rank: int, size: int) -> List[Tuple[int, int]]:
    """The CIE sites (layer, head) of ``rank``: layer pairs (l, L-1-l) dealt
    round-robin as whole pairs (every head), the remaining pairs and an odd
    L's middle layer split by head (h = rank mod size).  Every site exactly
    once over the ranks; equal staircase work per rank when size | H."""
    pairs = [(l, n_layers - 1 - l) for l in range(n_layers // 2)]
    whole = len(pairs) // size
    out = [(l, h) for p in range(whole * size) if p % size == rank for l in pairs[p] for h in range(n_heads)]
    rest = [l for p in pairs[whole * size:] for l in p] + ([n_layers // 2] if n_layers % 2 else [])
    out += [(l, h) for l in rest for h in strided_shard(n_heads, rank, size)]
    return sorted(out)


def sharded_cie(n_layers: int, n_heads: int, n_prompts: int,
                local_fn: Callable[[Sequence[Tuple[int, int]]], torch.Tensor], zeros: Callable[[], torch.Tensor],
                group=None) -> torch.Tensor:
    """CIE averaged over ``n_prompts`` with the sites split by
    ``balanced_site_shard``.  ``local_fn(sites)`` returns Σ_prompts Δp as
    [L, H] with zeros outside ``sites``; ``zeros()`` is a rank's empty share."""
    rank, size = world(group)
    sites = balanced_site_shard(n_layers, n_heads, rank, size)
    part = local_fn(sites).clone() if sites else zeros()
    return all_reduce_sum(part, group) / n_prompts


def sharded_mean_activation(prompts: Sequence[Sequence[int]],
                            local_fn: Callable[[Sequence[Sequence[int]]], Optional[torch.Tensor]],
                            project: Callable[[torch.Tensor], torch.Tensor], zeros: Callable[[], torch.Tensor],
                            group=None) -> torch.Tensor:
    """Mean hook_result over prompts, prompts split contiguously over ranks.
    ``local_fn(prompts)`` → Σ z [L, d]; ``zeros()`` → the [L, d] zero sum of
    a rank with no prompts; ``project`` → [L, H, d]."""
    rank, size = world(group)
    a, b = contiguous_shard(len(prompts), rank, size)
    zsum = local_fn(prompts[a:b]).clone() if b > a else zeros()
    zsum = all_reduce_sum(zsum, group)
    return project(zsum) / len(prompts)


# ------------------------------------------------------------ engine entry points
def cie_sharded(mean_head_activations, scrambled_prompts, prompt_answers, model, group=None) -> torch.Tensor:
    """``calculate_average_causal_indirect_effect`` (scratch2.py:171-197) on
    this rank's GPU with the (layer, head) sites split across the process
    group (``balanced_site_shard``).  Accepts the reference's forms: string
    prompts (BOS prepended) or token ids, answers as token-id lists (first
    token, B3) or ints."""
    from .experiments import causal_indirect_effect_sums, normalize_cie_inputs
    cfg = model.cfg
    if tuple(mean_head_activations.shape) != (cfg.n_layers, cfg.n_heads, cfg.d_model):
        raise ValueError("Mean head activations must be of shape (n_layers, n_heads, d_model)")
    if len(scrambled_prompts) != len(prompt_answers):
        raise ValueError("Prompt answers must be of the same length as scrambled prompts")
    prompts, answers = normalize_cie_inputs(model, scrambled_prompts, prompt_answers)
    return sharded_cie(cfg.n_layers, cfg.n_heads, len(prompts),
                       lambda sites: causal_indirect_effect_sums(mean_head_activations, prompts, answers,
                                                                 model, sites=sites),
                       lambda: torch.zeros(cfg.n_layers, cfg.n_heads, device=model.device), group)


cie_heads_sharded = cie_sharded  # the round-3 name


def mean_activation_sharded(prompts, model, group=None) -> torch.Tensor:
    """``generate_mean_activation`` over pre-built prompts, prompt-sharded."""
    from .experiments import sum_last_z
    cfg = model.cfg
    return sharded_mean_activation(prompts, lambda ps: sum_last_z(model, ps), model.project_heads,
                                   lambda: torch.zeros(cfg.n_layers, cfg.d_model, device=model.device), group)


def apply_layered_vectors_to_zero_shot_sharded(layered_vectors, contexts, function_token, model,
                                               reference_late_binding: bool = True, group=None):
    """``apply_layered_vectors_to_zero_shot`` (scratch2.py:114-127) with the
    (prompt, layer) sites round-robin over ranks; every rank returns the full
    per-layer accuracy list."""
    from .experiments import _zero_shot_accuracy
    return _zero_shot_accuracy(layered_vectors, contexts, function_token, model, reference_late_binding,
                               SiteShard(group))


def apply_layered_vectors_to_zero_shot_by_probability_sharded(layered_vectors, contexts, function_token, model,
                                                              reference_late_binding: bool = True, group=None):
    """``apply_layered_vectors_to_zero_shot_by_probability`` (scratch2.py:135-150),
    sites round-robin over ranks."""
    from .experiments import _zero_shot_dprob
    return _zero_shot_dprob(layered_vectors, contexts, function_token, model, reference_late_binding,
                            SiteShard(group))


def check_accuracy_of_added_task_vector_by_layer_sharded(task_vector, contexts, topk: int, model, group=None):
    """The FV top-k accuracy at every layer (scratch2.py:306-314 per layer),
    sites round-robin over ranks."""
    from .experiments import check_accuracy_of_added_task_vector_by_layer
    return check_accuracy_of_added_task_vector_by_layer(task_vector, contexts, topk, model, shard=SiteShard(group))


def function_vector_head_count_grid_sharded(mean_head_activations, causal_indirect_effects, contexts, model,
                                            heads_per_batch: int = 2, number_of_batches: int = 64, topk: int = 5,
                                            group=None):
    """The FV head-count grid (scratch2.py:411-425), sites round-robin over ranks."""
    from .experiments import function_vector_head_count_grid
    return function_vector_head_count_grid(mean_head_activations, causal_indirect_effects, contexts, model,
                                           heads_per_batch, number_of_batches, topk, shard=SiteShard(group))

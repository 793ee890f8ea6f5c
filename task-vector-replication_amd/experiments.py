"""The reference's experiment entry points, same names and signatures,
executed as batched sweeps on the HIP engine.

Each function replaces a Python loop of batch-1 TransformerLens forwards
(one per prompt x patch site) with one clean-forward launch sequence and one
patch-sweep launch sequence whose batch enumerates the sites:

  generate_mean_activation                     scratch2.py:81-100   (a1)
  gather_head_activations_to_layers            scratch2.py:103-104  (a2)
  apply_layered_vectors_to_zero_shot           scratch2.py:114-127  (a3, a4)
  apply_layered_vectors_to_zero_shot_by_probability  scratch2.py:135-150 (a5)
  calculate_average_causal_indirect_effect     scratch2.py:171-197  (a6, a7)
  assemble_task_vector                         scratch2.py:232-238  (a10)
  logits_to_next_k_tokens, check_accuracy_of_task_vector,
  check_accuracy_of_added_task_vector          scratch2.py:278-314  (a11)
  test_component_hypothesis                    scratch.py:106-147   (a12)
  substitute_task                              scratch.py:164-213

Drop-in notes
* ``model`` is an ``amd.Model`` instead of a HookedTransformer; it must be
  passed (the reference's defaults bind a module-global model).
* Late-binding closure (App. B1): the reference's layer sweeps add
  ``layered_vectors[-1]`` at every layer.  ``reference_late_binding=True``
  (default) reproduces that; ``False`` adds ``layered_vectors[i]`` at layer i.
* Accuracy compares decoded strings exactly as the reference (B5).
* ``assemble_task_vector`` accepts device tensors (the reference's
  ``.numpy()`` needs CPU tensors, B9).
"""
from __future__ import annotations

import random
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .model import Model, make_sites, range_checked
from .prompts import (Pairs, assemble_end_list_tasks, construct_query, generate_shuffled_prompt,  # noqa: F401
                      generate_shuffled_prompts, icl_multi_token, icl_single_token, sample_icl_prompts)

# Sites per patch_sweep launch (bounds the activation workspace: a CIE site
# of a T-token prompt holds T rows).
MAX_SITES_PER_LAUNCH = 16384
# Prompts per clean-forward launch during extraction.
EXTRACT_BATCH = 2048


def _chunks(n: int, size: int):
    """[a, b) ranges of at most ``size`` covering range(n), as equal as
    possible (12 prompts at 11 per launch run as 6 + 6, not 11 + 1: a
    1-prompt launch shares no prefix rows and runs small GEMMs)."""
    if n <= 0:
        return
    k = -(-n // size)
    for i in range(k):
        yield i * n // k, (i + 1) * n // k


# ------------------------------------------------------------------ a1 / a2
@range_checked
def generate_mean_activation(contexts: Pairs, function_token: str, seperator_token: str = ",",
                             model: Model = None, num_contexts: int = 1024, len_contexts: int = 4
                             ) -> torch.Tensor:
    """Mean over ``num_contexts`` ICL prompts of ``blocks.{l}.attn.hook_result``
    at the last position, for every layer and head: [n_layers, n_heads, d_model].
    Captured in z form on the GPU and projected once (mean is linear)."""
    prompts = sample_icl_prompts(model, contexts, function_token, seperator_token, num_contexts,
                                 len_contexts)
    return model.project_heads(sum_last_z(model, prompts)) / num_contexts


@range_checked
def sum_last_z(model: Model, prompts: Sequence[Sequence[int]]) -> torch.Tensor:
    """Σ over prompts of hook_z at the last position, [L, d] (fp32, device)."""
    total = None
    for a, b in _chunks(len(prompts), EXTRACT_BATCH):
        z = model.forward_clean(prompts[a:b], capture=True)["zsum"]
        total = z if total is None else total + z
    return total


def gather_head_activations_to_layers(mean_head_activations: torch.Tensor) -> torch.Tensor:
    return mean_head_activations.sum(1)


# ------------------------------------------------------------- a3 / a4 / a5
def _layer_vectors(layered_vectors: torch.Tensor, model: Model, late_binding: bool):
    v = layered_vectors.to(model.device, torch.float32)
    if late_binding:
        return v[-1:].contiguous(), lambda layer: 0
    if v.shape[0] != model.cfg.n_layers:
        raise ValueError("layered_vectors must have one row per layer")
    return v.contiguous(), lambda layer: layer


def _add_site_outputs(model: Model, seqs: List[List[int]], site_seq, site_layer, site_vec, vectors: torch.Tensor,
                      targets: Optional[List[int]], topk: int, shard=None, clean_outputs: bool = True):
    """Clean forward of ``seqs`` + the ADD_ATTN_OUT_LASTPOS sites
    (``hook_attn_out[0, -1] += vectors[vec]`` at ``layer``, scratch2.py:107-109)
    of the global site list (site_seq, site_layer, site_vec).  ``shard``
    (distributed.SiteShard) evaluates only this rank's sites and all-gathers
    the per-site outputs, so every rank returns every site in global order.
    ``clean_outputs=False``: the caller reads no clean outputs, so the clean
    rows skip their final LayerNorm + unembed statistics.
    Returns (clean outputs per prompt, patched outputs per site)."""
    n_sites = len(site_seq)
    sel = np.arange(n_sites) if shard is None else np.asarray(shard.select(n_sites), dtype=np.int64)
    trace = model._sweep_trace(len(seqs), sum(len(s) for s in seqs))
    # the clean rows run inside the first sweep launch when there is one
    clean = model.forward_clean(seqs, targets=targets if clean_outputs else None, topk=topk if clean_outputs else 0,
                                trace=trace, defer=len(sel) > 0)
    dev = model.device
    patched = {}
    if targets is not None:
        patched["prob"] = [torch.empty(0, device=dev)]
    if topk:
        patched["topk"] = [torch.empty(0, topk, dtype=torch.int32, device=dev)]
    if len(sel):
        patched = {k: [] for k in patched}
        sites = make_sites(len(sel))
        sites["kind"] = _lib.SITE_ADD_ATTN_OUT_LASTPOS
        sites["seq"] = np.asarray(site_seq)[sel]
        sites["layer"] = np.asarray(site_layer)[sel]
        sites["vec"] = np.asarray(site_vec)[sel]
        if targets is not None:
            sites["target"] = np.asarray(targets)[sites["seq"]]
        for a, b in _chunks(len(sites), MAX_SITES_PER_LAUNCH):
            out = model.patch_sweep(trace, sites[a:b], vectors, topk=topk, want_prob=targets is not None)
            for k in patched:
                patched[k].append(out[k])
    patched = {k: torch.cat(v) for k, v in patched.items()}
    if shard is not None:
        patched = {k: shard.gather(v, n_sites) for k, v in patched.items()}
    return clean, patched


def _injection_sweep(model: Model, seqs: List[List[int]], vectors: torch.Tensor, vec_of_layer,
                     layers: Sequence[int], targets: Optional[List[int]], topk: int, shard=None,
                     clean_outputs: bool = True):
    """One ADD_ATTN_OUT_LASTPOS site per (prompt, layer).  Returns (clean
    outputs, patched outputs [n, len(layers)])."""
    n, layers = len(seqs), list(layers)
    site_layer = np.tile(np.asarray(layers, dtype=np.int32), n)
    site_vec = np.tile(np.asarray([vec_of_layer(l) for l in layers], dtype=np.int32), n)
    clean, patched = _add_site_outputs(model, seqs, np.repeat(np.arange(n, dtype=np.int32), len(layers)), site_layer,
                                       site_vec, vectors, targets, topk, shard, clean_outputs)
    return clean, {k: v.view(n, len(layers), *v.shape[1:]) for k, v in patched.items()}


@range_checked
def _zero_shot_accuracy(layered_vectors, contexts: Pairs, function_token: str, model: Model,
                        reference_late_binding: bool, shard=None) -> List[float]:
    L = model.cfg.n_layers
    vectors, vec_of = _layer_vectors(layered_vectors, model, reference_late_binding)
    f = model.to_single_token(function_token)
    seqs = [[0, model.to_single_token(x), f] for x, _ in contexts]
    _, patched = _injection_sweep(model, seqs, vectors, vec_of, range(L), None, 1, shard, clean_outputs=False)
    # top-1 decoded == answer (scratch2.py's to_string comparison), decoding
    # each distinct token id once instead of once per (prompt, layer)
    ids, inv = np.unique(patched["topk"][..., 0].cpu().numpy(), return_inverse=True)
    words = [model.to_string(int(t)) for t in ids]
    want = {y: i for i, y in enumerate(dict.fromkeys(y for _, y in contexts))}
    eq = np.array([[w == y for y in want] for w in words], dtype=bool).reshape(len(ids), len(want))
    col = np.asarray([want[y] for _, y in contexts])
    hits = eq[inv.reshape(len(contexts), L), col[:, None]].sum(0)
    return [1.0 * int(h) / len(contexts) for h in hits]


@range_checked
def _zero_shot_dprob(layered_vectors, contexts: Pairs, function_token: str, model: Model,
                     reference_late_binding: bool, shard=None) -> torch.Tensor:
    L = model.cfg.n_layers
    vectors, vec_of = _layer_vectors(layered_vectors, model, reference_late_binding)
    f = model.to_single_token(function_token)
    enc = model.tokenizer.encode
    seqs = [[0] + enc(x) + [f] for x, _ in contexts]
    targets = [enc(y)[0] for _, y in contexts]
    clean, patched = _injection_sweep(model, seqs, vectors, vec_of, range(L), targets, 0, shard)
    return (patched["prob"] - clean["prob"][:, None]).sum(0) / len(contexts)


@range_checked
def apply_layered_vectors_to_zero_shot(layered_vectors: torch.Tensor, contexts: Pairs, function_token: str,
                                       model: Model = None, reference_late_binding: bool = True) -> List[float]:
    """Per-layer top-1 accuracy of zero-shot ``[BOS, x, f]`` prompts with a
    vector added to ``hook_attn_out[0, -1]`` at that layer."""
    return _zero_shot_accuracy(layered_vectors, contexts, function_token, model, reference_late_binding)


@range_checked
def apply_layered_vectors_to_zero_shot_by_probability(layered_vectors: torch.Tensor, contexts: Pairs,
                                                      function_token: str, model: Model = None,
                                                      reference_late_binding: bool = True) -> torch.Tensor:
    """Per-layer mean change of the first answer token's probability
    (patched − clean), [n_layers] on the device."""
    return _zero_shot_dprob(layered_vectors, contexts, function_token, model, reference_late_binding)


# ------------------------------------------------------------------- a6 / a7
def normalize_cie_inputs(model: Model, scrambled_prompts, prompt_answers):
    """The reference's prompt / answer forms → token-id prompts (BOS
    prepended to strings by ``to_tokens``, scratch2.py:182) and first answer
    token ids (``[answer][0]``, scratch2.py:184,192: B3)."""
    prompts = [model.to_tokens(p)[0].tolist() if isinstance(p, str) else [int(x) for x in p]
               for p in scrambled_prompts]
    answers = [int(a[0]) if isinstance(a, (list, tuple)) else int(a) for a in prompt_answers]
    return prompts, answers


@range_checked
def causal_indirect_effect_sums(mean_head_activations: torch.Tensor, prompts: Sequence[Sequence[int]],
                                answers: Sequence[int], model: Model,
                                layers: Optional[Sequence[int]] = None,
                                heads: Optional[Sequence[int]] = None,
                                sites: Optional[Sequence[Tuple[int, int]]] = None) -> torch.Tensor:
    """Σ over prompts of p_patched(answer) − p_clean(answer) for every
    (layer, head) site, [n_layers, n_heads] (zeros outside ``layers``/``heads``,
    or outside the explicit (layer, head) list ``sites``).
    ``prompts`` are token ids (BOS included); one clean forward + one
    staircase sweep per launch-sized group of prompts."""
    cfg = model.cfg
    L, H = cfg.n_layers, cfg.n_heads
    if sites is not None:
        if layers is not None or heads is not None:
            raise ValueError("give either sites or layers / heads")
        sl = np.asarray(sites, dtype=np.int32).reshape(-1, 2)
        if sl.size and (sl[:, 0].min() < 0 or sl[:, 0].max() >= L or sl[:, 1].min() < 0 or sl[:, 1].max() >= H):
            raise ValueError("site (layer, head) out of range")
        grid_l, grid_h = sl[:, 0].copy(), sl[:, 1].copy()
    else:
        layers = list(range(L)) if layers is None else list(layers)
        heads = list(range(H)) if heads is None else list(heads)
        grid_l = np.repeat(np.asarray(layers, dtype=np.int32), len(heads))
        grid_h = np.tile(np.asarray(heads, dtype=np.int32), len(layers))
    per_prompt = grid_l.size
    vectors = mean_head_activations.to(model.device, torch.float32).reshape(L * H, cfg.d_model).contiguous()
    out = torch.zeros(L, H, device=model.device)
    group = max(1, MAX_SITES_PER_LAUNCH // max(per_prompt, 1))
    for a, b in _chunks(len(prompts), group):
        seqs = [list(map(int, p)) for p in prompts[a:b]]
        tg = [int(t) for t in answers[a:b]]
        n = len(seqs)
        trace = model._sweep_trace(n, sum(len(s) for s in seqs))
        p0 = model.forward_clean(seqs, targets=tg, trace=trace, defer=per_prompt > 0)["prob"]
        sites = make_sites(n * per_prompt)
        sites["seq"] = np.repeat(np.arange(n, dtype=np.int32), per_prompt)
        sites["kind"] = _lib.SITE_REPLACE_HEAD_ALLPOS
        sites["layer"] = np.tile(grid_l, n)
        sites["head"] = np.tile(grid_h, n)
        sites["vec"] = sites["layer"] * H + sites["head"]
        sites["target"] = np.repeat(np.asarray(tg, dtype=np.int32), per_prompt)
        p = model.patch_sweep(trace, sites, vectors)["prob"].view(n, per_prompt)
        delta = (p - p0[:, None]).sum(0)
        out.index_put_((torch.as_tensor(grid_l, device=model.device).long(),
                        torch.as_tensor(grid_h, device=model.device).long()), delta, accumulate=True)
    return out


@range_checked
def calculate_average_causal_indirect_effect(mean_head_activations: torch.Tensor, scrambled_prompts,
                                             prompt_answers, model: Model = None) -> torch.Tensor:
    """CIE[l, h] = mean over prompts of softmax(patched)[answer[0]] −
    softmax(clean)[answer[0]], where the patch writes ``mean[l, h]`` into
    ``hook_result[0, :, h]`` at every position.  [n_layers, n_heads]."""
    cfg = model.cfg
    if tuple(mean_head_activations.shape) != (cfg.n_layers, cfg.n_heads, cfg.d_model):
        raise ValueError("Mean head activations must be of shape (n_layers, n_heads, d_model)")
    if len(scrambled_prompts) != len(prompt_answers):
        raise ValueError("Prompt answers must be of the same length as scrambled prompts")
    prompts, answers = normalize_cie_inputs(model, scrambled_prompts, prompt_answers)
    return causal_indirect_effect_sums(mean_head_activations, prompts, answers, model) / len(prompts)


# ---------------------------------------------------------------- a10 / a11
def assemble_task_vector(mean_head_activations: torch.Tensor, causal_indirect_effects: torch.Tensor,
                         layer: int, num_heads: int) -> torch.Tensor:
    """Sum of the mean outputs of the ``num_heads`` highest-CIE heads in
    layers ≤ ``layer`` (torch.topk order and tie rule, as the reference)."""
    sub = causal_indirect_effects[: layer + 1, :]
    _, idx = torch.topk(sub.flatten(), num_heads)
    H = sub.shape[1]
    rows = mean_head_activations[(idx // H).to(mean_head_activations.device),
                                 (idx % H).to(mean_head_activations.device)]
    vec = torch.zeros(mean_head_activations.shape[-1], dtype=mean_head_activations.dtype,
                      device=mean_head_activations.device)
    for r in rows:  # sequential adds, the reference's summation order
        vec += r
    return vec


def logits_to_next_k_tokens(k: int, logits: torch.Tensor, model: Model = None) -> List[str]:
    return [model.to_string(e) for e in torch.topk(logits[0, -1, :], k).indices.tolist()]


def _fv_topk(task_vector, layer: int, contexts: Pairs, topk: int, model: Model, with_baseline: bool):
    seqs = [model.to_tokens(x + ":")[0].tolist() for x, _ in contexts]
    firsts = [model.to_string(model.tokenizer.encode(y)[0]) for _, y in contexts]
    vec = task_vector.to(model.device, torch.float32).reshape(1, -1).contiguous()
    clean, patched = _injection_sweep(model, seqs, vec, lambda l: 0, [layer], None, topk=topk,
                                      clean_outputs=with_baseline)
    def hits(top):
        return sum(first in [model.to_string(t) for t in row] for first, row in zip(firsts, top.tolist()))
    fv = hits(patched["topk"][:, 0].cpu())
    base = hits(clean["topk"].cpu()) if with_baseline else None
    return base, fv


@range_checked
def check_accuracy_of_task_vector(task_vector: torch.Tensor, layer: int, contexts: Pairs, topk: int = 5,
                                  model: Model = None) -> Tuple[float, float]:
    """(zero-shot top-k accuracy, top-k accuracy with the FV added to
    ``hook_attn_out[0, -1]`` at ``layer``) for prompts ``x + ":"``."""
    base, fv = _fv_topk(task_vector, layer, contexts, topk, model, True)
    return (1.0 * base / len(contexts), 1.0 * fv / len(contexts))


@range_checked
def check_accuracy_of_added_task_vector(task_vector: torch.Tensor, layer: int, contexts: Pairs, topk: int = 5,
                                        model: Model = None) -> float:
    _, fv = _fv_topk(task_vector, layer, contexts, topk, model, False)
    return 1.0 * fv / len(contexts)


# ---------------------------------------------------------------------- a12
@range_checked
def test_component_hypothesis(contexts: Pairs, function_token: str, model: Model = None,
                              num_contexts: int = 256, len_contexts: int = 4, batch_contexts: int = 512):
    """Layer sweep of residual patching: the ICL run's ``hook_resid_pre[L][-2]``
    written into a dummy-query run, continued from layer L.  Returns
    (total, baseline hits, regular hits, [hits per layer])."""
    L = model.cfg.n_layers
    pool = list(contexts)
    draws = []
    for _ in range(num_contexts):
        random.shuffle(pool)
        demos, query = pool[:len_contexts], pool[len_contexts]
        draws.append((demos, query, pool[len_contexts + 1][0]))
    base_hits = normal_hits = 0
    per_layer = [0] * L
    for a, b in _chunks(len(draws), batch_contexts):
        seqs, answers = [], []
        for demos, query, dummy in draws[a:b]:
            seqs.append(model.to_tokens(construct_query(query, function_token)[0])[0].tolist())
            seqs.append(icl_single_token(model, demos, query[0], function_token, None))
            seqs.append(icl_single_token(model, demos, dummy, function_token, None))
            answers.append(query[1])
        n = len(answers)
        trace = model._sweep_trace(3 * n, sum(len(s) for s in seqs))
        top = model.forward_clean(seqs, topk=1, trace=trace)["topk"][:, 0].cpu().view(n, 3).tolist()
        sites = make_sites(n * L)
        T = np.asarray([len(seqs[3 * i + 2]) for i in range(n)], dtype=np.int32)
        sites["kind"] = _lib.SITE_SET_RESID_PRE_POS
        sites["seq"] = np.repeat(3 * np.arange(n) + 2, L)
        sites["src_seq"] = np.repeat(3 * np.arange(n) + 1, L)
        sites["pos"] = np.repeat(T - 2, L)
        sites["src_pos"] = np.repeat(T - 2, L)
        sites["layer"] = np.tile(np.arange(L), n)
        pt = model.patch_sweep(trace, sites, None, topk=1, want_prob=False)["topk"][:, 0].cpu().view(n, L).tolist()
        for i, ans in enumerate(answers):
            base_hits += model.to_string(top[i][0]) == ans
            normal_hits += model.to_string(top[i][1]) == ans
            for l in range(L):
                per_layer[l] += model.to_string(pt[i][l]) == ans
    return (num_contexts, base_hits, normal_hits, per_layer)


@range_checked
def substitute_task(taskA: Pairs, taskB: Pairs, layer: int, function_token: str = "→", model: Model = None,
                    num_contexts: int = 256, len_contexts: int = 4):
    """Swap ``hook_resid_pre[layer][-1]`` between a task-A and a task-B run of
    the same query.  Returns (n, A hits, B hits, A←B hits on B's answer,
    B←A hits on A's answer).  Sorts both task lists in place (App. B6)."""
    if len(taskA) != len(taskB):
        raise ValueError("The two tasks must have the same length")
    taskA.sort(key=lambda p: p[0])
    taskB.sort(key=lambda p: p[0])
    if any(a[0] != b[0] for a, b in zip(taskA, taskB)):
        raise ValueError("The two tasks must have the same domains")
    mixed = [(a[0], a[1], b[1]) for a, b in zip(taskA, taskB)]
    seqs, ans = [], []
    for _ in range(num_contexts):
        random.shuffle(mixed)
        ctx_a = [(m[0], m[1]) for m in mixed[:len_contexts]]
        ctx_b = [(m[0], m[2]) for m in mixed[:len_contexts]]
        q = mixed[len_contexts][0][0]  # first character of the query item, as scratch.py:189
        seqs.append(icl_single_token(model, ctx_a, q, function_token, None))
        seqs.append(icl_single_token(model, ctx_b, q, function_token, None))
        ans.append((mixed[len_contexts][1], mixed[len_contexts][2]))
    n = num_contexts
    trace = model._sweep_trace(2 * n, sum(len(s) for s in seqs))
    top = model.forward_clean(seqs, topk=1, trace=trace)["topk"][:, 0].cpu().view(n, 2).tolist()
    sites = make_sites(2 * n)
    T = np.asarray([len(s) for s in seqs], dtype=np.int32)
    sites["kind"] = _lib.SITE_SET_RESID_PRE_POS
    sites["layer"] = layer
    sites["seq"] = np.arange(2 * n)
    sites["src_seq"] = np.arange(2 * n) ^ 1  # A takes B's row, B takes A's
    sites["pos"] = T - 1
    sites["src_pos"] = T[np.arange(2 * n) ^ 1] - 1
    pt = model.patch_sweep(trace, sites, None, topk=1, want_prob=False)["topk"][:, 0].cpu().view(n, 2).tolist()
    a_hits = sum(model.to_string(top[i][0]) == ans[i][0] for i in range(n))
    b_hits = sum(model.to_string(top[i][1]) == ans[i][1] for i in range(n))
    a_to_b = sum(model.to_string(pt[i][0]) == ans[i][1] for i in range(n))
    b_to_a = sum(model.to_string(pt[i][1]) == ans[i][0] for i in range(n))
    return (num_contexts, a_hits, b_hits, a_to_b, b_to_a)


# ------------------------------------------------------- batched FV evaluation
def _fv_sites_topk(model: Model, contexts: Pairs, vectors: torch.Tensor, layer_vec: Sequence[Tuple[int, int]],
                   topk: int, shard=None):
    """Top-k hits of every (prompt, (layer, vector)) pair in ONE sweep:
    prompts ``x + ":"``, vector added to hook_attn_out[0, -1] at the layer
    (scratch2.py:306-314 semantics).  Returns hits [len(layer_vec)]."""
    seqs = [model.to_tokens(x + ":")[0].tolist() for x, _ in contexts]
    firsts = [model.to_string(model.tokenizer.encode(y)[0]) for _, y in contexts]
    n, m = len(seqs), len(layer_vec)
    lv = np.asarray(layer_vec, dtype=np.int32).reshape(m, 2)
    vecs = vectors.to(model.device, torch.float32).reshape(-1, model.cfg.d_model).contiguous()
    _, patched = _add_site_outputs(model, seqs, np.repeat(np.arange(n, dtype=np.int32), m), np.tile(lv[:, 0], n),
                                   np.tile(lv[:, 1], n), vecs, None, topk, shard, clean_outputs=False)
    top = patched["topk"].view(n, m, topk).cpu().tolist()
    hits = np.zeros(m, dtype=np.int64)
    for i, first in enumerate(firsts):
        for j in range(m):
            hits[j] += first in [model.to_string(t) for t in top[i][j]]
    return hits


@range_checked
def check_accuracy_of_added_task_vector_by_layer(task_vector: torch.Tensor, contexts: Pairs, topk: int = 5,
                                                 model: Model = None, shard=None) -> List[float]:
    """``check_accuracy_of_added_task_vector`` at every layer (one sweep;
    ``shard``: distributed.SiteShard, sites round-robin over ranks)."""
    L = model.cfg.n_layers
    hits = _fv_sites_topk(model, contexts, task_vector.reshape(1, -1), [(l, 0) for l in range(L)], topk, shard)
    return [float(h) / len(contexts) for h in hits]


@range_checked
def function_vector_head_count_grid(mean_head_activations: torch.Tensor, causal_indirect_effects: torch.Tensor,
                                    contexts: Pairs, model: Model = None, heads_per_batch: int = 2,
                                    number_of_batches: int = 64, topk: int = 5, shard=None) -> torch.Tensor:
    """The FV head-count grid of scratch2.py:411-425 as ONE batched sweep:
    accuracy[i, j] of the function vector made of the top (j+1)*heads_per_batch
    heads of layers <= i, added at layer i.  Where the reference skips the
    assembly ((j+1)*k >= (i+1)*n_heads, :416) its ``task_vectors[i, j]`` stays
    the zero vector it was created as (:413) and the accuracy loop (:420-424)
    still evaluates it: those cells are the zero vector added at layer i, i.e.
    layer i's zero-shot top-k accuracy.  [n_layers, number_of_batches]."""
    L, H = model.cfg.n_layers, model.cfg.n_heads
    d = mean_head_activations.shape[-1]
    vecs = [torch.zeros(d, dtype=torch.float32, device=model.device)]  # vector 0: the skipped cells
    cells = []  # (i, j, index of the evaluated (layer, vector) pair)
    pairs = []
    for i in range(L):
        zero_pair = None  # layer i's skipped cells share ONE (layer i, zero vector) evaluation
        for j in range(number_of_batches):
            k = (j + 1) * heads_per_batch
            if k < (i + 1) * H:
                vecs.append(assemble_task_vector(mean_head_activations, causal_indirect_effects, i, k)
                            .to(model.device, torch.float32))
                pairs.append((i, len(vecs) - 1))
                cells.append((i, j, len(pairs) - 1))
            else:
                if zero_pair is None:
                    pairs.append((i, 0))
                    zero_pair = len(pairs) - 1
                cells.append((i, j, zero_pair))
    hits = _fv_sites_topk(model, contexts, torch.stack(vecs), pairs, topk, shard)
    acc = torch.zeros(L, number_of_batches)
    for i, j, q in cells:
        acc[i, j] = float(hits[q]) / len(contexts)
    return acc

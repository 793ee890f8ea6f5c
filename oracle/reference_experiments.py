"""ORACLE (test infrastructure only) — the reference's experiment functions
restated on the CPU hooked model, one batch-1 forward per site, Python hook
callbacks, global ``random`` — i.e. the reference's loop structure, which is
also what bench.py's cpu_baseline leg times.

Every function cites the reference lines it restates.  Quirks are kept
(SURVEY.md App. B): late-binding hook closures (B1), all-position head
replacement (B2), first-answer-token probability (B3), double separator (B4),
string comparison of decoded tokens (B5), in-place shuffles (B6).  B7
(scratch.py passing ``model`` as the separator) is restated with its intended
meaning, ``seperator_token=None``.
"""
from __future__ import annotations

import random
from typing import List, Sequence, Tuple

import numpy as np
import torch

Pairs = List[Tuple[str, str]]


# --------------------------------------------------------------- prompts (a9)
def mix_contexts_and_query(contexts: Pairs, query: str, function_token: str = "→",
                           seperator_token=None, model=None) -> List[int]:
    """scratch2.py:50-62 / scratch.py:49-61: [BOS=0] + (x, f, y[, sep])* [+ sep] + q + f."""
    f_id = model.to_single_token(function_token)
    sep = None if seperator_token is None else model.to_single_token(seperator_token)
    ids = [0]
    for x, y in contexts:
        ids += [model.to_single_token(x), f_id, model.to_single_token(y)]
        if sep is not None:
            ids.append(sep)
    if sep is not None:
        ids.append(sep)  # the doubled separator before the query (App. B4)
    return ids + [model.to_single_token(query), f_id]


def mix_multitoken_contexts_and_query(contexts: Pairs, query: str, function_token: str = "→",
                                      seperator_token=None, model=None) -> List[int]:
    """scratch2.py:63-78 (multi-token items, same layout)."""
    toks = lambda s: model.to_tokens(s, prepend_bos=False).tolist()[0]  # noqa: E731
    f_ids = toks(function_token)
    sep_ids = toks(seperator_token) if seperator_token is not None else []
    ids = [0]
    for x, y in contexts:
        ids += toks(x) + f_ids + toks(y) + sep_ids
    ids += sep_ids
    return ids + toks(query) + f_ids


# ---------------------------------------------------------- extraction (a1)
def generate_mean_activation(contexts: Pairs, function_token: str, seperator_token=",", model=None,
                             num_contexts: int = 1024, len_contexts: int = 4) -> torch.Tensor:
    """scratch2.py:81-100: mean over prompts of hook_result[0, -1] per layer."""
    cfg = model.cfg
    pool = contexts.copy()
    acc = torch.zeros(cfg.n_layers, cfg.n_heads, cfg.d_model, dtype=model.dtype)
    saved = cfg.use_attn_result
    cfg.use_attn_result = True
    for _ in range(num_contexts):
        random.shuffle(pool)
        demos, query = pool[:len_contexts], pool[len_contexts]
        ids = mix_multitoken_contexts_and_query(demos, query[0], function_token, seperator_token, model)
        _, cache = model.run_with_cache(torch.tensor(ids))
        for l in range(cfg.n_layers):
            acc[l] += cache[f"blocks.{l}.attn.hook_result"][0, -1]
    cfg.use_attn_result = saved
    return acc / num_contexts


def gather_head_activations_to_layers(mean_head_activations: torch.Tensor) -> torch.Tensor:
    """scratch2.py:103-104."""
    return mean_head_activations.sum(1)


# -------------------------------------------------------- layer sweeps (a3-a5)
def layer_addition_hook(hook_value, hook, vector):
    """scratch2.py:107-109."""
    hook_value[0, -1, :] = hook_value[0, -1, :] + vector
    return hook_value


def logits_to_next_token(logits, model) -> str:
    """scratch2.py:111-112."""
    return model.to_string(int(torch.argmax(logits[0, -1, :])))


def apply_layered_vectors_to_zero_shot(layered_vectors, contexts: Pairs, function_token: str, model):
    """scratch2.py:114-127 (late-binding closure kept: every hook adds
    layered_vectors[-1], App. B1)."""
    hits = [0] * model.cfg.n_layers
    hook_functions = [lambda hv, hook: layer_addition_hook(hv, hook, vector) for vector in layered_vectors]
    for x, y in contexts:
        tokens = torch.tensor([0, model.to_single_token(x), model.to_single_token(function_token)])
        for i in range(model.cfg.n_layers):
            logits = model.run_with_hooks(tokens, fwd_hooks=[(f"blocks.{i}.hook_attn_out", hook_functions[i])])
            if logits_to_next_token(logits, model) == y:
                hits[i] += 1
    return [1.0 * h / len(contexts) for h in hits]


def apply_layered_vectors_to_zero_shot_by_probability(layered_vectors, contexts: Pairs, function_token: str,
                                                      model):
    """scratch2.py:135-150 (same closure quirk)."""
    sums = torch.zeros(model.cfg.n_layers, dtype=model.dtype)
    hook_functions = [lambda hv, hook: layer_addition_hook(hv, hook, vector) for vector in layered_vectors]
    for x, y in contexts:
        tokens = torch.tensor([0] + model.to_tokens(x, prepend_bos=False).tolist()[0]
                              + [model.to_single_token(function_token)])
        answer = model.to_tokens(y, prepend_bos=False)[0]
        base = torch.softmax(model.forward(tokens)[0, -1, :], dim=0)[answer]
        for i in range(model.cfg.n_layers):
            logits = model.run_with_hooks(tokens, fwd_hooks=[(f"blocks.{i}.hook_attn_out", hook_functions[i])])
            p = torch.softmax(logits[0, -1, :], dim=0)[answer]
            sums[i] += p[0] - base[0]
    return sums / len(contexts)


# ---------------------------------------------------------------- CIE (a6-a8)
def calculate_average_causal_indirect_effect(mean_head_activations, scrambled_prompts, prompt_answers, model,
                                             layers: Sequence[int] = None, heads: Sequence[int] = None):
    """scratch2.py:171-197.  ``layers``/``heads`` restrict the sweep (used by
    the stratified CPU baseline); by default the full layer x head grid."""
    cfg = model.cfg
    if tuple(mean_head_activations.shape) != (cfg.n_layers, cfg.n_heads, cfg.d_model):
        raise ValueError("Mean head activations must be of shape (n_layers, n_heads, d_model)")
    if len(scrambled_prompts) != len(prompt_answers):
        raise ValueError("Prompt answers must be of the same length as scrambled prompts")
    layers = range(cfg.n_layers) if layers is None else layers
    heads = range(cfg.n_heads) if heads is None else heads
    saved = cfg.use_attn_result
    cfg.use_attn_result = True
    cie = torch.zeros(cfg.n_layers, cfg.n_heads, dtype=model.dtype)
    for prompt, answer in zip(scrambled_prompts, prompt_answers):
        tokens = model.to_tokens(prompt) if isinstance(prompt, str) else torch.tensor([prompt])
        p0 = torch.softmax(model.forward(tokens)[0, -1, :], dim=0)[answer]
        for layer in layers:
            for head in heads:
                def hook(hook_value, hook, layer=layer, head=head):
                    hook_value[0, :, head, :] = mean_head_activations[layer, head, :]
                    return hook_value
                out = model.run_with_hooks(tokens, fwd_hooks=[(f"blocks.{layer}.attn.hook_result", hook)])
                p = torch.softmax(out[0, -1, :], dim=0)[answer]
                cie[layer, head] += p[0] - p0[0]
    cfg.use_attn_result = saved
    return cie / len(scrambled_prompts)


def generate_shuffled_prompt(contexts: Pairs, model, function_token: str = ":", seperator_token=None):
    """scratch2.py:200-211: demo answers shuffled, query answer kept."""
    answers = [y for _, y in contexts[:-1]]
    random.shuffle(answers)
    parts = []
    for (x, _), y in zip(contexts[:-1], answers):
        parts.append(x + function_token + y + (seperator_token if seperator_token is not None else ""))
    prompt = "".join(parts) + contexts[-1][0] + function_token
    return prompt, model.to_tokens(contexts[-1][1], prepend_bos=False).tolist()[0]


def generate_shuffled_prompts(contexts: Pairs, model, num_prompts: int, prompt_length: int,
                              function_token: str = ":", seperator_token=None):
    """scratch2.py:213-225."""
    if prompt_length >= len(contexts):
        raise ValueError("Prompt length must be less than the number of contexts")
    pool = contexts.copy()
    prompts, answers = [], []
    for _ in range(num_prompts):
        random.shuffle(pool)
        p, a = generate_shuffled_prompt(pool[:prompt_length + 1], model, function_token, seperator_token)
        prompts.append(p)
        answers.append(a)
    return prompts, answers


# ---------------------------------------------------- function vectors (a10-a11)
def assemble_task_vector(mean_head_activations, causal_indirect_effects, layer: int, num_heads: int):
    """scratch2.py:232-238."""
    sub = causal_indirect_effects[:layer + 1, :]
    _, idx = torch.topk(sub.flatten(), num_heads)
    heads = np.array(np.unravel_index(idx.numpy(), sub.shape)).T
    vec = torch.zeros(mean_head_activations.shape[-1], dtype=mean_head_activations.dtype)
    for l, h in heads:
        vec += mean_head_activations[l, h, :]
    return vec


def assemble_end_list_tasks(objects: List[str], num_lists: int, num_elements: int, seperator: str = ","):
    """scratch2.py:240-245 (shuffles ``objects`` in place, App. B6)."""
    tasks = []
    for _ in range(num_lists):
        random.shuffle(objects)
        tasks.append((seperator.join(objects[:num_elements]), objects[num_elements - 1]))
    return tasks


def logits_to_next_k_tokens(k: int, logits, model) -> List[str]:
    """scratch2.py:278-282."""
    return [model.to_string(e) for e in torch.topk(logits[0, -1, :], k).indices.tolist()]


def check_accuracy_of_task_vector(task_vector, layer: int, contexts: Pairs, topk: int = 5, model=None):
    """scratch2.py:292-304: (baseline top-k accuracy, with the FV added)."""
    base_hits, fv_hits = 0, 0
    for x, y in contexts:
        prompt = x + ":"
        first = model.to_string(model.to_tokens(y, prepend_bos=False).tolist()[0][0])
        if first in logits_to_next_k_tokens(topk, model.forward(prompt), model):
            base_hits += 1
        logits = model.run_with_hooks(prompt, fwd_hooks=[(f"blocks.{layer}.hook_attn_out",
                                                          lambda hv, hook: layer_addition_hook(hv, hook, task_vector))])
        if first in logits_to_next_k_tokens(topk, logits, model):
            fv_hits += 1
    return (1.0 * base_hits / len(contexts), 1.0 * fv_hits / len(contexts))


def check_accuracy_of_added_task_vector(task_vector, layer: int, contexts: Pairs, topk: int = 5, model=None):
    """scratch2.py:306-314."""
    hits = 0
    for x, y in contexts:
        prompt = x + ":"
        first = model.to_string(model.to_tokens(y, prepend_bos=False).tolist()[0][0])
        logits = model.run_with_hooks(prompt, fwd_hooks=[(f"blocks.{layer}.hook_attn_out",
                                                          lambda hv, hook: layer_addition_hook(hv, hook, task_vector))])
        if first in logits_to_next_k_tokens(topk, logits, model):
            hits += 1
    return 1.0 * hits / len(contexts)


# ------------------------------------------------------ residual patching (a12)
def construct_query(pair, function_token: str = "→"):
    """scratch.py:47-48."""
    return (pair[0] + function_token, pair[1])


def test_component_hypothesis(contexts: Pairs, function_token: str, model=None, num_contexts: int = 256,
                              len_contexts: int = 4):
    """scratch.py:106-147 with the separator argument as intended (None, B7)."""
    pool = contexts.copy()
    total, base_hits, normal_hits = 0, 0, 0
    per_layer = [0] * model.cfg.n_layers
    for _ in range(num_contexts):
        total += 1
        random.shuffle(pool)
        demos, query = pool[:len_contexts], pool[len_contexts]
        answer, dummy = query[1], pool[len_contexts + 1][0]
        if logits_to_next_token(model(model.to_tokens(construct_query(query, function_token)[0])), model) == answer:
            base_hits += 1
        normal_logits, normal_cache = model.run_with_cache(
            torch.tensor(mix_contexts_and_query(demos, query[0], function_token, None, model)))
        if logits_to_next_token(normal_logits, model) == answer:
            normal_hits += 1
        _, dummy_cache = model.run_with_cache(
            torch.tensor(mix_contexts_and_query(demos, dummy, function_token, None, model)))
        for layer in range(model.cfg.n_layers):
            resid = dummy_cache[f"blocks.{layer}.hook_resid_pre"]
            resid[0, -2, :] = normal_cache[f"blocks.{layer}.hook_resid_pre"][0, -2, :]
            if logits_to_next_token(model.forward(resid, start_at_layer=layer), model) == answer:
                per_layer[layer] += 1
    return (total, base_hits, normal_hits, per_layer)


def substitute_task(taskA: Pairs, taskB: Pairs, layer: int, function_token: str = "→", model=None,
                    num_contexts: int = 256, len_contexts: int = 4):
    """scratch.py:164-213 (sorts both task lists in place, App. B6)."""
    if len(taskA) != len(taskB):
        raise ValueError("The two tasks must have the same length")
    taskA.sort(key=lambda p: p[0])
    taskB.sort(key=lambda p: p[0])
    for a, b in zip(taskA, taskB):
        if a[0] != b[0]:
            raise ValueError("The two tasks must have the same domains")
    mixed = [(a[0], a[1], b[1]) for a, b in zip(taskA, taskB)]
    a_hits = b_hits = a_to_b = b_to_a = 0
    for _ in range(num_contexts):
        random.shuffle(mixed)
        ctx_a = [(m[0], m[1]) for m in mixed[:len_contexts]]
        ctx_b = [(m[0], m[2]) for m in mixed[:len_contexts]]
        query = mixed[len_contexts][0][0]
        ans_a, ans_b = mixed[len_contexts][1], mixed[len_contexts][2]
        la, ca = model.run_with_cache(torch.tensor(mix_contexts_and_query(ctx_a, query, function_token, None, model)))
        lb, cb = model.run_with_cache(torch.tensor(mix_contexts_and_query(ctx_b, query, function_token, None, model)))
        a_hits += logits_to_next_token(la, model) == ans_a
        b_hits += logits_to_next_token(lb, model) == ans_b
        ra = ca[f"blocks.{layer}.hook_resid_pre"].clone()
        rb = cb[f"blocks.{layer}.hook_resid_pre"].clone()
        ra[0, -1, :] = cb[f"blocks.{layer}.hook_resid_pre"][0, -1, :]
        rb[0, -1, :] = ca[f"blocks.{layer}.hook_resid_pre"][0, -1, :]
        a_to_b += logits_to_next_token(model.forward(ra, start_at_layer=layer), model) == ans_b
        b_to_a += logits_to_next_token(model.forward(rb, start_at_layer=layer), model) == ans_a
    return (num_contexts, a_hits, b_hits, a_to_b, b_to_a)

#!/usr/bin/env python3
"""Generate tests/golden/reference_outputs*.{json,safetensors}: the outputs of
the reference's OWN hot-path functions, run verbatim on the CPU oracle model.

Run here, where /root/reference exists (never on the GPU box):

    python tests/golden/make_reference_fixtures.py [--no-160m]

The reference scripts cannot be imported (their module top level fetches a
model by name: scratch.py:26, scratch2.py:26).  Their experiment functions,
however, only use TransformerLens' API through the ``model`` argument and the
module globals ``t``/``np``/``random``/``tqdm``/``device``/``model``, and
``HookedPythiaOracle`` implements that API (run_with_cache, run_with_hooks,
forward(start_at_layer=), cfg.use_attn_result, to_tokens, to_single_token,
to_string).  So the function definitions are AST-extracted from the source
text and executed in a namespace that binds those globals to torch, numpy,
an identity ``tqdm``, the CPU and the oracle model:

  scratch2.py  generate_mean_activation (:81-100), gather_head_activations_to_layers
               (:103-104), layer_addition_hook / logits_to_next_token (:107-112),
               apply_layered_vectors_to_zero_shot (:114-127), ..._by_probability
               (:135-150), calculate_average_causal_indirect_effect (:171-197),
               generate_shuffled_prompt(s) (:200-225), assemble_task_vector (:232-238),
               assemble_end_list_tasks (:240-245), logits_to_next_k_tokens,
               check_accuracy_of_task_vector, check_accuracy_of_added_task_vector
               (:278-314), mix_(multitoken_)contexts_and_query (:50-78)
  scratch.py   test_component_hypothesis (:106-147), substitute_task (:164-213),
               mix_contexts_and_query (:49-61), construct_query, logits_to_next_token

The FV head-count grid (scratch2.py:411-425) is top-level cell code, not a
function: its two loops are restated below around the reference's own
assemble_task_vector / check_accuracy_of_added_task_vector.

One deviation, recorded in the fixture metadata: scratch.py as committed
passes ``model`` positionally as ``seperator_token`` (scratch.py:131,137,
193,194), so ``to_single_token(model)`` cannot run.  The
extracted ``mix_contexts_and_query`` is wrapped so that a non-string separator
means "no separator" (the intended meaning, the one the recorded results in
Experimental Results.txt predate).  Everything else runs unmodified.

Only data is written: inputs (seeds, sizes, task names) and outputs.  No
reference source text is stored.
"""
import argparse
import json
import random
import sys
import types
import typing
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(HERE))

from make_prompt_fixtures import extract  # noqa: E402

OUT_JSON = HERE / "reference_outputs.json"
OUT_160M = HERE / "reference_outputs_160m.safetensors"

SCRATCH2 = ["mix_contexts_and_query", "mix_multitoken_contexts_and_query", "generate_mean_activation",
            "gather_head_activations_to_layers", "layer_addition_hook", "logits_to_next_token",
            "apply_layered_vectors_to_zero_shot", "apply_layered_vectors_to_zero_shot_by_probability",
            "calculate_average_causal_indirect_effect", "generate_shuffled_prompt", "generate_shuffled_prompts",
            "assemble_task_vector", "assemble_end_list_tasks", "logits_to_next_k_tokens",
            "check_accuracy_of_task_vector", "check_accuracy_of_added_task_vector"]
SCRATCH = ["construct_query", "mix_contexts_and_query", "logits_to_next_token", "test_component_hypothesis",
           "substitute_task"]

# the tiny fixture model (= tests/conftest.py tiny_sd / tiny_oracle)
TINY = {"config": "tiny", "weight_seed": 0, "std": 0.15, "ln_std": 0.1, "tokenizer": "SyntheticTokenizer(512)",
        "oracle_dtype": "float32"}
# the Pythia-160m-shape fixture model (C1); std 0.1 makes its next-token
# distributions peaked enough that per-layer accuracy / probability move
P160 = {"config": "pythia-160m", "weight_seed": 0, "std": 0.1, "ln_std": 0.1,
        "tokenizer": "SyntheticTokenizer(50304)", "oracle_dtype": "float32"}

B7_NOTE = ("scratch.py:131,137,193,194 pass `model` positionally as seperator_token (SURVEY App. B7); the "
           "extracted mix_contexts_and_query is wrapped so a non-string separator means None. No other change.")


def reference_namespace(fname, names, model):
    """Execute the extracted definitions with the reference's module globals
    bound to torch / numpy / random / the CPU / the oracle model."""
    ns = {"t": torch, "np": np, "random": random, "tqdm": lambda it, *a, **k: it, "device": torch.device("cpu"),
          "model": model, "Tensor": torch.Tensor, "Float": object, "List": typing.List, "Tuple": typing.Tuple,
          "Optional": typing.Optional, "HookedTransformer": object,
          "hook_points": types.SimpleNamespace(HookPoint=object)}
    exec(compile(extract(fname, names), f"<reference {fname} (extracted)>", "exec"), ns)
    return ns


def with_b7_fix(ns):
    ref_mix = ns["mix_contexts_and_query"]

    def mix_contexts_and_query(contexts, query, function_token="→", seperator_token=None, model=ns["model"]):
        if seperator_token is not None and not isinstance(seperator_token, str):
            model, seperator_token = seperator_token, None  # B7: the positional model landed in the separator
        return ref_mix(contexts, query, function_token, seperator_token, model)

    ns["mix_contexts_and_query"] = mix_contexts_and_query
    return ns


def make_oracle(name, spec):
    import tvr_amd
    from conftest import oracle_config  # noqa: E402  (tests/ on sys.path below)
    from oracle.hooked_pythia import HookedPythiaOracle
    cfg = tvr_amd.get_config(name)
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=spec["weight_seed"], std=spec["std"], ln_std=spec["ln_std"])
    tok = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
    return HookedPythiaOracle(oracle_config(cfg), sd, dtype=torch.float32, tokenizer=tok)


def model_task(model, xs, function_token, rank=0):
    """A task whose answers are the model's own zero-shot predictions: y = the
    rank-th most likely next token of [BOS] + tokens(x) + tokens(f) (the
    layout of scratch2.py:121,142).  Random weights know none of the
    reference's tasks, so on the reference's literal tasks every accuracy is 0
    and the comparisons would be vacuous; with these, baseline accuracy is 1
    and the injected vectors move it.  The pairs are stored in the fixture."""
    out = []
    for x in xs:
        ids = [0] + model.tokenizer.encode(x) + model.tokenizer.encode(function_token)
        logits = model.forward(torch.tensor(ids))[0, -1]
        out.append((x, model.to_string(int(torch.topk(logits, rank + 1).indices[rank]))))
    return out


def f32list(x):
    return [float(v) for v in torch.as_tensor(x).float().flatten().tolist()]


def tiny_cases():
    import tvr_amd
    T = tvr_amd.tasks
    model = make_oracle("tiny", TINY)
    s2 = reference_namespace("scratch2.py", SCRATCH2, model)
    s1 = with_b7_fix(reference_namespace("scratch.py", SCRATCH, model))
    out = {"model": TINY, "deviations": [B7_NOTE], "tasks": {}, "cases": {}}
    C = out["cases"]
    letters = [x for x, _ in T.letter_to_caps]
    # model-consistent tasks (see model_task): "→" zero-shot answers, ":" ones, and the
    # runner-up "→" answers (a second task over the same domain, for substitute_task)
    arrow_task = model_task(model, letters, T.ARROW)
    colon_task = model_task(model, letters, ":")
    runner_up_task = model_task(model, letters, T.ARROW, rank=1)
    out["tasks"] = {"arrow": arrow_task, "colon": colon_task, "arrow_runner_up": runner_up_task}

    # a1: extraction (scratch2.py:81-100) on the reference's letter_to_caps, "→", ",", 48 prompts x 4 demos
    random.seed(1234)
    mean = s2["generate_mean_activation"](list(T.letter_to_caps), T.ARROW, ",", model, num_contexts=48, len_contexts=4)
    C["generate_mean_activation"] = {"seed": 1234, "task": "letter_to_caps", "function_token": T.ARROW,
                                     "seperator_token": ",", "num_contexts": 48, "len_contexts": 4,
                                     "shape": list(mean.shape), "out": f32list(mean)}
    # a2-a5: layer sweeps with the summed means (B1 late-binding closure as committed)
    layered = s2["gather_head_activations_to_layers"](mean)
    acc = s2["apply_layered_vectors_to_zero_shot"](layered, list(arrow_task), T.ARROW, model)
    dp = s2["apply_layered_vectors_to_zero_shot_by_probability"](layered, list(arrow_task), T.ARROW, model)
    C["apply_layered_vectors_to_zero_shot"] = {"vectors": "gather(mean)", "task": "arrow",
                                               "out": [float(a) for a in acc]}
    C["apply_layered_vectors_to_zero_shot_by_probability"] = {"vectors": "gather(mean)", "task": "arrow",
                                                              "out": f32list(dp)}
    # a8 + a7: shuffled prompts and the CIE over every (layer, head)
    random.seed(99)
    prompts, answers = s2["generate_shuffled_prompts"](list(arrow_task), model, 6, 4, T.ARROW)
    cie = s2["calculate_average_causal_indirect_effect"](mean, prompts, answers, model)
    C["calculate_average_causal_indirect_effect"] = {"seed": 99, "task": "arrow", "num_prompts": 6,
                                                     "prompt_length": 4, "function_token": T.ARROW,
                                                     "prompts": prompts, "answers": answers,
                                                     "shape": list(cie.shape), "out": f32list(cie)}
    # a10 + a11: FV of the top-3 heads of layers <= 1, top-5 accuracy on the ":" task (x 2 so it moves)
    fv = s2["assemble_task_vector"](mean, cie, 1, 3)
    C["assemble_task_vector"] = {"layer": 1, "num_heads": 3, "out": f32list(fv)}
    ctx = list(colon_task[:40])
    C["check_accuracy_of_task_vector"] = {"vector": "fv * 2", "layer": 1, "contexts": "colon[:40]", "topk": 5,
                                          "out": list(s2["check_accuracy_of_task_vector"](fv * 2, 1, ctx, 5, model))}
    C["check_accuracy_of_added_task_vector"] = {
        "vector": "fv * 2", "layer": 0, "contexts": "colon[:40]", "topk": 5,
        "out": s2["check_accuracy_of_added_task_vector"](fv * 2, 0, ctx, 5, model)}
    # f3: the head-count grid, the scratch2.py:411-425 loops around the reference's functions
    # (mean x 2, 1 head per batch, 6 batches, 30 contexts; cells with (j+1)*k >= (i+1)*H keep
    # the zero vector, as task_vectors starts as zeros at :413)
    L, H, d = model.cfg.n_layers, model.cfg.n_heads, model.cfg.d_model
    hpb, nb = 1, 6
    vectors = torch.zeros(L, nb, d)
    for i in range(L):
        for j in range(nb):
            if (j + 1) * hpb < (i + 1) * H:
                vectors[i, j] = s2["assemble_task_vector"](mean * 2, cie, i, (j + 1) * hpb)
    grid = torch.zeros(L, nb)
    for i in range(L):
        for j in range(nb):
            grid[i, j] = s2["check_accuracy_of_added_task_vector"](vectors[i, j], i, list(colon_task[:30]), 5, model)
    C["function_vector_head_count_grid"] = {"means": "mean * 2", "heads_per_batch": hpb, "number_of_batches": nb,
                                            "contexts": "colon[:30]", "topk": 5, "shape": [L, nb],
                                            "out": f32list(grid)}
    # multi-token items: state -> capital extraction ("," separated, ":" function token) and the
    # end-of-list CIE with "|" separators (the scratch2.py:262-267, 376-379 cells, scaled down)
    random.seed(42)
    mean_s = s2["generate_mean_activation"](list(T.state_to_capital_task), ":", ",", model, num_contexts=24,
                                            len_contexts=5)
    C["generate_mean_activation_state_to_capital"] = {"seed": 42, "task": "state_to_capital",
                                                      "function_token": ":", "seperator_token": ",",
                                                      "num_contexts": 24, "len_contexts": 5,
                                                      "shape": list(mean_s.shape), "out": f32list(mean_s)}
    random.seed(43)
    states = list(T.us_states)
    last_state = s2["assemble_end_list_tasks"](states, 40, 5)
    prompts_l, answers_l = s2["generate_shuffled_prompts"](last_state, model, 4, 3, ":", "|")
    cie_l = s2["calculate_average_causal_indirect_effect"](mean_s * 4, prompts_l, answers_l, model)
    C["calculate_average_causal_indirect_effect_end_list"] = {
        "seed": 43, "lists": [40, 5], "num_prompts": 4, "prompt_length": 3, "function_token": ":",
        "seperator_token": "|", "means": "state_to_capital mean * 4", "prompts": prompts_l, "answers": answers_l,
        "shape": list(cie_l.shape), "out": f32list(cie_l)}
    # a12 and next #4: residual patching (scratch.py), B7 as noted
    random.seed(5)
    tch = s1["test_component_hypothesis"](list(arrow_task), T.ARROW, model, num_contexts=40, len_contexts=4)
    C["test_component_hypothesis"] = {"seed": 5, "task": "arrow", "num_contexts": 40, "len_contexts": 4,
                                      "out": [tch[0], tch[1], tch[2], list(tch[3])]}
    random.seed(6)
    sub = s1["substitute_task"](list(arrow_task), list(runner_up_task), 1, T.ARROW, model, 32, 4)
    C["substitute_task"] = {"seed": 6, "tasks": ["arrow", "arrow_runner_up"], "layer": 1,
                            "num_contexts": 32, "len_contexts": 4, "out": list(sub)}
    return out


def p160_cases():
    """C1 at the real Pythia-160m shape: extraction on state -> capital
    (5 demos, ":" / ","), the Δprobability layer sweep on the states with the
    model's own ":" answers (multi-token x) and the accuracy layer sweep on the
    letters with its own "→" answers (single-token x: to_single_token)."""
    import tvr_amd
    T = tvr_amd.tasks
    model = make_oracle("pythia-160m", P160)
    s2 = reference_namespace("scratch2.py", SCRATCH2, model)
    random.seed(2024)
    mean = s2["generate_mean_activation"](list(T.state_to_capital_task), ":", ",", model, num_contexts=16,
                                          len_contexts=5)
    layered = s2["gather_head_activations_to_layers"](mean)
    states = model_task(model, [x for x, _ in T.state_to_capital_task[:20]], ":")
    letters = model_task(model, [x for x, _ in T.letter_to_caps], T.ARROW)
    dp = s2["apply_layered_vectors_to_zero_shot_by_probability"](layered, list(states), ":", model)
    acc = s2["apply_layered_vectors_to_zero_shot"](layered, list(letters), T.ARROW, model)
    meta = {"model": P160, "seed": 2024, "task": "state_to_capital", "function_token": ":",
            "seperator_token": ",", "num_contexts": 16, "len_contexts": 5,
            "dprob_task": states, "accuracy_task": letters, "accuracy_function_token": T.ARROW,
            "vectors": "gather(mean) (B1 late binding as committed)",
            "accuracy_out": [float(a) for a in acc]}
    tensors = {"mean": mean.float().contiguous(), "dprob": dp.float().contiguous()}
    return meta, tensors


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-160m", action="store_true")
    a = ap.parse_args()
    sys.path.insert(0, str(ROOT / "tests"))
    torch.set_num_threads(8)
    out = tiny_cases()
    out["generator"] = "tests/golden/make_reference_fixtures.py"
    if not a.no_160m:
        from safetensors.torch import save_file
        meta, tensors = p160_cases()
        save_file(tensors, str(OUT_160M))
        out["pythia_160m"] = meta
    elif OUT_JSON.exists():
        old = json.loads(OUT_JSON.read_text())
        if "pythia_160m" in old:
            out["pythia_160m"] = old["pythia_160m"]
    OUT_JSON.write_text(json.dumps(out, indent=1) + "\n")
    print(f"wrote {OUT_JSON}" + ("" if a.no_160m else f" and {OUT_160M}"))


if __name__ == "__main__":
    main()

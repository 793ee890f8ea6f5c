"""GPU: the HIP engine (through the C ABI, every GEMM path) against the
outputs of the reference's OWN functions (tests/golden/reference_outputs*,
made by tests/golden/make_reference_fixtures.py on the CPU oracle model with
the same seeded weights, tokenizer and global-``random`` seeds).

Each product function gets the fixture's inputs, so every comparison isolates
one function.  Tolerances (fp32 engine vs the fp32 reference run; the GEMM
reduction order differs):
* mean vectors / function vectors: 1e-4 relative (north star)
* probabilities, Δp, CIE: |Δ| <= 1e-4 * max|ref| + 1e-7
* accuracies, hit counts, grids: identical
"""
import json
import random
from pathlib import Path

import pytest
import torch

import tvr_amd

pytestmark = pytest.mark.gpu

GOLD = Path(__file__).parent / "golden"
FIX = json.loads((GOLD / "reference_outputs.json").read_text())
C = FIX["cases"]
T = tvr_amd.tasks
ARROW = T.ARROW


def tensor(case):
    return torch.tensor(case["out"], dtype=torch.float32).view(*case.get("shape", [-1]))


def pairs(name):
    return [tuple(p) for p in FIX["tasks"][name]]


def rel_err(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def abs_ok(a, b, rel=1e-4):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return (a - b).abs().max().item() <= rel * b.abs().max().item() + 1e-7


def test_extraction(tiny_model):
    for key, task in (("generate_mean_activation", T.letter_to_caps),
                      ("generate_mean_activation_state_to_capital", T.state_to_capital_task)):
        c = C[key]
        random.seed(c["seed"])
        mean = tvr_amd.generate_mean_activation(list(task), c["function_token"], c["seperator_token"],
                                                model=tiny_model, num_contexts=c["num_contexts"],
                                                len_contexts=c["len_contexts"])
        assert rel_err(mean, tensor(c)) < 1e-4, key


def test_layer_sweeps(tiny_model):
    layered = tvr_amd.gather_head_activations_to_layers(tensor(C["generate_mean_activation"]).cuda())
    acc = tvr_amd.apply_layered_vectors_to_zero_shot(layered, pairs("arrow"), ARROW, model=tiny_model)
    assert acc == C["apply_layered_vectors_to_zero_shot"]["out"]
    dp = tvr_amd.apply_layered_vectors_to_zero_shot_by_probability(layered, pairs("arrow"), ARROW, model=tiny_model)
    assert abs_ok(dp, tensor(C["apply_layered_vectors_to_zero_shot_by_probability"]))


def test_shuffled_prompts_and_cie(tiny_model):
    c = C["calculate_average_causal_indirect_effect"]
    random.seed(c["seed"])
    prompts, answers = tvr_amd.generate_shuffled_prompts(pairs("arrow"), tiny_model, c["num_prompts"],
                                                         c["prompt_length"], c["function_token"])
    assert prompts == c["prompts"] and answers == c["answers"]
    mean = tensor(C["generate_mean_activation"]).cuda()
    cie = tvr_amd.calculate_average_causal_indirect_effect(mean, prompts, answers, model=tiny_model)
    assert abs_ok(cie, tensor(c))
    c = C["calculate_average_causal_indirect_effect_end_list"]
    mean_s = tensor(C["generate_mean_activation_state_to_capital"]).cuda() * 4
    cie = tvr_amd.calculate_average_causal_indirect_effect(mean_s, c["prompts"], c["answers"], model=tiny_model)
    assert abs_ok(cie, tensor(c))


def test_function_vector_accuracy_and_grid(tiny_model):
    mean = tensor(C["generate_mean_activation"]).cuda()
    cie = tensor(C["calculate_average_causal_indirect_effect"]).cuda()
    fv = tvr_amd.assemble_task_vector(mean, cie, 1, 3)
    assert rel_err(fv, tensor(C["assemble_task_vector"])) < 1e-4
    fv = tensor(C["assemble_task_vector"]).cuda()
    ctx = pairs("colon")[:40]
    assert list(tvr_amd.check_accuracy_of_task_vector(fv * 2, 1, ctx, 5, model=tiny_model)) == \
        C["check_accuracy_of_task_vector"]["out"]
    assert tvr_amd.check_accuracy_of_added_task_vector(fv * 2, 0, ctx, 5, model=tiny_model) == \
        C["check_accuracy_of_added_task_vector"]["out"]
    g = C["function_vector_head_count_grid"]
    grid = tvr_amd.experiments.function_vector_head_count_grid(mean * 2, cie, pairs("colon")[:30], model=tiny_model,
                                                               heads_per_batch=g["heads_per_batch"],
                                                               number_of_batches=g["number_of_batches"], topk=5)
    assert torch.equal(grid, tensor(g))


def test_residual_patching(tiny_model):
    c = C["test_component_hypothesis"]
    random.seed(c["seed"])
    got = tvr_amd.test_component_hypothesis(pairs("arrow"), ARROW, model=tiny_model, num_contexts=c["num_contexts"],
                                            len_contexts=c["len_contexts"], batch_contexts=16)
    assert [got[0], got[1], got[2], list(got[3])] == c["out"]
    c = C["substitute_task"]
    random.seed(c["seed"])
    got = tvr_amd.substitute_task(pairs("arrow"), pairs("arrow_runner_up"), c["layer"], ARROW, model=tiny_model,
                                  num_contexts=c["num_contexts"], len_contexts=c["len_contexts"])
    assert list(got) == c["out"]


@pytest.mark.slow
@pytest.mark.parametrize("gemm", ["x2f16", "f32"])
def test_pythia160m_c1_against_reference_functions(gemm):
    """C1 at the real Pythia-160m shape (d 768, 12 heads, d_head 64, V 50304):
    extraction on state -> capital, the Δprobability sweep and the accuracy
    sweep, against the reference functions' outputs."""
    from safetensors.torch import load_file
    meta = FIX["pythia_160m"]
    spec = meta["model"]
    want = load_file(str(GOLD / "reference_outputs_160m.safetensors"))
    cfg = tvr_amd.get_config(spec["config"])
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=spec["weight_seed"], std=spec["std"], ln_std=spec["ln_std"])
    model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda", gemm=gemm)
    random.seed(meta["seed"])
    mean = tvr_amd.generate_mean_activation(list(T.state_to_capital_task), meta["function_token"],
                                            meta["seperator_token"], model=model, num_contexts=meta["num_contexts"],
                                            len_contexts=meta["len_contexts"])
    assert rel_err(mean, want["mean"]) < 1e-4
    layered = tvr_amd.gather_head_activations_to_layers(want["mean"].cuda())
    dp = tvr_amd.apply_layered_vectors_to_zero_shot_by_probability(
        layered, [tuple(p) for p in meta["dprob_task"]], meta["function_token"], model=model)
    assert abs_ok(dp, want["dprob"])
    acc = tvr_amd.apply_layered_vectors_to_zero_shot(layered, [tuple(p) for p in meta["accuracy_task"]],
                                                     meta["accuracy_function_token"], model=model)
    assert acc == meta["accuracy_out"]

"""CPU: the oracle's restatement of the reference's hot-path loops
(oracle/reference_experiments.py) against the outputs of the reference's OWN
functions, run verbatim on the same oracle model and the same seeds
(tests/golden/make_reference_fixtures.py -> tests/golden/reference_outputs*.json).

This pins the oracle's experiment loops (a1, a4, a5, a7, a8, a10-a12, f3, f4) to
the reference code; the GPU tests then compare the engine with the same
fixtures (tests/test_gpu_reference_fixtures.py).  The restatement and the
reference run the same fp32 torch ops on the CPU, so the bar here is tight:
1e-6 relative on tensors, identical accuracies.
"""
import json
import random
from pathlib import Path

import pytest
import torch

import tvr_amd
from conftest import make_oracle
from oracle import reference_experiments as R

GOLD = Path(__file__).parent / "golden"
FIX = json.loads((GOLD / "reference_outputs.json").read_text())
C = FIX["cases"]
T = tvr_amd.tasks
ARROW = T.ARROW


def tensor(case):
    return torch.tensor(case["out"], dtype=torch.float32).view(*case.get("shape", [-1]))


def pairs(name):
    return [tuple(p) for p in FIX["tasks"][name]]


def close(a, b, rel=1e-6):
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    return (a - b).abs().max().item() <= rel * b.abs().max().item() + 1e-9


@pytest.fixture(scope="module")
def oracle():
    spec = FIX["model"]
    cfg = tvr_amd.get_config(spec["config"])
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=spec["weight_seed"], std=spec["std"], ln_std=spec["ln_std"])
    return make_oracle(cfg, sd, tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab))


def test_fixture_metadata_records_the_b7_deviation():
    assert any("B7" in d for d in FIX["deviations"])
    assert FIX["model"] == {"config": "tiny", "weight_seed": 0, "std": 0.15, "ln_std": 0.1,
                            "tokenizer": "SyntheticTokenizer(512)", "oracle_dtype": "float32"}


def test_extraction(oracle):
    c = C["generate_mean_activation"]
    random.seed(c["seed"])
    mean = R.generate_mean_activation(list(T.letter_to_caps), c["function_token"], c["seperator_token"], oracle,
                                      c["num_contexts"], c["len_contexts"])
    assert close(mean, tensor(c))
    c = C["generate_mean_activation_state_to_capital"]
    random.seed(c["seed"])
    mean = R.generate_mean_activation(list(T.state_to_capital_task), c["function_token"], c["seperator_token"],
                                      oracle, c["num_contexts"], c["len_contexts"])
    assert close(mean, tensor(c))


def test_layer_sweeps(oracle):
    layered = R.gather_head_activations_to_layers(tensor(C["generate_mean_activation"]))
    assert R.apply_layered_vectors_to_zero_shot(layered, pairs("arrow"), ARROW, oracle) == \
        C["apply_layered_vectors_to_zero_shot"]["out"]
    dp = R.apply_layered_vectors_to_zero_shot_by_probability(layered, pairs("arrow"), ARROW, oracle)
    assert close(dp, tensor(C["apply_layered_vectors_to_zero_shot_by_probability"]), 1e-5)


def test_shuffled_prompts_and_cie(oracle):
    c = C["calculate_average_causal_indirect_effect"]
    random.seed(c["seed"])
    prompts, answers = R.generate_shuffled_prompts(pairs("arrow"), oracle, c["num_prompts"], c["prompt_length"],
                                                   c["function_token"])
    assert prompts == c["prompts"] and answers == c["answers"]
    cie = R.calculate_average_causal_indirect_effect(tensor(C["generate_mean_activation"]), prompts, answers, oracle)
    assert close(cie, tensor(c), 1e-5)


def test_end_list_cie(oracle):
    c = C["calculate_average_causal_indirect_effect_end_list"]
    random.seed(c["seed"])
    states = list(T.us_states)
    last_state = R.assemble_end_list_tasks(states, *c["lists"])
    prompts, answers = R.generate_shuffled_prompts(last_state, oracle, c["num_prompts"], c["prompt_length"],
                                                   c["function_token"], c["seperator_token"])
    assert prompts == c["prompts"] and answers == c["answers"]
    assert any(len(a) > 1 for a in answers)  # multi-token answers: only the first token counts (B3)
    mean = tensor(C["generate_mean_activation_state_to_capital"]) * 4
    assert close(R.calculate_average_causal_indirect_effect(mean, prompts, answers, oracle), tensor(c), 1e-5)


def test_function_vector_and_accuracy(oracle):
    mean = tensor(C["generate_mean_activation"])
    cie = tensor(C["calculate_average_causal_indirect_effect"])
    fv = R.assemble_task_vector(mean, cie, 1, 3)
    assert close(fv, tensor(C["assemble_task_vector"]))
    ctx = pairs("colon")[:40]
    assert list(R.check_accuracy_of_task_vector(fv * 2, 1, ctx, 5, oracle)) == C["check_accuracy_of_task_vector"]["out"]
    assert R.check_accuracy_of_added_task_vector(fv * 2, 0, ctx, 5, oracle) == \
        C["check_accuracy_of_added_task_vector"]["out"]


def test_head_count_grid_cells(oracle):
    """The grid's skipped cells (scratch2.py:416) hold the zero vector and are
    still evaluated (:420-424): their accuracy is the layer's zero-shot one."""
    c = C["function_vector_head_count_grid"]
    grid = tensor(c)
    L, H = oracle.cfg.n_layers, oracle.cfg.n_heads
    ctx = pairs("colon")[:30]
    zero = torch.zeros(oracle.cfg.d_model)
    for i in range(L):
        for j in range(c["number_of_batches"]):
            if (j + 1) * c["heads_per_batch"] >= (i + 1) * H:
                assert grid[i, j].item() == pytest.approx(R.check_accuracy_of_added_task_vector(zero, i, ctx, 5, oracle))
    assert (grid > 0).any() and (grid < 1).any()  # informative: the vectors move the accuracy


def test_residual_patching(oracle):
    c = C["test_component_hypothesis"]
    random.seed(c["seed"])
    got = R.test_component_hypothesis(pairs("arrow"), ARROW, oracle, c["num_contexts"], c["len_contexts"])
    assert [got[0], got[1], got[2], list(got[3])] == c["out"]
    c = C["substitute_task"]
    random.seed(c["seed"])
    got = R.substitute_task(pairs("arrow"), pairs("arrow_runner_up"), c["layer"], ARROW, oracle, c["num_contexts"],
                            c["len_contexts"])
    assert list(got) == c["out"]


def test_fixtures_are_informative():
    """Accuracies strictly between 0 and 1 somewhere (the model-consistent
    tasks), CIE and Δp nonzero: the GPU comparisons are not vacuous."""
    acc = C["apply_layered_vectors_to_zero_shot"]["out"]
    assert any(0 < a < 1 for a in acc)
    assert C["test_component_hypothesis"]["out"][2] > 0
    assert 0 < C["check_accuracy_of_task_vector"]["out"][1] < 1
    assert tensor(C["calculate_average_causal_indirect_effect"]).abs().max() > 1e-3


def test_160m_extraction_pinned():
    """C1 at the Pythia-160m shape: the restatement's extraction equals the
    reference function's (state -> capital, 16 prompts x 5 demos)."""
    from safetensors.torch import load_file
    meta = FIX["pythia_160m"]
    spec = meta["model"]
    want = load_file(str(GOLD / "reference_outputs_160m.safetensors"))
    cfg = tvr_amd.get_config(spec["config"])
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=spec["weight_seed"], std=spec["std"], ln_std=spec["ln_std"])
    oracle = make_oracle(cfg, sd, tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab))
    random.seed(meta["seed"])
    mean = R.generate_mean_activation(list(T.state_to_capital_task), meta["function_token"], meta["seperator_token"],
                                      oracle, meta["num_contexts"], meta["len_contexts"])
    assert close(mean, want["mean"])
    assert any(0 < a < 1 for a in meta["accuracy_out"])
    assert want["dprob"].abs().max() > 1e-3

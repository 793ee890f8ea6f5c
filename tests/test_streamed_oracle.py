"""CPU: the layer-streamed fp64 oracle (oracle/streamed_pythia.py) equals the
whole-model hooked oracle running the reference's loops
(oracle/reference_experiments.py, scratch2.py:81-100,171-197,292-314) on the
same seeded weights, to fp64 reassociation (1e-12).  The full-depth GPU tests
(tests/test_gpu_full_depth.py) use the streamed form at 6.9B / 12B."""
import random

import pytest
import torch

import tvr_amd
from conftest import TINY_STD
from oracle import reference_experiments as R
from oracle.hooked_pythia import HookedPythiaOracle
from oracle.streamed_pythia import StreamedPythiaOracle

from conftest import oracle_config

ARROW = tvr_amd.tasks.ARROW


@pytest.fixture(scope="module")
def pair():
    cfg = tvr_amd.get_config("tiny").with_(n_layers=3)
    shapes = tvr_amd.weights.hf_param_shapes(cfg)
    sd = {n: tvr_amd.weights.synth_param(cfg, n, s, 5, "cpu", TINY_STD) for n, s in shapes.items()}
    tok = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
    calls = []

    def get_raw(name):
        calls.append(name)
        return sd[name].clone()
    streamed = StreamedPythiaOracle(oracle_config(cfg), get_raw)  # the fp32 reference's rotary tables
    full = HookedPythiaOracle(oracle_config(cfg), sd, dtype=torch.float64, tokenizer=tok,
                              rotary_table_dtype=torch.float32)
    return cfg, tok, full, streamed, calls


def rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-300)).item()


def test_weights_are_streamed_one_block_at_a_time(pair):
    cfg, _, _, streamed, calls = pair
    n0 = len(calls)
    streamed.block(1)
    streamed.block(1)  # cached
    assert len(calls) - n0 == 12  # the block's 12 HF parameters, once
    assert all(c.startswith("gpt_neox.layers.1.") for c in calls[n0:])


def test_clean_logits_equal_hooked_oracle(pair):
    cfg, tok, full, streamed, _ = pair
    g = random.Random(0)
    seqs = [[0] + [g.randrange(1, cfg.d_vocab) for _ in range(T - 1)] for T in (5, 9, 9, 14)]
    got = streamed.last_logits(seqs)
    for s, row in zip(seqs, got):
        assert rel(row, full.forward(torch.tensor([s]))[0, -1]) < 1e-12


def test_mean_activation_equals_reference_loop(pair):
    cfg, tok, full, streamed, _ = pair
    random.seed(7)
    want = R.generate_mean_activation(list(tvr_amd.tasks.letter_to_caps), ARROW, ",", full, 12, 4)

    class _M:
        pass
    m = _M()
    m.cfg, m.to_single_token, m.tokenizer = cfg, full.to_single_token, tok
    random.seed(7)
    prompts = tvr_amd.prompts.sample_icl_prompts(m, list(tvr_amd.tasks.letter_to_caps), ARROW, ",", 12, 4)
    assert rel(streamed.mean_activation(prompts), want) < 1e-12


def test_cie_equals_reference_loop(pair):
    cfg, tok, full, streamed, _ = pair
    g = torch.Generator().manual_seed(3)
    mean = torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, generator=g, dtype=torch.float64)
    r = random.Random(1)
    prompts = [[0] + [r.randrange(1, cfg.d_vocab) for _ in range(10)] for _ in range(3)]
    answers = [int(full.forward(torch.tensor([p]))[0, -1].argmax()) for p in prompts]
    want = R.calculate_average_causal_indirect_effect(mean, prompts, [[a] for a in answers], full)
    got = streamed.cie(mean, prompts, answers)
    assert (got - want).abs().max().item() <= 1e-12 * want.abs().max().item()
    assert want.abs().max().item() > 1e-3
    sub = streamed.cie(mean, prompts, answers, layers=[0, 2], heads=[1, 3])
    mask = torch.zeros_like(sub, dtype=torch.bool)
    mask[torch.tensor([0, 2])[:, None], torch.tensor([1, 3])[None, :]] = True
    assert (sub[mask] - want[mask]).abs().max().item() <= 1e-12 * want.abs().max().item()
    assert sub[~mask].abs().max().item() == 0.0


def test_added_vector_topk_equals_reference_hook(pair):
    cfg, tok, full, streamed, _ = pair
    r = random.Random(2)
    seqs = [[0, r.randrange(1, cfg.d_vocab), r.randrange(1, cfg.d_vocab)] for _ in range(6)]
    vec = torch.randn(cfg.d_model, generator=torch.Generator().manual_seed(4), dtype=torch.float64) * 3
    for layer in (0, 2):
        got = streamed.added_topk(seqs, layer, vec, 5)
        for s, row in zip(seqs, got):
            ref = full.run_with_hooks(torch.tensor([s]), fwd_hooks=[(f"blocks.{layer}.hook_attn_out",
                                      lambda hv, hook: R.layer_addition_hook(hv, hook, vec))])[0, -1]
            assert row.tolist() == torch.topk(ref, 5).indices.tolist()
    clean = streamed.added_topk(seqs, 0, None, 3)
    for s, row in zip(seqs, clean):
        assert row.tolist() == torch.topk(full.forward(torch.tensor([s]))[0, -1], 3).indices.tolist()


def test_rotary_tables_are_the_fp32_references():
    """The fp64 evaluation keeps the fp32 reference's sin / cos tables (TL
    computes them in fp32 for an fp32 model): identical to HookedPythiaOracle's
    fp32 tables; fp64 tables are a different (fp64 TL) model."""
    cfg = tvr_amd.get_config("tiny")
    shapes = tvr_amd.weights.hf_param_shapes(cfg)
    sd = {n: tvr_amd.weights.synth_param(cfg, n, s, 0, "cpu") for n, s in shapes.items()}
    st = StreamedPythiaOracle(oracle_config(cfg), lambda n: sd[n])
    h32 = HookedPythiaOracle(oracle_config(cfg), sd)
    h64 = HookedPythiaOracle(oracle_config(cfg), sd, dtype=torch.float64)
    assert torch.equal(st._sin, h32._sin.double()) and torch.equal(st._cos, h32._cos.double())
    assert not torch.equal(st._sin, h64._sin)


def test_layer_sweep_equals_reference_loops(pair):
    """StreamedPythiaOracle.layer_sweep against the reference's two layer sweeps
    (scratch2.py:114-127 accuracy, :135-150 Δprob; late-binding closure: the
    last vector at every layer) run on the whole-model hooked oracle."""
    cfg, tok, full, streamed, _ = pair
    r = random.Random(6)
    xs = [f"<|{r.randrange(100, cfg.d_vocab)}|>" for _ in range(8)]
    seqs = [[0, tok.encode(x)[0], tok.encode(ARROW)[0]] for x in xs]
    g = torch.Generator().manual_seed(8)
    layered = torch.randn(cfg.n_layers, cfg.d_model, generator=g, dtype=torch.float64) * 2
    # answers: half the clean top-1, half the top-1 with the vector at layer 1 (accuracies neither 0 nor 1)
    top_clean = streamed.added_topk(seqs, 0, None, 1)[:, 0]
    top_l1 = streamed.added_topk(seqs, 1, layered[-1], 1)[:, 0]
    ys = [tok.decode_one(int((top_clean if i % 2 else top_l1)[i])) for i in range(len(xs))]
    contexts = list(zip(xs, ys))
    acc_ref = R.apply_layered_vectors_to_zero_shot(layered, contexts, ARROW, full)
    dp_ref = R.apply_layered_vectors_to_zero_shot_by_probability(layered, contexts, ARROW, full)
    targets = [tok.encode(y)[0] for y in ys]
    p0, P, ids, vals = streamed.layer_sweep(seqs, layered[-1], targets)
    acc = [sum(tok.decode_one(int(ids[i, l, 0])) == ys[i] for i in range(len(xs))) / len(xs)
           for l in range(cfg.n_layers)]
    assert acc == acc_ref
    assert any(0 < a < 1 for a in acc)
    dp = (P - p0[:, None]).mean(0)
    assert (dp - dp_ref.double()).abs().max().item() <= 1e-12 * dp_ref.abs().max().item()
    assert (vals[..., 0] >= vals[..., 1]).all()
    sub = streamed.layer_sweep(seqs, layered[-1], targets, layers=[2, 0])
    assert torch.equal(sub[1], P[:, [2, 0]]) and torch.equal(sub[2], ids[:, [2, 0]])


def test_rounded_engine_entry_form_is_the_same_cie(pair):
    """oracle/rounded_pythia.py's ``entry_engine`` rule (the engine's REPLACE_HEAD
    entry: clean attention output − z_h W_O[h] + vector, fp32 operands) with no
    operand rounding gives the reference's CIE to fp32 operand precision."""
    from oracle.rounded_pythia import Rounded
    cfg, tok, full, streamed, _ = pair
    emu = Rounded(streamed.cfg, streamed._get, {"entry_engine": True})
    g = torch.Generator().manual_seed(3)
    mean = torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, generator=g, dtype=torch.float64)
    r = random.Random(1)
    prompts = [[0] + [r.randrange(1, cfg.d_vocab) for _ in range(10)] for _ in range(2)]
    answers = [int(row.argmax()) for row in streamed.last_logits(prompts)]
    want = streamed.cie(mean, prompts, answers)
    got = emu.cie(mean, prompts, answers)
    assert (got - want).abs().max().item() <= 1e-5 * want.abs().max().item()
    assert want.abs().max().item() > 1e-3

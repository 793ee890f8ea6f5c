"""Stream-K GEMM launches (csrc/gemm_pingpong.hpp ``sk_blocks``,
splitk_sk_reduce_kernel; engine.hip plan_pp) against the plain / split-K
launches (``TVR_STREAM_K=0``), on the small-M shapes they serve: the C2
layer sweeps (52 prompts x T0 = 3: M = 156 + 52 l rows, 70 column tiles of
the QKV + MLP-in GEMM, 10 of the O + MLP-out one) and a CIE sweep, at the
Pythia-2.8B width (3 layers, std-0.1 weights so the outputs are
informative).  The two differ only in fp32 summation order: logits within
1e-5 relative, probabilities / CIE within 1e-4 of the largest + 1e-7,
top-1 identical; both against the fp32 CPU oracle at the same bars."""
import pytest
import torch

import tvr_amd
from conftest import make_oracle
from oracle import reference_experiments as R

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


@pytest.mark.timeout(900)
def test_stream_k_matches_plain_launches(monkeypatch):
    cfg = tvr_amd.get_config("pythia-2.8b").with_(n_layers=3)
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0, std=0.1)
    tok = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
    model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda", tokenizer=tok)
    oracle = make_oracle(cfg, sd, tok)
    task = list(tvr_amd.tasks.letter_to_caps)
    arrow = tvr_amd.tasks.ARROW
    prompts, _ = tvr_amd.prompts.synthetic_cie_prompts(model, 2, 4, seed=1234)
    answers = [int(t) for t in model.forward_clean(prompts, topk=1)["topk"][:, 0].tolist()]
    g = torch.Generator().manual_seed(5)
    mean = (torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, generator=g) * 0.5).cuda()
    layered = tvr_amd.gather_head_activations_to_layers(mean)
    out = {}
    for sk in ("1", "0"):
        monkeypatch.setenv("TVR_STREAM_K", sk)
        clean = model.forward_clean([[0, 5, 9]] * 52, topk=1, return_logits=True)  # 156 rows: 70 + 10 tiles
        dp = tvr_amd.apply_layered_vectors_to_zero_shot_by_probability(layered, task, arrow, model=model)
        acc = tvr_amd.apply_layered_vectors_to_zero_shot(layered, task, arrow, model=model)
        cie = tvr_amd.experiments.causal_indirect_effect_sums(mean, prompts, answers, model).cpu().double()
        out[sk] = (clean["logits"][0].cpu().double(), dp.cpu().double(), acc, cie)
    (l1, d1, a1, c1), (l0, d0, a0, c0) = out["1"], out["0"]
    assert ((l1 - l0).abs().max() / l0.abs().max()).item() < 1e-5
    assert (d1 - d0).abs().max().item() <= 1e-4 * d0.abs().max().item() + 1e-7
    assert a1 == a0
    assert (c1 - c0).abs().max().item() <= 1e-4 * c0.abs().max().item() + 1e-7
    # both against the CPU oracle (the reference's loops)
    ref = oracle.forward(torch.tensor([[0, 5, 9]]))[0, -1].double()
    assert ((l1 - ref).abs().max() / ref.abs().max()).item() < 1e-4
    ref_dp = R.apply_layered_vectors_to_zero_shot_by_probability(layered.cpu(), task, arrow, oracle).double()
    assert (d1 - ref_dp).abs().max().item() <= 1e-4 * ref_dp.abs().max().item() + 1e-7
    model._check_range("stream-K test")


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", ["pythia-2.8b", "pythia-12b"])
def test_row_attention_matches_tile_kernel(name, monkeypatch):
    """attention_row_kernel (one query row per sequence: last-position sites,
    every sweep's trimmed last layer) against attention_mfma_kernel
    (TVR_ROW_ATTN=0) at d_head 80 / 128, and against the CPU oracle: a layer
    sweep's Δprob / accuracy, a clean forward's last-row logits and a CIE
    (whose last layer is single-row)."""
    cfg = tvr_amd.get_config(name).with_(n_layers=3)
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0, std=0.1)
    tok = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
    model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda", tokenizer=tok)
    oracle = make_oracle(cfg, sd, tok)
    task = list(tvr_amd.tasks.letter_to_caps)[:20]
    arrow = tvr_amd.tasks.ARROW
    prompts, _ = tvr_amd.prompts.synthetic_cie_prompts(model, 2, 4, seed=1234)
    answers = [int(t) for t in model.forward_clean(prompts, topk=1)["topk"][:, 0].tolist()]
    g = torch.Generator().manual_seed(5)
    mean = (torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, generator=g) * 0.5).cuda()
    layered = tvr_amd.gather_head_activations_to_layers(mean)
    out = {}
    for ra in ("1", "0"):
        monkeypatch.setenv("TVR_ROW_ATTN", ra)
        logits = model.forward_clean(prompts, topk=1, return_logits=True)["logits"].cpu().double()
        dp = tvr_amd.apply_layered_vectors_to_zero_shot_by_probability(layered, task, arrow, model=model)
        acc = tvr_amd.apply_layered_vectors_to_zero_shot(layered, task, arrow, model=model)
        cie = tvr_amd.experiments.causal_indirect_effect_sums(mean, prompts, answers, model).cpu().double()
        out[ra] = (logits, dp.cpu().double(), acc, cie)
    (l1, d1, a1, c1), (l0, d0, a0, c0) = out["1"], out["0"]
    assert ((l1 - l0).abs().max() / l0.abs().max()).item() < 1e-5
    assert (d1 - d0).abs().max().item() <= 1e-4 * d0.abs().max().item() + 1e-7
    assert a1 == a0
    assert (c1 - c0).abs().max().item() <= 1e-4 * c0.abs().max().item() + 1e-7
    ref = torch.stack([oracle.forward(torch.tensor([p]))[0, -1] for p in prompts]).double()
    assert ((l1 - ref).abs().max() / ref.abs().max()).item() < 1e-4
    ref_dp = R.apply_layered_vectors_to_zero_shot_by_probability(layered.cpu(), task, arrow, oracle).double()
    assert (d1 - ref_dp).abs().max().item() <= 1e-4 * ref_dp.abs().max().item() + 1e-7
    assert a1 == R.apply_layered_vectors_to_zero_shot(layered.cpu(), task, arrow, oracle)
    model._check_range("row attention test")


def _sweeps(model, prompts, answers, mean, layered, task, arrow):
    logits = model.forward_clean(prompts, topk=1, return_logits=True)["logits"].cpu().double()
    dp = tvr_amd.apply_layered_vectors_to_zero_shot_by_probability(layered, task, arrow, model=model)
    acc = tvr_amd.apply_layered_vectors_to_zero_shot(layered, task, arrow, model=model)
    cie = tvr_amd.experiments.causal_indirect_effect_sums(mean, prompts, answers, model).cpu().double()
    return logits, dp.cpu().double(), acc, cie


def _ab_against_oracle(name, kshot, env, monkeypatch, n_prompts=3):
    """The same sweeps with ``env`` = "1" and "0" (an engine A/B switch read per
    launch), compared with each other and the CPU oracle (the reference's
    loops): clean logits 1e-5 between forms / 1e-4 vs the oracle, Δprob and
    CIE 1e-4 of the largest + 1e-7, accuracies identical."""
    cfg = tvr_amd.get_config(name).with_(n_layers=3)
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0, std=0.1)
    tok = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
    model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda", tokenizer=tok)
    oracle = make_oracle(cfg, sd, tok)
    # the CIE against fp64 (the fp32 reference's own accumulation error reaches ~1e-4 of max |CIE| at 12B width)
    oracle64 = make_oracle(cfg, sd, tok, dtype=torch.float64, rotary_table_dtype=torch.float32)
    task = list(tvr_amd.tasks.letter_to_caps)[:20]
    arrow = tvr_amd.tasks.ARROW
    # several prompts share their leading tokens (BOS and, for the CIE, the sites' prefix rows)
    prompts, _ = tvr_amd.prompts.synthetic_cie_prompts(model, n_prompts, kshot, seed=1234)
    answers = [int(t) for t in model.forward_clean(prompts, topk=1)["topk"][:, 0].tolist()]
    g = torch.Generator().manual_seed(5)
    mean = (torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, generator=g) * 0.5).cuda()
    layered = tvr_amd.gather_head_activations_to_layers(mean)
    out = {}
    for v in ("1", "0"):
        monkeypatch.setenv(env, v)
        out[v] = _sweeps(model, prompts, answers, mean, layered, task, arrow)
    (l1, d1, a1, c1), (l0, d0, a0, c0) = out["1"], out["0"]
    assert ((l1 - l0).abs().max() / l0.abs().max()).item() < 1e-5
    assert (d1 - d0).abs().max().item() <= 1e-4 * d0.abs().max().item() + 1e-7
    assert a1 == a0
    assert (c1 - c0).abs().max().item() <= 1e-4 * c0.abs().max().item() + 1e-7
    ref = torch.stack([oracle.forward(torch.tensor([p]))[0, -1] for p in prompts]).double()
    assert ((l1 - ref).abs().max() / ref.abs().max()).item() < 1e-4
    heads = [0, 1, cfg.n_heads - 1]  # the CPU oracle's batch-1 loop on a subset of the heads (time)
    ref_cie = R.calculate_average_causal_indirect_effect(mean.cpu().double(), prompts, [[a] for a in answers], oracle64,
                                                         heads=heads).double()[:, heads]
    c1m = c1[:, heads] / len(prompts)
    err = (c1m - ref_cie).abs().max().item()
    print(f"{name} {env} k={kshot} T={len(prompts[0])}: CIE err {err:.2e} of max {ref_cie.abs().max():.2e}")
    assert err <= 1e-4 * ref_cie.abs().max().item() + 1e-7
    ref_dp = R.apply_layered_vectors_to_zero_shot_by_probability(layered.cpu(), task, arrow, oracle).double()
    assert (d1 - ref_dp).abs().max().item() <= 1e-4 * ref_dp.abs().max().item() + 1e-7
    model._check_range(f"{env} A/B test")


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name,kshot", [("pythia-2.8b", 5), ("pythia-2.8b", 9), ("pythia-12b", 6)])
def test_vstage_attention_matches_direct_loads(name, kshot, monkeypatch):
    """Two-key-tile attention (16 < T <= 32: T = 18 / 30 / 21 here) with V
    staged through LDS (STAGE 3, TVR_ATT_VSTAGE=1, the default) against V
    loaded directly (=0), at d_head 80 and 128, including the CIE sweep's
    shared-prefix (K / V cache) rows — ADVICE r4."""
    _ab_against_oracle(name, kshot, "TVR_ATT_VSTAGE", monkeypatch)


@pytest.mark.timeout(900)
def test_sliced_split_and_stream_k_at_12b_width(monkeypatch):
    """Pythia-12B width (O + MLP-out K = 25,600: every x2f16 GEMM of the model
    runs the sliced accumulation) at small M, so the planner splits: the sliced
    split-K (TVR_STREAM_K=0) and sliced stream-K (=1) instantiations against
    each other and the CPU oracle — ADVICE r4."""
    _ab_against_oracle("pythia-12b", 4, "TVR_STREAM_K", monkeypatch, n_prompts=2)

"""GPU: the linearised entry layer of head-replacement sites (lin_entry.hpp).

In a fused sweep (clean rows inside the sweep, as the CIE runs it), the first
layer after a REPLACE_HEAD site's layer computes its entering rows' QKV +
MLP-in outputs from the clean rows' outputs and a K = d_head GEMM against
W1[l] W_O[l-1] instead of the full K = d_model GEMM.  These tests run models
of >= 3 layers (the 2-layer tiny model has no such layer) and compare

* the CIE over every (layer, head) site with the fp32 CPU oracle running the
  reference's loop (scratch2.py:171-197, oracle/reference_experiments.py),
* patched logits / top-k / probabilities with the same sweep through the full
  GEMM (TVR_LIN_ENTRY=0): within 1e-5 relative (fp32-level reassociation),
* sweeps whose entry layers mix kinds (the linearised path is skipped for a
  layer with a non-REPLACE entering site, kept for the others), shared
  prefixes (followers enter at position 1) and ragged prompts,

on both planar GEMM paths (x2f16: fp32-accurate; bf16 at its own tolerance).
"""
import random

import pytest
import torch

import tvr_amd
from conftest import TINY_STD, make_oracle
from oracle import reference_experiments as R
from tvr_amd import experiments as E

pytestmark = pytest.mark.gpu

L4 = 4


def rel_err(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def deep():
    cfg = tvr_amd.get_config("tiny").with_(n_layers=L4)
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=3, std=TINY_STD)
    tok = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
    return cfg, sd, tok, make_oracle(cfg, sd, tok)


def prompts_with_shared_prefixes(cfg, n, seed):
    rng = random.Random(seed)
    base = [0] + [rng.randrange(1, cfg.d_vocab) for _ in range(40)]
    out = []
    for i in range(n):
        T = rng.randrange(5, 30)
        keep = rng.choice([1, 1, 3, 8])  # BOS only (most), or a longer common prefix
        out.append(base[:keep] + [rng.randrange(1, cfg.d_vocab) for _ in range(T - keep)])
    return out


def sweep(model, prompts, sites, vecs, monkeypatch, lin):
    monkeypatch.setenv("TVR_LIN_ENTRY", "1" if lin else "0")
    trace = model.trace(len(prompts), sum(map(len, prompts)))
    clean = model.forward_clean(prompts, targets=[p[1] for p in prompts], topk=3, trace=trace, defer=True)
    out = model.patch_sweep(trace, sites, vecs, topk=3, return_logits=True)
    torch.cuda.synchronize()
    return out, clean


@pytest.mark.parametrize("gemm", ["x2f16", "bf16"])
def test_cie_matches_oracle_with_lin_entry(deep, gemm):
    cfg, sd, tok, oracle = deep
    model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda", tokenizer=tok, gemm=gemm)
    random.seed(5)
    task = tvr_amd.tasks.letter_to_caps
    mean_ref = R.generate_mean_activation(list(task), tvr_amd.tasks.ARROW, ",", oracle, 16, 4)
    prompts, answers = tvr_amd.generate_shuffled_prompts(task, model, 4, 4, tvr_amd.tasks.ARROW)
    cie_ref = R.calculate_average_causal_indirect_effect(mean_ref, prompts, answers, oracle)
    cie = tvr_amd.calculate_average_causal_indirect_effect(mean_ref.cuda(), prompts, answers, model=model).cpu()
    bound = cie_ref.abs().max().item()
    err = (cie.double() - cie_ref.double()).abs().max().item()
    if gemm == "x2f16":
        bar = 1e-4 * bound + 1e-7
    else:  # bf16: the north star's 2e-2, of the largest probability involved (as the headline-width tests)
        tp, ta = tvr_amd.experiments.normalize_cie_inputs(model, prompts, answers)
        p_clean = model.forward_clean(tp, targets=ta)["prob"]
        bar = 2e-2 * (p_clean.max().item() + bound)  # p_clean + |CIE| bounds the patched probabilities
    print(f"{gemm}: CIE err {err:.3e} (max |CIE| {bound:.3e}, bar {bar:.3e})")
    assert err <= bar
    if gemm == "x2f16":  # the highest-effect heads are the same
        assert torch.topk(cie.flatten(), 5).indices.tolist() == torch.topk(cie_ref.flatten(), 5).indices.tolist()
    model._check_range("lin entry test")


@pytest.mark.parametrize("gemm", ["x2f16", "bf16"])
def test_lin_entry_equals_full_entry_gemm(deep, gemm, monkeypatch):
    cfg, sd, tok, oracle = deep
    model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda", tokenizer=tok, gemm=gemm)
    prompts = prompts_with_shared_prefixes(cfg, 6, seed=11)
    g = torch.Generator().manual_seed(2)
    vecs = (torch.randn(cfg.n_layers * cfg.n_heads + 2, cfg.d_model, generator=g) * 0.5).cuda()
    # every (layer, head) of every prompt, plus: layer 2's entering sites mixed with an
    # ADD_ATTN_OUT site and a SET_RESID site (entry layer 2 -> full GEMM there; layer 1 stays linearised)
    combos = [(l, h) for l in range(cfg.n_layers) for h in range(cfg.n_heads)]
    n = len(prompts) * len(combos) + 2
    sites = tvr_amd.make_sites(n)
    k = 0
    for i, p in enumerate(prompts):
        for l, h in combos:
            s = sites[k]
            s["seq"], s["kind"], s["layer"], s["head"], s["vec"], s["target"] = (
                i, tvr_amd._lib.SITE_REPLACE_HEAD_ALLPOS, l, h, l * cfg.n_heads + h, p[1])
            k += 1
    s = sites[k]
    s["seq"], s["kind"], s["layer"], s["vec"], s["target"] = 0, tvr_amd._lib.SITE_ADD_ATTN_OUT_LASTPOS, 1, \
        cfg.n_layers * cfg.n_heads, prompts[0][1]
    s = sites[k + 1]
    s["seq"], s["kind"], s["layer"], s["pos"], s["src_seq"], s["src_pos"], s["target"] = (
        1, tvr_amd._lib.SITE_SET_RESID_PRE_POS, 2, len(prompts[1]) - 2, 2, len(prompts[2]) - 2, prompts[1][1])
    on, clean_on = sweep(model, prompts, sites, vecs, monkeypatch, True)
    off, clean_off = sweep(model, prompts, sites, vecs, monkeypatch, False)
    tol = 1e-5 if gemm == "x2f16" else 2e-2
    assert rel_err(on["logits"], off["logits"]) < tol
    assert (on["prob"] - off["prob"]).abs().max().item() <= tol * off["prob"].abs().max().item() + 1e-7
    if gemm == "x2f16":
        assert torch.equal(on["topk"], off["topk"])
        assert torch.equal(clean_on["topk"], clean_off["topk"])
    assert rel_err(clean_on["prob"], clean_off["prob"]) < 1e-6
    # and each REPLACE site against the oracle's hook on its own prompt (x2f16: fp32 bar)
    if gemm == "x2f16":
        oracle.cfg.use_attn_result = True
        try:
            for j in range(0, len(prompts) * len(combos), 7):
                s = sites[j]
                v = vecs[int(s["vec"])].cpu()

                def hook(x, hook, h=int(s["head"]), v=v):
                    x[0, :, h, :] = v
                    return x
                ref = oracle.run_with_hooks(torch.tensor([prompts[int(s["seq"])]]),
                                            fwd_hooks=[(f"blocks.{int(s['layer'])}.attn.hook_result", hook)])[0, -1]
                assert rel_err(on["logits"][j], ref) < 1e-4, (j, s)
                assert on["topk"][j].tolist() == torch.topk(ref, 3).indices.tolist(), j
        finally:
            oracle.cfg.use_attn_result = False
    model._check_range("lin entry test")


# real widths, 3 layers (layer 1 is the linearised entry layer of the layer-0
# sites): kernels at their headline shapes (KP 96 for d_head 80, 128 for 128;
# N = D1 17920 / 35840 / 28672).  std-0.1 weights make these models sensitive
# (the answer's probability moves by up to half).  Each entry path (linearised
# and full GEMM) against the fp64 oracle running the reference's loop
# (scratch2.py:171-197) on every site of one prompt, the fp32 reference's rotary
# tables (oracle/streamed_pythia.py):
# * x2f16: the north star's 1e-4 of the largest |CIE| + 1e-7, top-5 heads
#   identical, and the two paths within the same bar of each other;
# * bf16: no more than 1.5x the error bf16 rounding of the same GEMM operands
#   produces in the fp64 oracle (oracle/rounded_pythia.py, variant
#   "engine_bf16": the bf16 planes and the fp16 Q / K operands of csrc/), so a
#   regression in code both entry paths share shows against the oracle, not
#   only against the other path; and the paths within 5e-2 of p_max of each
#   other (each rounds its own way).
# (fp16w: fp16-valued weights — the exact-fp16 GEMMs, the linearised entry's G = v W1'^T as ((v - mean) o gamma)
# W1^T on the raw rows, lin_entry.hpp lin_gamma_rows_kernel)
WIDE = [("pythia-2.8b", "x2f16", 4), ("pythia-12b", "x2f16", 10), ("pythia-6.9b", "bf16", 5),
        ("pythia-2.8b", "x2f16-fp16w", 4), ("pythia-12b", "x2f16-fp16w", 10)]


@pytest.mark.slow
@pytest.mark.timeout(900)
@pytest.mark.parametrize("name,gemm,kshot", WIDE, ids=[f"{n}-{g}" for n, g, _ in WIDE])
def test_lin_entry_at_headline_widths(name, gemm, kshot, monkeypatch):
    fp16 = gemm.endswith("-fp16w")
    gemm = gemm.replace("-fp16w", "")
    cfg = tvr_amd.get_config(name).with_(n_layers=3)
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0, std=0.1, fp16=fp16)
    tok = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
    model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda", tokenizer=tok, gemm=gemm)
    assert model.exact16 == fp16
    prompts, _ = tvr_amd.prompts.synthetic_cie_prompts(model, 2, kshot, seed=1234)
    clean = model.forward_clean(prompts, topk=1)
    answers = [[int(t)] for t in clean["topk"][:, 0].tolist()]  # p ~ 1e-9 for random pairs: use the argmax
    pmax = model.forward_clean(prompts, targets=[a[0] for a in answers])["prob"].max().item()
    random.seed(3)
    letters = list(tvr_amd.tasks.letter_to_caps)
    mean = tvr_amd.generate_mean_activation(letters, tvr_amd.tasks.ARROW, ",", model=model, num_contexts=8,
                                            len_contexts=4)
    cies = {}
    for lin in ("1", "0"):
        monkeypatch.setenv("TVR_LIN_ENTRY", lin)
        cies[lin] = tvr_amd.calculate_average_causal_indirect_effect(mean, prompts, answers,
                                                                     model=model).cpu().double()
    big = cies["0"].abs().max().item()
    assert big > 1e-3  # informative: the patches move the answer's probability
    ref = R.calculate_average_causal_indirect_effect(
        mean.cpu().double(), prompts[:1], answers[:1],
        make_oracle(cfg, sd, tok, dtype=torch.float64, rotary_table_dtype=torch.float32))
    rmax = ref.abs().max().item()
    lin_full = (cies["1"] - cies["0"]).abs().max().item()
    errs = {}
    for lin in ("1", "0"):
        monkeypatch.setenv("TVR_LIN_ENTRY", lin)
        one = tvr_amd.calculate_average_causal_indirect_effect(mean, prompts[:1], answers[:1], model=model)
        errs[lin] = ((one.cpu().double() - ref).abs().max().item(), one.cpu())
    if gemm == "x2f16":
        bar = 1e-4 * rmax + 1e-7
        print(f"{name} x2f16: max |CIE| {rmax:.3e}; err vs fp64 linearised {errs['1'][0]:.2e}, full "
              f"{errs['0'][0]:.2e} (bar {bar:.2e}); linearised vs full entry {lin_full:.2e}")
        assert lin_full <= 1e-4 * big + 1e-7, lin_full  # fp32 summation order only
        for lin in ("1", "0"):
            assert errs[lin][0] <= bar, (lin, errs[lin][0], bar)
            assert torch.topk(errs[lin][1].flatten(), 5).indices.tolist() == \
                torch.topk(ref.flatten(), 5).indices.tolist(), lin
    else:
        from oracle.rounded_pythia import Rounded, variants
        from oracle.streamed_pythia import StreamedPythiaOracle
        from conftest import oracle_config
        get = lambda n: sd[n].cuda()  # noqa: E731
        base = StreamedPythiaOracle(oracle_config(cfg), get)
        emu = Rounded(oracle_config(cfg), get, variants()["engine_bf16"])
        m64 = mean.double()
        floor = (emu.cie(m64, prompts[:1], [a[0] for a in answers[:1]]) -
                 base.cie(m64, prompts[:1], [a[0] for a in answers[:1]])).abs().max().item()
        print(f"{name} bf16: p_max {pmax:.3f}; CIE err vs fp64 linearised {errs['1'][0]:.3e}, full {errs['0'][0]:.3e}"
              f"; emulated bf16-operand floor {floor:.3e}; linearised vs full entry {lin_full:.3e}")
        assert lin_full <= 5e-2 * pmax, (lin_full, pmax)
        for lin in ("1", "0"):
            assert errs[lin][0] <= 1.5 * floor, (lin, errs[lin][0], floor)
    model._check_range("lin entry headline widths")


@pytest.mark.slow
@pytest.mark.timeout(900)
@pytest.mark.parametrize("name,gemm,kshot", [("pythia-2.8b", "x2f16", 4), ("pythia-6.9b", "bf16", 5),
                                             ("pythia-2.8b", "x2f16-fp16w", 4)],
                         ids=["pythia-2.8b-x2f16", "pythia-6.9b-bf16", "pythia-2.8b-x2f16-fp16w"])
def test_lin_entry_head_shard_at_headline_widths(name, gemm, kshot, monkeypatch):
    """One rank's share of an 8-way head split (heads h = 0 mod 8): 4 distinct
    vectors per entry layer, so the linearised entry's G = v W1^T runs on
    gemm_skinny_kernel (<= 16 rows) at the real K / N (2560 / 17920, 4096 /
    28672), against the full entry GEMM at the bars of the test above.  fp16w:
    the one-plane G on the raw W1 with NON-centred vectors (the random means
    below: the centring in lin_gamma_rows_kernel is what makes it exact)."""
    fp16 = gemm.endswith("-fp16w")
    gemm = gemm.replace("-fp16w", "")
    cfg = tvr_amd.get_config(name).with_(n_layers=3)
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0, std=0.1, fp16=fp16)
    tok = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
    model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda", tokenizer=tok, gemm=gemm)
    assert model.exact16 == fp16
    prompts, _ = tvr_amd.prompts.synthetic_cie_prompts(model, 2, kshot, seed=1234)
    answers = [int(t) for t in model.forward_clean(prompts, topk=1)["topk"][:, 0].tolist()]
    pmax = model.forward_clean(prompts, targets=answers)["prob"].max().item()
    g = torch.Generator().manual_seed(5)
    mean = (torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, generator=g) * 0.5).cuda()
    heads = list(range(0, cfg.n_heads, 8))
    sums = {}
    for lin in ("1", "0"):
        monkeypatch.setenv("TVR_LIN_ENTRY", lin)
        sums[lin] = E.causal_indirect_effect_sums(mean, prompts, answers, model, heads=heads).cpu().double()
    big = sums["0"].abs().max().item()
    assert big > 1e-3
    other = [h for h in range(cfg.n_heads) if h not in heads]
    assert sums["1"][:, other].abs().max().item() == 0.0
    bar = 1e-4 * big + 1e-7 if gemm == "x2f16" else 5e-2 * pmax  # bf16: two bf16 paths, rounded differently
    d = (sums["1"] - sums["0"]).abs().max().item()
    print(f"{name} {gemm} head shard: linearised vs full entry {d:.3e} (bar {bar:.3e})")
    assert d <= bar
    model._check_range("lin entry head shard")

"""Exact-fp16 weights (include/tvr.h ``tvr_model_set_exact16``, engine.hip x16).

Every released Pythia checkpoint stores its tensors as float16.  With such
weights the x2f16 GEMMs run on the checkpoint's own W1 rows (LN gamma applied
to the LNPre rows: Q | K | V columns read x̂·γ1, MLP-in columns x̂·γ2) and its
uncentred W2, whose residual-plane product is exactly zero: 2 matrix products
per slice instead of 3 (gemm_pingpong.hpp WX).  The residual stream then
carries one constant per row (every LayerNorm removes it; the trace export
subtracts it).  Checked here, on fp16-valued synthetic weights:

* the reference functions at the 2.8B (one launch, per-tile A operand) and 12B
  (sliced accumulation) widths against the fp32 oracle on the SAME weights, at
  tests/test_gpu_headline_shapes.py's fp32 bars (1e-4);
* the exact-fp16 path against the processed-weight path of the same model
  (set_exact16(False)): clean logits, every CIE site, the extraction and the
  trace's hook_resid_pre export agree to fp32 rounding (bar 2e-5 of max; the CIE 5e-5);
* the tiny model (d 64: the Q | K | V / MLP-in boundary inside a 256-column
  tile, two launches) the same way.
"""
import random

import pytest
import torch

import tvr_amd
import test_gpu_headline_shapes as H

pytestmark = [pytest.mark.gpu]

ARROW = tvr_amd.tasks.ARROW
# exact16 vs the processed-weight path: fp32 rounding differences of two exact rewrites only — 2e-5 of max
# (measured <= 9.4e-6: logits 3.3e-6, extraction 7.0e-6, the centred trace export 8.1e-6 at the 12B width,
# fused-statistics probabilities 9.4e-6); the CIE, a difference of two probabilities, cancels: 5e-5 of
# max |CIE| (measured 1.3-2.7e-5; each path is within the fp32 bar of 1e-4 of the oracle)
X16_TOL = 2e-5
X16_TOL_CIE = 5e-5
X16_TOL_PROB = 2e-5


def rel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _run(model, prompts, answers, mean_in):
    out = model.forward_clean(prompts, targets=answers, topk=5, return_logits=True)
    # without logits: the fused-statistics unembed (exact-fp16 W_U when bound)
    fused = model.forward_clean(prompts, targets=answers, topk=5)
    out["prob_fused"], out["topk_fused"] = fused["prob"], fused["topk"]
    sums = tvr_amd.experiments.causal_indirect_effect_sums(mean_in, prompts, answers, model)
    tr = model.trace(len(prompts), sum(len(p) for p in prompts))
    model.forward_clean(prompts, trace=tr)
    resid = [tr.resid_pre(l).clone() for l in range(model.cfg.n_layers + 1)]
    random.seed(3)
    mean = tvr_amd.generate_mean_activation(list(tvr_amd.tasks.letter_to_caps), ARROW, ",", model=model,
                                            num_contexts=8, len_contexts=4)
    return out, sums.clone(), resid, mean


def _compare_paths(model, prompts, answers, mean_in):
    assert model.exact16
    a = _run(model, prompts, answers, mean_in)
    model.set_exact16(False)
    try:
        b = _run(model, prompts, answers, mean_in)
    finally:
        model.set_exact16(True)
    (oa, sa, ra, ma), (ob, sb, rb, mb) = a, b
    errs = {"logits": rel(oa["logits"], ob["logits"]), "prob": rel(oa["prob"], ob["prob"]),
            "prob_fused": rel(oa["prob_fused"], ob["prob_fused"]),
            "cie": rel(sa, sb), "extraction": rel(ma, mb),
            "resid_pre": max(rel(x, y) for x, y in zip(ra, rb))}
    print("exact16 vs processed weights:", {k: f"{v:.2e}" for k, v in errs.items()})
    for k, v in errs.items():
        assert v <= (X16_TOL_CIE if k == "cie" else X16_TOL_PROB if k.startswith("prob") else X16_TOL), (k, v)
    assert oa["topk"].tolist() == ob["topk"].tolist()
    assert oa["topk_fused"].tolist() == ob["topk_fused"].tolist() == oa["topk"].tolist()
    assert model.weights.raw16_unembed is not None
    # the raw path's trace rows are centred on export, as TL's residual stream is
    for x in ra:
        assert x.double().mean(dim=1).abs().max().item() <= 1e-5 * x.abs().max().item()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("width", ["2.8b", "12b"])
def test_exact16_width_parity(width):
    r = H.reference(width, fp16=True)
    model = tvr_amd.Model.from_hf_state_dict(r["cfg"], r["sd"], device="cuda", tokenizer=r["tok"], gemm="x2f16")
    try:
        assert model.exact16 and model.weights.raw16 is not None
        H.check_width(r, model, "x2f16")
        _compare_paths(model, r["prompts"], r["answers"], r["mean"].cuda())
    finally:
        del model
        torch.cuda.empty_cache()


def test_exact16_tiny_two_launch_boundary(tiny_cfg, tokenizer):
    sd = tvr_amd.weights.synth_hf_state_dict(tiny_cfg, seed=0, std=0.3, fp16=True)
    model = tvr_amd.Model.from_hf_state_dict(tiny_cfg, sd, device="cuda", tokenizer=tokenizer, gemm="x2f16")
    assert model.exact16 and (3 * tiny_cfg.d_model) % 256 != 0
    g = torch.Generator().manual_seed(5)
    prompts = [[0] + torch.randint(1, tiny_cfg.d_vocab, (int(n),), generator=g).tolist() for n in (5, 9, 12)]
    answers = [int(x) for x in torch.randint(0, tiny_cfg.d_vocab, (3,), generator=g)]
    mean = torch.randn(tiny_cfg.n_layers, tiny_cfg.n_heads, tiny_cfg.d_model, generator=g).cuda() * 0.3
    _compare_paths(model, prompts, answers, mean)


def test_exact16_off_other_modes_and_fp32_weights(tiny_cfg, tiny_sd, tokenizer):
    """fp32-valued weights keep the processed path; other GEMM modes ignore the binding."""
    m32 = tvr_amd.Model.from_hf_state_dict(tiny_cfg, tiny_sd, device="cuda", tokenizer=tokenizer)
    assert not m32.exact16 and m32.weights.raw16 is None
    with pytest.raises(ValueError):
        m32.set_exact16(True)
    sd = tvr_amd.weights.synth_hf_state_dict(tiny_cfg, seed=0, std=0.3, fp16=True)
    m = tvr_amd.Model.from_hf_state_dict(tiny_cfg, sd, device="cuda", tokenizer=tokenizer, gemm="f32")
    ids = [[0, 5, 7, 9, 11]]
    a = m.forward_clean(ids, return_logits=True)["logits"]
    m.set_exact16(False)
    b = m.forward_clean(ids, return_logits=True)["logits"]
    assert torch.equal(a, b)  # f32 mode: the binding changes nothing

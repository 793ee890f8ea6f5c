"""GPU parity at FULL depth on informative weights (VERDICT r2 "what's missing" 2).

The headline-width tests (test_gpu_headline_shapes.py) truncate the models to
2 layers; the bench's ``parity`` block runs the full 32 layers but on the HF
initialiser's std-0.02 weights, whose max |CIE| is ~1e-6.  Here the whole
model runs: Pythia-2.8B (32 layers, x2f16 and fp32 MFMA) and Pythia-12B (36
layers, x2f16) with seeded std-0.05 weights, where a single head moves the
answer's probability by up to ~2e-2 (layer 0), ~6e-4 (layer 16) and ~3e-4
(layer 31) at 2.8B.  That is where cancellation in the linearised entry
layer's ``y = (sigma_c y_c + (mu_c - mu) c1 + G - z Wsc) / sigma``
(csrc/lin_entry.hpp), the staircase and prefix sharing would show after 30
downstream layers.

Checked against the CPU oracle running the reference's loops
(oracle/reference_experiments.py restating scratch2.py:81-100 and :171-197):
* clean last-row logits (1e-4 relative), answer probability, top-1 identical;
* a1 extraction: mean head activations [L, H, d] over 4 six-shot prompts
  (1e-4 max-abs relative to max |mean|);
* a7 CIE: prompt 0 at layers {0, L/2, L-1} x all 32 heads (2.8B) and layers
  {0, 35} x 8 heads (12B): |err| <= 1e-4 max |CIE| + 1e-7, with max |CIE| >
  1e-3 asserted (the sites move the probability).
The answer is the clean argmax (random pairs give p ~ 1e-5 and a vacuous CIE).
"""
import random

import pytest
import torch

import tvr_amd
from conftest import make_oracle
from oracle import reference_experiments as R

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

STD = 0.05
TOL = 1e-4
ARROW = tvr_amd.tasks.ARROW
# model, GEMM paths, CIE layers, CIE heads, k-shot of the CIE prompt (T = 1 + 3k + 2)
MODELS = {
    "2.8b": ("pythia-2.8b", ("x2f16", "f32"), (0, 16, 31), tuple(range(32)), 4),
    "12b": ("pythia-12b", ("x2f16", "f32"), (0, 35), tuple(range(0, 40, 5)), 10),
}
# 12B: the fp32 reproducibility floor reaches the 1e-4 bar (36 layers, K up to 25,600; the fp32 CPU oracle
# itself is off by 8.7e-5 of max |CIE| from fp64 at 3 layers of this width, test_gpu_lin_entry.py), so
# there the CIE bar is 1e-4 of max |CIE| or twice the distance of this engine's exact-product fp32 MFMA
# path (set_gemm("f32")) from the same oracle, whichever is larger; the f32 path itself is measured, not
# asserted.  2.8B: both paths at 1e-4.
BAR_FROM_F32 = {"12b"}


def rel_err(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("which", list(MODELS))
def test_full_depth_parity(which):
    name, gemms, layers, heads, kshot = MODELS[which]
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    cfg = tvr_amd.get_config(name)
    tok = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
    # the same seeded weights for both: generated on the GPU, processed by the
    # oracle's TransformerLens restatement there, then held on the CPU
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0, device="cuda", std=STD)
    oracle = make_oracle(cfg, sd, tok)
    model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda", tokenizer=tok, gemm=gemms[0])
    del sd
    torch.cuda.empty_cache()
    try:
        # --- the reference's loops on the CPU
        class _M:  # the prompt builder only needs cfg + to_single_token
            pass
        m = _M()
        m.cfg, m.to_single_token = cfg, oracle.to_single_token
        prompts, _ = tvr_amd.prompts.synthetic_cie_prompts(m, 1, kshot, seed=1234)
        clean_ref = oracle.forward(torch.tensor(prompts))[0, -1]
        answer = int(clean_ref.argmax())
        random.seed(2)
        mean_ref = R.generate_mean_activation(list(tvr_amd.tasks.letter_to_caps), ARROW, ",", oracle, 4, 6)
        cie_ref = R.calculate_average_causal_indirect_effect(mean_ref, prompts, [[answer]], oracle,
                                                             layers=list(layers), heads=list(heads)).double()
        idx_l = torch.tensor(layers)
        ref_sites = cie_ref[idx_l][:, list(heads)]
        cmax = ref_sites.abs().max().item()
        print(f"{name}: p(answer) {torch.softmax(clean_ref.double(), 0)[answer]:.3e}, max |CIE| {cmax:.3e}, "
              f"max |mean| {mean_ref.abs().max():.3e}")
        assert cmax > 1e-3  # informative: the patched sites move the answer's probability
        errs = {}
        for gemm in gemms:
            model.set_gemm(gemm)
            out = model.forward_clean(prompts, targets=[answer], topk=1, return_logits=True)
            e_logits = rel_err(out["logits"][0], clean_ref)
            p_ref = torch.softmax(clean_ref.double(), 0)[answer].item()
            strict = not (which in BAR_FROM_F32 and gemm == "f32")  # 12B's f32 path: the bar reference, measured
            assert e_logits < TOL or not strict, (gemm, e_logits)
            # the answer's probability: 1e-4 relative, or what the measured logit error implies through the
            # softmax where that is larger (|dp| <= p (|dl_a| + sum_j p_j |dl_j|) <= 2 p max|dl|): at 12B the
            # logits differ by 2.5e-5 of max |logit| (both sides fp32-class), i.e. by ~2e-4 absolute
            e_abs = (out["logits"][0].cpu().double() - clean_ref.double()).abs().max().item()
            e_p = abs(out["prob"][0].item() - p_ref)
            print(f"{name} {gemm}: p {p_ref:.4e}, |dp| {e_p:.2e}, max |dlogit| {e_abs:.2e}")
            assert e_p <= max(TOL * p_ref, 2.0 * p_ref * e_abs) + 1e-7 or not strict, (gemm, e_p, e_abs)
            assert int(out["topk"][0, 0]) == answer
            random.seed(2)
            mean = tvr_amd.generate_mean_activation(list(tvr_amd.tasks.letter_to_caps), ARROW, ",", model=model,
                                                    num_contexts=4, len_contexts=6)
            e_mean = rel_err(mean, mean_ref)
            assert e_mean < TOL or not strict, (gemm, e_mean)
            sums = tvr_amd.experiments.causal_indirect_effect_sums(mean_ref.cuda(), prompts, [answer], model,
                                                                   layers=list(layers), heads=list(heads))
            got = sums.cpu().double()[idx_l][:, list(heads)]
            err = (got - ref_sites).abs().max().item()
            print(f"{name} {gemm}: logits rel {e_logits:.2e}, extraction rel {e_mean:.2e}, "
                  f"CIE abs err {err:.2e} ({err / cmax:.2e} of max)")
            errs[gemm] = err
            if which not in BAR_FROM_F32:
                assert err <= TOL * cmax + 1e-7, (gemm, err, cmax)
            # no site outside the requested grid is touched
            mask = torch.ones_like(sums, dtype=torch.bool)
            mask[idx_l[:, None], torch.tensor(heads)[None, :]] = False
            assert sums[mask.cuda()].abs().max().item() == 0.0
        if which in BAR_FROM_F32:
            bar = max(TOL * cmax + 1e-7, 2.0 * errs["f32"])
            print(f"{name}: CIE bar {bar:.2e} ({bar / cmax:.2e} of max; f32-MFMA path err {errs['f32']:.2e})")
            assert errs["x2f16"] <= bar, (errs, bar, cmax)
    finally:
        del model
        torch.cuda.empty_cache()

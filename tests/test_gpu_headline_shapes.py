"""GPU parity at the headline widths (VERDICT r1 "configs_untested").

Truncated-depth models with the REAL widths of the benchmark configs, so the
kernels the bench times run at their real shapes and are compared with the
fp32 CPU oracle running the reference's loops (oracle/reference_experiments.py):

  2.8B width  d 2560, 32 heads, d_head 80, rotary 20, d_mlp 10240, V 50304
              (C2 / C3: attention_mfma_kernel<*, 80, *>, GEMM N 17920 / K 12800,
              the lnpre register path at d 2560, unembed at V 50304)
  12B width   d 5120, 40 heads, d_head 128, rotary 32, d_mlp 20480, V 50688 (C5)
  6.9B width  d 4096, 32 heads, d_head 128, d_mlp 16384, V 50432, bf16 (C4)

Weights are seeded synthetic with std 0.1 (not the HF init's 0.02, whose
next-token distributions at these widths are flat: every accuracy 0 and
|CIE| ~ 1e-5) so that top-1 / top-5 / accuracy identity means something; the
zero-shot tasks are model-consistent (answers = the oracle's own zero-shot
predictions, as in tests/golden/make_reference_fixtures.py), so baseline
accuracy is 1 and the injected vectors move it.

Checked per width: clean last-row logits / top-5 / target probability,
extraction (a1), both layer sweeps (a4 accuracy, a5 Δprob), the CIE over every
(layer, head) site of every prompt (a7), the FV top-5 accuracy (a10, a11).
Tolerances: fp32 paths as tests/test_gpu_engine.py (1e-4 relative on logits
and vectors, |Δ| <= 1e-4 max|ref| + 1e-7 on probabilities / CIE, accuracies and
top-k identical); bf16 at the north star's 2e-2 (extracted vectors and logits
max-abs relative, the fp32 paths' metric), probabilities, Δprob and CIE within 2e-2
of the largest probability involved, accuracies within 0.1.
"""
import random

import pytest
import torch

import tvr_amd
from conftest import make_oracle
from oracle import reference_experiments as R

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

ARROW = tvr_amd.tasks.ARROW
WIDTHS = {
    # name, layers, prompts, k-shot (T = 1 + 3k + 2), contexts of the zero-shot sweeps
    "2.8b": ("pythia-2.8b", 2, 3, 4, 20),
    "12b": ("pythia-12b", 2, 1, 10, 10),
    "6.9b": ("pythia-6.9b", 2, 2, 5, 12),
}
CASES = [("2.8b", "x2f16"), ("2.8b", "f32"), ("12b", "x2f16"), ("6.9b", "bf16")]
STD = 0.1
# bf16: the north star's 2e-2 bar (stated for extracted vectors) applied to the
# probabilities, Δprob and CIE as well, relative to the largest probability
# involved: with the attention-score projections on fp16 operands (csrc/split.hpp
# store_ln4) the 6.9B-width CIE is off by 1.87e-2 of p_max (2.7e-2 when Q / K
# were bf16, which is what the round-2 bar of 5e-2 covered), Δprob by 4.9e-3
BF16_PROB_TOL = 2e-2
_CACHE = {}


def rel_err(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def fro_err(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm()).item()


def model_task(oracle, xs, f):
    out = []
    for x in xs:
        ids = [0] + oracle.tokenizer.encode(x) + oracle.tokenizer.encode(f)
        out.append((x, oracle.to_string(int(oracle.forward(torch.tensor(ids))[0, -1].argmax()))))
    return out


def reference(width, fp16=False):
    """Oracle + everything the reference loops compute at this width (once).
    ``fp16``: fp16-valued weights, as the released checkpoints (the engine then
    binds its exact-fp16 GEMMs: tests/test_gpu_exact16.py)."""
    key = (width, fp16)
    if key in _CACHE:
        return _CACHE[key]
    _CACHE.clear()
    name, L, n_prompts, kshot, n_ctx = WIDTHS[width]
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    cfg = tvr_amd.get_config(name).with_(n_layers=L)
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0, std=STD, fp16=fp16)
    tok = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
    oracle = make_oracle(cfg, sd, tok)
    letters = [x for x, _ in tvr_amd.tasks.letter_to_caps][:n_ctx]
    r = {"cfg": cfg, "sd": sd, "tok": tok, "oracle": oracle,
         "arrow": model_task(oracle, letters, ARROW), "colon": model_task(oracle, letters, ":")}
    random.seed(2)
    r["mean"] = R.generate_mean_activation(list(tvr_amd.tasks.letter_to_caps), ARROW, ",", oracle, 16, 6)
    layered = R.gather_head_activations_to_layers(r["mean"])
    r["acc"] = R.apply_layered_vectors_to_zero_shot(layered, r["arrow"], ARROW, oracle)
    r["dprob"] = R.apply_layered_vectors_to_zero_shot_by_probability(layered, r["arrow"], ARROW, oracle)

    class _M:  # the prompt builder only needs cfg + to_single_token
        pass
    m = _M()
    m.cfg, m.to_single_token = cfg, oracle.to_single_token
    r["prompts"], _ = tvr_amd.prompts.synthetic_cie_prompts(m, n_prompts, kshot, seed=1234)
    r["clean"] = [oracle.forward(torch.tensor([p]))[0, -1] for p in r["prompts"]]
    # answers = the clean argmax (random pairs give p ~ 1e-9 and a vacuous CIE)
    r["answers"] = [int(c.argmax()) for c in r["clean"]]
    r["cie"] = R.calculate_average_causal_indirect_effect(r["mean"], r["prompts"], [[a] for a in r["answers"]],
                                                         oracle)
    r["fv"] = R.assemble_task_vector(r["mean"], r["cie"], L - 1, 5) * 4  # x 4: it moves the top-5 at 2.8B width
    r["fv_acc"] = R.check_accuracy_of_task_vector(r["fv"], L - 1, r["colon"], 5, oracle)
    _CACHE[key] = r
    return r


@pytest.mark.timeout(900)
@pytest.mark.parametrize("width,gemm", CASES, ids=[f"{w}-{g}" for w, g in CASES])
def test_headline_width_parity(width, gemm):
    r = reference(width)
    model = tvr_amd.Model.from_hf_state_dict(r["cfg"], r["sd"], device="cuda", tokenizer=r["tok"], gemm=gemm)
    assert not model.exact16
    check_width(r, model, gemm)


def check_width(r, model, gemm):
    """Every reference function at this width against the oracle's results in r."""
    cfg = r["cfg"]
    bf16 = gemm == "bf16"
    tol = 2e-2 if bf16 else 1e-4
    try:
        # clean forward: last-row logits, probability of the answer, top-5
        out = model.forward_clean(r["prompts"], targets=r["answers"], topk=5, return_logits=True)
        pmax = 0.0
        for i, ref in enumerate(r["clean"]):
            assert rel_err(out["logits"][i], ref) < tol, i
            pr = torch.softmax(ref.double(), 0)
            pmax = max(pmax, pr.max().item())
            ptol = BF16_PROB_TOL if bf16 else tol
            if bf16:
                print(f"bf16 clean prob {i}: err {abs(out['prob'][i].item() - pr[r['answers'][i]].item()):.3e}, "
                      f"p_max {pr.max().item():.3f}")
            assert abs(out["prob"][i].item() - pr[r["answers"][i]].item()) <= ptol * pr.max().item() + 1e-7
            if not bf16:
                assert out["topk"][i].tolist() == torch.topk(ref, 5).indices.tolist(), i
        # a1: extraction (16 prompts, 6-shot letter_to_caps)
        random.seed(2)
        mean = tvr_amd.generate_mean_activation(list(tvr_amd.tasks.letter_to_caps), ARROW, ",", model=model,
                                                num_contexts=16, len_contexts=6)
        # the same metric on every path: max-abs error relative to max |mean| (bf16: the north star's 2e-2;
        # the Q / K projections run on fp16 operands in the bf16 mode, csrc/split.hpp store_ln4)
        print(f"{gemm} extraction: max-abs rel {rel_err(mean, r['mean']):.3e}, "
              f"frobenius rel {fro_err(mean, r['mean']):.3e}")
        assert rel_err(mean, r["mean"]) < tol
        # a4 / a5 on the oracle's means (each function isolated)
        layered = tvr_amd.gather_head_activations_to_layers(r["mean"].cuda())
        acc = tvr_amd.apply_layered_vectors_to_zero_shot(layered, r["arrow"], ARROW, model=model)
        dp = tvr_amd.apply_layered_vectors_to_zero_shot_by_probability(layered, r["arrow"], ARROW, model=model)
        if bf16:
            print(f"bf16 layer sweeps: accuracy {acc} vs {r['acc']}, max |d dprob| "
                  f"{(dp.cpu().double() - r['dprob'].double()).abs().max().item():.3e}")
            assert max(abs(a - b) for a, b in zip(acc, r["acc"])) <= 0.1, (acc, r["acc"])
            assert (dp.cpu().double() - r["dprob"].double()).abs().max().item() <= BF16_PROB_TOL
        else:
            assert acc == r["acc"]
            assert (dp.cpu().double() - r["dprob"].double()).abs().max().item() <= \
                tol * r["dprob"].abs().max().item() + 1e-7
        # a7: every (layer, head) site of every prompt
        sums = tvr_amd.experiments.causal_indirect_effect_sums(r["mean"].cuda(), r["prompts"], r["answers"], model)
        cie = sums.cpu().double() / len(r["prompts"])
        err = (cie - r["cie"].double()).abs().max().item()
        if bf16:  # bf16 rounding of the GEMM inputs on std-6 logits: 1.87e-2 of p at p = 0.91
            print(f"bf16 CIE: max abs err {err:.3e} = {err / pmax:.3e} of p_max {pmax:.3f}")
            assert err <= BF16_PROB_TOL * pmax, (err, pmax)
        else:
            assert err <= tol * r["cie"].abs().max().item() + 1e-7, (err, r["cie"].abs().max().item())
            assert r["cie"].abs().max().item() > 1e-4  # the sites move the probability
        # a10 / a11: FV from the oracle's CIE, top-5 accuracy clean and injected
        fv_acc = tvr_amd.check_accuracy_of_task_vector(r["fv"].cuda(), cfg.n_layers - 1, r["colon"], 5, model=model)
        if bf16:
            assert all(abs(a - b) <= 0.1 for a, b in zip(fv_acc, r["fv_acc"])), (fv_acc, r["fv_acc"])
        else:
            assert tuple(fv_acc) == tuple(r["fv_acc"])
    finally:
        del model
        torch.cuda.empty_cache()

"""GPU parity at FULL depth on informative weights, against a layer-streamed
fp64 oracle (VERDICT r3 "next round" 1).

The headline-width tests (test_gpu_headline_shapes.py) truncate the models to
2 layers; the bench's ``parity`` block runs the full 32 layers but on the HF
initialiser's std-0.02 weights, whose max |CIE| is ~1e-6.  Here the whole
model runs with seeded std-0.05 weights, where one head moves the answer's
probability by percents, and is checked against
``oracle.streamed_pythia.StreamedPythiaOracle``: the reference's loops
(scratch2.py:81-100 extraction, :171-197 CIE, :232-238 FV assembly, :292-314
FV top-k accuracy) on TransformerLens-semantics Pythia in fp64, one block's
weights at a time, run on cuda:0 through torch's fp64 (hipBLAS DGEMM: none of
the engine's kernels), pinned to the whole-model CPU oracle at 1e-12 by
tests/test_streamed_oracle.py.  No bar depends on the engine under test.

* fp32-accurate paths (``test_full_depth_fp32_paths``), the north star's fp32
  bars against fp64: clean last-row logits 1e-4 relative, answer probability
  1e-4 relative, top-1 identical, a1 extraction 1e-4 max-abs relative, CIE
  |err| <= 1e-4 max |CIE| + 1e-7 — Pythia-2.8B (32 layers; x2f16 and the exact-
  product fp32 MFMA) at layers {0, 16, 31} x all 32 heads, Pythia-12B (36
  layers, 10-shot T = 33; x2f16, the C5 path; the fp32 MFMA path is reported)
  at layers {0, 18, 35} x all 40 heads.  Max |CIE| > 1e-3 is asserted (the
  sites move the probability).
* C4, Pythia-6.9B in the bf16 configuration (``test_c4_bf16_function_vector_
  pipeline``): extraction over 64 five-shot prompts (max-abs relative < 2e-2,
  the north star's bf16 bar); the CIE of 12 prompts over layers 0 .. 10, 16,
  31 x all heads with the oracle's means (error reported as a fraction of
  max |CIE|); the top-10 function-vector head set of layers <= 10
  (scratch2.py:232-238, C4's FV) identical to the oracle's; then the whole C4
  chain on the engine's own means and CIE — FV assembled, added at layer 10
  of 50 zero-shot prompts, top-5 accuracy (scratch2.py:292-304) identical to
  the oracle chain's, clean and with the FV.
The CIE answers are the clean argmax (random pairs give p ~ 1e-5 and a
vacuous CIE); the zero-shot task's answers are the oracle's own clean top-1.
"""
import random

import pytest
import torch

import tvr_amd
from conftest import oracle_config
from oracle.streamed_pythia import StreamedPythiaOracle
from tvr_amd import experiments as E

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

STD = 0.05
TOL = 1e-4
ARROW = tvr_amd.tasks.ARROW
# model, asserted GEMM paths, reported-only paths, CIE layers, k-shot of the CIE prompt (T = 1 + 3k + 2)
FP32_MODELS = {
    "2.8b": ("pythia-2.8b", ("x2f16", "f32"), (), (0, 16, 31), 4),
    "12b": ("pythia-12b", ("x2f16",), ("f32",), (0, 18, 35), 10),
}


def rel_err(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def streamed_oracle(cfg, std=STD):
    """fp64 oracle on cuda:0 over the SAME seeded weights the engine got
    (synth_param on the same device: identical fp32 values, then fp64)."""
    shapes = tvr_amd.weights.hf_param_shapes(cfg)
    return StreamedPythiaOracle(oracle_config(cfg),
                                lambda n: tvr_amd.weights.synth_param(cfg, n, shapes[n], 0, "cuda", std))


class _Builder:  # the prompt builders need cfg, to_single_token and the tokenizer only
    def __init__(self, cfg):
        self.cfg = cfg
        self.tokenizer = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
        self.to_single_token = lambda s: self.tokenizer.encode(s)[0]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("which", list(FP32_MODELS))
def test_full_depth_fp32_paths(which):
    name, gemms, reported, layers, kshot = FP32_MODELS[which]
    cfg = tvr_amd.get_config(name)
    b = _Builder(cfg)
    model = tvr_amd.Model.from_pretrained(name, device="cuda", seed=0, std=STD, gemm=gemms[0])
    oracle = streamed_oracle(cfg)
    heads = list(range(cfg.n_heads))
    try:
        prompts, _ = tvr_amd.prompts.synthetic_cie_prompts(b, 1, kshot, seed=1234)
        clean_ref = oracle.last_logits(prompts)[0]
        answer = int(clean_ref.argmax())
        p_ref = torch.softmax(clean_ref, 0)[answer].item()
        random.seed(2)
        ex = tvr_amd.prompts.sample_icl_prompts(b, list(tvr_amd.tasks.letter_to_caps), ARROW, ",", 4, 6)
        mean_ref = oracle.mean_activation(ex)
        mean32 = mean_ref.float()  # the vectors both sides patch with
        cie_ref = oracle.cie(mean32.double(), prompts, [answer], layers=layers, heads=heads)
        idx = torch.tensor(layers)
        ref_sites = cie_ref[idx]
        cmax = ref_sites.abs().max().item()
        print(f"{name}: p(answer) {p_ref:.3e}, max |CIE| {cmax:.3e} (by layer "
              f"{[round(ref_sites[i].abs().max().item(), 6) for i in range(len(layers))]}), "
              f"max |mean| {mean_ref.abs().max():.3e}")
        assert cmax > 1e-3  # informative: the patched sites move the answer's probability
        for gemm in gemms + reported:
            strict = gemm in gemms
            model.set_gemm(gemm)
            out = model.forward_clean(prompts, targets=[answer], topk=1, return_logits=True)
            e_logits = rel_err(out["logits"][0], clean_ref)
            e_p = abs(out["prob"][0].item() - p_ref)
            mean = model.project_heads(E.sum_last_z(model, ex)) / len(ex)
            e_mean = rel_err(mean, mean_ref)
            sums = E.causal_indirect_effect_sums(mean32.cuda(), prompts, [answer], model, layers=list(layers),
                                                 heads=heads)
            got = sums.cpu().double()[idx]
            err = (got - ref_sites).abs().max().item()
            by_layer = [(got[i] - ref_sites[i]).abs().max().item() / cmax for i in range(len(layers))]
            print(f"{name} {gemm}{'' if strict else ' (reported)'}: logits rel {e_logits:.2e}, |dp| {e_p:.2e} "
                  f"(p {p_ref:.3e}), extraction rel {e_mean:.2e}, CIE abs err {err:.2e} = {err / cmax:.2e} of max "
                  f"(by layer {[f'{x:.1e}' for x in by_layer]})")
            if strict:
                assert e_logits < TOL, (gemm, e_logits)
                assert e_p <= TOL * p_ref + 1e-7, (gemm, e_p)
                assert int(out["topk"][0, 0]) == answer
                assert e_mean < TOL, (gemm, e_mean)
                assert err <= TOL * cmax + 1e-7, (gemm, err, cmax)
            # no site outside the requested grid is touched
            mask = torch.ones_like(sums, dtype=torch.bool)
            mask[idx] = False
            assert sums[mask.cuda()].abs().max().item() == 0.0
    finally:
        del model
        torch.cuda.empty_cache()


FV_LAYER, FV_HEADS = 10, 10  # C4: the function vector of the top-10 heads with layer <= 10 (scratch2.py:270 scaled)


@pytest.mark.timeout(900)
def test_c4_bf16_function_vector_pipeline():
    name = "pythia-6.9b"
    cfg = tvr_amd.get_config(name)
    b = _Builder(cfg)
    model = tvr_amd.Model.from_pretrained(name, device="cuda", seed=0, std=STD, gemm="bf16")
    oracle = streamed_oracle(cfg)
    L, H = cfg.n_layers, cfg.n_heads
    try:
        # --- a1: extraction over 64 five-shot prompts of a synthetic 50-pair task (C4's prompt form)
        task = tvr_amd.tasks.synthetic_task(50, cfg.d_vocab, seed=101)
        random.seed(5)
        ex = tvr_amd.prompts.sample_icl_prompts(b, task, ARROW, ",", 64, 5)
        mean_ref = oracle.mean_activation(ex)
        mean_eng = model.project_heads(E.sum_last_z(model, ex)) / len(ex)
        e_mean = rel_err(mean_eng, mean_ref)
        print(f"C4 bf16 extraction: max-abs rel {e_mean:.3e} (max |mean| {mean_ref.abs().max():.3e})")
        # --- a7: CIE over 12 prompts (T = 18), layers 0..10, 16, 31 x all heads, with the oracle's means
        prompts, _ = tvr_amd.prompts.synthetic_cie_prompts(b, 12, 5, seed=1234)
        clean_ref = oracle.last_logits(prompts)
        answers = [int(r.argmax()) for r in clean_ref]
        p_max = torch.softmax(clean_ref, -1).max().item()
        layers = list(range(FV_LAYER + 1)) + [16, 31]
        mean32 = mean_ref.float()
        cie_ref = oracle.cie(mean32.double(), prompts, answers, layers=layers)
        cie = (E.causal_indirect_effect_sums(mean32.cuda(), prompts, answers, model, layers=layers).cpu().double()
               / len(prompts))
        cmax = cie_ref.abs().max().item()
        err = (cie - cie_ref).abs()
        rep = {l: err[l].max().item() / cmax for l in (0, 16, 31)}
        print(f"C4 bf16 CIE: max |CIE| {cmax:.3e}, p_max {p_max:.3f}; |err| / max|CIE| at layers 0/16/31 "
              f"{rep[0]:.2e} / {rep[16]:.2e} / {rep[31]:.2e}, over layers <= {FV_LAYER} "
              f"{err[:FV_LAYER + 1].max().item() / cmax:.2e}")
        top_ref = torch.topk(cie_ref[:FV_LAYER + 1].flatten(), FV_HEADS + 1)
        top_eng = torch.topk(cie[:FV_LAYER + 1].flatten(), FV_HEADS)
        set_ref = sorted(divmod(int(i), H) for i in top_ref.indices[:FV_HEADS])
        set_eng = sorted(divmod(int(i), H) for i in top_eng.indices)
        gap = (top_ref.values[FV_HEADS - 1] - top_ref.values[FV_HEADS]).item()
        print(f"C4 bf16 top-{FV_HEADS} heads (layer <= {FV_LAYER}): oracle {set_ref}, engine {set_eng}; oracle gap "
              f"10th-11th {gap:.2e}, engine max |err| there {err[:FV_LAYER + 1].max().item():.2e}")
        # --- the whole C4 chain on the engine's own means and CIE vs the oracle's chain
        cie_chain = (E.causal_indirect_effect_sums(mean_eng, prompts, answers, model,
                                                   layers=list(range(FV_LAYER + 1))).cpu().double() / len(prompts))
        fv_ref = E.assemble_task_vector(mean_ref, cie_ref, FV_LAYER, FV_HEADS)
        fv_eng = E.assemble_task_vector(mean_eng, cie_chain.to(mean_eng.device), FV_LAYER, FV_HEADS)
        set_chain = sorted(divmod(int(i), H) for i in torch.topk(cie_chain[:FV_LAYER + 1].flatten(), FV_HEADS).indices)
        print(f"C4 bf16 chain: top-{FV_HEADS} heads {set_chain}, FV rel err {rel_err(fv_eng, fv_ref):.3e}")
        # zero-shot task: 50 items whose answers are the oracle's clean top-1 of [BOS, x, ":"]
        xs = [f"<|{t}|>" for t in random.Random(9).sample(range(1000, cfg.d_vocab), 50)]
        zs = [[0, b.tokenizer.encode(x)[0], b.tokenizer.encode(":")[0]] for x in xs]
        base_top = oracle.added_topk(zs, FV_LAYER, None, 5)
        contexts = [(x, b.tokenizer.decode_one(int(t[0]))) for x, t in zip(xs, base_top)]
        fv_top = oracle.added_topk(zs, FV_LAYER, fv_ref, 5)
        dec = b.tokenizer.decode_one
        firsts = [dec(b.tokenizer.encode(y)[0]) for _, y in contexts]  # scratch2.py:298: decoded strings

        def acc(tops):
            return sum(f in [dec(int(t)) for t in row] for f, row in zip(firsts, tops)) / len(zs)
        acc_ref = (acc(base_top), acc(fv_top))
        acc_eng = E.check_accuracy_of_task_vector(fv_eng, FV_LAYER, contexts, 5, model=model)
        print(f"C4 bf16 FV top-5 accuracy at layer {FV_LAYER} (clean, with FV): engine {acc_eng}, oracle {acc_ref}")
        assert e_mean < 2e-2, e_mean
        assert cmax > 1e-3
        assert set_eng == set_ref, (set_eng, set_ref)
        assert set_chain == set_ref, (set_chain, set_ref)
        assert tuple(acc_eng) == tuple(acc_ref), (acc_eng, acc_ref)
    finally:
        del model
        torch.cuda.empty_cache()

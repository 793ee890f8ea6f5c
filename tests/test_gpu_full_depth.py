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
* C4, Pythia-6.9B (``test_c4_function_vector_pipeline``): extraction over 64
  five-shot prompts; the CIE of 12 prompts over layers 0 .. 10, 16, 31 x all
  heads with the oracle's means; the top-10 function-vector head set of layers
  <= 10 (scratch2.py:232-238, C4's FV); then the whole C4 chain on the
  engine's own means and CIE — FV assembled, added at layer 10 of 50 zero-shot
  prompts, top-5 accuracy (scratch2.py:292-304), clean and with the FV.  On
  the fp32-accurate x2f16 path every one of these is held to the fp32 bars
  (head set and accuracies identical); on bf16, the north star's 2e-2 on the
  extracted vectors and a CIE error no larger than 1.5x the error bf16
  rounding of the same GEMM operands produces in the fp64 oracle
  (oracle/rounded_pythia.py) — see the test's docstring for why the head set
  cannot be a bf16 requirement.
The CIE answers are the clean argmax (random pairs give p ~ 1e-5 and a
vacuous CIE); the zero-shot task's answers are the oracle's clean second
choice (top-5 accuracy 1 without the FV; the FV moves them).
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
_C4 = {}


def c4_reference():
    """Pythia-6.9B (32 layers, std-0.05 weights) and the oracle's side of the
    C4 chain, computed once: extraction over 64 five-shot prompts, the CIE of
    12 prompts over layers 0..10, 16, 31, the top-10 FV heads of layers <= 10,
    the FV's top-5 accuracy on 50 zero-shot prompts."""
    if _C4:
        return _C4
    name = "pythia-6.9b"
    cfg = tvr_amd.get_config(name)
    b = _Builder(cfg)
    oracle = streamed_oracle(cfg)
    H = cfg.n_heads
    task = tvr_amd.tasks.synthetic_task(50, cfg.d_vocab, seed=101)
    random.seed(5)
    ex = tvr_amd.prompts.sample_icl_prompts(b, task, ARROW, ",", 64, 5)
    mean_ref = oracle.mean_activation(ex)
    prompts, _ = tvr_amd.prompts.synthetic_cie_prompts(b, 12, 5, seed=1234)
    answers = [int(r.argmax()) for r in oracle.last_logits(prompts)]
    layers = list(range(FV_LAYER + 1)) + [16, 31]
    mean32 = mean_ref.float()  # the vectors both sides patch with
    cie_ref = oracle.cie(mean32.double(), prompts, answers, layers=layers)
    top = torch.topk(cie_ref[:FV_LAYER + 1].flatten(), FV_HEADS + 1)
    fv_ref = E.assemble_task_vector(mean_ref, cie_ref, FV_LAYER, FV_HEADS)
    # zero-shot task: the answers are the oracle's clean SECOND choice after [BOS, x, ":"] (clean top-5 accuracy 1;
    # the FV moves them in and out of the top 5)
    xs = [f"<|{t}|>" for t in random.Random(9).sample(range(1000, cfg.d_vocab), 50)]
    zs = [[0, b.tokenizer.encode(x)[0], b.tokenizer.encode(":")[0]] for x in xs]
    base_top = oracle.added_topk(zs, FV_LAYER, None, 5)
    dec = b.tokenizer.decode_one
    contexts = [(x, dec(int(t[1]))) for x, t in zip(xs, base_top)]
    firsts = [dec(b.tokenizer.encode(y)[0]) for _, y in contexts]  # scratch2.py:298: decoded strings

    def acc(tops):
        return sum(f in [dec(int(t)) for t in row] for f, row in zip(firsts, tops)) / len(zs)
    _C4.update(cfg=cfg, name=name, oracle=oracle, ex=ex, mean_ref=mean_ref, mean32=mean32, prompts=prompts,
               answers=answers, layers=layers, cie_ref=cie_ref, cmax=cie_ref.abs().max().item(),
               set_ref=sorted(divmod(int(i), H) for i in top.indices[:FV_HEADS]),
               gap=(top.values[FV_HEADS - 1] - top.values[FV_HEADS]).item(), contexts=contexts,
               acc_ref=(acc(base_top), acc(oracle.added_topk(zs, FV_LAYER, fv_ref, 5))))
    return _C4


@pytest.mark.timeout(900)
@pytest.mark.parametrize("gemm", ["x2f16", "bf16"])
def test_c4_function_vector_pipeline(gemm):
    """C4 at full depth.  x2f16 (fp32-accurate): the north star's fp32 bars —
    extraction 1e-4, CIE 1e-4 max|CIE| + 1e-7, the top-10 FV head set and the
    FV top-5 accuracy identical, in isolation (the oracle's means) and along
    the engine's own chain.  bf16: the north star's bf16 bar on the extracted
    vectors (2e-2); its CIE error must not exceed 1.5x what bf16 rounding of
    the GEMM operands alone produces (oracle/rounded_pythia.py: the fp64
    oracle with the engine's operand roundings, measured on the same sites):
    the 10th and 11th oracle CIE values are ~1e-3 of max |CIE| apart, two
    orders of magnitude inside bf16's ~1e-1 CIE noise, so the top-10 set is a
    fp32-accurate requirement (asserted on x2f16) and reported for bf16."""
    r = c4_reference()
    cfg, H = r["cfg"], r["cfg"].n_heads
    model = tvr_amd.Model.from_pretrained(r["name"], device="cuda", seed=0, std=STD, gemm=gemm)
    try:
        ex, prompts, answers, layers, cmax = r["ex"], r["prompts"], r["answers"], r["layers"], r["cmax"]
        mean_eng = model.project_heads(E.sum_last_z(model, ex)) / len(ex)
        e_mean = rel_err(mean_eng, r["mean_ref"])
        cie = (E.causal_indirect_effect_sums(r["mean32"].cuda(), prompts, answers, model, layers=layers)
               .cpu().double() / len(prompts))
        err = (cie - r["cie_ref"]).abs()
        set_eng = sorted(divmod(int(i), H) for i in torch.topk(cie[:FV_LAYER + 1].flatten(), FV_HEADS).indices)
        # the chain on the engine's own means and CIE (bench C4's computation)
        cie_chain = (E.causal_indirect_effect_sums(mean_eng, prompts, answers, model,
                                                   layers=list(range(FV_LAYER + 1))).cpu().double() / len(prompts))
        set_chain = sorted(divmod(int(i), H) for i in torch.topk(cie_chain[:FV_LAYER + 1].flatten(), FV_HEADS).indices)
        fv_eng = E.assemble_task_vector(mean_eng, cie_chain.to(mean_eng.device), FV_LAYER, FV_HEADS)
        acc_eng = tuple(E.check_accuracy_of_task_vector(fv_eng, FV_LAYER, r["contexts"], 5, model=model))
        overlap = len(set(set_eng) & set(r["set_ref"]))
        print(f"C4 {gemm}: extraction max-abs rel {e_mean:.3e}; CIE max |CIE| {cmax:.3e}, |err| / max|CIE| at "
              f"layers 0/16/31 {err[0].max() / cmax:.2e} / {err[16].max() / cmax:.2e} / {err[31].max() / cmax:.2e}, "
              f"all {err.max() / cmax:.2e}; top-{FV_HEADS} heads (layer <= {FV_LAYER}) oracle {r['set_ref']}, engine "
              f"{set_eng} ({overlap} shared; oracle 10th-11th gap {r['gap']:.2e}), chain {set_chain}; FV top-5 "
              f"accuracy (clean, FV) engine {acc_eng} oracle {r['acc_ref']}")
        assert cmax > 1e-3
        if gemm == "x2f16":
            assert e_mean < TOL, e_mean
            assert err.max().item() <= TOL * cmax + 1e-7, (err.max().item(), cmax)
            assert set_eng == r["set_ref"], (set_eng, r["set_ref"])
            assert set_chain == r["set_ref"], (set_chain, r["set_ref"])
            assert acc_eng == r["acc_ref"], (acc_eng, r["acc_ref"])
        else:
            from oracle.rounded_pythia import Rounded, variants
            shapes = tvr_amd.weights.hf_param_shapes(cfg)
            emu = Rounded(oracle_config(cfg), lambda n: tvr_amd.weights.synth_param(cfg, n, shapes[n], 0, "cuda", STD),
                          variants()["engine_bf16"])
            floor = (emu.cie(r["mean32"].double(), prompts, answers, layers=layers) - r["cie_ref"]).abs().max().item()
            print(f"C4 bf16: emulated bf16-operand floor {floor / cmax:.2e} of max |CIE|, engine {err.max() / cmax:.2e}")
            assert e_mean < 2e-2, e_mean
            assert err.max().item() <= 1.5 * floor, (err.max().item(), floor)
    finally:
        del model
        torch.cuda.empty_cache()

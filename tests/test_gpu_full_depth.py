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
  layers, 10-shot T = 33; x2f16, the C5 path, and the fp32 MFMA path with its
  sliced accumulation) at layers {0, 18, 35} x all 40 heads.  Max |CIE| > 1e-3 is asserted (the
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
# model, asserted GEMM paths, reported-only paths, CIE layers, k-shot of the CIE prompt (T = 1 + 3k + 2),
# fp16-valued weights (the released checkpoints' dtype: the x2f16 GEMMs then run on the exact fp16 weights,
# 2 products, tests/test_gpu_exact16.py)
FP32_MODELS = {
    "2.8b": ("pythia-2.8b", ("x2f16", "f32"), (), (0, 16, 31), 4, False),
    # 12B f32: the exact-product fp32 MFMA path with the sliced accumulation (gemm_f32.hpp SLICE_KT; VERDICT r4:
    # unsliced it measured 2.7e-4 of max |CIE|, over the bar)
    "12b": ("pythia-12b", ("x2f16", "f32"), (), (0, 18, 35), 10, False),
    "2.8b-fp16w": ("pythia-2.8b", ("x2f16",), (), (0, 16, 31), 4, True),
    "12b-fp16w": ("pythia-12b", ("x2f16",), (), (0, 18, 35), 10, True),
}


def rel_err(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def streamed_oracle(cfg, std=STD, fp16=False):
    """fp64 oracle on cuda:0 over the SAME seeded weights the engine got
    (synth_param on the same device: identical fp32 values, then fp64)."""
    shapes = tvr_amd.weights.hf_param_shapes(cfg)
    return StreamedPythiaOracle(oracle_config(cfg),
                                lambda n: tvr_amd.weights.synth_param(cfg, n, shapes[n], 0, "cuda", std, fp16=fp16))


class _Builder:  # the prompt builders need cfg, to_single_token and the tokenizer only
    def __init__(self, cfg):
        self.cfg = cfg
        self.tokenizer = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
        self.to_single_token = lambda s: self.tokenizer.encode(s)[0]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("which", list(FP32_MODELS))
def test_full_depth_fp32_paths(which):
    name, gemms, reported, layers, kshot, fp16 = FP32_MODELS[which]
    cfg = tvr_amd.get_config(name)
    b = _Builder(cfg)
    model = tvr_amd.Model.from_pretrained(name, device="cuda", seed=0, std=STD, gemm=gemms[0], fp16_weights=fp16)
    assert model.exact16 == fp16
    oracle = streamed_oracle(cfg, fp16=fp16)
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


def c4_reference(fp16=False):
    """Pythia-6.9B (32 layers, std-0.05 weights) and the oracle's side of the
    C4 chain, computed once: extraction over 64 five-shot prompts, the CIE of
    12 prompts over layers 0..10, 16, 31, the top-10 FV heads of layers <= 10,
    the FV's top-5 accuracy on 50 zero-shot prompts."""
    if fp16 in _C4:
        return _C4[fp16]
    name = "pythia-6.9b"
    cfg = tvr_amd.get_config(name)
    b = _Builder(cfg)
    oracle = streamed_oracle(cfg, fp16=fp16)
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
    # zero-shot task (accuracies neither 0 nor 1): after [BOS, x, ":"] the answer is the oracle's clean
    # SECOND choice for even prompts (inside the clean top 5) and its clean 6th..10th choice for odd ones (outside
    # it), so the clean top-5 accuracy is 0.5 and the FV moves answers in and out of the top 5 both ways
    xs = [f"<|{t}|>" for t in random.Random(9).sample(range(1000, cfg.d_vocab), 50)]
    zs = [[0, b.tokenizer.encode(x)[0], b.tokenizer.encode(":")[0]] for x in xs]
    base_top = oracle.added_topk(zs, FV_LAYER, None, 10)
    dec = b.tokenizer.decode_one
    contexts = [(x, dec(int(t[1] if i % 2 == 0 else t[5 + (i // 2) % 5]))) for i, (x, t) in enumerate(zip(xs, base_top))]
    firsts = [dec(b.tokenizer.encode(y)[0]) for _, y in contexts]  # scratch2.py:298: decoded strings

    def acc(tops):
        return sum(f in [dec(int(t)) for t in row] for f, row in zip(firsts, tops)) / len(zs)
    _C4[fp16] = dict(cfg=cfg, name=name, oracle=oracle, ex=ex, mean_ref=mean_ref, mean32=mean32, prompts=prompts,
                     answers=answers, layers=layers, cie_ref=cie_ref, cmax=cie_ref.abs().max().item(),
                     set_ref=sorted(divmod(int(i), H) for i in top.indices[:FV_HEADS]),
                     gap=(top.values[FV_HEADS - 1] - top.values[FV_HEADS]).item(), contexts=contexts,
                     acc_ref=(acc(base_top[:, :5]), acc(oracle.added_topk(zs, FV_LAYER, fv_ref, 5))))
    return _C4[fp16]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("gemm", ["x2f16", "x2f16-fp16w", "bf16"])
def test_c4_function_vector_pipeline(gemm, monkeypatch):
    """C4 at full depth.  x2f16 (fp32-accurate): the north star's fp32 bars —
    extraction 1e-4, CIE 1e-4 max|CIE| + 1e-7, the top-10 FV head set and the
    FV top-5 accuracy identical, in isolation (the oracle's means) and along
    the engine's own chain.  bf16: the north star's bf16 bar on the extracted
    vectors (2e-2); its CIE error must not exceed 1.5x what bf16 rounding of
    the GEMM operands alone produces (oracle/rounded_pythia.py: the fp64
    oracle with the engine's operand roundings, measured on the same sites):
    the 10th and 11th oracle CIE values are ~1e-3 of max |CIE| apart, two
    orders of magnitude inside bf16's ~1e-1 CIE noise, so the top-10 set is a
    fp32-accurate requirement (asserted on x2f16) and reported for bf16.
    ``x2f16-fp16w``: fp16-valued weights (the released checkpoints' dtype) —
    the exact-fp16 GEMMs, incl. the linearised entry's G on the raw W1 — at the
    x2f16 bars against the oracle on the same weights."""
    fp16 = gemm.endswith("-fp16w")
    gemm = gemm.replace("-fp16w", "")
    r = c4_reference(fp16)
    cfg, H = r["cfg"], r["cfg"].n_heads
    model = tvr_amd.Model.from_pretrained(r["name"], device="cuda", seed=0, std=STD, gemm=gemm, fp16_weights=fp16)
    assert model.exact16 == fp16
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
        print(f"C4 {gemm}{' fp16 weights' if fp16 else ''}: extraction max-abs rel {e_mean:.3e}; CIE max |CIE| "
              f"{cmax:.3e}, |err| / max|CIE| at "
              f"layers 0/16/31 {err[0].max() / cmax:.2e} / {err[16].max() / cmax:.2e} / {err[31].max() / cmax:.2e}, "
              f"all {err.max() / cmax:.2e}; top-{FV_HEADS} heads (layer <= {FV_LAYER}) oracle {r['set_ref']}, engine "
              f"{set_eng} ({overlap} shared; oracle 10th-11th gap {r['gap']:.2e}), chain {set_chain}; FV top-5 "
              f"accuracy (clean, FV) engine {acc_eng} oracle {r['acc_ref']}")
        assert cmax > 1e-3
        # informative FV accuracies: neither 0 nor 1, clean and with the FV
        assert all(0 < a < 1 for a in r["acc_ref"]), r["acc_ref"]
        if gemm == "x2f16":
            assert e_mean < TOL, e_mean
            assert err.max().item() <= TOL * cmax + 1e-7, (err.max().item(), cmax)
            assert set_eng == r["set_ref"], (set_eng, r["set_ref"])
            assert set_chain == r["set_ref"], (set_chain, r["set_ref"])
            assert acc_eng == r["acc_ref"], (acc_eng, r["acc_ref"])
        else:
            m = c4_bf16_metrics(model, r, cie, e_mean, monkeypatch)
            set_emu = m.pop("set_emu")
            print(f"C4 bf16: {m}; top-{FV_HEADS} heads emulation {set_emu} "
                  f"({len(set(set_emu) & set(set_eng))} shared with the engine)")
            failed = c4_bf16_bars_failed(m)
            assert not failed, failed
    finally:
        del model
        torch.cuda.empty_cache()


_C4_EMU = {}


def c4_bf16_metrics(model, r, cie, e_mean, monkeypatch):
    """The engine (bf16) against the bf16-EMULATING fp64 oracle site by site (the engine's operand roundings —
    bf16, fp16 Q / K — and its REPLACE_HEAD entry form, everything else fp64; computed once).  At this depth two
    bf16 implementations that differ at the fp32 level partly decorrelate (test_bf16_value_level_one_block's
    docstring), so the bars are the magnitude against fp64 and the direction against the emulation; the
    value-level one is test_bf16_value_level_one_block.  Ratios are of the emulation's distance to fp64."""
    from oracle.rounded_pythia import Rounded, variants
    cfg, prompts, answers, layers = r["cfg"], r["prompts"], r["answers"], r["layers"]
    if "cie" not in _C4_EMU:
        shapes = tvr_amd.weights.hf_param_shapes(cfg)
        emu = Rounded(oracle_config(cfg), lambda n: tvr_amd.weights.synth_param(cfg, n, shapes[n], 0, "cuda", STD),
                      variants()["engine_bf16_entry"])
        _C4_EMU["cie"] = emu.cie(r["mean32"].double(), prompts, answers, layers=layers)
        del emu
    cie_emu = _C4_EMU["cie"]
    floor = (cie_emu - r["cie_ref"]).abs().max().item()
    e_emu = (cie - cie_emu).abs().max().item()
    monkeypatch.setenv("TVR_LIN_ENTRY", "0")  # the full entry GEMM: the emulation's arithmetic exactly
    cie_full = (E.causal_indirect_effect_sums(r["mean32"].cuda(), prompts, answers, model, layers=layers)
                .cpu().double() / len(prompts))
    monkeypatch.delenv("TVR_LIN_ENTRY")
    e_full = (cie_full - cie_emu).abs().max().item()
    H = cfg.n_heads
    return {"extraction": e_mean, "floor_of_max_cie": floor / r["cmax"],
            "vs_fp64": (cie - r["cie_ref"]).abs().max().item() / floor,
            "full_entry_vs_emu": e_full / floor, "lin_entry_vs_emu": e_emu / floor,
            "set_emu": sorted(divmod(int(i), H) for i in torch.topk(cie_emu[:FV_LAYER + 1].flatten(), FV_HEADS).indices)}


def c4_bf16_bars_failed(m):
    """The C4 bf16 bars a metrics dict misses: the north star's 2e-2 on the extraction, the CIE error against
    fp64 within 1.5x the emulated bf16-operand floor, and the direction — engine − emulation at most 1.0x that
    floor on either entry path (independent errors of the floor's size would put it at ~1.41x; measured 0.55 -
    0.66, profiles/r05/gpu_tests_r05d.log)."""
    bars = {"extraction": 2e-2, "vs_fp64": 1.5, "full_entry_vs_emu": 1.0, "lin_entry_vs_emu": 1.0}
    return {k: m[k] for k, b in bars.items() if not m[k] <= b}


# ------------------------------------------------------------------ C2 at full depth
C2_CONTEXTS = 52  # BASELINE C2: 52 zero-shot prompts x all layers (scratch2.py:160,163 on letter_to_caps)


def c2_contexts(oracle, b, cfg, vector, n=C2_CONTEXTS, seed=11):
    """Zero-shot prompts [BOS, x, →] (scratch2.py:121) with answers chosen so
    the per-layer accuracies are informative (neither all 0 nor all 1): for
    even prompts the most frequent patched top-1 over the layers (the vector
    moves the answer there at some layers and not at others), for odd ones the
    clean top-1 (the vector moves it away at some layers).  Returns the
    contexts (x, y) as strings, the prompts and the answer ids."""
    xs = [f"<|{t}|>" for t in random.Random(seed).sample(range(1000, cfg.d_vocab), n)]
    seqs = [[0, b.tokenizer.encode(x)[0], b.tokenizer.encode(ARROW)[0]] for x in xs]
    clean_top = oracle.last_logits(seqs).argmax(-1)
    _, _, ids, _ = oracle.layer_sweep(seqs, vector, [0] * n, k=1)
    answers = []
    for i in range(n):
        if i % 2:
            answers.append(int(clean_top[i]))
        else:
            vals, counts = ids[i, :, 0].unique(return_counts=True)
            answers.append(int(vals[counts.argmax()]))
    dec = b.tokenizer.decode_one
    return [(x, dec(a)) for x, a in zip(xs, answers)], seqs, answers


def oracle_layer_sweeps(oracle, b, seqs, contexts, answers, vector):
    """(accuracy [L], Δprob [L], smallest top-1 / top-2 logit margin over the
    sites) of the reference's two layer sweeps on ``oracle``."""
    p0, P, ids, vals = oracle.layer_sweep(seqs, vector, answers, k=2)
    dec = b.tokenizer.decode_one
    n, L = P.shape
    acc = [sum(dec(int(ids[i, l, 0])) == contexts[i][1] for i in range(n)) / n for l in range(L)]
    dp = (P - p0[:, None]).mean(0)
    return acc, dp, (vals[..., 0] - vals[..., 1]).min().item()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("fp16", [False, True], ids=["processed", "fp16w"])
def test_c2_layer_sweeps_full_depth_x2f16(fp16):
    """C2 (scratch2.py:114-127 accuracy and :135-150 Δprob sweeps, the repo's
    headline plots) on the whole 32-layer Pythia-2.8B with std-0.05 weights,
    52 zero-shot prompts x 32 layers, against the fp64 streamed oracle: the
    per-layer accuracy list identical, Δprob within 1e-4 of the largest |Δprob|
    + 1e-7 (the north star's fp32 bars).  The vector is the reference's
    layered_vectors[-1] (late binding, App. B1) of the oracle's own extraction
    (scratch2.py:156-163: 2048 six-shot prompts there, 64 here).  ``fp16w``:
    fp16-valued weights, as the released checkpoints and the bench — the
    exact-fp16 GEMMs (2 products) and the exact-fp16 fused-statistics unembed,
    the path the bench's C2 number runs."""
    name = "pythia-2.8b"
    cfg = tvr_amd.get_config(name)
    b = _Builder(cfg)
    oracle = streamed_oracle(cfg, fp16=fp16)
    random.seed(3)
    ex = tvr_amd.prompts.sample_icl_prompts(b, list(tvr_amd.tasks.letter_to_caps), ARROW, ",", 64, 6)
    layered = E.gather_head_activations_to_layers(oracle.mean_activation(ex)).float()  # [L, d] fp32
    vec = layered[-1].double()
    contexts, seqs, answers = c2_contexts(oracle, b, cfg, vec)
    acc_ref, dp_ref, margin = oracle_layer_sweeps(oracle, b, seqs, contexts, answers, vec)
    model = tvr_amd.Model.from_pretrained(name, device="cuda", seed=0, std=STD, gemm="x2f16", fp16_weights=fp16)
    assert model.exact16 == fp16
    try:
        acc = E.apply_layered_vectors_to_zero_shot(layered.cuda(), contexts, ARROW, model=model)
        dp = E.apply_layered_vectors_to_zero_shot_by_probability(layered.cuda(), contexts, ARROW, model=model)
        dp = dp.cpu().double()
        dmax = dp_ref.abs().max().item()
        err = (dp - dp_ref).abs().max().item()
        print(f"C2 {name} x2f16{' fp16 weights' if fp16 else ''}, 32 layers: accuracy engine {acc}\n  oracle {acc_ref}\n"
              f"  Δprob max |ref| {dmax:.3e}, "
              f"|err| {err:.2e} = {err / dmax:.2e} of max; smallest oracle top-1 margin {margin:.2e}")
        informative = [a for a in acc_ref if 0 < a < 1]
        assert len(informative) >= 4 and dmax > 1e-3, (acc_ref, dmax)
        assert acc == acc_ref
        assert err <= TOL * dmax + 1e-7, (err, dmax)
    finally:
        del model
        torch.cuda.empty_cache()


@pytest.mark.timeout(900)
def test_c2_layer_sweeps_full_depth_bf16():
    """The same two layer sweeps on the whole 32-layer Pythia-6.9B in the bf16
    mode (BASELINE C4's precision), against fp64 and the bf16-emulating fp64
    oracle (oracle/rounded_pythia.py ``engine_bf16``: the engine's operand
    roundings, everything else fp64).  At 32 layers two bf16 implementations
    decorrelate: any fp32-level difference (accumulation order, fp32 LN /
    softmax) flips a few bf16 roundings per block and the flips compound
    (tools/bf16_probe.py, profiles/r05/bf16_probe_r05c.log: engine vs emulation
    4 % of the emulation's own distance to fp64 after block 0, 21 % after block
    1, ~50 % from block 10 on), so the value-level check is the shallow
    test_bf16_value_level_shallow; here: the engine's Δprob error against fp64
    within 1.5x the emulation's (the bf16 operand-rounding floor at this
    depth) and the accuracies within 2 of the 52 prompts of the emulation's at
    every layer (bf16 flips near-tied top-1s)."""
    from oracle.rounded_pythia import Rounded, variants
    name = "pythia-6.9b"
    cfg = tvr_amd.get_config(name)
    b = _Builder(cfg)
    oracle = streamed_oracle(cfg)
    random.seed(4)
    ex = tvr_amd.prompts.sample_icl_prompts(b, tvr_amd.tasks.synthetic_task(50, cfg.d_vocab, seed=101), ARROW, ",",
                                            64, 5)
    layered = E.gather_head_activations_to_layers(oracle.mean_activation(ex)).float()
    vec = layered[-1].double()
    contexts, seqs, answers = c2_contexts(oracle, b, cfg, vec, seed=12)
    acc_ref, dp_ref, margin = oracle_layer_sweeps(oracle, b, seqs, contexts, answers, vec)
    shapes = tvr_amd.weights.hf_param_shapes(cfg)
    emu = Rounded(oracle_config(cfg), lambda n: tvr_amd.weights.synth_param(cfg, n, shapes[n], 0, "cuda", STD),
                  variants()["engine_bf16"])
    acc_emu, dp_emu, _ = oracle_layer_sweeps(emu, b, seqs, contexts, answers, vec)
    del emu
    model = tvr_amd.Model.from_pretrained(name, device="cuda", seed=0, std=STD, gemm="bf16")
    try:
        acc = E.apply_layered_vectors_to_zero_shot(layered.cuda(), contexts, ARROW, model=model)
        dp = E.apply_layered_vectors_to_zero_shot_by_probability(layered.cuda(), contexts, ARROW, model=model)
        dp = dp.cpu().double()
        dmax = dp_ref.abs().max().item()
        floor = (dp_emu - dp_ref).abs().max().item()
        e_emu = (dp - dp_emu).abs().max().item()
        e_ref = (dp - dp_ref).abs().max().item()
        dacc = max(abs(a - c) for a, c in zip(acc, acc_emu)) * len(contexts)
        print(f"C2 {name} bf16, 32 layers: accuracy engine {acc}\n  emulated {acc_emu}\n  fp64 {acc_ref}\n"
              f"  Δprob max |fp64| {dmax:.3e}: emulation vs fp64 {floor / dmax:.2e}, engine vs fp64 {e_ref / dmax:.2e}, "
              f"engine vs emulation {e_emu / dmax:.2e} of max; accuracy vs emulation at most {dacc:.0f} prompts; "
              f"smallest fp64 top-1 margin {margin:.2e}")
        assert len([a for a in acc_ref if 0 < a < 1]) >= 4 and dmax > 1e-3, (acc_ref, dmax)
        assert e_ref <= 1.5 * floor + 1e-7, (e_ref, floor)
        assert dacc <= 2, (acc, acc_emu)
    finally:
        del model
        torch.cuda.empty_cache()


@pytest.mark.timeout(900)
def test_bf16_value_level_one_block():
    """The bf16 mode at VALUE level, at the depth where a
    value-level bar can hold: Pythia-6.9B width, ONE block (std-0.05
    weights), against the bf16-emulating fp64 oracle (oracle/rounded_pythia.py
    ``engine_bf16_entry``: the engine's operand roundings — bf16 weights and
    activations, fp16 Q / K — and its REPLACE_HEAD entry form; everything
    else fp64).  Clean last-row logits of 12 prompts, the CIE of every
    (layer 0, head) site over them and the Δprob sweep of 52 prompts: engine −
    emulation at most HALF of emulation − fp64 (max over the values): an
    engine whose bf16 error had the emulation's size but an independent
    direction would measure sqrt(2) ~ 1.41 there, so one wrong in another
    direction than its operand roundings explain fails.  Why not closer, and
    why one block: the engine's fp32 arithmetic (accumulation order, fp32 LN /
    softmax) differs from the emulation's fp64 by ~1e-6 relative, which flips
    a fraction of the next bf16 roundings (each flip is a whole bf16 ulp on
    that element); the flips compound block by block (tools/bf16_probe.py,
    profiles/r05/bf16_probe_r05c.log: residual stream engine vs emulation 4 %
    of the emulation's distance to fp64 after block 0, 21 % after block 1,
    ~50 % from block 10 on; 2 / 3-layer truncations 0.33 / 0.36 on the logits,
    profiles/r05/gpu_tests_r05d.log), so at depth two correct bf16
    implementations decorrelate and the full-depth tests hold bf16 to the
    1.5x-floor bars."""
    ratios = bf16_one_block_ratios()
    assert all(r <= 0.5 for r in ratios.values()), ratios


_ONE_BLOCK = {}


def bf16_one_block_ratios():
    """test_bf16_value_level_one_block's measurement: engine − emulation over emulation − fp64 for the clean
    logits, the CIE and the Δprob sweep (the references computed once; the engine built afresh, so a
    diagnostic knob set in the environment applies)."""
    from oracle.rounded_pythia import Rounded, variants
    name = "pythia-6.9b"
    cfg = tvr_amd.get_config(name).with_(n_layers=1)
    if _ONE_BLOCK:
        return _one_block_engine(name, cfg, **_ONE_BLOCK)
    b = _Builder(cfg)
    shapes = tvr_amd.weights.hf_param_shapes(cfg)
    get = lambda n: tvr_amd.weights.synth_param(cfg, n, shapes[n], 0, "cuda", STD)  # noqa: E731
    f64 = StreamedPythiaOracle(oracle_config(cfg), get)
    emu = Rounded(oracle_config(cfg), get, variants()["engine_bf16_entry"])
    prompts, _ = tvr_amd.prompts.synthetic_cie_prompts(b, 12, 5, seed=1234)
    random.seed(6)
    ex = tvr_amd.prompts.sample_icl_prompts(b, tvr_amd.tasks.synthetic_task(50, cfg.d_vocab, seed=101), ARROW, ",",
                                            32, 5)
    mean = f64.mean_activation(ex).float()
    lg = {k: o.last_logits(prompts) for k, o in (("f64", f64), ("emu", emu))}
    answers = [int(r.argmax()) for r in lg["f64"]]
    cie = {k: o.cie(mean.double(), prompts, answers) for k, o in (("f64", f64), ("emu", emu))}
    layered = E.gather_head_activations_to_layers(mean)
    contexts, seqs, targets = c2_contexts(f64, b, cfg, layered[-1].double(), seed=13)
    dp = {}
    for k, o in (("f64", f64), ("emu", emu)):
        p0, P, _, _ = o.layer_sweep(seqs, layered[-1].double(), targets, k=1)
        dp[k] = (P - p0[:, None]).mean(0)
    assert cie["f64"].abs().max().item() > 1e-3
    _ONE_BLOCK.update(prompts=prompts, mean=mean, answers=answers, layered=layered, contexts=contexts,
                      refs=(lg, cie, dp))
    return _one_block_engine(name, cfg, **_ONE_BLOCK)


def _one_block_engine(name, cfg, prompts, mean, answers, layered, contexts, refs):
    model = tvr_amd.Model.from_pretrained(name, cfg=cfg, device="cuda", seed=0, std=STD, gemm="bf16")
    try:
        o = model.forward_clean(prompts, topk=1, return_logits=True)
        c = E.causal_indirect_effect_sums(mean.cuda(), prompts, answers, model).cpu().double() / len(prompts)
        d = E.apply_layered_vectors_to_zero_shot_by_probability(layered.cuda(), contexts, ARROW, model=model)
        got = (o["logits"].cpu().double(), c, d.cpu().double())
        names = ("clean logits", "CIE", "layer-sweep Δprob")
        ratios = {}
        for i, what in enumerate(names):
            floor = (refs[i]["emu"] - refs[i]["f64"]).abs().max().item()
            e = (got[i] - refs[i]["emu"]).abs().max().item()
            ratios[what] = e / floor
            print(f"bf16 {name} x 1 block, {what}: emulation vs fp64 {floor:.3e} (max |fp64| "
                  f"{refs[i]['f64'].abs().max():.3e}); engine vs emulation {e:.3e} = {e / floor:.3f} of it")
        return ratios
    finally:
        del model
        torch.cuda.empty_cache()


# the two wrong bf16 implementations the negative controls build (engine diagnostic knobs, engine.hip
# tvr_model_set_gemm): the fp16 Q / K operands dropped (round 2's bug: Q / K on bf16), and the bf16 weight
# planes truncated instead of rounded to nearest even (a conversion bug: a systematic bias of half an ulp)
WRONG_BF16 = {"qk_on_bf16": ("TVR_DEBUG_BF16_QK", "0"), "weights_truncated": ("TVR_DEBUG_BF16_TRUNC", "1")}


@pytest.mark.timeout(900)
@pytest.mark.parametrize("wrong", list(WRONG_BF16))
def test_bf16_bars_reject_a_wrong_bf16_path(wrong, monkeypatch):
    """Negative controls of the bf16 bars (the bars were set after the measurement, so they
    must be shown to catch a wrong bf16 implementation): with the engine deliberately wrong, the value-level
    one-block bar (0.5 of the emulation's distance) and the C4 full-depth bars (magnitude 1.5x, direction 1.0x
    of the floor) must FAIL, while the same measurements on the correct engine pass them (the two tests above)."""
    var, val = WRONG_BF16[wrong]
    monkeypatch.setenv(var, val)
    ratios = bf16_one_block_ratios()
    print(f"one block, {wrong}: {ratios}")
    r = c4_reference()
    model = tvr_amd.Model.from_pretrained(r["name"], device="cuda", seed=0, std=STD, gemm="bf16")
    try:
        mean_eng = model.project_heads(E.sum_last_z(model, r["ex"])) / len(r["ex"])
        e_mean = rel_err(mean_eng, r["mean_ref"])
        cie = (E.causal_indirect_effect_sums(r["mean32"].cuda(), r["prompts"], r["answers"], model,
                                             layers=r["layers"]).cpu().double() / len(r["prompts"]))
        m = c4_bf16_metrics(model, r, cie, e_mean, monkeypatch)
        m.pop("set_emu")
    finally:
        del model
        torch.cuda.empty_cache()
    failed = c4_bf16_bars_failed(m)
    print(f"C4 bf16, {wrong}: {m}; bars missed: {failed}")
    assert not all(x <= 0.5 for x in ratios.values()), ("the one-block value bar accepts", wrong, ratios)
    assert failed, ("the C4 bf16 bars accept", wrong, m)

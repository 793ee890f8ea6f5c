"""Engine robustness paths a real checkpoint or a C caller can reach.

* x2f16 range fallback: with the exact-fp16
  GEMMs the QKV + MLP-in GEMM's A operand is LNPre(x)·γ, so a checkpoint with a
  large LayerNorm gamma can push it past the fp16 split's limit (|a| < 4095).
  The experiment functions then fall back inside the same process — exact-fp16
  → processed weights (x2f16, A = LNPre(x), bounded by sqrt(d_model)) →
  x3bf16 — re-run the call from the same global ``random`` state and warn.
  Forced here with one gamma of 2000 on the tiny model; the results must still
  equal the fp64 oracle on the same weights at the fp32 bars, with the same
  prompts the reference functions draw.
* ``tvr_trace_read`` into a destination that is only float-aligned (a C
  caller's offset view) gives the same centred rows as an aligned one.
* ``set_exact16`` / ``set_gemm`` re-plan on the model's device, not the
  current one (needs two GPUs; skipped on a one-GPU box).
"""
import random

import pytest
import torch

import tvr_amd
from tvr_amd import _lib
from oracle import reference_experiments as R
from conftest import make_oracle

pytestmark = [pytest.mark.gpu]

ARROW = tvr_amd.tasks.ARROW
BIG_GAMMA = 2000.0  # exact in fp16; LNPre rows reach |x| ~ 3 at d 64, so |x * gamma| passes 4095


def _big_gamma_sd(cfg):
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0, std=0.15, fp16=True)
    sd["gpt_neox.layers.1.input_layernorm.weight"][3] = BIG_GAMMA
    return sd


def test_range_fallback_large_gamma(tiny_cfg, tokenizer):
    sd = _big_gamma_sd(tiny_cfg)
    oracle = make_oracle(tiny_cfg, sd, tokenizer, torch.float64)
    task = list(tvr_amd.tasks.letter_to_caps)

    model = tvr_amd.Model.from_hf_state_dict(tiny_cfg, sd, device="cuda", tokenizer=tokenizer, gemm="x2f16")
    assert model.exact16
    # without the fallback the call fails loudly instead of returning inaccurate numbers
    model.range_fallback = False
    random.seed(0)
    with pytest.raises(_lib.RangeError):
        tvr_amd.generate_mean_activation(task, ARROW, ",", model=model, num_contexts=16, len_contexts=4)

    model.range_fallback = True
    random.seed(0)
    with pytest.warns(RuntimeWarning, match="retrying on x2f16"):
        mean = tvr_amd.generate_mean_activation(task, ARROW, ",", model=model, num_contexts=16, len_contexts=4)
    assert model.range_fallbacks[0] == ("generate_mean_activation", "x2f16 (processed weights)")
    assert not model.exact16 and model.gemm in ("x2f16", "x3bf16")
    random.seed(0)  # the retry re-drew the same prompts: the reference function from the same seed agrees
    mean_ref = R.generate_mean_activation(task, ARROW, ",", model=oracle, num_contexts=16, len_contexts=4)
    err = ((mean.cpu().double() - mean_ref).abs().max() / mean_ref.abs().max()).item()
    assert err < 1e-4, err

    random.seed(1)
    prompts, answers = tvr_amd.generate_shuffled_prompts(task, model, 3, 4, ARROW)
    cie = tvr_amd.calculate_average_causal_indirect_effect(mean, prompts, answers, model=model)
    cie_ref = R.calculate_average_causal_indirect_effect(mean_ref, prompts, answers, oracle)
    cerr = (cie.cpu().double() - cie_ref.double()).abs().max().item()
    assert cerr <= 1e-4 * cie_ref.abs().max().item() + 1e-7, cerr
    print("range fallbacks:", model.range_fallbacks, f"extraction {err:.2e}, CIE {cerr:.2e}")


def test_range_fallback_chain_ends_on_x3bf16(tiny_cfg, tokenizer):
    """Processed x2f16 weights that still trip the check move to x3bf16; x3bf16 has no limit, so nothing
    is left to fall back to and a RangeError (were one raised) propagates."""
    sd = _big_gamma_sd(tiny_cfg)
    model = tvr_amd.Model.from_hf_state_dict(tiny_cfg, sd, device="cuda", tokenizer=tokenizer, gemm="x2f16")
    model.set_exact16(False)
    assert model._fall_back("probe", RuntimeError("forced")) and model.gemm == "x3bf16"
    assert not model._fall_back("probe", RuntimeError("forced"))
    assert model.range_fallbacks == [("probe", "x3bf16")]


def test_trace_read_offset_destination(tiny_cfg, tokenizer):
    """The exact-fp16 path's trace export centres its rows on the device; a destination that is only
    float-aligned (an offset view, as a C caller may pass) takes the element-wise form: the same rows."""
    sd = tvr_amd.weights.synth_hf_state_dict(tiny_cfg, seed=0, std=0.15, fp16=True)
    model = tvr_amd.Model.from_hf_state_dict(tiny_cfg, sd, device="cuda", tokenizer=tokenizer, gemm="x2f16")
    assert model.exact16
    prompts = [[0, 5, 9, 13, 2], [0, 7, 1, 4]]
    tr = model.trace(len(prompts), sum(map(len, prompts)))
    model.forward_clean(prompts, trace=tr)
    n, d = sum(map(len, prompts)), tiny_cfg.d_model
    for layer in (0, 1, tiny_cfg.n_layers):
        ref = tr.resid_pre(layer)
        big = torch.full((n * d + 3,), float("nan"), device="cuda")
        _lib.check(model._lib.tvr_trace_read(tr._h, _lib.TRACE_RESID_PRE, layer, big.data_ptr() + 4,
                                             model._stream()), "tvr_trace_read")
        torch.cuda.synchronize()
        got = big[1:1 + n * d].view(n, d)
        # same rows; the row mean summed in another order (float4 vs element-wise): fp32 rounding only
        assert (got - ref).abs().max().item() <= 1e-6 * ref.abs().max().item(), layer
        assert torch.isnan(big[0]) and torch.isnan(big[-2:]).all()  # nothing written outside
        assert ref.double().mean(dim=1).abs().max().item() <= 1e-5 * ref.abs().max().item()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs")
def test_replan_on_the_model_device(tiny_cfg, tokenizer):
    """set_exact16 / set_gemm allocate and convert the weight planes on the model's device while another
    device is current, and leave the current device as it was."""
    sd = tvr_amd.weights.synth_hf_state_dict(tiny_cfg, seed=0, std=0.15, fp16=True)
    model = tvr_amd.Model.from_hf_state_dict(tiny_cfg, sd, device="cuda:1", tokenizer=tokenizer, gemm="x2f16")
    ids = [[0, 5, 7, 9, 11]]
    a = model.forward_clean(ids, return_logits=True)["logits"]
    with torch.cuda.device(0):
        model.set_exact16(False)
        model.set_exact16(True)
        model.set_gemm("x3bf16")
        model.set_gemm("x2f16")
        assert torch.cuda.current_device() == 0
    b = model.forward_clean(ids, return_logits=True)["logits"]
    assert torch.equal(a, b)


def test_replan_round_trip_one_device(tiny_cfg, tokenizer):
    """The one-GPU form of the test above: exact16 off / on and x3bf16 / x2f16 re-plans come back to the same
    binding bit for bit (the x2f16 planes rebuilt from the kept weights), the mode mirrors follow the engine,
    and the current device is unchanged."""
    sd = tvr_amd.weights.synth_hf_state_dict(tiny_cfg, seed=0, std=0.15, fp16=True)
    model = tvr_amd.Model.from_hf_state_dict(tiny_cfg, sd, device="cuda:0", tokenizer=tokenizer, gemm="x2f16")
    ids = [[0, 5, 7, 9, 11], [0, 3, 2]]
    a = model.forward_clean(ids, return_logits=True)["logits"]
    dev = torch.cuda.current_device()
    model.set_exact16(False)
    assert not model.exact16 and model.gemm == "x2f16"
    p = model.forward_clean(ids, return_logits=True)["logits"]
    assert (p - a).abs().max().item() <= 1e-5 * a.abs().max().item()  # processed weights: fp32-level agreement
    model.set_gemm("x3bf16")
    assert model.gemm == "x3bf16"
    model.set_gemm("x2f16")
    model.set_exact16(True)
    assert model.exact16 and model.gemm == "x2f16"
    assert torch.cuda.current_device() == dev
    b = model.forward_clean(ids, return_logits=True)["logits"]
    assert torch.equal(a, b)

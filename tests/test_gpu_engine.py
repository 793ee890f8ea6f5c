"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle.

Tolerances (fp32 engine vs fp32 oracle; the GEMM reduction order differs):
* logits / residuals / z: |Δ| ≤ 1e-4 · max|ref| (typically ~1e-6)
* extracted mean vectors: ≤ 1e-4 relative (north-star bar)
* probabilities: |Δp| ≤ 1e-5 · max p, CIE: |Δ| ≤ 1e-4 · max|CIE| + 1e-7
* top-1 / top-k ids and string accuracies: identical (near-ties excluded
  where the fp64 oracle's gap is below 1e-5)
"""
import random

import numpy as np
import pytest
import torch

import tvr_amd
from oracle import reference_experiments as R

pytestmark = pytest.mark.gpu

ARROW = tvr_amd.tasks.ARROW
X2F16, BF16 = tvr_amd._lib.GEMM_MODES["x2f16"], tvr_amd._lib.GEMM_MODES["bf16"]


def rel_err(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


# ------------------------------------------------------------------ kernels
@pytest.mark.parametrize("M,N,K", [(1, 1, 32), (37, 130, 64), (128, 128, 32), (300, 257, 320),
                                   (1000, 2560, 2560), (129, 50304, 64),
                                   (4096, 8192, 256), (3001, 17920, 96), (1025, 50304, 64)])
def test_gemm_f32_matches_torch(M, N, K):
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g)
    b = torch.randn(N, generator=g)
    C = torch.empty(M, N, device="cuda")
    lib = tvr_amd._lib.load()
    Ad, Wd, bd = A.cuda(), W.cuda(), b.cuda()
    tvr_amd._lib.check(lib.tvr_gemm_f32(Ad.data_ptr(), K, Wd.data_ptr(), K, bd.data_ptr(), C.data_ptr(), N,
                                        M, N, K, torch.cuda.current_stream().cuda_stream), "gemm")
    ref = A.double() @ W.double().T + b.double()
    err = (C.cpu().double() - ref).abs().max().item()
    bound = 4e-7 * (A.double().abs() @ W.double().abs().T).max().item() + 1e-6
    assert err <= bound, (err, bound)
    # fp32 torch reference of the same op, as a sanity anchor
    t32 = (Ad @ Wd.T + bd).cpu().double()
    assert (t32 - ref).abs().max().item() <= 2 * bound


@pytest.mark.parametrize("M,N,K", [(1, 1, 32), (37, 130, 64), (128, 128, 32), (300, 257, 320),
                                   (1000, 2560, 2560), (129, 50304, 64),
                                   (4096, 8192, 256), (3001, 17920, 96), (1025, 50304, 64)])
def test_gemm_x3bf16_matches_torch(M, N, K):
    """The 3-plane bf16 split GEMM meets the SAME bound as the fp32 MFMA GEMM."""
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) * 1e-3  # planes keep their own exponents
    b = torch.randn(N, generator=g)
    C = torch.empty(M, N, device="cuda")
    lib = tvr_amd._lib.load()
    st = torch.cuda.current_stream().cuda_stream
    Ad, Wd, bd = A.cuda(), W.cuda(), b.cuda()
    planes = torch.empty(3, N, K, dtype=torch.int16, device="cuda")
    tvr_amd._lib.check(lib.tvr_split_planes(Wd.data_ptr(), planes.data_ptr(), N * K, st), "split")
    # the planes sum back to W exactly
    bf = planes.view(torch.bfloat16).double()
    assert torch.equal(bf.sum(0), Wd.double())
    tvr_amd._lib.check(lib.tvr_gemm_x3bf16(Ad.data_ptr(), K, planes.data_ptr(), K, N * K, bd.data_ptr(),
                                           C.data_ptr(), N, M, N, K, st), "gemm_x3")
    ref = A.double() @ W.double().T + b.double()
    err = (C.cpu().double() - ref).abs().max().item()
    bound = 4e-7 * (A.double().abs() @ W.double().abs().T).max().item() + 1e-6
    assert err <= bound, (err, bound)


@pytest.mark.parametrize("M,N,K", [(1, 1, 32), (37, 130, 64), (128, 128, 32), (300, 257, 320),
                                   (1000, 2560, 2560), (129, 50304, 64),
                                   (4096, 8192, 256), (3001, 17920, 96), (1025, 50304, 64)])
def test_gemm_x2f16_matches_torch(M, N, K):
    """The 2-plane fp16 split GEMM meets the SAME bound as the fp32 MFMA GEMM,
    with weights far from fp16's natural range (the power-of-two scale)."""
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N)
    A = torch.randn(M, K, generator=g)
    A[:, ::7] *= 1e-4  # tiny inputs: the residual plane's subnormal range
    W = torch.randn(N, K, generator=g) * 1e-3
    b = torch.randn(N, generator=g)
    C = torch.empty(M, N, device="cuda")
    lib = tvr_amd._lib.load()
    st = torch.cuda.current_stream().cuda_stream
    Ad, Wd, bd = A.cuda(), W.cuda(), b.cuda()
    e = int(np.frexp(W.abs().max().item())[1])
    scale = float(2.0 ** (15 - e))
    planes = torch.empty(2, N, K, dtype=torch.int16, device="cuda")
    tvr_amd._lib.check(lib.tvr_weight_planes(X2F16, Wd.data_ptr(), scale, planes.data_ptr(), N * K, st), "split")
    # the planes sum back to W * scale within 2^-22 relative, or half the fp16
    # subnormal spacing (2^-25) where the residual plane is subnormal
    hp = planes.view(torch.float16).double()
    ws = Wd.double() * scale
    assert ((hp.sum(0) - ws).abs() <= 2.0 ** -22 * ws.abs() + 2.0 ** -25).all()
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    tvr_amd._lib.check(lib.tvr_gemm_x2f16(Ad.data_ptr(), K, planes.data_ptr(), K, N * K, scale, bd.data_ptr(),
                                          C.data_ptr(), N, M, N, K, flag.data_ptr(), st), "gemm_x2")
    ref = A.double() @ W.double().T + b.double()
    err = (C.cpu().double() - ref).abs().max().item()
    bound = 4e-7 * (A.double().abs() @ W.double().abs().T).max().item() + 1e-6
    assert err <= bound, (err, bound)
    assert flag.item() == 0


@pytest.mark.parametrize("M,N,K", [(1, 1, 32), (37, 130, 64), (300, 257, 320), (1000, 2560, 2560),
                                   (129, 50304, 64), (4096, 8192, 256), (3001, 17920, 96), (600, 2560, 12800)])
def test_gemm_x2f16_planar_matches_torch(M, N, K):
    """The engine's X2F16 GEMM (pre-split activations, LDS-DMA staging,
    16x16x32 MFMA) meets the fp32 MFMA GEMM's bound."""
    g = torch.Generator(device="cpu").manual_seed(M * 11 + N)
    A = torch.randn(M, K, generator=g)
    A[:, ::5] *= 1e-4
    W = torch.randn(N, K, generator=g) * 2e-2
    b = torch.randn(N, generator=g)
    lib = tvr_amd._lib.load()
    st = torch.cuda.current_stream().cuda_stream
    Ad, Wd, bd = A.cuda(), W.cuda(), b.cuda()
    scale = float(2.0 ** (15 - int(np.frexp(W.abs().max().item())[1])))
    planes = torch.empty(2, N, K, dtype=torch.int16, device="cuda")
    tvr_amd._lib.check(lib.tvr_weight_planes(X2F16, Wd.data_ptr(), scale, planes.data_ptr(), N * K, st), "split")
    lda = K + 32  # a padded logical row: the format's stride is independent of K
    Ap = torch.zeros(M, lda, device="cuda")
    Ap[:, :K] = Ad
    Ah = torch.empty(M, 2, lda, dtype=torch.int16, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    tvr_amd._lib.check(lib.tvr_act_rows(X2F16, Ap.data_ptr(), lda, Ah.data_ptr(), M, lda, flag.data_ptr(), st),
                       "split rows")
    # plane 0 + plane 1 = 16 a within 2^-22 relative (+ half the fp16 subnormal spacing)
    hs = Ah.view(torch.float16).double().sum(1)[:, :K]
    assert ((hs - 16 * Ad.double()).abs() <= 2.0 ** -22 * 16 * Ad.double().abs() + 2.0 ** -25).all()
    C = torch.empty(M, N, device="cuda")
    tvr_amd._lib.check(lib.tvr_gemm_planar(X2F16, Ah.data_ptr(), lda, planes.data_ptr(), K, N * K, scale,
                                                 bd.data_ptr(), C.data_ptr(), N, M, N, K, st), "gemm_x2p")
    ref = A.double() @ W.double().T + b.double()
    err = (C.cpu().double() - ref).abs().max().item()
    bound = 4e-7 * (A.double().abs() @ W.double().abs().T).max().item() + 1e-6
    assert err <= bound, (err, bound)
    assert flag.item() == 0


@pytest.mark.parametrize("M,N,K", [(1, 1, 64), (37, 130, 64), (300, 257, 320), (1000, 2560, 2560),
                                   (129, 50304, 64), (3001, 17920, 128), (600, 2560, 12800)])
def test_gemm_bf16_planar_matches_torch(M, N, K):
    """The bf16 planar GEMM equals an fp64 GEMM of the bf16-rounded operands
    up to fp32 accumulation error (the bf16 rounding itself is the mode)."""
    g = torch.Generator(device="cpu").manual_seed(M * 13 + N)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) * 2e-2
    b = torch.randn(N, generator=g)
    lib = tvr_amd._lib.load()
    st = torch.cuda.current_stream().cuda_stream
    Ad, Wd, bd = A.cuda(), W.cuda(), b.cuda()
    plane = torch.empty(N, K, dtype=torch.int16, device="cuda")
    tvr_amd._lib.check(lib.tvr_weight_planes(BF16, Wd.data_ptr(), 1.0, plane.data_ptr(), N * K, st), "bf16 W")
    assert torch.equal(plane.view(torch.bfloat16), Wd.to(torch.bfloat16))
    Ah = torch.empty(M, 2, K, dtype=torch.int16, device="cuda")
    tvr_amd._lib.check(lib.tvr_act_rows(BF16, Ad.data_ptr(), K, Ah.data_ptr(), M, K, None, st), "bf16 A")
    assert torch.equal(Ah[:, 0].view(torch.bfloat16), Ad.to(torch.bfloat16))
    C = torch.empty(M, N, device="cuda")
    tvr_amd._lib.check(lib.tvr_gemm_planar(BF16, Ah.data_ptr(), K, plane.data_ptr(), K, N * K, 1.0, bd.data_ptr(),
                                           C.data_ptr(), N, M, N, K, st), "gemm_bf16")
    Ab, Wb = Ad.to(torch.bfloat16).double().cpu(), Wd.to(torch.bfloat16).double().cpu()
    ref = Ab @ Wb.T + b.double()
    err = (C.cpu().double() - ref).abs().max().item()
    bound = 4e-7 * (Ab.abs() @ Wb.abs().T).max().item() + 1e-6
    assert err <= bound, (err, bound)


def test_gemm_x2f16_range_flag():
    """An input at the split's range limit (|a| >= 4095) is reported, not hidden."""
    M, N, K = 64, 64, 64
    lib = tvr_amd._lib.load()
    st = torch.cuda.current_stream().cuda_stream
    A = torch.randn(M, K, device="cuda")
    W = torch.randn(N, K, device="cuda") * 0.02
    planes = torch.empty(2, N, K, dtype=torch.int16, device="cuda")
    tvr_amd._lib.check(lib.tvr_weight_planes(X2F16, W.data_ptr(), 2.0 ** 16, planes.data_ptr(), N * K, st), "split")
    C = torch.empty(M, N, device="cuda")
    for big, want in ((4000.0, 0), (4100.0, 1)):
        A[5, 9] = big
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        tvr_amd._lib.check(lib.tvr_gemm_x2f16(A.data_ptr(), K, planes.data_ptr(), K, N * K, 2.0 ** 16, None,
                                              C.data_ptr(), N, M, N, K, flag.data_ptr(), st), "gemm_x2")
        assert flag.item() == want, big
        # the activation-format producers raise the same flag
        flag.zero_()
        Ah = torch.empty(M, 2, K, dtype=torch.int16, device="cuda")
        tvr_amd._lib.check(lib.tvr_act_rows(X2F16, A.data_ptr(), K, Ah.data_ptr(), M, K, flag.data_ptr(), st), "rows")
        assert flag.item() == want, big


@pytest.mark.parametrize("d", [64, 100, 768, 2560, 4096, 5120, 6144])  # register path: d % 256 == 0, d <= 5120
def test_lnpre_matches_torch(d):
    x = torch.randn(77, d, device="cuda") * 3 + 1
    y = torch.empty_like(x)
    lib = tvr_amd._lib.load()
    tvr_amd._lib.check(lib.tvr_lnpre_f32(x.data_ptr(), d, y.data_ptr(), d, 77, d, 1e-5,
                                         torch.cuda.current_stream().cuda_stream), "lnpre")
    xd = x.double()
    xd = xd - xd.mean(-1, keepdim=True)
    ref = xd / (xd.pow(2).mean(-1, keepdim=True) + 1e-5).sqrt()
    assert (y.double() - ref).abs().max().item() < 2e-6


# ------------------------------------------------------------ clean forward
def ragged_prompts(n, vocab, seed, lo=2, hi=40):
    rng = random.Random(seed)
    return [[0] + [rng.randrange(1, vocab) for _ in range(rng.randrange(lo, hi))] for _ in range(n)]


def test_forward_clean_matches_oracle(tiny_model, tiny_oracle):
    prompts = ragged_prompts(9, tiny_model.cfg.d_vocab, 1) + [[0], [0, 5], list(range(128))]
    targets = [p[-1] for p in prompts]
    out = tiny_model.forward_clean(prompts, targets=targets, topk=5, return_logits=True)
    for i, p in enumerate(prompts):
        ref = tiny_oracle.forward(torch.tensor([p]))[0, -1]
        assert rel_err(out["logits"][i], ref) < 1e-4, i
        pr = torch.softmax(ref, 0)
        assert abs(out["prob"][i].item() - pr[targets[i]].item()) <= 1e-5 * pr.max().item()
        assert out["topk"][i].tolist() == torch.topk(ref, 5).indices.tolist()


def test_forward_clean_shared_prefix_rows(tiny_model, tiny_oracle, monkeypatch):
    """Without a trace, prompts sharing leading tokens with an earlier prompt
    compute only their own suffix rows (engine.hip tvr_forward_clean):
    duplicates, 1-token prompts before and after longer ones, a prefix that
    is a whole earlier prompt, different first tokens; last-row logits and
    the z capture equal the oracle and the unshared run."""
    cfg = tiny_model.cfg
    rng = random.Random(23)
    base = [0] + [rng.randrange(1, cfg.d_vocab) for _ in range(40)]
    prompts = [[0], base[:30], base[:30], base[:12], base[:31] + [7, 9], [3] + base[1:20], [3] + base[1:5],
               [0, 5], base[:2], [0] + [rng.randrange(1, cfg.d_vocab) for _ in range(17)]]
    targets = [p[-1] for p in prompts]
    out = tiny_model.forward_clean(prompts, targets=targets, topk=5, return_logits=True, capture=True)
    for i, p in enumerate(prompts):
        ref = tiny_oracle.forward(torch.tensor([p]))[0, -1]
        assert rel_err(out["logits"][i], ref) < 1e-4, i
        assert out["topk"][i].tolist() == torch.topk(ref, 5).indices.tolist(), i
    monkeypatch.setenv("TVR_PREFIX_SHARE", "0")
    off = tiny_model.forward_clean(prompts, targets=targets, topk=5, return_logits=True, capture=True)
    assert rel_err(out["logits"], off["logits"]) < 1e-5
    assert torch.equal(out["topk"], off["topk"])
    assert rel_err(out["zsum"], off["zsum"]) < 1e-5


def test_trace_matches_run_with_cache(tiny_model, tiny_oracle):
    prompts = ragged_prompts(5, tiny_model.cfg.d_vocab, 2)
    trace = tiny_model.trace(len(prompts), sum(map(len, prompts)))
    tiny_model.forward_clean(prompts, trace=trace)
    off = 0
    L = tiny_model.cfg.n_layers
    resid = [trace.resid_pre(l).cpu() for l in range(L + 1)]
    zs = [trace.z(l).cpu() for l in range(L)]
    for p in prompts:
        _, cache = tiny_oracle.run_with_cache(torch.tensor([p]))
        T = len(p)
        for l in range(L):
            assert rel_err(resid[l][off:off + T], cache[f"blocks.{l}.hook_resid_pre"][0]) < 1e-4
            assert rel_err(zs[l][off:off + T], cache[f"blocks.{l}.attn.hook_z"][0].reshape(T, -1)) < 1e-4
        assert rel_err(resid[L][off:off + T], cache[f"blocks.{L - 1}.hook_resid_post"][0]) < 1e-4
        off += T


def test_forward_rejects_bad_input(tiny_model):
    with pytest.raises(ValueError):
        tiny_model.forward_clean([[0, 1], []])
    with pytest.raises(ValueError):
        tiny_model.forward_clean([[0, tiny_model.cfg.d_vocab]])
    with pytest.raises(RuntimeError):  # longer than the model's n_ctx (256 for "tiny")
        tiny_model.forward_clean([[0] * 257])


# --------------------------------------------------------------- experiments
@pytest.fixture(scope="module")
def mean_pair(tiny_model, tiny_oracle):
    random.seed(1234)
    ours = tvr_amd.generate_mean_activation(tvr_amd.tasks.letter_to_caps, ARROW, ",", model=tiny_model,
                                            num_contexts=96, len_contexts=4)
    random.seed(1234)
    ref = R.generate_mean_activation(tvr_amd.tasks.letter_to_caps, ARROW, ",", model=tiny_oracle,
                                     num_contexts=96, len_contexts=4)
    return ours, ref


def test_generate_mean_activation(mean_pair):
    ours, ref = mean_pair
    assert ours.shape == ref.shape
    assert rel_err(ours, ref) < 1e-4


def test_layer_sweeps_late_binding(tiny_model, tiny_oracle, mean_pair):
    ours_mean, ref_mean = mean_pair
    ctx = tvr_amd.tasks.letter_to_caps
    lv_ours = tvr_amd.gather_head_activations_to_layers(ours_mean)
    lv_ref = R.gather_head_activations_to_layers(ref_mean)
    acc = tvr_amd.apply_layered_vectors_to_zero_shot(lv_ours * 8, ctx, ARROW, model=tiny_model)
    acc_ref = R.apply_layered_vectors_to_zero_shot(lv_ref * 8, ctx, ARROW, tiny_oracle)
    assert acc == acc_ref
    dp = tvr_amd.apply_layered_vectors_to_zero_shot_by_probability(lv_ours * 8, ctx, ARROW, model=tiny_model)
    dp_ref = R.apply_layered_vectors_to_zero_shot_by_probability(lv_ref * 8, ctx, ARROW, tiny_oracle)
    assert (dp.cpu().double() - dp_ref.double()).abs().max().item() <= 1e-4 * dp_ref.abs().max().item() + 1e-7


def test_layer_sweep_per_layer_vectors(tiny_model, tiny_oracle, mean_pair):
    """Intended per-layer semantics (no closure quirk) = the reference hooks
    with one vector per layer."""
    ours_mean, ref_mean = mean_pair
    ctx = tvr_amd.tasks.fruit_to_color
    lv = tvr_amd.gather_head_activations_to_layers(ours_mean) * 8
    acc = tvr_amd.apply_layered_vectors_to_zero_shot(lv, ctx, ARROW, model=tiny_model,
                                                     reference_late_binding=False)
    lv_ref = R.gather_head_activations_to_layers(ref_mean) * 8
    hits = [0] * tiny_oracle.cfg.n_layers
    for x, y in ctx:
        tokens = torch.tensor([0, tiny_oracle.to_single_token(x), tiny_oracle.to_single_token(ARROW)])
        for i in range(tiny_oracle.cfg.n_layers):
            logits = tiny_oracle.run_with_hooks(tokens, fwd_hooks=[
                (f"blocks.{i}.hook_attn_out", lambda hv, hook, v=lv_ref[i]: R.layer_addition_hook(hv, hook, v))])
            hits[i] += R.logits_to_next_token(logits, tiny_oracle) == y
    assert acc == [h / len(ctx) for h in hits]


def test_causal_indirect_effect(tiny_model, tiny_oracle, mean_pair):
    ours_mean, ref_mean = mean_pair
    random.seed(99)
    prompts, answers = tvr_amd.generate_shuffled_prompts(tvr_amd.tasks.letter_to_caps, tiny_model, 6, 4, ARROW)
    random.seed(99)
    prompts_r, answers_r = R.generate_shuffled_prompts(tvr_amd.tasks.letter_to_caps, tiny_oracle, 6, 4, ARROW)
    assert prompts == prompts_r and answers == answers_r
    cie = tvr_amd.calculate_average_causal_indirect_effect(ours_mean, prompts, answers, model=tiny_model)
    cie_ref = R.calculate_average_causal_indirect_effect(ref_mean, prompts_r, answers_r, tiny_oracle)
    assert cie.shape == cie_ref.shape
    assert (cie.cpu().double() - cie_ref.double()).abs().max().item() <= 1e-4 * cie_ref.abs().max().item() + 1e-7
    # function vector from the top heads, then its zero-shot top-5 accuracy
    fv = tvr_amd.assemble_task_vector(ours_mean, cie, 1, 3)
    fv_ref = R.assemble_task_vector(ref_mean, cie_ref, 1, 3)
    assert rel_err(fv, fv_ref) < 1e-4
    ctx = tvr_amd.tasks.letter_to_caps[:40]
    acc = tvr_amd.check_accuracy_of_task_vector(fv * 4, 1, ctx, model=tiny_model)
    acc_ref = R.check_accuracy_of_task_vector(fv_ref * 4, 1, ctx, model=tiny_oracle)
    assert acc == acc_ref
    assert tvr_amd.check_accuracy_of_added_task_vector(fv * 4, 0, ctx, model=tiny_model) == \
        R.check_accuracy_of_added_task_vector(fv_ref * 4, 0, ctx, model=tiny_oracle)


def test_cie_validation(tiny_model):
    with pytest.raises(ValueError, match="Mean head activations"):
        tvr_amd.calculate_average_causal_indirect_effect(torch.zeros(1, 2, 3, device="cuda"), ["a"], [[1]],
                                                         model=tiny_model)
    cfg = tiny_model.cfg
    with pytest.raises(ValueError, match="same length"):
        tvr_amd.calculate_average_causal_indirect_effect(
            torch.zeros(cfg.n_layers, cfg.n_heads, cfg.d_model, device="cuda"), ["a", "b"], [[1]], model=tiny_model)


def test_component_hypothesis(tiny_model, tiny_oracle):
    random.seed(5)
    ours = tvr_amd.test_component_hypothesis(tvr_amd.tasks.low_to_caps, ARROW, model=tiny_model, num_contexts=40,
                                             len_contexts=4, batch_contexts=16)
    random.seed(5)
    ref = R.test_component_hypothesis(tvr_amd.tasks.low_to_caps, ARROW, model=tiny_oracle, num_contexts=40,
                                      len_contexts=4)
    assert ours == ref


def test_substitute_task(tiny_model, tiny_oracle):
    random.seed(6)
    ours = tvr_amd.substitute_task(list(tvr_amd.tasks.letter_to_caps), list(tvr_amd.tasks.letter_to_low), 1,
                                   ARROW, model=tiny_model, num_contexts=32, len_contexts=4)
    random.seed(6)
    ref = R.substitute_task(list(tvr_amd.tasks.letter_to_caps), list(tvr_amd.tasks.letter_to_low), 1, ARROW,
                            model=tiny_oracle, num_contexts=32, len_contexts=4)
    assert ours == ref


def test_patch_sweep_site_kinds_against_hooks(tiny_model, tiny_oracle):
    """Every site kind on ragged prompts, compared with the oracle's hook on
    the same prompt (logits of the last position)."""
    cfg = tiny_model.cfg
    prompts = ragged_prompts(4, cfg.d_vocab, 11, lo=3, hi=30)
    trace = tiny_model.trace(4, sum(map(len, prompts)))
    tiny_model.forward_clean(prompts, trace=trace)
    g = torch.Generator().manual_seed(3)
    vecs = torch.randn(5, cfg.d_model, generator=g)
    sites = tvr_amd.make_sites(4 * 4)
    want = []
    k = 0
    for i, p in enumerate(prompts):
        T = len(p)
        for kind in range(4):
            s = sites[k]
            s["seq"], s["kind"], s["target"] = i, kind, p[1]
            tokens = torch.tensor([p])
            if kind == 0:
                ref = tiny_oracle.forward(tokens)
            elif kind == 1:
                l, h = (i + 1) % cfg.n_layers, i % cfg.n_heads
                s["layer"], s["head"], s["vec"] = l, h, i
                tiny_oracle.cfg.use_attn_result = True
                def hook(hv, hook, h=h, v=vecs[i]):
                    hv[0, :, h, :] = v
                    return hv
                ref = tiny_oracle.run_with_hooks(tokens, fwd_hooks=[(f"blocks.{l}.attn.hook_result", hook)])
                tiny_oracle.cfg.use_attn_result = False
            elif kind == 2:
                l = i % cfg.n_layers
                s["layer"], s["vec"] = l, 4
                ref = tiny_oracle.run_with_hooks(tokens, fwd_hooks=[
                    (f"blocks.{l}.hook_attn_out", lambda hv, hook: R.layer_addition_hook(hv, hook, vecs[4]))])
            else:
                l, src = i % cfg.n_layers, (i + 1) % len(prompts)
                pos, spos = T // 2, len(prompts[src]) // 3
                s["layer"], s["pos"], s["src_seq"], s["src_pos"] = l, pos, src, spos
                _, c_dst = tiny_oracle.run_with_cache(tokens)
                _, c_src = tiny_oracle.run_with_cache(torch.tensor([prompts[src]]))
                r = c_dst[f"blocks.{l}.hook_resid_pre"].clone()
                r[0, pos] = c_src[f"blocks.{l}.hook_resid_pre"][0, spos]
                ref = tiny_oracle.forward(r, start_at_layer=l)
            want.append(ref[0, -1])
            k += 1
    out = tiny_model.patch_sweep(trace, sites, vecs.cuda(), topk=3, return_logits=True)
    for j, ref in enumerate(want):
        assert rel_err(out["logits"][j], ref) < 1e-4, (j, sites[j])
        assert out["topk"][j].tolist() == torch.topk(ref, 3).indices.tolist(), j
        pr = torch.softmax(ref, 0)[int(sites[j]["target"])].item()
        assert abs(out["prob"][j].item() - pr) <= 1e-5 * torch.softmax(ref, 0).max().item()


def test_patch_sweep_shared_prefix_rows(tiny_model, tiny_oracle, monkeypatch):
    """Head-replacement sites on prompts that share prefixes (BOS only, 20
    tokens, a whole duplicate prompt, none): followers read the prefix K/V
    from their leader's rows (engine.hip tvr_patch_sweep).  Each site equals
    the oracle's hook on its own prompt, and the sweep equals the same sweep
    with sharing off (TVR_PREFIX_SHARE=0)."""
    cfg = tiny_model.cfg
    rng = random.Random(17)
    base = [0] + [rng.randrange(1, cfg.d_vocab) for _ in range(29)]
    prompts = [base[:24], base[:20] + [rng.randrange(1, cfg.d_vocab) for _ in range(7)], base[:24],
               [5] + base[1:16], [0] + [rng.randrange(1, cfg.d_vocab) for _ in range(12)], base[:2]]
    trace = tiny_model.trace(len(prompts), sum(map(len, prompts)))
    tiny_model.forward_clean(prompts, trace=trace)
    g = torch.Generator().manual_seed(4)
    vecs = torch.randn(3, cfg.d_model, generator=g)
    combos = [(0, 1, 0), (1, 3, 1), (0, 1, 2), (1, 3, 1)]  # (layer, head, vec); the last one twice
    sites = tvr_amd.make_sites(len(prompts) * len(combos))
    want = []
    k = 0
    tiny_oracle.cfg.use_attn_result = True
    try:
        for i, p in enumerate(prompts):
            for l, h, v in combos:
                s = sites[k]
                s["seq"], s["kind"], s["target"] = i, tvr_amd._lib.SITE_REPLACE_HEAD_ALLPOS, p[1]
                s["layer"], s["head"], s["vec"] = l, h, v
                def hook(hv, hook, h=h, v=vecs[v]):
                    hv[0, :, h, :] = v
                    return hv
                want.append(tiny_oracle.run_with_hooks(torch.tensor([p]), fwd_hooks=[
                    (f"blocks.{l}.attn.hook_result", hook)])[0, -1])
                k += 1
    finally:
        tiny_oracle.cfg.use_attn_result = False
    out = tiny_model.patch_sweep(trace, sites, vecs.cuda(), topk=3, return_logits=True)
    monkeypatch.setenv("TVR_PREFIX_SHARE", "0")
    off = tiny_model.patch_sweep(trace, sites, vecs.cuda(), topk=3, return_logits=True)
    for j, ref in enumerate(want):
        assert rel_err(out["logits"][j], ref) < 1e-4, (j, sites[j])
        assert out["topk"][j].tolist() == torch.topk(ref, 3).indices.tolist(), j
    assert rel_err(out["logits"], off["logits"]) < 1e-5
    assert torch.equal(out["topk"], off["topk"])


@pytest.mark.slow
@pytest.mark.parametrize("gemm", ["x2f16", "x3bf16", "f32"])
def test_pythia160m_shape_cie_subset(tokenizer, gemm):
    """Pythia-160m shape (d 768, 12 heads, d_head 64): clean logits and a CIE
    stripe (3 layers x 12 heads, 2 prompts) against the fp32 oracle."""
    from conftest import make_oracle
    cfg = tvr_amd.get_config("pythia-160m")
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0)
    model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda", gemm=gemm)
    oracle = make_oracle(cfg, sd, model.tokenizer)
    prompts, answers = tvr_amd.prompts.synthetic_cie_prompts(model, 2, 4, seed=1234)
    g = torch.Generator().manual_seed(0)
    mean = torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, generator=g) * 0.5
    layers = [0, 6, 11]
    ours = tvr_amd.experiments.causal_indirect_effect_sums(mean.cuda(), prompts, answers, model, layers=layers)
    ref = R.calculate_average_causal_indirect_effect(mean, prompts, [[a] for a in answers], oracle,
                                                     layers=layers) * len(prompts)
    assert (ours.cpu().double() - ref.double()).abs().max().item() <= 1e-4 * ref.abs().max().item() + 1e-9
    out = model.forward_clean(prompts, return_logits=True)
    for i, p in enumerate(prompts):
        assert rel_err(out["logits"][i], oracle.forward(torch.tensor([p]))[0, -1]) < 1e-4


@pytest.mark.slow
def test_gemm_launch_shapes_full_cie_match_fp32_kernel(tokenizer):
    """Every GEMM launch shape of the engine's planar path in one sweep: a full
    Pythia-160m-shape CIE (12 x 12 sites, 12 prompts) runs launches from 6 to
    ~2,100 tiles, i.e. split-K (< 192 tiles), plain multi-round launches and
    the last-round tail split (engine.hip plan_pp), all on gemm_pingpong_kernel
    with the LDS epilogue.  Checked against the same sweep on the independent
    fp32-MFMA kernel family (gemm_f32_nt_kernel) at the north star's
    tolerance, and clean probabilities likewise."""
    cfg = tvr_amd.get_config("pythia-160m")
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0)
    prompts = answers = None
    res = {}
    for gemm in ("x2f16", "f32"):
        model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda", gemm=gemm)
        if prompts is None:
            prompts, answers = tvr_amd.prompts.synthetic_cie_prompts(model, 12, 4, seed=99)
        g = torch.Generator().manual_seed(5)
        mean = torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, generator=g) * 0.5
        cie = tvr_amd.experiments.causal_indirect_effect_sums(mean.cuda(), prompts, answers, model)
        p0 = model.forward_clean(prompts, targets=answers)["prob"]
        res[gemm] = (cie.cpu().double(), p0.cpu().double())
        del model
        torch.cuda.empty_cache()
    (c1, p1), (c2, p2) = res["x2f16"], res["f32"]
    assert (c1 - c2).abs().max().item() <= 1e-4 * c2.abs().max().item() + 1e-9
    assert (p1 - p2).abs().max().item() <= 1e-5 * p2.abs().max().item()


def test_batched_fv_helpers_match_reference_loops(tiny_model, tiny_oracle, mean_pair):
    """check_accuracy_of_added_task_vector_by_layer and the head-count grid
    (scratch2.py:411-425) = the reference's per-cell loops on the oracle."""
    ours_mean, ref_mean = mean_pair
    random.seed(3)
    prompts, answers = tvr_amd.generate_shuffled_prompts(tvr_amd.tasks.letter_to_caps, tiny_model, 4, 4, ARROW)
    cie = tvr_amd.calculate_average_causal_indirect_effect(ours_mean, prompts, answers, model=tiny_model)
    cie_ref = R.calculate_average_causal_indirect_effect(ref_mean, prompts, answers, tiny_oracle)
    ctx = tvr_amd.tasks.letter_to_caps[:30]
    fv = tvr_amd.assemble_task_vector(ours_mean, cie, 1, 3) * 4
    fv_ref = R.assemble_task_vector(ref_mean, cie_ref, 1, 3) * 4
    by_layer = tvr_amd.experiments.check_accuracy_of_added_task_vector_by_layer(fv, ctx, 5, model=tiny_model)
    assert by_layer == [R.check_accuracy_of_added_task_vector(fv_ref, l, ctx, 5, tiny_oracle)
                        for l in range(tiny_oracle.cfg.n_layers)]
    # the grid from the SAME CIE on both sides (the head ranking is an input,
    # so the comparison always runs); skipped cells keep the zero vector and
    # are still evaluated, as scratch2.py:413-424 does
    grid = tvr_amd.experiments.function_vector_head_count_grid(ref_mean.cuda() * 4, cie_ref.cuda(), ctx,
                                                               model=tiny_model, heads_per_batch=1,
                                                               number_of_batches=6)
    L, H = tiny_oracle.cfg.n_layers, tiny_oracle.cfg.n_heads
    want = torch.zeros(L, 6)
    for i in range(L):
        for j in range(6):
            v = torch.zeros(tiny_oracle.cfg.d_model)
            if (j + 1) < (i + 1) * H:
                v = R.assemble_task_vector(ref_mean * 4, cie_ref, i, j + 1)
            want[i, j] = R.check_accuracy_of_added_task_vector(v, i, ctx, 5, tiny_oracle)
    assert torch.equal(grid, want)


def test_x2f16_range_error_is_loud(tiny_cfg, tokenizer):
    """An activation outside the fp16 split's range fails the call (EngineError)
    instead of returning inaccurate results; the other modes run the same model."""
    sd = tvr_amd.weights.synth_hf_state_dict(tiny_cfg, seed=0, std=0.15)
    for k in list(sd):
        if k.endswith("mlp.dense_h_to_4h.weight"):
            sd[k] = sd[k] * 1e5  # GELU(h) ~ 1e5 >> 4095
    prompts = [[0, 5, 9, 13], [0, 7]]
    m = tvr_amd.Model.from_hf_state_dict(tiny_cfg, sd, device="cuda", tokenizer=tokenizer, gemm="x2f16")
    with pytest.raises(tvr_amd._lib.EngineError, match="X2F16"):
        m.forward_clean(prompts, targets=[1, 2])
    m.set_gemm("x3bf16")
    out = m.forward_clean(prompts, targets=[1, 2])
    assert torch.isfinite(out["prob"]).all()


# ------------------------------------------------------------------ bf16 mode
# The north star's bf16 bar: extracted vectors within 2e-2 relative of the fp32
# reference (only the GEMMs run in bf16; LayerNorm, attention, the residual
# stream and softmax stay fp32).  Probabilities and CIE are bounded relative
# to the largest probability involved.
BF16_TOL = 2e-2


@pytest.fixture(scope="module")
def tiny_model_bf16(tiny_cfg, tiny_sd, tokenizer):
    return tvr_amd.Model.from_hf_state_dict(tiny_cfg, tiny_sd, device="cuda", tokenizer=tokenizer, gemm="bf16")


def test_bf16_forward_and_extraction(tiny_model_bf16, tiny_oracle):
    m = tiny_model_bf16
    prompts = ragged_prompts(9, m.cfg.d_vocab, 1) + [[0], list(range(128))]
    targets = [p[-1] for p in prompts]
    out = m.forward_clean(prompts, targets=targets, return_logits=True)
    for i, p in enumerate(prompts):
        ref = tiny_oracle.forward(torch.tensor([p]))[0, -1]
        assert rel_err(out["logits"][i], ref) < BF16_TOL, i
        pr = torch.softmax(ref, 0)
        assert abs(out["prob"][i].item() - pr[targets[i]].item()) <= BF16_TOL * pr.max().item()
    random.seed(1234)
    ours = tvr_amd.generate_mean_activation(tvr_amd.tasks.letter_to_caps, ARROW, ",", model=m,
                                            num_contexts=96, len_contexts=4)
    random.seed(1234)
    ref = R.generate_mean_activation(tvr_amd.tasks.letter_to_caps, ARROW, ",", model=tiny_oracle,
                                     num_contexts=96, len_contexts=4)
    assert rel_err(ours, ref) < BF16_TOL


def test_bf16_cie(tiny_model_bf16, tiny_oracle):
    m = tiny_model_bf16
    task = tvr_amd.tasks.letter_to_caps
    random.seed(7)
    mean = R.generate_mean_activation(task, ARROW, ",", model=tiny_oracle, num_contexts=32, len_contexts=4)
    random.seed(8)
    prompts, answers = tvr_amd.generate_shuffled_prompts(task, m, 3, 4, ARROW)
    cie = tvr_amd.calculate_average_causal_indirect_effect(mean.cuda(), prompts, answers, model=m)
    cie_ref = R.calculate_average_causal_indirect_effect(mean, prompts, answers, tiny_oracle)
    pmax = max(torch.softmax(tiny_oracle.forward(m.to_tokens(p).cpu())[0, -1], 0).max().item() for p in prompts)
    assert (cie.cpu().double() - cie_ref.double()).abs().max().item() <= BF16_TOL * pmax


def test_sweeps_are_deterministic(tiny_model):
    """No atomics or unordered reductions on the result path: the same sweep
    twice is bitwise identical (capture is a fixed-order two-pass sum)."""
    task = tvr_amd.tasks.letter_to_caps
    outs = []
    for _ in range(2):
        random.seed(11)
        mean = tvr_amd.generate_mean_activation(task, ARROW, ",", model=tiny_model, num_contexts=40, len_contexts=4)
        random.seed(12)
        prompts, answers = tvr_amd.generate_shuffled_prompts(task, tiny_model, 3, 4, ARROW)
        cie = tvr_amd.calculate_average_causal_indirect_effect(mean, prompts, answers, model=tiny_model)
        outs.append((mean.cpu(), cie.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_profile_counts_gemm_and_hbm_kernels(tiny_model):
    """tvr_profile_read / tvr_profile_read_hbm: every kernel family of a CIE
    sweep and of an extraction is timed, with positive algorithmic bytes."""
    task = tvr_amd.tasks.letter_to_caps
    random.seed(5)
    tiny_model.profile(True)
    mean = tvr_amd.generate_mean_activation(task, ARROW, ",", model=tiny_model, num_contexts=16, len_contexts=4)
    ex = tiny_model.profile_hbm_stats()
    tiny_model.profile(True)  # reset
    random.seed(6)
    prompts, answers = tvr_amd.generate_shuffled_prompts(task, tiny_model, 2, 4, ARROW)
    tvr_amd.calculate_average_causal_indirect_effect(mean, prompts, answers, model=tiny_model)
    gemm = tiny_model.profile_stats()
    hbm = tiny_model.profile_hbm_stats()
    tiny_model.profile(False)
    L = tiny_model.cfg.n_layers
    # every layer's capture in ONE reduction (one launch pair per forward, after the layer loop)
    assert ex["capture"]["launches"] == 1 and ex["capture"]["bytes"] > 0 and ex["capture"]["ms"] > 0
    assert gemm["all"]["launches"] > 0 and gemm["all"]["flops"] > 0
    for k in ("entry", "lnpre", "attention", "row_stats"):
        assert hbm[k]["launches"] > 0 and hbm[k]["bytes"] > 0 and hbm[k]["gbps"] > 0, k
    assert hbm["capture"]["launches"] == 0
    assert hbm["entry"]["launches"] <= L  # one injection launch per entry layer


def test_string_prompt_paths_with_bpe_tokenizer(tiny_cfg, tiny_sd):
    """The reference's string-prompt paths (to_tokens with BOS, multi-token
    answers, decoded-string accuracy) through a byte-level BPE tokenizer.json
    (tests/golden/make_tokenizer.py): CIE on state -> capital prompts and the
    FV top-5 accuracy, engine vs oracle with the same tokenizer."""
    from pathlib import Path
    from conftest import make_oracle
    tok = tvr_amd.tokenizer.HFTokenizer(Path(__file__).parent / "golden" / "tokenizer.json")
    model = tvr_amd.Model.from_hf_state_dict(tiny_cfg, tiny_sd, device="cuda", tokenizer=tok)
    oracle = make_oracle(tiny_cfg, tiny_sd, tok)
    task = list(tvr_amd.tasks.state_to_capital_task)
    random.seed(8)
    mean = R.generate_mean_activation(task, ":", ",", model=oracle, num_contexts=16, len_contexts=3)
    random.seed(9)
    prompts, answers = tvr_amd.generate_shuffled_prompts(task, model, 3, 3, ":", ",")
    assert all(isinstance(p, str) for p in prompts) and any(len(a) > 1 for a in answers)
    cie = tvr_amd.calculate_average_causal_indirect_effect(mean.cuda() * 4, prompts, answers, model=model)
    cie_ref = R.calculate_average_causal_indirect_effect(mean * 4, prompts, answers, oracle)
    assert (cie.cpu().double() - cie_ref.double()).abs().max().item() <= 1e-4 * cie_ref.abs().max().item() + 1e-7
    fv = R.assemble_task_vector(mean, cie_ref, 1, 3) * 4
    ctx = task[:20]
    assert tvr_amd.check_accuracy_of_task_vector(fv.cuda(), 1, ctx, model=model) == \
        R.check_accuracy_of_task_vector(fv, 1, ctx, model=oracle)


@pytest.mark.parametrize("shape", ["tiny", "pythia-160m"])
@pytest.mark.parametrize("gemm", ["x2f16", "bf16"])
def test_fused_unembed_statistics_match_logits_path(shape, gemm):
    """The unembed GEMM's fused statistics epilogue (EPI_STATS: per 256-column
    tile max / sum exp / top-k candidates / target logit, no logits in HBM) +
    stats_merge_kernel equals the materialised-logits path (same GEMM, then
    row_stats_kernel) and torch on those logits: probabilities to 1e-6 of the
    largest, top-k ids identical for k = 1, 5, 16, on clean prompts and on
    patch sites.  V = 512 (2 tiles) and 50304 (196 full tiles + one of 128)."""
    cfg = tvr_amd.get_config(shape)
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=1, std=0.1)
    model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda", gemm=gemm)
    prompts = ragged_prompts(37, cfg.d_vocab, 5, lo=2, hi=30)
    trace = model.trace(len(prompts), sum(map(len, prompts)))
    with_logits = model.forward_clean(prompts, trace=trace, return_logits=True)["logits"]
    targets = [int(torch.topk(l, 3).indices[i % 3]) for i, l in enumerate(with_logits)]  # high-probability targets
    targets[1] = cfg.d_vocab - 1  # the last column of the last (partial) tile
    for k in (1, 5, 16):
        fused = model.forward_clean(prompts, targets=targets, topk=k)
        ref = model.forward_clean(prompts, targets=targets, topk=k, return_logits=True)
        p = torch.softmax(ref["logits"].double(), -1)
        assert (fused["prob"].double() - ref["prob"].double()).abs().max().item() <= 1e-6 * p.max().item()
        assert torch.equal(fused["topk"], ref["topk"])
        assert fused["topk"].long().tolist() == torch.topk(ref["logits"], k).indices.tolist()
    g = torch.Generator().manual_seed(2)
    vecs = (torch.randn(4, cfg.d_model, generator=g) * 2).cuda()
    sites = tvr_amd.make_sites(len(prompts) * 3)
    for i in range(len(prompts)):
        for j, kind in enumerate((tvr_amd._lib.SITE_REPLACE_HEAD_ALLPOS, tvr_amd._lib.SITE_ADD_ATTN_OUT_LASTPOS,
                                  tvr_amd._lib.SITE_NONE)):
            s = sites[3 * i + j]
            s["seq"], s["kind"], s["layer"], s["head"], s["vec"] = i, kind, (i + j) % cfg.n_layers, i % cfg.n_heads, j
            s["target"] = targets[i]
    fused = model.patch_sweep(trace, sites, vecs, topk=5)
    ref = model.patch_sweep(trace, sites, vecs, topk=5, return_logits=True)
    p = torch.softmax(ref["logits"].double(), -1)
    assert (fused["prob"].double() - ref["prob"].double()).abs().max().item() <= 1e-6 * p.max().item()
    assert torch.equal(fused["topk"], ref["topk"])


def test_forward_all_positions_and_start_at_layer(tiny_model, tiny_oracle):
    """Model.forward is TransformerLens' forward: [1, T, V] logits of every
    position (scratch2.py:143,183,297) and forward(resid, start_at_layer=L)
    (scratch.py:143,206,209), through tvr_forward_logits."""
    rng = random.Random(41)
    ids = [0] + [rng.randrange(1, tiny_model.cfg.d_vocab) for _ in range(20)]
    ref = tiny_oracle.forward(torch.tensor([ids]))
    out = tiny_model.forward(ids)
    assert out.shape == ref.shape
    assert rel_err(out[0], ref[0]) < 1e-4
    assert rel_err(tiny_model.forward(torch.tensor([ids]), last_only=True)[0, 0], ref[0, -1]) < 1e-4
    assert torch.equal(tiny_model(ids).argmax(-1).cpu(), ref.argmax(-1))
    _, cache = tiny_oracle.run_with_cache(torch.tensor([ids]))
    for layer in range(tiny_oracle.cfg.n_layers):
        resid = cache[f"blocks.{layer}.hook_resid_pre"].clone()
        resid[0, 5] = cache[f"blocks.{layer}.hook_resid_pre"][0, 9]  # scratch.py:141-142 style surgery
        want = tiny_oracle.forward(resid, start_at_layer=layer)
        got = tiny_model.forward(resid.cuda(), start_at_layer=layer)
        assert rel_err(got[0], want[0]) < 1e-4, layer


def test_sequences_longer_than_128(tiny_cfg, tiny_sd, tokenizer):
    """Prompts past 128 tokens (TransformerLens n_ctx 2048): the attention
    kernel's chunked online-softmax form, the chunked entry staging and the
    compact last-row z capture, against the oracle: last-row and all-position
    logits, extraction sums, every site kind on a 300-token prompt."""
    from conftest import make_oracle
    cfg = tiny_cfg.with_(n_ctx=2048)
    oracle = make_oracle(cfg, tiny_sd, tokenizer)
    rng = random.Random(43)
    prompts = [[0] + [rng.randrange(1, cfg.d_vocab) for _ in range(n - 1)] for n in (300, 17, 700, 129, 150)]
    for gemm in ("x2f16", "f32"):
        model = tvr_amd.Model.from_hf_state_dict(cfg, tiny_sd, device="cuda", tokenizer=tokenizer, gemm=gemm)
        out = model.forward_clean(prompts, targets=[p[3] for p in prompts], topk=3, return_logits=True, capture=True)
        zsum = torch.zeros(cfg.n_layers, cfg.d_model, dtype=torch.float64)
        for i, p in enumerate(prompts):
            logits, cache = oracle.run_with_cache(torch.tensor([p]))
            assert rel_err(out["logits"][i], logits[0, -1]) < 1e-4, (gemm, i)
            assert out["topk"][i].tolist() == torch.topk(logits[0, -1], 3).indices.tolist()
            for l in range(cfg.n_layers):
                zsum[l] += cache[f"blocks.{l}.attn.hook_z"][0, -1].reshape(-1).double()
        assert rel_err(out["zsum"], zsum) < 1e-4
        assert rel_err(model.forward(prompts[2])[0], oracle.forward(torch.tensor([prompts[2]]))[0]) < 1e-4
        # patch sites on the 300-token prompt
        p = prompts[0]
        trace = model.trace(len(prompts), sum(map(len, prompts)))
        model.forward_clean(prompts, trace=trace)
        vecs = torch.randn(2, cfg.d_model, generator=torch.Generator().manual_seed(7))
        sites = tvr_amd.make_sites(3)
        sites[0]["kind"], sites[0]["layer"], sites[0]["head"], sites[0]["vec"] = 1, 0, 2, 0
        sites[1]["kind"], sites[1]["layer"], sites[1]["vec"] = 2, 1, 1
        sites[2]["kind"], sites[2]["layer"], sites[2]["pos"], sites[2]["src_seq"], sites[2]["src_pos"] = 3, 1, 100, 2, 600
        sites["seq"] = 0
        got = model.patch_sweep(trace, sites, vecs.cuda(), return_logits=True, want_prob=False)["logits"]
        oracle.cfg.use_attn_result = True
        try:
            def rep(hv, hook):
                hv[0, :, 2, :] = vecs[0]
                return hv
            w0 = oracle.run_with_hooks(torch.tensor([p]), fwd_hooks=[("blocks.0.attn.hook_result", rep)])[0, -1]
        finally:
            oracle.cfg.use_attn_result = False
        w1 = oracle.run_with_hooks(torch.tensor([p]), fwd_hooks=[
            ("blocks.1.hook_attn_out", lambda hv, hook: R.layer_addition_hook(hv, hook, vecs[1]))])[0, -1]
        _, c0 = oracle.run_with_cache(torch.tensor([p]))
        _, c2 = oracle.run_with_cache(torch.tensor([prompts[2]]))
        r = c0["blocks.1.hook_resid_pre"].clone()
        r[0, 100] = c2["blocks.1.hook_resid_pre"][0, 600]
        w2 = oracle.forward(r, start_at_layer=1)[0, -1]
        for j, want in enumerate((w0, w1, w2)):
            assert rel_err(got[j], want) < 1e-4, (gemm, j)
        # the same sites with the clean forward deferred into the sweep (long rows in the fused launches)
        trace2 = model.trace(len(prompts), sum(map(len, prompts)))
        model.forward_clean(prompts, trace=trace2, defer=True)
        fused = model.patch_sweep(trace2, sites, vecs.cuda(), return_logits=True, want_prob=False)["logits"]
        assert rel_err(fused, got) < 1e-5, gemm
        assert rel_err(trace2.z(1), trace.z(1)) < 1e-5 and rel_err(trace2.resid_pre(2), trace.resid_pre(2)) < 1e-5
        del model


def _all_kind_sites(cfg, prompts):
    """Every site kind on every prompt (the kinds test's layout, no oracle)."""
    sites = tvr_amd.make_sites(4 * len(prompts))
    k = 0
    for i, p in enumerate(prompts):
        for kind in range(4):
            s = sites[k]
            s["seq"], s["kind"], s["target"] = i, kind, p[1]
            if kind == 1:
                s["layer"], s["head"], s["vec"] = (i + 1) % cfg.n_layers, i % cfg.n_heads, i % 5
            elif kind == 2:
                s["layer"], s["vec"] = i % cfg.n_layers, 4
            elif kind == 3:
                src = (i + 1) % len(prompts)
                s["layer"], s["pos"], s["src_seq"], s["src_pos"] = i % cfg.n_layers, len(p) // 2, src, \
                    len(prompts[src]) // 3
            k += 1
    return sites


def test_deferred_clean_forward_fused_into_sweep(tiny_model):
    """tvr_forward_clean_deferred + tvr_patch_sweep (the clean rows run inside
    the sweep's launches) gives the outputs of tvr_forward_clean +
    tvr_patch_sweep: every site kind, shared-prefix prompts, clean prob /
    top-k, and a trace filled as the clean forward fills it (resid_pre, z,
    and a second sweep that reads its K/V)."""
    cfg = tiny_model.cfg
    rng = random.Random(23)
    base = [0] + [rng.randrange(1, cfg.d_vocab) for _ in range(29)]
    prompts = ragged_prompts(4, cfg.d_vocab, 12, lo=3, hi=30) + [base[:24], base[:20] + [7, 9, 11], base[:24]]
    n, ntok = len(prompts), sum(map(len, prompts))
    tg = [p[1] for p in prompts]
    vecs = torch.randn(5, cfg.d_model, generator=torch.Generator().manual_seed(5)).cuda()
    sites = _all_kind_sites(cfg, prompts)
    head = tvr_amd.make_sites(2 * n)  # head replacement on every prompt (prefix sharing between 4..6)
    for i in range(n):
        for j in range(2):
            s = head[2 * i + j]
            s["seq"], s["kind"], s["target"] = i, tvr_amd._lib.SITE_REPLACE_HEAD_ALLPOS, tg[i]
            s["layer"], s["head"], s["vec"] = j, (i + j) % cfg.n_heads, j
    sites = np.concatenate([sites, head])

    ref_trace = tiny_model.trace(n, ntok)
    ref_clean = tiny_model.forward_clean(prompts, targets=tg, topk=3, trace=ref_trace)
    ref = tiny_model.patch_sweep(ref_trace, sites, vecs, topk=3, return_logits=True)

    trace = tiny_model.trace(n, ntok)
    clean = tiny_model.forward_clean(prompts, targets=tg, topk=3, trace=trace, defer=True)
    out = tiny_model.patch_sweep(trace, sites, vecs, topk=3, return_logits=True)
    assert rel_err(out["logits"], ref["logits"]) < 1e-5
    assert torch.equal(out["topk"], ref["topk"])
    assert (out["prob"] - ref["prob"]).abs().max().item() <= 1e-6
    assert (clean["prob"] - ref_clean["prob"]).abs().max().item() <= 1e-6
    assert torch.equal(clean["topk"], ref_clean["topk"])
    for layer in (0, 1, cfg.n_layers):
        assert rel_err(trace.resid_pre(layer), ref_trace.resid_pre(layer)) < 1e-5, layer
    for layer in range(cfg.n_layers):
        assert rel_err(trace.z(layer), ref_trace.z(layer)) < 1e-5, layer
    again = tiny_model.patch_sweep(trace, sites, vecs, topk=3, return_logits=True)  # the filled trace, reused
    assert rel_err(again["logits"], ref["logits"]) < 1e-5


def test_deferred_clean_forward_runs_on_other_use(tiny_model):
    """A deferred clean forward that no sweep picks up runs on its own when
    the trace is read (or re-used by tvr_forward_clean): outputs written, trace
    equal to the plain clean forward's."""
    cfg = tiny_model.cfg
    prompts = ragged_prompts(3, cfg.d_vocab, 31, lo=4, hi=20)
    n, ntok = len(prompts), sum(map(len, prompts))
    tg = [p[2] for p in prompts]
    ref_trace = tiny_model.trace(n, ntok)
    ref = tiny_model.forward_clean(prompts, targets=tg, topk=2, trace=ref_trace)
    trace = tiny_model.trace(n, ntok)
    clean = tiny_model.forward_clean(prompts, targets=tg, topk=2, trace=trace, defer=True)
    assert rel_err(trace.resid_pre(1), ref_trace.resid_pre(1)) < 1e-5  # runs the deferred forward
    assert (clean["prob"] - ref["prob"]).abs().max().item() <= 1e-6
    assert torch.equal(clean["topk"], ref["topk"])
    clean2 = tiny_model.forward_clean(prompts, targets=tg, trace=trace, defer=True)
    tiny_model.forward_clean(prompts[:1], trace=trace)  # flushes clean2 first
    assert (clean2["prob"] - ref["prob"]).abs().max().item() <= 1e-6
    with pytest.raises(ValueError):
        tiny_model.forward_clean(prompts, trace=trace, defer=True, return_logits=True)


def test_model_freed_on_del_and_traces_closed_first(tiny_cfg, tiny_sd, tokenizer):
    """The experiment functions' scratch trace does not keep the model alive (no model <-> trace cycle: `del
    model` frees it at once), and a caller's trace with a deferred forward pending is run and closed by the
    model before the engine model is destroyed (never after, on a freed model)."""
    import gc
    import weakref
    m = tvr_amd.Model.from_hf_state_dict(tiny_cfg, tiny_sd, device="cuda", tokenizer=tokenizer)
    mean = torch.randn(tiny_cfg.n_layers, tiny_cfg.n_heads, tiny_cfg.d_model, device="cuda") * 0.1
    tvr_amd.experiments.causal_indirect_effect_sums(mean, [[0, 5, 9, 3]], [7], m)  # creates the scratch trace
    assert m._trace_cache is not None
    r = weakref.ref(m)
    gc.disable()
    try:
        del m
        assert r() is None  # freed by reference counting alone
    finally:
        gc.enable()
    m = tvr_amd.Model.from_hf_state_dict(tiny_cfg, tiny_sd, device="cuda", tokenizer=tokenizer)
    t = m.trace(1, 8)
    out = m.forward_clean([[0, 5, 9, 3]], targets=[7], trace=t, defer=True)
    m.__del__()  # as the collector would, with the trace still alive: the pending forward runs first
    assert t._h is None and out["prob"].isfinite().all()

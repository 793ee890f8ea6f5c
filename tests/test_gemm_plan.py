"""CPU: the GEMM launch planner (include/tvr.h tvr_gemm_plan, engine.hip
plan_pp) on the launch shapes of the benchmark configs — a host-only entry
point, so it runs without a GPU.

* C3 (Pythia-2.8B CIE, M up to ~180k rows): the large launches keep one plain
  grid (a split tail only when the last round is nearly empty);
* C2 (52 prompts x T0 = 3: M = 156 + 52 l): the small-M launches get a K
  split that fills the 256 CUs (the 70-tile QKV and 10..70-tile O launches),
  chosen by the dispatch simulation;
* every plan is well formed (split >= 1, k-tiles per block >= 8, tail inside
  the grid) and stream-K stays off unless TVR_STREAM_K=1."""
import ctypes

import pytest

import tvr_amd

X2F16 = tvr_amd._lib.GEMM_MODES["x2f16"]
BF16 = tvr_amd._lib.GEMM_MODES["bf16"]
D, DMLP = 2560, 10240
D1, K2 = 3 * D + DMLP, D + DMLP


def plan(M, N, K, mode=X2F16, gelu=False, model_sliced=False, exact16=False):
    lib = tvr_amd._lib.load()
    out = (ctypes.c_int32 * 5)()
    flags = (1 if gelu else 0) | (2 if model_sliced else 0) | (4 if exact16 else 0)
    assert lib.tvr_gemm_plan(M, N, K, mode, flags, out) == 0
    return {"ksplit": out[0], "tail_base": out[1], "tail_split": out[2], "sk_base": out[3], "sk_blocks": out[4]}


def tiles(M, N):
    return ((M + 255) // 256) * ((N + 255) // 256)


def well_formed(p, M, N, K, bk=32):
    nkt = K // bk
    assert p["ksplit"] >= 1 and nkt // p["ksplit"] >= 8 or p["ksplit"] == 1
    if p["tail_base"]:
        assert p["ksplit"] == 1 and 0 < p["tail_base"] < tiles(M, N) and p["tail_split"] >= 2
        assert nkt // p["tail_split"] >= 8
    assert p["sk_base"] == -1 and p["sk_blocks"] == 0


@pytest.mark.parametrize("exact16", [False, True])
@pytest.mark.parametrize("l", range(32))
def test_c2_layer_launches(l, exact16, monkeypatch):
    monkeypatch.delenv("TVR_STREAM_K", raising=False)
    M = 156 + 52 * l
    q = plan(M, D1, D, gelu=True, exact16=exact16)
    o = plan(M, D, K2, exact16=exact16)
    well_formed(q, M, D1, D)
    well_formed(o, M, D, K2)
    # O + MLP-out: 10 column tiles per m-block -- never a plain launch on <= 70 of 256 CUs
    assert o["ksplit"] > 1 or o["tail_base"] > 0
    if tiles(M, D1) == 70:  # one m-block: 70 of 256 CUs plain
        assert q["ksplit"] > 1


@pytest.mark.parametrize("M", [5376 * l + 168 for l in (4, 8, 16, 24, 31)])
def test_c3_large_launches_stay_plain(M, monkeypatch):
    monkeypatch.delenv("TVR_STREAM_K", raising=False)
    for N, K, g in ((D1, D, True), (D, K2, False)):
        p = plan(M, N, K, gelu=g)
        well_formed(p, M, N, K)
        assert p["ksplit"] == 1
        if p["tail_base"]:
            assert p["tail_base"] == 256 * ((tiles(M, N) - 1) // 256)


def test_stream_k_is_opt_in(monkeypatch):
    monkeypatch.delenv("TVR_STREAM_K", raising=False)
    assert plan(156, D1, D, gelu=True)["sk_base"] == -1
    monkeypatch.setenv("TVR_STREAM_K", "1")
    p = plan(156, D1, D, gelu=True)  # 70 tiles x 80 k-tiles over 256 blocks
    assert p["sk_base"] == 0 and p["sk_blocks"] == 256


def test_bad_arguments():
    lib = tvr_amd._lib.load()
    out = (ctypes.c_int32 * 5)()
    assert lib.tvr_gemm_plan(0, D1, D, X2F16, 0, out) == tvr_amd._lib.TVR_ERR_INVALID
    assert lib.tvr_gemm_plan(16, D1, D, 0, 0, out) == tvr_amd._lib.TVR_ERR_INVALID  # f32 has no planar plan
    assert lib.tvr_gemm_plan(16, D1, 100, X2F16, 0, out) == tvr_amd._lib.TVR_ERR_UNSUPPORTED
    assert lib.tvr_gemm_plan(16, D1, D, X2F16, 8, out) == tvr_amd._lib.TVR_ERR_INVALID  # unknown flag bit
    p = plan(300, 4096 * 3 + 16384, 4096, BF16, True)
    well_formed(p, 300, 4096 * 3 + 16384, 4096, bk=64)


# Pythia-12B (C5): every x2f16 GEMM of the model runs the sliced accumulation (its O + MLP-out K = 25,600
# reaches the threshold), which the planner prices at ~13 % more per k-tile (the host entry point
# must plan with the same rule as launch_gemm)
D12, DMLP12 = 5120, 20480


@pytest.mark.parametrize("M", [40 * 33, 40 * 33 * 5, 40 * 33 * 17, 40 * 33 * 35 + 12 * 33])
def test_c5_plans_use_the_sliced_rule(M, monkeypatch):
    monkeypatch.delenv("TVR_STREAM_K", raising=False)
    D1_, K2_ = 3 * D12 + DMLP12, D12 + DMLP12
    q = plan(M, D1_, D12, gelu=True, model_sliced=True)
    o = plan(M, D12, K2_, model_sliced=True)
    well_formed(q, M, D1_, D12)
    well_formed(o, M, D12, K2_)
    # K >= the threshold is sliced whatever the flag says: the O + MLP-out plan does not depend on it
    assert plan(M, D12, K2_) == o

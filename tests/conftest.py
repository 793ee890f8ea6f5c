import os
import sys
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

import tvr_amd  # noqa: E402
from oracle.hooked_pythia import HookedPythiaOracle, OracleConfig  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP engine); run with -m gpu")
    config.addinivalue_line("markers", "slow: larger shapes")


def pytest_collection_modifyitems(config, items):
    have_gpu = torch.cuda.is_available()
    for it in items:
        if "gpu" in it.keywords and not have_gpu:
            it.add_marker(pytest.mark.skip(reason="no GPU in this container"))


def oracle_config(cfg) -> OracleConfig:
    return OracleConfig(n_layers=cfg.n_layers, d_model=cfg.d_model, n_heads=cfg.n_heads, d_mlp=cfg.d_mlp,
                        d_vocab=cfg.d_vocab, rotary_dim=cfg.rotary_dim, n_ctx=cfg.n_ctx, eps=cfg.ln_eps,
                        rotary_base=cfg.rotary_base)


# Larger-than-HF-init weights for the tiny model make its distributions peaked
# enough that argmax / top-k / accuracy comparisons are informative.
TINY_STD = 0.15


@pytest.fixture(scope="session")
def tiny_cfg():
    return tvr_amd.get_config("tiny")


@pytest.fixture(scope="session")
def tiny_sd(tiny_cfg):
    return tvr_amd.weights.synth_hf_state_dict(tiny_cfg, seed=0, std=TINY_STD)


@pytest.fixture(scope="session")
def tokenizer(tiny_cfg):
    return tvr_amd.tokenizer.SyntheticTokenizer(tiny_cfg.d_vocab)


def make_oracle(cfg, sd, tokenizer, dtype=torch.float32, rotary_table_dtype=None):
    """``rotary_table_dtype=torch.float32`` with an fp64 ``dtype``: the fp32
    reference evaluated in fp64 (TL computes an fp32 model's sin / cos tables
    in fp32: oracle/streamed_pythia.py)."""
    return HookedPythiaOracle(oracle_config(cfg), sd, dtype=dtype, tokenizer=tokenizer,
                              rotary_table_dtype=rotary_table_dtype)


@pytest.fixture(scope="session")
def tiny_oracle(tiny_cfg, tiny_sd, tokenizer):
    return make_oracle(tiny_cfg, tiny_sd, tokenizer)


@pytest.fixture(scope="session")
def tiny_oracle64(tiny_cfg, tiny_sd, tokenizer):
    return make_oracle(tiny_cfg, tiny_sd, tokenizer, torch.float64)


GEMM_MODES = ("x2f16", "x3bf16", "f32")


@pytest.fixture(scope="session", params=GEMM_MODES)
def tiny_model(request, tiny_cfg, tiny_sd, tokenizer):
    """The engine on the tiny model, once per GEMM path (every parity test
    runs against every matrix-core path at the same tolerance)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    m = tvr_amd.Model.from_hf_state_dict(tiny_cfg, tiny_sd, device="cuda", tokenizer=tokenizer,
                                         gemm=request.param)
    assert m._lib.tvr_model_get_gemm(m._h) == tvr_amd._lib.GEMM_MODES[request.param]
    return m

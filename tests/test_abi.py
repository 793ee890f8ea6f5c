"""CPU: the C-ABI library builds, loads, and exports every symbol that
include/tvr.h declares (no compute calls without a GPU)."""
import ctypes
import re
from pathlib import Path

import tvr_amd

ROOT = Path(__file__).resolve().parents[1]


def declared_functions():
    text = (ROOT / "include" / "tvr.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(tvr_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_entry_points():
    names = declared_functions()
    for want in ("tvr_model_create", "tvr_forward_clean", "tvr_patch_sweep", "tvr_project_heads",
                 "tvr_trace_create", "tvr_trace_read", "tvr_trace_flush", "tvr_gemm_f32"):
        assert want in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(str(tvr_amd._lib.LIB_PATH))
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    assert set(declared_functions()) == set(tvr_amd._lib.SIGNATURES)


def test_version_and_errors_without_gpu():
    lib = tvr_amd._lib.load()
    assert lib.tvr_abi_version() == tvr_amd._lib.ABI_VERSION == 11
    assert b"gfx950" in lib.tvr_version()
    # argument validation runs before any device call
    out = ctypes.c_void_p()
    rc = lib.tvr_model_create(None, None, None, None, None, ctypes.byref(out))
    assert rc == tvr_amd._lib.TVR_ERR_INVALID
    assert b"null" in lib.tvr_last_error()
    assert lib.tvr_model_set_exact16(None, None) == tvr_amd._lib.TVR_ERR_INVALID
    assert lib.tvr_model_set_exact16_unembed(None, None, None) == tvr_amd._lib.TVR_ERR_INVALID


def test_exact16_layer_record_matches_header():
    text = (ROOT / "include" / "tvr.h").read_text()
    body = re.search(r"typedef struct \{(.*?)\} tvr_exact16_layer;", text, re.S).group(1)
    assert re.findall(r"\*\s*(\w+);", body) == [f for f, _ in tvr_amd._lib.CExact16Layer._fields_]


def test_raw16_weights_only_for_fp16_values(tiny_cfg):
    """weights.py keeps the checkpoint's own GEMM weights (fp16) only when every one is fp16-valued."""
    import torch
    w16 = tvr_amd.weights.synth_engine_weights(tiny_cfg, seed=0, fp16=True)
    assert w16.raw16 is not None and len(w16.raw16) == tiny_cfg.n_layers
    r = w16.raw16[0]
    d, D1, K2 = tiny_cfg.d_model, 3 * tiny_cfg.d_model + tiny_cfg.d_mlp, tiny_cfg.d_model + tiny_cfg.d_mlp
    assert r.w1.dtype == torch.float16 and tuple(r.w1.shape) == (D1, d)
    assert r.w2.dtype == torch.float16 and tuple(r.w2.shape) == (d, K2)
    assert r.g1.dtype == torch.float32 and tuple(r.g1.shape) == (d,)
    # the processed W1 is fold_ln of the raw rows: W1' = W1 * gamma - row mean (TL fold_ln + centring)
    w1p = r.w1.float().clone()
    w1p[: 3 * d] = r.w1[: 3 * d].float() * r.g1
    w1p[3 * d:] = r.w1[3 * d:].float() * r.g2
    w1p = w1p - w1p.mean(dim=1, keepdim=True)
    assert torch.allclose(w1p, w16.layers[0].w1, atol=1e-6, rtol=0)
    # the processed W2 is the raw one centred over d_model
    w2 = r.w2.float()
    assert torch.allclose(w2 - w2.mean(dim=0, keepdim=True), w16.layers[0].w2, atol=1e-6, rtol=0)
    wu, gf = w16.raw16_unembed
    assert wu.dtype == torch.float16 and tuple(wu.shape) == (tiny_cfg.d_vocab, d) and gf.dtype == torch.float32
    assert tvr_amd.weights.synth_engine_weights(tiny_cfg, seed=0).raw16 is None


def test_site_record_layout_matches_header():
    text = (ROOT / "include" / "tvr.h").read_text()
    body = re.search(r"typedef struct tvr_site \{(.*?)\} tvr_site;", text, re.S).group(1)
    fields = re.findall(r"int32_t\s+(\w+);", body)
    assert fields == tvr_amd._lib.SITE_FIELDS
    assert tvr_amd.model.SITE_DTYPE.itemsize == 4 * len(fields)


def test_model_refuses_cpu_device(tiny_cfg):
    import pytest
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    w = tvr_amd.weights.synth_engine_weights(tiny_cfg, seed=0)
    with pytest.raises(tvr_amd._lib.EngineError, match="no CPU fallback"):
        tvr_amd.Model(tiny_cfg, w)


# the façade calls torch.ops.tvr.*, registered by _tvr_ops.so over the C ABI
OP_SCHEMAS = {
    "forward_clean": "tvr::forward_clean(int model, int trace, Tensor tokens, Tensor seq_lens, Tensor? targets, "
                     "int topk, bool want_logits, bool capture, bool defer, int n_layers, int d_model, int d_vocab, "
                     "Device device) -> (Tensor, Tensor, Tensor, Tensor)",
    "patch_sweep": "tvr::patch_sweep(int model, int trace, Tensor sites, Tensor? vectors, int topk, bool want_prob, "
                   "bool want_logits, int d_vocab, Device device) -> (Tensor, Tensor, Tensor)",
    "project_heads": "tvr::project_heads(int model, Tensor zsum, int n_heads) -> Tensor",
    "forward_logits": "tvr::forward_logits(int model, Tensor? tokens, Tensor? resid, int start_layer, "
                      "Tensor seq_lens, int d_vocab, Device device) -> Tensor",
}


def test_torch_ops_schemas():
    ops = tvr_amd._lib.load_ops()
    assert set(OP_SCHEMAS) == set(tvr_amd._lib.OPS)
    for name, schema in OP_SCHEMAS.items():
        assert str(getattr(ops, name).default._schema) == schema


def test_torch_ops_refuse_cpu_and_bad_arguments():
    import pytest
    import torch
    ops = tvr_amd._lib.load_ops()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.project_heads(1, torch.zeros(2, 4), 2)
    with pytest.raises(ValueError, match=r"\[n_sites, 9\]"):
        ops.patch_sweep(1, 1, torch.zeros(3, 8, dtype=torch.int32), None, 0, True, False, 8, torch.device("cuda", 0))

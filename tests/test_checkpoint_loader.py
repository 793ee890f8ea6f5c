"""The local checkpoint path that replaces the by-name fetch
(``HookedTransformer.from_pretrained("pythia-410m")``, scratch.py:26 /
scratch2.py:26): a GPTNeoXForCausalLM-layout safetensors file
with the key set real Pythia checkpoints carry — per-layer buffers
``attention.bias`` (causal mask), ``attention.masked_bias``,
``attention.rotary_emb.inv_freq`` — in fp16, single-file and sharded, plus
its config.json.

CPU: the loader keeps exactly the parameters, in fp32, and TL processing of
the loaded dict equals processing of the in-memory one.  GPU: a model built
from the file gives the same logits as one built from the state dict.
"""
import json

import pytest
import torch

import tvr_amd
from tvr_amd import weights as W


def write_checkpoint(tmp_path, cfg, sd, shards=1, lm_head=False):
    from safetensors.torch import save_file
    full = {}
    for k, v in sd.items():
        full[("lm_head.weight" if lm_head and k == "embed_out.weight" else k)] = v.half()
    rd = cfg.rotary_dim
    for l in range(cfg.n_layers):
        p = f"gpt_neox.layers.{l}.attention."
        full[p + "bias"] = torch.tril(torch.ones(cfg.n_ctx, cfg.n_ctx, dtype=torch.bool)).view(1, 1, cfg.n_ctx,
                                                                                                cfg.n_ctx)
        full[p + "masked_bias"] = torch.tensor(-1e9)
        full[p + "rotary_emb.inv_freq"] = 1.0 / (10000 ** (torch.arange(0, rd, 2).float() / rd))
    keys = sorted(full)
    if shards == 1:
        save_file(full, str(tmp_path / "model.safetensors"))
    else:
        wm = {}
        for i in range(shards):
            name = f"model-{i + 1:05d}-of-{shards:05d}.safetensors"
            part = {k: full[k] for k in keys[i::shards]}
            save_file(part, str(tmp_path / name))
            wm.update({k: name for k in part})
        (tmp_path / "model.safetensors.index.json").write_text(json.dumps({"weight_map": wm}))
    (tmp_path / "config.json").write_text(json.dumps({
        "model_type": "gpt_neox", "num_hidden_layers": cfg.n_layers, "hidden_size": cfg.d_model,
        "num_attention_heads": cfg.n_heads, "intermediate_size": cfg.d_mlp, "vocab_size": cfg.d_vocab,
        "rotary_pct": cfg.rotary_pct, "rotary_emb_base": 10000, "max_position_embeddings": cfg.n_ctx,
        "layer_norm_eps": 1e-5, "use_parallel_residual": True, "hidden_act": "gelu", "_name_or_path": "tiny-ckpt"}))
    return tmp_path


@pytest.fixture(scope="module")
def tiny():
    cfg = tvr_amd.get_config("tiny")
    return cfg, W.synth_hf_state_dict(cfg, seed=0, std=0.15)


@pytest.mark.parametrize("shards,lm_head", [(1, False), (3, False), (1, True)])
def test_loader_keeps_parameters_drops_buffers(tmp_path, tiny, shards, lm_head):
    cfg, sd = tiny
    path = write_checkpoint(tmp_path, cfg, sd, shards, lm_head)
    got = W.load_hf_safetensors(path, cfg)
    assert set(got) == set(W.hf_param_shapes(cfg))
    for k, v in sd.items():
        assert got[k].dtype == torch.float32
        assert torch.equal(got[k], v.half().float()), k
    if shards == 1:  # the file itself, not the directory
        assert set(W.load_hf_safetensors(path / "model.safetensors", cfg)) == set(got)


def test_loader_reports_missing_and_misshaped(tmp_path, tiny):
    cfg, sd = tiny
    bad = dict(sd)
    del bad["gpt_neox.layers.1.mlp.dense_4h_to_h.bias"]
    bad["gpt_neox.final_layer_norm.weight"] = torch.ones(cfg.d_model + 1)
    path = write_checkpoint(tmp_path, cfg, bad)
    with pytest.raises(ValueError, match=r"dense_4h_to_h.bias.*final_layer_norm"):
        W.load_hf_safetensors(path, cfg)


def test_config_json(tmp_path, tiny):
    cfg, sd = tiny
    c = W.config_from_hf_json(write_checkpoint(tmp_path, cfg, sd))
    for f in ("n_layers", "d_model", "n_heads", "d_mlp", "d_vocab", "rotary_dim", "n_ctx", "ln_eps", "rotary_base"):
        assert getattr(c, f) == getattr(cfg, f), f
    cj = json.loads((tmp_path / "config.json").read_text())
    cj["use_parallel_residual"] = False
    (tmp_path / "config.json").write_text(json.dumps(cj))
    with pytest.raises(ValueError, match="parallel residual"):
        W.config_from_hf_json(tmp_path)


def test_processing_of_loaded_checkpoint(tmp_path, tiny):
    cfg, sd = tiny
    got = W.load_hf_safetensors(write_checkpoint(tmp_path, cfg, sd), cfg)
    a = W.process_to_engine(cfg, got)
    b = W.process_to_engine(cfg, {k: v.half().float() for k, v in sd.items()})
    for x, y in zip(a.tensors(), b.tensors()):
        assert torch.equal(x, y)
    # a float16 checkpoint (every released Pythia) keeps its raw GEMM weights for the exact-fp16 GEMMs
    assert a.raw16 is not None and a.raw16_unembed is not None
    for ra, rb in zip(a.raw16, b.raw16):
        assert torch.equal(ra.w1, rb.w1) and torch.equal(ra.w2, rb.w2) and torch.equal(ra.g1, rb.g1)
    assert torch.equal(a.raw16_unembed[0], sd["embed_out.weight"].half())
    assert W.process_to_engine(cfg, got, raw16=False).raw16 is None


@pytest.mark.parametrize("raw16", [False, True])
def test_free_source_empties_the_state_dict(tmp_path, tiny, raw16):
    """free_source pops every tensor it processed, with or without the raw fp16 copies (the raw
    GEMM weights were kept alive when raw16 was off), and the result equals processing a kept dict."""
    cfg, sd = tiny
    got = W.load_hf_safetensors(write_checkpoint(tmp_path, cfg, sd), cfg)
    ref = W.process_to_engine(cfg, dict(got), raw16=raw16)
    out = W.process_to_engine(cfg, got, free_source=True, raw16=raw16)
    assert got == {}
    for x, y in zip(out.tensors(), ref.tensors()):
        assert torch.equal(x, y)
    assert (out.raw16 is not None) == raw16


@pytest.mark.gpu
def test_model_from_checkpoint_matches_state_dict(tmp_path, tiny):
    cfg, sd = tiny
    path = write_checkpoint(tmp_path, cfg, sd, shards=2)
    m1 = tvr_amd.Model.from_pretrained("tiny", checkpoint=str(path), device="cuda")
    m2 = tvr_amd.Model.from_hf_state_dict(cfg, {k: v.half().float() for k, v in sd.items()}, device="cuda")
    m3 = tvr_amd.Model.from_pretrained("tiny-ckpt-by-config", checkpoint=str(path), device="cuda")
    assert m3.cfg.n_layers == cfg.n_layers and m3.cfg.d_vocab == cfg.d_vocab
    prompts = [[0, 5, 9, 13, 2], [0, 7, 1]]
    l1 = m1.forward_clean(prompts, return_logits=True)["logits"]
    l2 = m2.forward_clean(prompts, return_logits=True)["logits"]
    l3 = m3.forward_clean(prompts, return_logits=True)["logits"]
    assert torch.equal(l1, l2) and torch.equal(l1, l3)

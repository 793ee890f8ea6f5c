"""CPU: pin the oracle's forward against HuggingFace GPTNeoX (the only
executable Pythia implementation offline) and the product's weight processing
against the oracle's.

TransformerLens' processing makes logits mean-centred over the vocab and the
residual mean-centred over d_model, without changing the softmax:
  TL_logits = HF_logits - mean_v(HF_logits)           
"""
import pytest
import torch

import tvr_amd
from conftest import TINY_STD, make_oracle

transformers = pytest.importorskip("transformers")


def hf_model(cfg, sd):
    from transformers import GPTNeoXConfig, GPTNeoXForCausalLM
    hcfg = GPTNeoXConfig(vocab_size=cfg.d_vocab, hidden_size=cfg.d_model, num_hidden_layers=cfg.n_layers,
                         num_attention_heads=cfg.n_heads, intermediate_size=cfg.d_mlp, rotary_pct=cfg.rotary_pct,
                         rotary_emb_base=int(cfg.rotary_base), max_position_embeddings=cfg.n_ctx,
                         layer_norm_eps=cfg.ln_eps, use_parallel_residual=True, hidden_act="gelu",
                         tie_word_embeddings=False, attention_bias=True)
    hcfg._attn_implementation = "eager"
    m = GPTNeoXForCausalLM(hcfg).eval()
    # real Pythia checkpoints call the unembed "embed_out"; transformers 5 names it "lm_head"
    renamed = {("lm_head.weight" if k == "embed_out.weight" else k): v.clone() for k, v in sd.items()}
    missing, unexpected = m.load_state_dict(renamed, strict=False)
    assert not unexpected, unexpected
    assert all("rotary" in k or "masked_bias" in k for k in missing), missing
    return m


# HF builds its rotary cos/sin in fp32 even for an fp64 model (GPTNeoXRotaryEmbedding
# forces fp32), TL in the model dtype: positions > 0 differ at ~1e-7 relative in fp64.
@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-6), (torch.float32, 2e-5)])
def test_oracle_logits_match_hf(tiny_cfg, tiny_sd, tokenizer, dtype, tol):
    hf = hf_model(tiny_cfg, tiny_sd).to(dtype)
    oracle = make_oracle(tiny_cfg, tiny_sd, tokenizer, dtype)
    g = torch.Generator().manual_seed(7)
    tokens = torch.randint(0, tiny_cfg.d_vocab, (1, 23), generator=g)
    with torch.no_grad():
        ref = hf(tokens).logits.to(dtype)
    ours = oracle.forward(tokens)
    ref_c = ref - ref.mean(-1, keepdim=True)
    scale = ref_c.abs().max()
    assert (ours - ref_c).abs().max() / scale < tol
    assert torch.equal(ours[0].argmax(-1), ref[0].argmax(-1))
    torch.testing.assert_close(torch.softmax(ours, -1), torch.softmax(ref, -1), rtol=tol * 10, atol=tol)


def test_oracle_resid_is_centred_hf_resid(tiny_cfg, tiny_sd, tokenizer):
    hf = hf_model(tiny_cfg, tiny_sd).double()
    oracle = make_oracle(tiny_cfg, tiny_sd, tokenizer, torch.float64)
    tokens = torch.tensor([[0, 5, 9, 33, 2, 101, 7]])
    with torch.no_grad():
        hs = hf(tokens, output_hidden_states=True).hidden_states
    _, cache = oracle.run_with_cache(tokens)
    for l in range(tiny_cfg.n_layers):
        want = hs[l] - hs[l].mean(-1, keepdim=True)
        torch.testing.assert_close(cache[f"blocks.{l}.hook_resid_pre"], want, rtol=0, atol=1e-6)


def test_hook_result_sums_to_attn_out(tiny_cfg, tiny_sd, tokenizer):
    """hook_result excludes b_O (and the folded value bias): Σ_h result + b_O = attn_out."""
    oracle = make_oracle(tiny_cfg, tiny_sd, tokenizer, torch.float64)
    oracle.cfg.use_attn_result = True
    try:
        _, cache = oracle.run_with_cache(torch.tensor([[0, 3, 4, 5, 6]]))
    finally:
        oracle.cfg.use_attn_result = False
    for l in range(tiny_cfg.n_layers):
        res = cache[f"blocks.{l}.attn.hook_result"]
        out = cache[f"blocks.{l}.hook_attn_out"]
        torch.testing.assert_close(res.sum(-2) + oracle.w["blocks"][l]["b_O"], out, rtol=0, atol=1e-12)


def engine_layout_forward(cfg, w, tokens):
    """Torch restatement of the engine's fused-layout math (test helper):
    the product's processed weights must reproduce the oracle's logits."""
    d, H, dh, rd = cfg.d_model, cfg.n_heads, cfg.d_head, cfg.rotary_dim
    x = w.w_embed[tokens].double()
    T = x.shape[0]

    def lnpre(v):
        v = v - v.mean(-1, keepdim=True)
        return v / (v.pow(2).mean(-1, keepdim=True) + cfg.ln_eps).sqrt()

    pos = torch.arange(T, dtype=torch.float64)
    freq = cfg.rotary_base ** (torch.arange(rd // 2, dtype=torch.float64) / (rd / 2))
    ang = pos[:, None] / torch.cat([freq, freq])[None]
    cos, sin = ang.cos(), ang.sin()

    def rot(v):  # [T, H, dh]
        r, p = v[..., :rd], v[..., rd:]
        flip = torch.cat([-r[..., rd // 2:], r[..., : rd // 2]], -1)
        return torch.cat([r * cos[:, None] + flip * sin[:, None], p], -1)

    for L in w.layers:
        y = lnpre(x) @ L.w1.double().T + L.b1.double()
        q, k, v = (y[:, i * d:(i + 1) * d].view(T, H, dh) for i in range(3))
        q, k = rot(q), rot(k)
        s = torch.einsum("qhe,khe->hqk", q, k) / dh ** 0.5
        s = s.masked_fill(torch.triu(torch.ones(T, T, dtype=torch.bool), 1), float("-inf"))
        z = torch.einsum("hqk,khe->qhe", s.softmax(-1), v).reshape(T, d)
        a2 = torch.cat([z, torch.nn.functional.gelu(y[:, 3 * d:])], -1)
        x = x + a2 @ L.w2.double().T + L.b2.double()
    return lnpre(x) @ w.w_unembed_t.double().T + w.b_unembed.double()


def test_engine_weight_processing_matches_oracle(tiny_cfg, tiny_sd, tokenizer):
    w = tvr_amd.weights.process_to_engine(tiny_cfg, tiny_sd, dtype=torch.float64)
    oracle = make_oracle(tiny_cfg, tiny_sd, tokenizer, torch.float64)
    tokens = torch.tensor([0, 17, 1, 99, 12, 1, 250, 3, 1])
    ours = engine_layout_forward(tiny_cfg, w, tokens)
    want = oracle.forward(tokens[None])[0]
    torch.testing.assert_close(ours, want, rtol=0, atol=1e-10)


def test_synth_engine_weights_equal_processed_state_dict(tiny_cfg):
    sd = tvr_amd.weights.synth_hf_state_dict(tiny_cfg, seed=3, std=TINY_STD)
    a = tvr_amd.weights.process_to_engine(tiny_cfg, sd)
    b = tvr_amd.weights.synth_engine_weights(tiny_cfg, seed=3, std=TINY_STD)
    for x, y in zip(a.tensors(), b.tensors()):
        assert torch.equal(x, y)

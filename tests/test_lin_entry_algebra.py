"""CPU: the algebra behind the linearised entry layer (csrc/lin_entry.hpp),
pinned on the fp64 oracle (TransformerLens semantics, oracle/hooked_pythia.py).

For a head-replacement site (layer l-1, head h, vector v: the hook writes v
into ``blocks.{l-1}.attn.hook_result[0, :, h]`` at every position,
scratch2.py:187-189), the residual entering block l is
    r = r_c + v - z_h W_O[h]                     (r_c, z_h: the clean run's)
and block l's first projections read LNPre(r).  The engine computes them as
    y = (sigma_c y_c + (mu_c - mu) c1 + v W - z_h (W_O[h] W)) / sigma + b
with y_c = LNPre(r_c) W the clean row's own projection, c1 = 1^T W, and
(mu, sigma) the row's LayerNormPre statistics.  Both identities are checked
here against the oracle's own hooked forward in fp64 for Q, K, V and MLP-in.
"""
import torch

import tvr_amd
from conftest import make_oracle


def test_linearised_entry_identity_fp64(tiny_cfg, tokenizer):
    cfg = tiny_cfg.with_(n_layers=3)
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=5, std=0.15)
    oracle = make_oracle(cfg, sd, tokenizer, dtype=torch.float64)
    g = torch.Generator().manual_seed(0)
    tokens = torch.tensor([[0] + torch.randint(1, cfg.d_vocab, (13,), generator=g).tolist()])
    v = torch.randn(cfg.d_model, generator=g, dtype=torch.float64)
    H, eps = cfg.n_heads, cfg.ln_eps
    for l in (1, 2):
        for h in (0, H - 1):
            _, clean = oracle.run_with_cache(tokens)
            got = {}

            def replace(x, hook, h=h):
                x[0, :, h, :] = v
                return x

            def grab(x, hook):
                got["r"] = x.detach().clone()
                return x
            oracle.cfg.use_attn_result = True
            try:
                oracle.run_with_hooks(tokens, fwd_hooks=[(f"blocks.{l - 1}.attn.hook_result", replace),
                                                         (f"blocks.{l}.hook_resid_pre", grab)])
            finally:
                oracle.cfg.use_attn_result = False
            r_hooked = got["r"][0]
            b = oracle.w["blocks"]
            r_c = clean[f"blocks.{l}.hook_resid_pre"][0]
            z_h = clean[f"blocks.{l - 1}.attn.hook_z"][0][:, h, :]            # [T, dh]
            W_O = b[l - 1]["W_O"][h]                                           # [dh, d]
            # the entry kernel's residual
            r = r_c + (v - z_h @ W_O)
            assert torch.allclose(r, r_hooked, rtol=0, atol=1e-12 * r_hooked.abs().max().item())
            # block l's first projections, direct and linearised
            W = torch.cat([b[l]["W_Q"].permute(1, 0, 2).reshape(cfg.d_model, -1),
                           b[l]["W_K"].permute(1, 0, 2).reshape(cfg.d_model, -1),
                           b[l]["W_V"].permute(1, 0, 2).reshape(cfg.d_model, -1), b[l]["W_in"]], dim=1)

            def ln_stats(x):
                mu = x.mean(-1, keepdim=True)
                return mu, ((x - mu).pow(2).mean(-1, keepdim=True) + eps).sqrt()
            mu, sig = ln_stats(r)
            mu_c, sig_c = ln_stats(r_c)
            direct = ((r - mu) / sig) @ W
            y_c = ((r_c - mu_c) / sig_c) @ W
            c1 = W.sum(0)
            lin = (sig_c * y_c + (mu_c - mu) * c1 + v @ W - z_h @ (W_O @ W)) / sig
            assert torch.allclose(lin, direct, rtol=0, atol=1e-11 * direct.abs().max().item()), (l, h)

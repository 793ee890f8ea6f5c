"""ORACLE (test infrastructure only) — the reference's experiment loops on a
LAYER-STREAMED fp64 TransformerLens-semantics Pythia, for full-depth parity at
the 6.9B / 12B widths.

``HookedPythiaOracle`` holds every processed weight of the model at once
(12B in fp64 would be 95 GB) and runs one batch-1 forward per site, which at
full depth and these widths takes hours.  This restatement keeps ONE block's
weights at a time: ``get_raw(name)`` produces an HF GPT-NeoX parameter on
demand (the seeded generator, or a checkpoint reader), the block is processed
with the same TL steps (``hooked_pythia.tl_process_block``: fold_ln,
center_writing_weights, fold_value_biases) in fp64, every sequence that needs
that block goes through it as one batch, and the block is dropped.

Semantics are the reference's, row by row (each batch row is an independent
batch-1 forward):
* ``cie``: scratch2.py:171-197 — per prompt a clean forward (p0 =
  softmax(logits[0, -1])[answer], :183-184) and one forward per (layer, head)
  with ``hook_result[0, :, head, :] = mean[layer, head]`` at every position
  (:187-191), p - p0 accumulated and divided by the prompt count (:194,197).
  Rows of a site at layer l equal the clean rows before block l (the hook is
  the only difference), so a site joins the batch at its layer from the clean
  row's ``hook_resid_pre`` — the same numbers as a separate forward from
  token 0.
* ``mean_activation``: scratch2.py:87-100 — mean over the given prompts of
  ``hook_result[0, -1]`` per layer (prompts built by the caller with the
  reference's prompt builder, scratch2.py:88-95).
* ``added_topk``: scratch2.py:292-314 — top-k ids of the last row with
  ``hook_attn_out[0, -1] += vector`` at ``layer`` (layer_addition_hook,
  :107-109); ``vector=None`` is the plain forward (:297).
Per-head results are formed (``einsum(z, W_O)``, then ``sum(-2) + b_O``, as TL
with ``use_attn_result``) only where a hook reads or writes them; elsewhere the
attention output is ``z_flat @ W_O_flat + b_O``, the same sum in another order
(fp64: ~1e-16 relative; tests/test_streamed_oracle.py pins the whole oracle to
``HookedPythiaOracle`` + ``reference_experiments`` at 1e-12).

It runs on whatever device ``get_raw`` returns tensors on: the CPU tests keep
it on the CPU; the full-depth GPU tests keep it on cuda:0 in fp64 (torch /
hipBLAS DGEMM — none of the engine's kernels), which is what makes a 32-layer
6.9B CIE over hundreds of sites take seconds instead of hours.  Results come
back as CPU fp64 tensors.  Only tests/ and tools/ probes use this module.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

from .hooked_pythia import OracleConfig, tl_process_block, tl_process_embed, tl_process_unembed


class StreamedPythiaOracle:
    def __init__(self, cfg: OracleConfig, get_raw: Callable[[str], torch.Tensor], dtype=torch.float64,
                 rotary_table_dtype=torch.float32):
        self.cfg = cfg
        self.dtype = dtype
        self._get = get_raw
        g = lambda n: get_raw(n).to(dtype)  # noqa: E731
        self.W_E = tl_process_embed(g("gpt_neox.embed_in.weight"))
        self.device = self.W_E.device
        self.W_U, self.b_U = tl_process_unembed(g("embed_out.weight"), g("gpt_neox.final_layer_norm.weight"),
                                                g("gpt_neox.final_layer_norm.bias"))
        # TL calculate_sin_cos_rotary computes the tables in fp32 for any model dtype but fp64: the reference
        # runs fp32 (TL's default), so its tables are the fp32 ones, which this fp64 evaluation keeps
        # (``rotary_table_dtype``; float64 restates an fp64 TL model instead).  At 12B (T = 33) the fp32
        # angles pos / freq differ from fp64 by up to ~2e-6 rad — 30x the fp32 rounding of q / k, and the
        # largest single difference between the fp32 reference and an fp64-table model
        # (tools/precision_probe.py): a model definition, not arithmetic error.
        rd = cfg.rotary_dim
        hp = rotary_table_dtype
        pos = torch.arange(cfg.n_ctx, dtype=hp, device=self.device)
        dim = torch.arange(max(rd // 2, 1), dtype=hp, device=self.device)
        freq = cfg.rotary_base ** (dim / max(rd / 2, 1))
        ang = pos[:, None] / torch.cat([freq, freq])[None, :]
        self._sin = torch.sin(ang).to(dtype)
        self._cos = torch.cos(ang).to(dtype)
        self._block_cache: Tuple[int, Optional[Dict[str, torch.Tensor]]] = (-1, None)

    # ------------------------------------------------------------- weights
    def block(self, l: int) -> Dict[str, torch.Tensor]:
        """Block l's TL-processed weights (generated and processed on demand; the last one is kept)."""
        if self._block_cache[0] != l:
            self._block_cache = (-1, None)
            p = f"gpt_neox.layers.{l}."
            self._block_cache = (l, tl_process_block(lambda n: self._get(p + n).to(self.dtype), self.cfg))
        return self._block_cache[1]

    # ------------------------------------------------------------- the model
    def _ln_pre(self, x):
        x = x - x.mean(-1, keepdim=True)
        return x / (x.pow(2).mean(-1, keepdim=True) + self.cfg.eps).sqrt()

    def _rotate(self, x):
        rd = self.cfg.rotary_dim
        if rd == 0:
            return x
        T, n = x.shape[1], rd // 2
        xr, xp = x[..., :rd], x[..., rd:]
        flip = torch.cat([-xr[..., n:], xr[..., :n]], dim=-1)
        return torch.cat([xr * self._cos[:T][None, :, None, :] + flip * self._sin[:T][None, :, None, :], xp], dim=-1)

    def _block(self, l: int, resid: torch.Tensor, replace: Sequence[Tuple[int, int, torch.Tensor]] = (),
               add_last: Sequence[Tuple[int, torch.Tensor]] = (), want_result_last: bool = False):
        """Block l over a batch [b, T, d] of same-length rows.  ``replace``:
        (row, head, vector) — hook_result[row, :, head] = vector (all
        positions); ``add_last``: (row, vector) — hook_attn_out[row, -1] +=
        vector.  Returns (resid_post, per-head result at the last position
        [b, H, d] if ``want_result_last``)."""
        w = self.block(l)
        x = self._ln_pre(resid)
        q = self._rotate(torch.einsum("bpd,hde->bphe", x, w["W_Q"]) + w["b_Q"])
        k = self._rotate(torch.einsum("bpd,hde->bphe", x, w["W_K"]) + w["b_K"])
        v = torch.einsum("bpd,hde->bphe", x, w["W_V"]) + w["b_V"]
        T = x.shape[1]
        scores = torch.einsum("bqhe,bkhe->bhqk", q, k) / math.sqrt(self.cfg.d_head)
        mask = torch.triu(torch.ones(T, T, dtype=torch.bool, device=x.device), diagonal=1)
        z = torch.einsum("bkhe,bhqk->bqhe", v, torch.softmax(scores.masked_fill(mask, float("-inf")), dim=-1))
        H, dh, d = self.cfg.n_heads, self.cfg.d_head, self.cfg.d_model
        attn = z.reshape(z.shape[0], T, H * dh) @ w["W_O"].reshape(H * dh, d) + w["b_O"]
        if replace:
            rows = sorted({r for r, _, _ in replace})
            ri = torch.tensor(rows, device=x.device)
            result = torch.einsum("bqhe,hed->bqhd", z[ri], w["W_O"])
            at = {r: i for i, r in enumerate(rows)}
            for r, h, vec in replace:
                result[at[r], :, h, :] = vec.to(result)
            attn[ri] = result.sum(-2) + w["b_O"]
        for r, vec in add_last:
            attn[r, -1] = attn[r, -1] + vec.to(attn)
        mlp = torch.nn.functional.gelu(x @ w["W_in"] + w["b_in"]) @ w["W_out"] + w["b_out"]
        res_last = torch.einsum("bhe,hed->bhd", z[:, -1], w["W_O"]) if want_result_last else None
        return resid + attn + mlp, res_last

    def _final_last(self, resid):
        """Last-position logits [b, V] (ln_final + unembed)."""
        return self._ln_pre(resid[:, -1]) @ self.W_U + self.b_U

    def _embed(self, seqs: Sequence[Sequence[int]]):
        return self.W_E[torch.tensor([list(s) for s in seqs], device=self.device)]

    # ------------------------------------------------------------ experiments
    @torch.no_grad()
    def last_logits(self, seqs: Sequence[Sequence[int]], batch: int = 256) -> torch.Tensor:
        """Clean last-row logits [n, V] of token-id prompts (grouped by length)."""
        out = [None] * len(seqs)
        for idx in _by_length(seqs, batch):
            r = self._embed([seqs[i] for i in idx])
            for l in range(self.cfg.n_layers):
                r, _ = self._block(l, r)
            lg = self._final_last(r).cpu()
            for j, i in enumerate(idx):
                out[i] = lg[j]
        return torch.stack(out).double()

    @torch.no_grad()
    def cie(self, mean: torch.Tensor, prompts: Sequence[Sequence[int]], answers: Sequence[int],
            layers: Optional[Sequence[int]] = None, heads: Optional[Sequence[int]] = None) -> torch.Tensor:
        """scratch2.py:171-197 restricted to ``layers`` x ``heads``: [L, H] fp64
        (zeros elsewhere), the mean over prompts of p_patched - p_clean."""
        cfg = self.cfg
        L, H = cfg.n_layers, cfg.n_heads
        layers = list(range(L)) if layers is None else list(layers)
        heads = list(range(H)) if heads is None else list(heads)
        mean = mean.to(self.device, self.dtype)
        out = torch.zeros(L, H, dtype=torch.float64)
        sites = [(l, h) for l in layers for h in heads]
        for prompt, ans in zip(prompts, answers):
            clean = self._embed([prompt])  # [1, T, d]
            active = clean[:0]             # sites' rows, in the order they joined
            joined: List[Tuple[int, int]] = []
            for l in range(L):
                new = [s for s in sites if s[0] == l]
                batch = torch.cat([clean, active] + ([clean.expand(len(new), -1, -1)] if new else []))
                rep = [(1 + len(joined) + i, h, mean[l, h]) for i, (_, h) in enumerate(new)]
                batch, _ = self._block(l, batch, replace=rep)
                joined += new
                clean, active = batch[:1], batch[1:]
            p = torch.softmax(self._final_last(torch.cat([clean, active])), dim=-1)[:, int(ans)].cpu().double()
            for i, (l, h) in enumerate(joined):
                out[l, h] += p[1 + i] - p[0]
        return out / len(prompts)

    @torch.no_grad()
    def mean_activation(self, prompts: Sequence[Sequence[int]], batch: int = 256) -> torch.Tensor:
        """scratch2.py:87-100: mean of hook_result[0, -1] over the prompts, [L, H, d] fp64."""
        cfg = self.cfg
        acc = torch.zeros(cfg.n_layers, cfg.n_heads, cfg.d_model, dtype=self.dtype, device=self.device)
        for idx in _by_length(prompts, batch):
            r = self._embed([prompts[i] for i in idx])
            for l in range(cfg.n_layers):
                r, res = self._block(l, r, want_result_last=True)
                acc[l] += res.sum(0)
        return (acc / len(prompts)).cpu().double()

    @torch.no_grad()
    def layer_sweep(self, seqs: Sequence[Sequence[int]], vector: torch.Tensor, targets: Sequence[int],
                    layers: Optional[Sequence[int]] = None, k: int = 2):
        """The layer sweeps of scratch2.py:114-127 / :135-150 on one batch of
        equal-length prompts: for every (prompt, layer i) a forward with
        ``hook_attn_out[0, -1] += vector`` at block i (layer_addition_hook,
        :107-109; the reference's late-binding closure adds the same vector at
        every layer, App. B1), and the clean forward (:143).  A site row joins
        the batch at its layer from the clean row's hook_resid_pre — the same
        numbers as a separate forward from token 0 (the rows before block i are
        the clean ones).  Returns CPU tensors: clean softmax prob of each
        target [n], patched prob [n, len(layers)], patched top-k ids
        [n, len(layers), k] and top-k logits [n, len(layers), k] (the margins)."""
        cfg = self.cfg
        L = cfg.n_layers
        layers = list(range(L)) if layers is None else list(layers)
        if len({len(s) for s in seqs}) != 1:
            raise ValueError("layer_sweep: one prompt length per call")
        n = len(seqs)
        vec = vector.to(self.device, self.dtype)
        clean = self._embed(seqs)      # [n, T, d]
        active = clean[:0]
        joined: List[Tuple[int, int]] = []  # (prompt, layer) of the site rows, in join order
        for l in range(L):
            new = [(i, l) for i in range(n)] if l in layers else []
            batch = torch.cat([clean, active] + ([clean] if new else []))
            add = [(n + len(joined) + j, vec) for j in range(len(new))]
            batch, _ = self._block(l, batch, add_last=add)
            joined += new
            clean, active = batch[:n], batch[n:]
        logits = self._final_last(torch.cat([clean, active]))
        tg = torch.as_tensor([int(t) for t in targets], device=logits.device)
        p = torch.softmax(logits, dim=-1)
        p_clean = p[torch.arange(n, device=p.device), tg].cpu()
        top = torch.topk(logits[n:], k, dim=-1)
        p_site = p[n:][torch.arange(len(joined), device=p.device), tg[[i for i, _ in joined]]].cpu()
        col = {l: c for c, l in enumerate(layers)}
        P = torch.zeros(n, len(layers), dtype=torch.float64)
        ids = torch.zeros(n, len(layers), k, dtype=torch.long)
        vals = torch.zeros(n, len(layers), k, dtype=torch.float64)
        for j, (i, l) in enumerate(joined):
            P[i, col[l]] = p_site[j]
            ids[i, col[l]] = top.indices[j].cpu()
            vals[i, col[l]] = top.values[j].cpu().double()
        return p_clean.double(), P, ids, vals

    @torch.no_grad()
    def added_topk(self, seqs: Sequence[Sequence[int]], layer: int, vector: Optional[torch.Tensor], k: int,
                   batch: int = 256) -> torch.Tensor:
        """Top-k ids [n, k] of the last row with ``hook_attn_out[0, -1] += vector``
        at ``layer`` (scratch2.py:301,311); ``vector=None``: the clean forward (:297)."""
        out = [None] * len(seqs)
        vec = None if vector is None else vector.to(self.device, self.dtype)
        for idx in _by_length(seqs, batch):
            r = self._embed([seqs[i] for i in idx])
            for l in range(self.cfg.n_layers):
                add = [(j, vec) for j in range(len(idx))] if (vec is not None and l == layer) else ()
                r, _ = self._block(l, r, add_last=add)
            top = torch.topk(self._final_last(r), k, dim=-1).indices.cpu()
            for j, i in enumerate(idx):
                out[i] = top[j]
        return torch.stack(out)


def _by_length(seqs: Sequence[Sequence[int]], batch: int):
    """Index groups of equal-length sequences, at most ``batch`` per group."""
    groups: Dict[int, List[int]] = {}
    for i, s in enumerate(seqs):
        groups.setdefault(len(s), []).append(i)
    for idx in groups.values():
        for a in range(0, len(idx), batch):
            yield idx[a:a + batch]

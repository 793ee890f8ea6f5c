#!/usr/bin/env python3
"""Which rounding drives the engine's CIE error at full depth?

Runs the layer-streamed fp64 oracle (oracle/streamed_pythia.py) on cuda:0 with
selected intermediates rounded to a narrower type (fp32 / bf16 / fp16), the
way a GEMM path rounds them, and reports for each variant the CIE error
against the plain fp64 run (fraction of max |CIE|), the clean logits' error
and — for the bf16 / 6.9B case — whether the top-10 heads of layers <= 10
(scratch2.py:232-238) stay the same.  Test infrastructure only (a probe,
never the product).

  python tools/precision_probe.py --model pythia-12b --kshot 10 --prompts 1 --layers 0,18,35 \
      --variants fp64,fp32_all,resid32,ln32,attn32,gemm32
  python tools/precision_probe.py --model pythia-6.9b --kshot 5 --prompts 4 --layers 0-10 \
      --variants fp64,engine_bf16,all_bf16,w_bf16,act_bf16,all_f16
"""
import argparse
import json
import math
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import tvr_amd  # noqa: E402
from oracle.hooked_pythia import OracleConfig  # noqa: E402
from oracle.streamed_pythia import StreamedPythiaOracle  # noqa: E402


def r16(x, dtype):
    """Round to a 16-bit type; fp16 with a power-of-two scale into its range (as the engine's planes)."""
    if dtype == torch.bfloat16:
        return x.to(torch.bfloat16).to(x.dtype)
    m = x.abs().max().item()
    s = 2.0 ** (14 - math.ceil(math.log2(m))) if m > 0 else 1.0
    return (x * s).to(torch.float16).to(x.dtype) / s


class Rounded(StreamedPythiaOracle):
    """fp64 streamed oracle with rounding points.  ``rules``: name -> callable(x)."""

    def __init__(self, cfg, get_raw, rules):
        self.rules = rules
        super().__init__(cfg, get_raw)
        self._wcache = {}

    def R(self, name, x):
        f = self.rules.get(name)
        return f(x) if f else x

    def block(self, l):
        b = super().block(l)
        if self._wcache.get("l") != l:
            self._wcache = {"l": l, "w": {k: self.R("w_" + k, v) for k, v in b.items()}}
        return self._wcache["w"]

    def _ln_pre(self, x):
        x = self.R("ln_in", x)
        y = super()._ln_pre(x)
        return self.R("ln_out", y)

    def _block(self, l, resid, replace=(), add_last=(), want_result_last=False):
        w = self.block(l)
        x = self._ln_pre(resid)
        xq = self.R("a_qk", x)
        xv = self.R("a_v", x)
        q = self._rotate(self.R("gemm_out", torch.einsum("bpd,hde->bphe", xq, w["W_Q"]) + w["b_Q"]))
        k = self._rotate(self.R("gemm_out", torch.einsum("bpd,hde->bphe", xq, w["W_K"]) + w["b_K"]))
        v = self.R("gemm_out", torch.einsum("bpd,hde->bphe", xv, w["W_V"]) + w["b_V"])
        T = x.shape[1]
        scores = self.R("attn", torch.einsum("bqhe,bkhe->bhqk", q, k) / math.sqrt(self.cfg.d_head))
        mask = torch.triu(torch.ones(T, T, dtype=torch.bool, device=x.device), diagonal=1)
        pat = self.R("attn", torch.softmax(scores.masked_fill(mask, float("-inf")), dim=-1))
        z = self.R("attn", torch.einsum("bkhe,bhqk->bqhe", v, pat))
        H, dh, d = self.cfg.n_heads, self.cfg.d_head, self.cfg.d_model
        zo = self.R("a_z", z)
        attn = self.R("gemm_out", zo.reshape(z.shape[0], T, H * dh) @ w["W_O"].reshape(H * dh, d))
        if replace:
            rows = sorted({r for r, _, _ in replace})
            ri = torch.tensor(rows, device=x.device)
            result = torch.einsum("bqhe,hed->bqhd", zo[ri], w["W_O"])
            at = {r: i for i, r in enumerate(rows)}
            for r, h, vec in replace:
                result[at[r], :, h, :] = vec.to(result)
            attn[ri] = result.sum(-2)
        for r, vec in add_last:
            attn[r, -1] = attn[r, -1] + vec.to(attn)
        h = self.R("gemm_out", xv @ w["W_in"] + w["b_in"])
        g = self.R("a_gelu", torch.nn.functional.gelu(h))
        mlp = self.R("gemm_out", g @ w["W_out"])
        res_last = torch.einsum("bhe,hed->bhd", z[:, -1], w["W_O"]) if want_result_last else None
        return self.R("resid", resid + (attn + w["b_O"]) + (mlp + w["b_out"])), res_last

    def _final_last(self, resid):
        x = self.R("a_u", self._ln_pre(resid[:, -1]))
        return x @ self.R("w_U", self.W_U) + self.b_U


F32 = lambda x: x.float().double()  # noqa: E731
BF = lambda x: r16(x, torch.bfloat16)  # noqa: E731
FH = lambda x: r16(x, torch.float16)  # noqa: E731
WEIGHTS = ["w_W_Q", "w_W_K", "w_W_V", "w_W_O", "w_W_in", "w_W_out", "w_U"]
ACTS = ["a_qk", "a_v", "a_z", "a_gelu", "a_u"]


def variants():
    v = {"fp64": {},
         "fp32_all": {k: F32 for k in ["ln_in", "ln_out", "gemm_out", "attn", "resid", "a_gelu"] + WEIGHTS},
         "resid32": {"resid": F32}, "ln32": {"ln_in": F32, "ln_out": F32}, "attn32": {"attn": F32},
         "gemm32": {"gemm_out": F32}, "gelu32": {"a_gelu": F32}, "w32": {k: F32 for k in WEIGHTS}}
    allbf = {k: BF for k in WEIGHTS + ACTS}
    v["all_bf16"] = allbf
    eng = dict(allbf, a_qk=FH, w_W_Q=FH, w_W_K=FH)
    v["engine_bf16"] = eng
    v["w_bf16"] = {k: BF for k in WEIGHTS}
    v["act_bf16"] = {k: BF for k in ACTS}
    v["all_f16"] = {k: FH for k in WEIGHTS + ACTS}
    for k in WEIGHTS + ACTS:  # the engine's bf16 mode with ONE operand group kept exact
        v["engine_bf16_but_" + k] = {kk: vv for kk, vv in eng.items() if kk != k}
    return v


def parse_layers(s):
    out = []
    for part in s.split(","):
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="pythia-12b")
    ap.add_argument("--std", type=float, default=0.05)
    ap.add_argument("--kshot", type=int, default=10)
    ap.add_argument("--prompts", type=int, default=1)
    ap.add_argument("--layers", default="0")
    ap.add_argument("--heads", default="all")
    ap.add_argument("--variants", default="fp64,fp32_all")
    ap.add_argument("--n-layers", type=int, default=0, help="truncate the model (0: full depth)")
    ap.add_argument("--fv-layer", type=int, default=10)
    ap.add_argument("--device", default="cuda")
    args = ap.parse_args()
    cfg = tvr_amd.get_config(args.model)
    if args.n_layers:
        cfg = cfg.with_(n_layers=args.n_layers)
    shapes = tvr_amd.weights.hf_param_shapes(cfg)
    ocfg = OracleConfig(cfg.n_layers, cfg.d_model, cfg.n_heads, cfg.d_mlp, cfg.d_vocab, cfg.rotary_dim, cfg.n_ctx,
                        cfg.ln_eps, cfg.rotary_base)
    get = lambda n: tvr_amd.weights.synth_param(cfg, n, shapes[n], 0, args.device, args.std)  # noqa: E731
    tok = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)

    class B:
        pass
    b = B()
    b.cfg, b.tokenizer, b.to_single_token = cfg, tok, lambda s: tok.encode(s)[0]
    prompts, _ = tvr_amd.prompts.synthetic_cie_prompts(b, args.prompts, args.kshot, seed=1234)
    layers = parse_layers(args.layers)
    heads = None if args.heads == "all" else parse_layers(args.heads)
    base = Rounded(ocfg, get, {})
    clean = base.last_logits(prompts)
    answers = [int(r.argmax()) for r in clean]
    # means: the extraction of 16 prompts on the fp64 model (fp32-rounded, as both sides patch with)
    import random
    random.seed(2)
    ex = tvr_amd.prompts.sample_icl_prompts(b, list(tvr_amd.tasks.letter_to_caps), tvr_amd.tasks.ARROW, ",", 16, 6)
    mean = base.mean_activation(ex).float().double()
    ref = base.cie(mean, prompts, answers, layers=layers, heads=heads)
    cmax = ref.abs().max().item()
    fvl = [l for l in layers if l <= args.fv_layer]
    top_ref = None
    if len(fvl) == args.fv_layer + 1:
        top_ref = sorted(torch.topk(ref[:args.fv_layer + 1].flatten(), 10).indices.tolist())
    print(json.dumps({"model": args.model, "layers": cfg.n_layers, "std": args.std, "T": len(prompts[0]),
                      "max_cie": cmax, "p_max": torch.softmax(clean, -1).max().item()}), flush=True)
    V = variants()
    for name in args.variants.split(","):
        t0 = time.time()
        o = Rounded(ocfg, get, V[name]) if name != "fp64" else base
        lg = o.last_logits(prompts)
        c = o.cie(mean, prompts, answers, layers=layers, heads=heads)
        err = (c - ref).abs()
        row = {"variant": name, "cie_err_frac": err.max().item() / cmax,
               "cie_err_frac_by_layer": {l: round(err[l].max().item() / cmax, 7) for l in layers[:3] + layers[-1:]},
               "logits_rel": ((lg - clean).abs().max() / clean.abs().max()).item(), "s": round(time.time() - t0, 1)}
        if top_ref is not None:
            top = sorted(torch.topk(c[:args.fv_layer + 1].flatten(), 10).indices.tolist())
            row["top10_same"] = top == top_ref
            row["top10_diff"] = sorted(set(top) ^ set(top_ref))
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

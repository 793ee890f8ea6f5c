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
from oracle.rounded_pythia import Rounded, variants  # noqa: E402


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

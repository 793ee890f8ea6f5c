#!/usr/bin/env python3
"""Linearised entry layer (lin_entry.hpp): C3 sweep time with TVR_LIN_ENTRY
on / off in one process, the profiled HBM-kind breakdown, and the CIE
difference between the two paths; optionally a truncated-depth model of
another width (--model pythia-12b --layers 3).
  python tools/lin_probe.py [--model pythia-2.8b] [--layers 0] [--prompts 12] [--reps 2]"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import tvr_amd  # noqa: E402
from tvr_amd.experiments import causal_indirect_effect_sums  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="pythia-2.8b")
ap.add_argument("--layers", type=int, default=0)
ap.add_argument("--prompts", type=int, default=12)
ap.add_argument("--kshot", type=int, default=4)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--std", type=float, default=0.02)
a = ap.parse_args()
cfg = tvr_amd.get_config(a.model)
if a.layers:
    cfg = cfg.with_(n_layers=a.layers)
sd = None
if a.layers or a.std != 0.02:
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0, std=a.std)
    model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda",
                                             tokenizer=tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab))
else:
    model = tvr_amd.Model.from_pretrained(a.model, device="cuda", seed=0)
g = torch.Generator(device="cuda").manual_seed(4321)
mean = torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, device="cuda", generator=g) * 0.5
prompts, answers = tvr_amd.prompts.synthetic_cie_prompts(model, a.prompts, a.kshot, seed=1234)
res = {"model": a.model, "layers": cfg.n_layers, "prompts": a.prompts, "T": len(prompts[0])}
cies = {}
for rep in range(a.reps):
    for lin in ("1", "0"):
        os.environ["TVR_LIN_ENTRY"] = lin
        causal_indirect_effect_sums(mean, prompts, answers, model)
        torch.cuda.synchronize()
        t = time.perf_counter()
        cie = causal_indirect_effect_sums(mean, prompts, answers, model)
        torch.cuda.synchronize()
        res.setdefault(f"ms_lin{lin}", []).append(round((time.perf_counter() - t) * 1e3, 2))
        cies[lin] = cie.double().cpu()
        print(f"rep {rep} lin {lin}: {res[f'ms_lin{lin}'][-1]} ms", file=sys.stderr, flush=True)
for lin in ("1", "0"):
    os.environ["TVR_LIN_ENTRY"] = lin
    model.profile(True)
    causal_indirect_effect_sums(mean, prompts, answers, model)
    h = model.profile_hbm_stats()
    gs = model.profile_stats()
    model.profile(False)
    res[f"hbm_lin{lin}"] = {k: {"launches": v["launches"], "ms": round(v["ms"], 3)} for k, v in h.items()}
    res[f"gemm_ms_lin{lin}"] = round(gs["all"]["ms"], 3)
d = (cies["1"] - cies["0"]).abs().max().item()
res["max_abs_cie_diff"] = d
res["max_abs_cie"] = cies["0"].abs().max().item()
model._check_range("lin probe")
print(json.dumps(res))

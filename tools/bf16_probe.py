#!/usr/bin/env python3
"""Where the engine's bf16 mode departs from its fp64 emulation (VERDICT r4
item 1b): the clean forward of Pythia-6.9B (seeded std-0.05 weights) layer by
layer — hook_resid_pre of the engine (bf16 GEMM mode) against the fp64
streamed oracle with the engine's operand roundings (oracle/rounded_pythia.py
``engine_bf16``) and against plain fp64.  Prints, per layer, the max-abs and
RMS distances engine-emulation and emulation-fp64 (relative to the fp64
residual's RMS) — a value-level departure shows where it starts.

  python tools/bf16_probe.py [--layers 32] [--prompts 12]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import torch  # noqa: E402

import tvr_amd  # noqa: E402
from conftest import oracle_config  # noqa: E402
from oracle.rounded_pythia import Rounded, variants  # noqa: E402
from oracle.streamed_pythia import StreamedPythiaOracle  # noqa: E402


class _B:
    def __init__(self, cfg):
        self.cfg = cfg
        self.tokenizer = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
        self.to_single_token = lambda s: self.tokenizer.encode(s)[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="pythia-6.9b")
    ap.add_argument("--layers", type=int, default=0)
    ap.add_argument("--prompts", type=int, default=12)
    ap.add_argument("--variant", default="engine_bf16")
    ap.add_argument("--gemm", default="bf16")
    a = ap.parse_args()
    cfg = tvr_amd.get_config(a.model)
    if a.layers:
        cfg = cfg.with_(n_layers=a.layers)
    shapes = tvr_amd.weights.hf_param_shapes(cfg)
    get = lambda n: tvr_amd.weights.synth_param(cfg, n, shapes[n], 0, "cuda", 0.05)  # noqa: E731
    prompts, _ = tvr_amd.prompts.synthetic_cie_prompts(_B(cfg), a.prompts, 5, seed=1234)
    sd = {n: get(n) for n in shapes}
    model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda", gemm=a.gemm)
    del sd
    tr = model.trace(len(prompts), sum(len(p) for p in prompts))
    out = model.forward_clean(prompts, topk=1, return_logits=True, trace=tr)
    T = len(prompts[0])
    eng = [tr.resid_pre(l).double().view(len(prompts), T, -1) for l in range(cfg.n_layers + 1)]
    eng_logits = out["logits"].double()
    res = {}
    for tag, orc in (("fp64", StreamedPythiaOracle(oracle_config(cfg), get)),
                     ("emu", Rounded(oracle_config(cfg), get, variants()[a.variant]))):
        r = orc._embed(prompts)
        rs = [r]
        for l in range(cfg.n_layers):
            r, _ = orc._block(l, r)
            rs.append(r)
        res[tag] = (rs, orc._final_last(r))
        del orc
        torch.cuda.empty_cache()
    f64, emu = res["fp64"][0], res["emu"][0]
    for l in range(cfg.n_layers + 1):
        scale = f64[l].pow(2).mean().sqrt().item()
        d_ee = (eng[l] - emu[l]).cpu()
        d_ef = (emu[l] - f64[l]).cpu()
        d_gf = (eng[l] - f64[l]).cpu()
        print(json.dumps({"layer": l, "rms_scale": round(scale, 4),
                          "eng_emu_max": float(d_ee.abs().max() / scale), "eng_emu_rms": float(d_ee.pow(2).mean().sqrt() / scale),
                          "emu_f64_max": float(d_ef.abs().max() / scale), "emu_f64_rms": float(d_ef.pow(2).mean().sqrt() / scale),
                          "eng_f64_rms": float(d_gf.pow(2).mean().sqrt() / scale)}), flush=True)
    lf, le = res["fp64"][1].cpu(), res["emu"][1].cpu()
    lg = eng_logits.cpu()
    s = lf.abs().max().item()
    print(json.dumps({"logits": True, "eng_emu_max": float((lg - le).abs().max() / s),
                      "emu_f64_max": float((le - lf).abs().max() / s), "eng_f64_max": float((lg - lf).abs().max() / s)}))


if __name__ == "__main__":
    main()

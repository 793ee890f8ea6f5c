#!/usr/bin/env python3
"""Split one C3 bench step (CIE sweep, 12 prompts x 1024 sites, Pythia-2.8B
shape) into its clean forward and its patch sweep, timed on the GPU.

  python tools/step_anatomy.py [--gemm x2f16] [--reps 3]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import tvr_amd  # noqa: E402
from tvr_amd import _lib  # noqa: E402
from tvr_amd.model import make_sites  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gemm", default="x2f16")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = tvr_amd.Model.from_pretrained("pythia-2.8b", device=dev, seed=0, gemm=args.gemm)
    cfg = model.cfg
    L, H = cfg.n_layers, cfg.n_heads
    prompts, answers = tvr_amd.prompts.synthetic_cie_prompts(model, 12, 4, seed=1234)
    g = torch.Generator(device=dev).manual_seed(4321)
    vectors = (torch.randn(L * H, cfg.d_model, device=dev, generator=g) * 0.5).contiguous()
    seqs = [list(map(int, p)) for p in prompts]
    n = len(seqs)
    trace = model.trace(n, sum(len(s) for s in seqs))
    per = L * H
    sites = make_sites(n * per)
    sites["seq"] = np.repeat(np.arange(n, dtype=np.int32), per)
    sites["kind"] = _lib.SITE_REPLACE_HEAD_ALLPOS
    sites["layer"] = np.tile(np.repeat(np.arange(L, dtype=np.int32), H), n)
    sites["head"] = np.tile(np.tile(np.arange(H, dtype=np.int32), L), n)
    sites["vec"] = sites["layer"] * H + sites["head"]
    sites["target"] = np.repeat(np.asarray(answers, dtype=np.int32), per)

    def t(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.reps * 1e3

    clean = lambda: model.forward_clean(seqs, targets=answers, trace=trace)  # noqa: E731
    sweep = lambda: model.patch_sweep(trace, sites, vectors)  # noqa: E731
    clean()
    sweep()
    out = {"workload": "C3 step: 12 prompts (T=15) x 1024 REPLACE_HEAD sites", "gemm": args.gemm,
           "clean_forward_ms": round(t(clean), 3), "patch_sweep_ms": round(t(sweep), 3)}
    model.profile(True)
    clean()
    torch.cuda.synchronize()
    st = model.profile_stats()["all"]
    hb = model.profile_hbm_stats()
    model.profile(False)
    out["clean_forward_gemm_ms"] = round(st["ms"], 3)
    out["clean_forward_gemm_launches"] = st["launches"]
    out["clean_forward_hbm_ms"] = {k: round(v["ms"], 3) for k, v in hb.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

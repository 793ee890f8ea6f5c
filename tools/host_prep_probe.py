#!/usr/bin/env python3
"""Host-side cost of one C3 sweep (bench.py's workload): the wall time of the
tvr_patch_sweep call (table building + uploads + enqueueing the launches,
no synchronisation) against the whole step.  Diagnostic only.
  python tools/host_prep_probe.py"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tvr_amd  # noqa: E402
from tvr_amd import _lib  # noqa: E402
from tvr_amd.experiments import causal_indirect_effect_sums  # noqa: E402

model = tvr_amd.Model.from_pretrained("pythia-2.8b", device="cuda", seed=0)
cfg = model.cfg
prompts, answers = tvr_amd.prompts.synthetic_cie_prompts(model, 12, 4, seed=1234)
g = torch.Generator(device="cuda").manual_seed(4321)
mean = torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, device="cuda", generator=g) * 0.5
orig = model._lib.tvr_patch_sweep
calls = []


def timed_sweep(*a):
    t = time.perf_counter()
    rc = orig(*a)
    calls.append(time.perf_counter() - t)
    return rc


class LibProxy:
    def __getattr__(self, n):
        return timed_sweep if n == "tvr_patch_sweep" else getattr(model.__dict__["_lib_real"], n)


model.__dict__["_lib_real"] = model._lib
model._lib = LibProxy()
for _ in range(2):
    causal_indirect_effect_sums(mean, prompts, answers, model)
torch.cuda.synchronize()
calls.clear()
steps = []
for _ in range(3):
    t = time.perf_counter()
    causal_indirect_effect_sums(mean, prompts, answers, model)
    torch.cuda.synchronize()
    steps.append(time.perf_counter() - t)
print(json.dumps({"patch_sweep_host_ms": [round(c * 1e3, 2) for c in calls],
                  "step_ms": [round(s * 1e3, 2) for s in steps]}))

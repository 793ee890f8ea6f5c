#!/usr/bin/env python3
"""C2 layer sweep anatomy: the accuracy sweep (52 prompts x 32 layers, T0 = 3,
ADD_ATTN_OUT_LASTPOS) timed, then profiled (GEMM variants + HBM kinds).
  python tools/c2_probe.py [--reps 3]"""
import argparse
import json
import random
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import tvr_amd  # noqa: E402
from tvr_amd import experiments as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--weights", default="fp16", choices=["fp16", "fp32"],
                help="fp16-valued weights (the bench's default: exact-fp16 GEMMs) or fp32-valued")
a = ap.parse_args()
model = tvr_amd.Model.from_pretrained("pythia-2.8b", device="cuda", fp16_weights=a.weights == "fp16")
task, arrow = tvr_amd.tasks.letter_to_caps, tvr_amd.tasks.ARROW
random.seed(0)
mean = E.generate_mean_activation(task, arrow, model=model, num_contexts=64, len_contexts=6)
lv = E.gather_head_activations_to_layers(mean)
res = {}
E.apply_layered_vectors_to_zero_shot(lv, task, arrow, model)
ts = []
for _ in range(a.reps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    E.apply_layered_vectors_to_zero_shot(lv, task, arrow, model)
    torch.cuda.synchronize()
    ts.append(round((time.perf_counter() - t) * 1e3, 3))
res["accuracy_sweep_ms"] = ts
model.profile(True)
E.apply_layered_vectors_to_zero_shot(lv, task, arrow, model)
st = model.profile_stats()
hb = model.profile_hbm_stats()
model.profile(False)
res["gemm"] = {k: {"launches": v["launches"], "ms": round(v["ms"], 3),
                   "tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 1) if v["ms"] else None}
               for k, v in st.items()}
res["hbm"] = {k: {"launches": v["launches"], "ms": round(v["ms"], 3)} for k, v in hb.items() if v["launches"]}
print(json.dumps(res))

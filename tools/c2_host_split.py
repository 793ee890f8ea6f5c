#!/usr/bin/env python3
"""Where the C2 accuracy sweep's wall time goes on the host side.  Diagnostic.

Per call of apply_layered_vectors_to_zero_shot (52 prompts x 32 layers):
  wall        perf_counter around the call (synchronised on both sides)
  gpu_span    HIP events on the engine's stream: one recorded just before the
              call (the device is idle, so it marks the call's start) and one
              recorded right after patch_sweep returns (after every kernel)
  head_ms     host time from the call's start to patch_sweep's entry (Python
              site preparation, the deferred clean forward's registration)
  op_ms       host time inside patch_sweep (the engine's preparation and the
              enqueue of its launches; the GPU runs meanwhile)
  tail_ms     wall - (time at which patch_sweep returned + the wait for the GPU)
              ~ the read-back and top-1 decode after the last kernel
  python tools/c2_host_split.py [--reps 5]"""
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
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
model = tvr_amd.Model.from_pretrained("pythia-2.8b", device="cuda")
task, arrow = tvr_amd.tasks.letter_to_caps, tvr_amd.tasks.ARROW
random.seed(0)
mean = E.generate_mean_activation(task, arrow, model=model, num_contexts=64, len_contexts=6)
lv = E.gather_head_activations_to_layers(mean)
E.apply_layered_vectors_to_zero_shot(lv, task, arrow, model)

marks = {}
orig = model.patch_sweep


def timed_patch_sweep(*args, **kw):
    marks["op_in"] = time.perf_counter()
    out = orig(*args, **kw)
    marks["op_out"] = time.perf_counter()
    marks["ev_after"] = torch.cuda.Event(enable_timing=True)
    marks["ev_after"].record()
    return out


model.patch_sweep = timed_patch_sweep
rows = []
for _ in range(a.reps):
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    E.apply_layered_vectors_to_zero_shot(lv, task, arrow, model)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    gpu = e0.elapsed_time(marks["ev_after"])
    rows.append({"wall_ms": round((t1 - t0) * 1e3, 3), "gpu_span_ms": round(gpu, 3),
                 "head_ms": round((marks["op_in"] - t0) * 1e3, 3),
                 "op_ms": round((marks["op_out"] - marks["op_in"]) * 1e3, 3),
                 "after_gpu_ms": round((t1 - t0) * 1e3 - gpu, 3)})
for r in rows:
    print(json.dumps(r))

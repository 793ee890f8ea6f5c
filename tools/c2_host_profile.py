#!/usr/bin/env python3
"""Host-side cost of the C2 accuracy sweep: wall time vs. GPU busy time, and a
cProfile of the Python + engine host work per sweep (what the GPU waits for
between sweeps).
  python tools/c2_host_profile.py [--reps 20]"""
import argparse
import cProfile
import io
import pstats
import random
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import tvr_amd  # noqa: E402
from tvr_amd import experiments as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
model = tvr_amd.Model.from_pretrained("pythia-2.8b", device="cuda")
task, arrow = tvr_amd.tasks.letter_to_caps, tvr_amd.tasks.ARROW
random.seed(0)
mean = E.generate_mean_activation(task, arrow, model=model, num_contexts=64, len_contexts=6)
lv = E.gather_head_activations_to_layers(mean)
for fn in (E.apply_layered_vectors_to_zero_shot, E.apply_layered_vectors_to_zero_shot_by_probability):
    fn(lv, task, arrow, model)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.reps):
        fn(lv, task, arrow, model)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / a.reps * 1e3
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.reps):
        fn(lv, task, arrow, model)
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(f"== {fn.__name__}: {wall:.3f} ms per sweep (wall)")
    print(s.getvalue())

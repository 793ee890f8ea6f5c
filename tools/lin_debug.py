#!/usr/bin/env python3
"""Localise lin-entry vs full-GEMM differences (debug aid): the headline-width
test's CIE computed with TVR_LIN_ENTRY on / off / off again, per layer."""
import os
import random
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import tvr_amd  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "pythia-2.8b"
std = float(sys.argv[2]) if len(sys.argv) > 2 else 0.1
cfg = tvr_amd.get_config(name).with_(n_layers=3)
sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0, std=std)
tok = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda", tokenizer=tok, gemm="x2f16")
prompts, _ = tvr_amd.prompts.synthetic_cie_prompts(model, 2, 4, seed=1234)
clean = model.forward_clean(prompts, topk=1)
answers = [[int(t)] for t in clean["topk"][:, 0].tolist()]
random.seed(3)
mean = tvr_amd.generate_mean_activation(list(tvr_amd.tasks.letter_to_caps), tvr_amd.tasks.ARROW, ",", model=model,
                                        num_contexts=8, len_contexts=4)
print("mean max", mean.abs().max().item())
res = {}
for tag, lin in (("on", "1"), ("off", "0"), ("off2", "0"), ("on2", "1")):
    os.environ["TVR_LIN_ENTRY"] = lin
    res[tag] = tvr_amd.calculate_average_causal_indirect_effect(mean, prompts, answers, model=model).cpu().double()
    tr = model._trace_cache
    print(tag, "clean probs via sweep:", [float(x) for x in model.forward_clean(prompts, targets=[a[0] for a in answers])["prob"]])
for a, b in (("on", "off"), ("off", "off2"), ("on", "on2")):
    d = (res[a] - res[b]).abs()
    print(a, "vs", b, "max", d.max().item(), "per layer", [round(x, 6) for x in d.amax(1).tolist()])
print("cie max", res["off"].abs().max().item())

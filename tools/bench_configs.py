#!/usr/bin/env python3
"""Measure the SURVEY.md §8(d) configurations on one GPU through the façade
(the reference's own experiment functions), seeded synthetic weights.

  python tools/bench_configs.py --configs C2,C3,C4 [--gemm x2f16] [--c4-gemm bf16] [--c4-tasks 20] \
      > profiles/configs_rNN.json

C2  Pythia-2.8B: extraction N=2048, 6-shot (T=28) on letter_to_caps; per-layer
    accuracy + Δprob sweeps over the 52 zero-shot prompts (1664 sites each).
C3  Pythia-2.8B: CIE over 12 shuffled 4-shot letter_to_caps prompts (12,288 sites).
C4  Pythia-6.9B: per synthetic 50-pair task: extraction N=512 5-shot (T=24), CIE
    over 12 prompts, FV = top-10 heads of layers <= 10, FV added at every layer
    for 50 zero-shot prompts (top-5 accuracy).  Timed per task.
C5 is bench.py --model pythia-12b --kshot 10.
"""
import argparse
import json
import random
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import tvr_amd  # noqa: E402
from tvr_amd import experiments as E  # noqa: E402


def timed(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = fn()
    torch.cuda.synchronize()
    return out, time.perf_counter() - t


def c2_c3(which, gemm):
    res = {}
    model = tvr_amd.Model.from_pretrained("pythia-2.8b", device="cuda", gemm=gemm)
    task, arrow = tvr_amd.tasks.letter_to_caps, tvr_amd.tasks.ARROW
    random.seed(0)
    E.generate_mean_activation(task, arrow, model=model, num_contexts=64, len_contexts=6)  # warm
    random.seed(1)
    mean, t_ex = timed(lambda: E.generate_mean_activation(task, arrow, model=model, num_contexts=2048, len_contexts=6))
    if "C2" in which:
        lv = E.gather_head_activations_to_layers(mean)
        acc, t_acc = timed(lambda: E.apply_layered_vectors_to_zero_shot(lv, task, arrow, model))
        dp, t_dp = timed(lambda: E.apply_layered_vectors_to_zero_shot_by_probability(lv, task, arrow, model))
        n_sites = len(task) * model.cfg.n_layers
        res["C2"] = {"extraction_prompts_per_s": round(2048 / t_ex, 1), "extraction_s": round(t_ex, 3),
                     "layer_sweep_accuracy_sites_per_s": round(n_sites / t_acc, 1), "accuracy_s": round(t_acc, 3),
                     "layer_sweep_prob_sites_per_s": round(n_sites / t_dp, 1), "prob_s": round(t_dp, 3),
                     "accuracy_by_layer": acc, "dprob_by_layer": [round(x, 8) for x in dp.tolist()]}
    if "C3" in which:
        random.seed(2)
        prompts, answers = E.generate_shuffled_prompts(task, model, 12, 4, arrow)
        E.calculate_average_causal_indirect_effect(mean, prompts[:1], answers[:1], model)  # warm
        cie, t_cie = timed(lambda: E.calculate_average_causal_indirect_effect(mean, prompts, answers, model))
        top = torch.topk(cie.flatten(), 5)
        res["C3"] = {"cie_sites": 12 * 1024, "cie_s": round(t_cie, 3),
                     "patched_prompts_per_s": round(12 * 1024 / t_cie, 1),
                     "top5_heads": [[int(i) // model.cfg.n_heads, int(i) % model.cfg.n_heads] for i in top.indices],
                     "top5_cie": [float(v) for v in top.values]}
    return res


def c4(n_tasks, gemm):
    """C4 through the multi-GPU entry points (distributed.py), which are the
    plain functions when run as one process: extraction prompt-sharded (one
    all-reduce of [L, d]), CIE head-sharded (one all-reduce of [L, H]), the FV
    layer sweep with (prompt, layer) sites round-robin (one all_gather).
    torchrun: every rank builds the same seeded prompts and gets the same
    results; rank 0 reports."""
    from tvr_amd import distributed as D
    rank, world = D.world()
    dev = torch.device("cuda", torch.cuda.current_device())
    model = tvr_amd.Model.from_pretrained("pythia-6.9b", device=dev, gemm=gemm)
    arrow = tvr_amd.tasks.ARROW
    per_task = []
    for ti in range(n_tasks):
        task = tvr_amd.tasks.synthetic_task(50, model.cfg.d_vocab, seed=100 + ti)
        random.seed(ti)
        t0 = time.perf_counter()
        ex_prompts = tvr_amd.prompts.sample_icl_prompts(model, task, arrow, ",", 512, 5)
        mean, t_ex = timed(lambda: D.mean_activation_sharded(ex_prompts, model))
        prompts, answers = E.generate_shuffled_prompts(task, model, 12, 5, arrow)
        cie, t_cie = timed(lambda: D.cie_sharded(mean, prompts, answers, model))
        fv = E.assemble_task_vector(mean, cie, 10, 10)
        acc, t_fv = timed(lambda: D.check_accuracy_of_added_task_vector_by_layer_sharded(fv, task, 5, model))
        per_task.append({"task_seed": 100 + ti, "extraction_s": round(t_ex, 3), "cie_s": round(t_cie, 3),
                         "cie_patched_prompts_per_s": round(12 * 1024 / t_cie, 1), "fv_layer_sweep_s": round(t_fv, 3),
                         "total_s": round(time.perf_counter() - t0, 3), "fv_top5_acc_by_layer": acc})
    cie_rate = sum(12 * 1024 / t["cie_s"] for t in per_task) / len(per_task)
    return {"C4": {"gemm": gemm, "world": world, "tasks": per_task, "mean_cie_patched_prompts_per_s": round(cie_rate, 1),
                   "mean_task_s": round(sum(t["total_s"] for t in per_task) / len(per_task), 3),
                   "sharding": "extraction prompt-sharded + all-reduce; CIE heads = rank mod world + all-reduce; FV "
                               "layer sweep sites round-robin + all_gather"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C3,C4")
    ap.add_argument("--gemm", default="x2f16", help="GEMM path of C2/C3 (fp32-accurate by default)")
    ap.add_argument("--c4-gemm", default="bf16", help="GEMM path of C4 (BASELINE.json: bf16)")
    ap.add_argument("--c4-tasks", type=int, default=20)
    ap.add_argument("--dist-backend", default="nccl", help="torchrun runs: nccl (RCCL) or gloo")
    a = ap.parse_args()
    import os
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world > 1:  # torchrun: one rank per GPU, RCCL (C4 only)
        local = int(os.environ.get("LOCAL_RANK", 0))
        torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group(a.dist_backend)
    which = set(a.configs.split(","))
    out = {"gpu": torch.cuda.get_device_name(0), "weights": "seeded synthetic (no checkpoints offline)",
           "gemm": a.gemm}
    if which & {"C2", "C3"}:
        out.update(c2_c3(which, a.gemm))
        torch.cuda.empty_cache()
    if "C4" in which:
        out.update(c4(a.c4_tasks, a.c4_gemm))
    if world == 1 or dist.get_rank() == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

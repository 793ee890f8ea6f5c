#!/usr/bin/env python3
"""bench.py — patched-forward prompts/sec on the Pythia-2.8B layer x head
causal-indirect-effect sweep (BASELINE.json metric).

One step = one full CIE sweep of ``--prompts`` label-shuffled 4-shot prompts
(T = 15 tokens) over all 32 x 32 (layer, head) sites: the clean forward of the
prompts plus 12 x 1024 patched forwards, each evaluated to the probability of
the prompt's first answer token (scratch2.py:171-197), i.e. 12,288 units per
GPU per step.  Weights are seeded synthetic Pythia-2.8B (no checkpoints
offline), fp16-valued as the released checkpoints store them (``--weights
fp16``, default; ``fp32`` draws fp32-valued ones as rounds 1-5 did) and
computed on in fp32 like the reference (TransformerLens loads the float16
checkpoint into its default fp32 dtype).  With fp16-valued weights the engine
binds the checkpoint's own GEMM weights (include/tvr.h tvr_model_set_exact16):
their residual plane is zero, so the x2f16 GEMMs run 2 products instead of 3
(``roofline.peak`` is then the 2-product ceiling), and a
``processed_weights_leg`` re-times the sweep on the TL-processed weights
(3 products) for comparison.

GEMMs (95 % of the step) run on the fp32-accurate two-plane fp16 split
(``--gemm x2f16``, default: every fp32 operand split into 2 power-of-two-scaled
fp16 planes, 3 products on v_mfma_f32_16x16x32_f16, fp32 accumulation — the
fp16 form of 3xTF32; GEMM inputs limited to |a| < 4095, checked on the device),
the three-plane bf16 split (``--gemm x3bf16``: 6 products) or
``v_mfma_f32_32x32x2_f32`` (``--gemm f32``).  Both splits measure at or below
the fp32 MFMA GEMM's error against fp64 (tests/test_gpu_engine.py,
profiles/gemm_split_probe_r01.jsonl); ``dtype`` names the emulation.  At N=1
an ``f32_leg`` re-times the same sweep on the fp32 MFMA path and reports the
max CIE difference between the two paths; ``parity`` compares the engine with
the CPU oracle on informative weights (a 4-layer std-0.05 copy at the same
width: extraction, clean logits and every CIE site of one prompt) and
``parity_bench_weights`` on the sites the ``cpu_baseline`` leg computes.

``configs``: C2 (N = 1 only: a one-GPU config), C4 and C5 — at N > 1 sharded
over the ranks as their BASELINE 8-GPU configs say (max-over-ranks times).

Multi-GPU (torchrun, one rank per GPU, RCCL), ``--shard``:
* ``sites`` (default; BASELINE's C3 "one 32 x 32 sweep sharded across the
  GPUs"): the SAME 12 prompts on every rank, each rank owns a balanced block
  of (layer, head) sites (distributed.balanced_site_shard: whole layer pairs
  (l, L-1-l), every pair the same staircase work; at N = 8 on 2.8B, 2 pairs =
  4 whole layers per rank), one SUM all-reduce of the [L, H] CIE sums per
  step — strong scaling, 12,288 units per step in total whatever N is
  (``--emulate-world N`` times rank 0's share of it on one GPU);
  ``heads`` is the round-3 split (head ≡ rank mod N in every layer), kept for
  A/B.  At N > 1 a short ``weak_prompt_partition`` leg follows:
  every rank sweeps its own 12 prompts (seed 1234 + rank) over all sites, the
  weak-scaling figure, reported under its own key and never as ``value``;
* ``prompts``: that weak form as the headline (12,288 units per GPU per step;
  no data-path collective, one all-reduce).
value = units of all ranks / max-rank time.  The timed region runs with no
profiling; the kernel timings of ``roofline`` / ``hbm_kernels`` come from a
separate profiled pass of the same step.

``--gpus N`` without torchrun (no ``WORLD_SIZE`` in the environment): this
process touches no GPU and starts N child ranks of itself (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free MASTER_PORT), each on GPU
LOCAL_RANK, waits for them and exits with the worst exit status; rank 0 prints
the JSON line, whose ``n_gpus`` is the world size the process group saw.
``--dist-backend gloo`` rehearses several ranks on one GPU;
``--launch-check`` runs only the rendezvous and the timing collectives (no
GPU: the CPU test of the launcher).

Extra JSON objects: ``roofline`` (dominant kernel = the GEMM family, achieved
from HIP events on the engine's launch stream), ``cpu_baseline`` (the CPU
oracle running the reference's loop structure on a bounded sample, rank 0 at
N=1 only).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "patched-forward prompts/sec, Pythia-2.8B layer×head CIE sweep, 1–8 GPUs"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 spec (155 measured)
BF16_MFMA_PEAK_TFLOPS = 2516.6  # 1024 FLOP/clk/SIMD x 1024 SIMDs x 2.4 GHz (guide: "~2.5 PF dense")
# 16-bit MFMA products per fp32-equivalent product (fp16 and bf16 MFMA run at one rate)
PRODUCTS = {"x3bf16": 6, "x2f16": 3, "bf16": 1}
PEAKS = {"f32": FP32_MFMA_PEAK_TFLOPS, **{k: BF16_MFMA_PEAK_TFLOPS / v for k, v in PRODUCTS.items()}}
KERNELS = {"f32": "gemm_f32_nt_kernel (v_mfma_f32_32x32x2_f32; all three fused epilogues)",
           "x3bf16": "gemm_x3bf16_nt_kernel (3-plane bf16 split on v_mfma_f32_32x32x16_bf16, 6 products, "
                     "fp32 accumulate; all three fused epilogues)",
           "x2f16": "gemm_pingpong_kernel<ACT_X2F16> (2-plane fp16 split activations written by their producers, "
                    "LDS-DMA staging with counted waits, 4 phases per k-tile, two wave groups one barrier apart, "
                    "3 products on v_mfma_f32_16x16x32_f16, fp32 accumulate; all three fused epilogues)",
           "x2f16-exact16": "gemm_pingpong_kernel<ACT_X2F16, WX> (2-plane fp16 split activations written by their "
                            "producers against ONE exact fp16 weight plane (the checkpoint's own), 2 products on "
                            "v_mfma_f32_16x16x32_f16, fp32 accumulate; wide wave tile (4 x 2 waves of 64 x 128), "
                            "LDS-DMA staging with counted waits, 2 phases per k-tile over 3 LDS buffers (4 when "
                            "sliced), two wave groups one barrier apart; all three fused epilogues)",
           "bf16": "gemm_pingpong_kernel<ACT_BF16> (bf16 weights and activations, LDS-DMA staging with counted "
                   "waits, two wave groups one barrier apart, v_mfma_f32_16x16x32_bf16, fp32 accumulate; all "
                   "three fused epilogues)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="pythia-2.8b")
    ap.add_argument("--prompts", type=int, default=12, help="CIE prompts per GPU per step")
    ap.add_argument("--kshot", type=int, default=4)
    ap.add_argument("--c4-prompts", dest="c4_prompts", action="store_true",
                    help="profiling: the headline sweep on C4's shuffled string prompts (a synthetic 50-pair task, "
                         "--kshot demos, tokenised: T=23 at 5-shot) instead of the single-token ones, so a rocprofv3 "
                         "pass of it is C4's CIE sweep at C4's own prompt length (tools/prof_cmd.sh)")
    ap.add_argument("--extract", type=int, default=2048,
                    help="prompts of the mean extraction (a1, C2's N = 2048, 6-shot, T = 28) that supplies the CIE "
                         "means; timed separately (extraction prompts/s, capture kernel GB/s); 0 = seeded random "
                         "means, so every GEMM launch of the process belongs to a CIE step (the rocprof runs: "
                         "rocprof averages == bench averages)")
    ap.add_argument("--cpu-baseline", dest="cpu_baseline", action="store_true", default=True)
    ap.add_argument("--no-cpu-baseline", dest="cpu_baseline", action="store_false")
    ap.add_argument("--shard", default="sites", choices=("sites", "heads", "prompts"),
                    help="N>1: sites = the same 12 prompts, (layer, head) sites in balanced layer-pair blocks per "
                         "rank (strong scaling: BASELINE's C3, default); heads = the same prompts split by head mod N "
                         "(round-3 form); prompts = 12 prompts per GPU, sites partitioned by prompt (weak scaling)")
    ap.add_argument("--weak-leg", dest="weak_leg", action="store_true", default=True,
                    help="N>1 with a strong split: also time the prompt-partitioned weak form (own key, not value)")
    ap.add_argument("--no-weak-leg", dest="weak_leg", action="store_false")
    ap.add_argument("--profile-steps", type=int, default=2, help="steps of the separate profiled pass")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="N=1 only, planning aid: time rank 0's share of a strong-split run (--shard sites / heads) "
                         "on this many GPUs on this one GPU; value = the units of that share / its time")
    ap.add_argument("--weights", default="fp16", choices=("fp16", "fp32"),
                    help="synthetic weight values: fp16-valued as the released checkpoints (default) or fp32")
    ap.add_argument("--gemm", default="x2f16", choices=("x2f16", "x3bf16", "f32", "bf16"),
                    help="matrix-core path of the GEMMs (x2f16 / x3bf16 / f32 fp32-accurate; bf16 is the "
                         "north star's bf16 configuration, not the fp32 headline)")
    ap.add_argument("--f32-leg", dest="f32_leg", action="store_true", default=True,
                    help="N=1: also time the sweep on the fp32 MFMA GEMM and compare CIE")
    ap.add_argument("--no-f32-leg", dest="f32_leg", action="store_false")
    ap.add_argument("--no-processed-leg", dest="processed_leg", action="store_false", default=True,
                    help="skip the 3-product re-timing on the processed weights (profiling runs)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI) for real runs; gloo to rehearse several ranks on one GPU")
    ap.add_argument("--configs", default="C2,C4,C5",
                    help="N=1: the other BASELINE.json configs timed after the headline, reported under 'configs' "
                         "(C2 = the Pythia-2.8B layer sweeps on the headline model, C4 = the Pythia-6.9B bf16 "
                         "function-vector suite per task, C5 = the Pythia-12B 36x40 10-shot CIE sweep); '' skips them")
    ap.add_argument("--c5-layers", dest="c5_layers", type=int, default=0,
                    help="rehearsals only: C5 on the first N of Pythia-12B's 36 layers (two 12B replicas on one GPU); "
                         "the workload string says so, and 0 (default) is the BASELINE config")
    ap.add_argument("--launch-check", dest="launch_check", action="store_true",
                    help="only the rank launch, rendezvous and max-over-ranks timing (no GPU work; CPU test)")
    return ap.parse_args()


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """``--gpus N`` without torchrun: start N child ranks of this script and
    wait for them.  Called before anything in this process touches the GPU
    (children are fresh processes, never an exec of this one).  A rank that
    fails ends the others (they would block in a collective) by their PIDs."""
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, "-u", str(Path(__file__).resolve())] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = rc or code
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    for p in procs:
        p.wait()
    return rc


def launch_check(rank: int, world: int, backend: str) -> None:
    """The launcher's CPU rehearsal: rendezvous, barrier, max-over-ranks time."""
    dist.init_process_group(backend)
    t0 = time.perf_counter()
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    times = [torch.zeros(1, dtype=torch.float64) for _ in range(dist.get_world_size())]
    dist.all_gather(times, el)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        w = dist.get_world_size()
        # the workloads a real run at this world size times (C2 is a one-GPU config: N = 1 only)
        workloads = {"C3": describe_workload("pythia-2.8b", 32, 32, 12, 4, 15, w, "sites")[0],
                     "C4": c4_workload(w), "C5": c5_workload(w)}
        if w == 1:
            workloads["C2"] = "52 zero-shot prompts (T0=3) x 32 layers"
        print(json.dumps({"launch_check": True, "n_gpus": w, "backend": backend,
                          "rank_elapsed_s": [t.item() for t in times], "max_elapsed_s": el.item(),
                          "workloads": workloads}), flush=True)
    dist.destroy_process_group()


def pmc_summary(family, workload, any_len=False):
    """The committed rocprofv3 PMC summary of this bench command on the same
    GEMM family (profiles/pmc_gemm_<family>.json, written by
    tools/prof_summary.py): HBM bytes per GEMM launch from separate FETCH_SIZE /
    WRITE_SIZE passes (gfx950 x2 FETCH_SIZE correction) and MFMA utilisation
    from SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE.  (None, None) if absent."""
    p = ROOT / "profiles" / f"pmc_gemm_{family}.json"
    if not p.exists():
        return None, None
    d = json.loads(p.read_text())
    same = d.get("workload") == workload
    if any_len and not same:  # C4: the same sweep (model, sites, prompts, shots) at another prompt length
        same = str(d.get("workload", "")).rsplit(", T=", 1)[0] == workload.rsplit(", T=", 1)[0]
    if d.get("family") != family or not same:
        return None, None  # counters of another kernel or workload do not apply
    return d, f"{p.relative_to(ROOT)} ({d.get('source', '?')}; workload {d.get('workload')})"


HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E ~8 TB/s


def hbm_kernels(hbm, hbm_ex, steps, workload=None):
    """Achieved GB/s of the HBM-bound kernels (HIP events around each launch,
    algorithmic bytes per include/tvr.h tvr_hbm_kind): injection, LayerNorm,
    attention and target-probability rows from the timed CIE region; capture
    from the timed extraction.  ``traffic``: memory-side bytes per launch from
    the committed rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this command
    (profiles/pmc_hbm_kernels.json, tools/prof_summary.py) when the workload
    matches."""
    out = {"peak_gbps": HBM_PEAK_GBPS,
           "basis": "algorithmic bytes / summed HIP-event launch time (engine stream), per kernel kind"}
    pm = {}
    p = ROOT / "profiles" / "pmc_hbm_kernels.json"
    if p.exists():
        d = json.loads(p.read_text())
        if workload is not None and d.get("workload") == workload:
            pm = d.get("kernels", {})
            out["traffic_source"] = f"{p.relative_to(ROOT)} ({d.get('source', '?')}; {d.get('note', '')})"

    def row(v, per):
        if not v["launches"]:
            return None
        g = v["gbps"]
        return {"launches" + per: round(v["launches"] / (steps if per else 1), 1),
                "avg_launch_us": round(v["ms"] * 1e3 / v["launches"], 2),
                "bytes_per_launch": round(v["bytes"] / v["launches"]),
                "achieved_gbps": round(g, 1), "frac": round(g / HBM_PEAK_GBPS, 4)}
    for k in ("entry", "lnpre", "attention", "row_stats", "lin_entry"):
        out[k] = row(hbm[k], "_per_step") if k in hbm else None
        if out[k] and k in pm:
            out[k]["traffic"] = pm[k]["fetch_bytes_x2_per_launch"] + pm[k]["write_bytes_per_launch"]
    out["capture"] = row(hbm_ex["capture"], "") if hbm_ex else None
    return out


def log(*a):
    print(*a, file=sys.stderr, flush=True)


SPLITS = {"sites": "sites in balanced layer-pair blocks per rank", "heads": "sites h = rank (mod {n})"}


def describe_workload(model_name: str, n_layers: int, n_heads: int, prompts: int, kshot: int, T: int, world: int,
                      shard: str, emulate: int = 0, n_sites_rank: int = 0):
    """(workload string, scaling label) of the bench line.  The headline at
    any N is BASELINE's C3: ONE sweep of the same prompts over all L x H sites
    (strong scaling; at N > 1 the sites split across the ranks, ``sites`` or
    ``heads``).  ``shard == "prompts"`` at N > 1 is the weak form (prompts per
    GPU)."""
    base = f"{model_name} CIE sweep {n_layers}x{n_heads} sites"
    if emulate:
        return (f"{model_name} CIE sweep, rank 0's share of a {emulate}-GPU split "
                f"({SPLITS.get(shard, shard).format(n=emulate)}: {n_sites_rank} of {n_layers * n_heads} sites), "
                f"{prompts} prompts/step, {kshot}-shot, T={T} (planning emulation on one GPU, not the metric)",
                "strong")
    if world > 1 and shard == "prompts":
        return f"{base}, {prompts} prompts/GPU/step, {kshot}-shot, T={T}", "weak"
    if world > 1:
        return f"{base}, {prompts} prompts/step, {kshot}-shot, T={T}, {SPLITS[shard].format(n=world)}", "strong"
    return f"{base}, {prompts} prompts/step, {kshot}-shot, T={T}", "strong"


def _sync_time(fn, reps):
    """fn() run `reps` times between synchronize calls; seconds per call."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, out


def config_c2(model, mean, peak, reps=3):
    """C2: the per-layer accuracy and Δprob sweeps of a 52-pair
    task over all layers (52 zero-shot [BOS, x, f] prompts x L layers = 1,664
    ADD_ATTN_OUT_LASTPOS sites per sweep, scratch2.py:114-150), with the
    layer-(L-1) vector of the headline's 2048-prompt extraction (late binding,
    App. B1).  Roofline: F_alg = (L-1-l)(2 P_l + 4 T0 d) + 2 d V per site,
    averaged over l (T0 = 3)."""
    import tvr_amd
    from tvr_amd import experiments as E
    cfg = model.cfg
    L, d, V = cfg.n_layers, cfg.d_model, cfg.d_vocab
    P_l = 4 * d * d + 2 * d * cfg.d_mlp
    f_alg = sum((L - 1 - l) * (2 * P_l + 4 * 3 * d) + 2 * d * V for l in range(L)) / L
    task = tvr_amd.tasks.letter_to_caps
    lv = E.gather_head_activations_to_layers(mean)
    out = {"workload": f"{len(task)} zero-shot prompts (T0=3) x {L} layers = {len(task) * L} sites per sweep, "
                       "vector = layer-(L-1) sum of the headline's extraction means",
           "gflop_per_site": round(f_alg / 1e9, 3), "reps": reps}
    for key, fn in (("accuracy", lambda: E.apply_layered_vectors_to_zero_shot(lv, task, tvr_amd.tasks.ARROW, model)),
                    ("dprob", lambda: E.apply_layered_vectors_to_zero_shot_by_probability(lv, task, tvr_amd.tasks.ARROW,
                                                                                          model))):
        fn()  # warm (trace / workspace sizing)
        sec, _ = _sync_time(fn, reps)
        rate = len(task) * L / sec
        out[key] = {"ms_per_sweep": round(sec * 1e3, 3), "sites_per_s": round(rate, 1),
                    "site_tflops": round(rate * f_alg / 1e12, 2), "site_frac": round(rate * f_alg / 1e12 / peak, 4)}
    out["peak_tflops"] = round(peak, 1)
    if model.exact16 and model.gemm == "x2f16":
        # the same work against the 3-product ceiling of rounds 1-4 (838.9 TF), for comparison across rounds
        for key in ("accuracy", "dprob"):
            out[key]["site_frac_vs_3product_ceiling"] = round(out[key]["site_tflops"] / PEAKS["x2f16"], 4)
    return out


def config_c5(args, dev, peak, world=1, rank=0, emulate=0, return_cie=False):
    """C5: Pythia-12B, the full 36 x 40 CIE sweep of 12
    shuffled 10-shot prompts (T = 33): 17,280 patched prompts per step.  At
    N > 1 the SAME sweep is split across the ranks as the headline's C3 is
    (distributed.balanced_site_shard: whole layer pairs per rank, one SUM
    all-reduce of the [L, H] sums; strong scaling, max-over-ranks time);
    ``emulate`` times rank 0's share of that split on one GPU.  Seeded
    synthetic weights and means; one warmup step, ``steps`` timed.  F_alg per
    SURVEY §8d.  ``args.c5_layers`` > 0 (rehearsals): the first that many
    layers only.  ``return_cie``: the step's all-reduced [L, H] CIE sums too
    (tests/test_gpu_distributed.py compares the sharded sweep with one process)."""
    import tvr_amd
    from tvr_amd.distributed import balanced_site_shard
    from tvr_amd.experiments import causal_indirect_effect_sums
    t0 = time.time()
    cfg12 = tvr_amd.get_config("pythia-12b")
    layers = getattr(args, "c5_layers", 0)
    if layers:
        cfg12 = cfg12.with_(n_layers=layers)
    model = tvr_amd.Model.from_pretrained("pythia-12b", cfg=cfg12, device=dev, seed=0, gemm=args.gemm,
                                          fp16_weights=args.weights == "fp16")
    cfg = model.cfg
    x16 = bool(model.exact16)
    g = torch.Generator(device=dev).manual_seed(4321)
    mean = torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, device=dev, generator=g) * 0.5
    prompts, answers = tvr_amd.prompts.synthetic_cie_prompts(model, args.prompts, 10, seed=1234)
    build_s = time.time() - t0
    n_split = emulate or world
    sites = balanced_site_shard(cfg.n_layers, cfg.n_heads, rank, n_split) if n_split > 1 else None

    def step():
        cie = causal_indirect_effect_sums(mean, prompts, answers, model, sites=sites)
        if world > 1:
            dist.all_reduce(cie)
        return cie
    cie = step()
    steps = max(1, min(args.steps, 2))
    if world > 1:
        dist.barrier()
    with model.range_scope("C5 steps"):  # one range check at the end, as the headline's timed steps
        sec, _ = _sync_time(step, steps)
    rt = None
    if world > 1:
        rt = rank_times(sec, dev)
        sec = max(rt)
    L, d, V, T = cfg.n_layers, cfg.d_model, cfg.d_vocab, len(prompts[0])
    P_l = 4 * d * d + 2 * d * cfg.d_mlp
    f_alg = sum((L - 1 - l) * (2 * P_l * T + 2 * T * (T + 1) * d) + 2 * d * V for l in range(L)) / L
    units = len(prompts) * (len(sites) if emulate else L * cfg.n_heads)
    rate = units / sec
    peak_all = peak * (1 if emulate else world)
    del model
    torch.cuda.empty_cache()
    extra = {"cie": cie.cpu()} if return_cie else {}
    return {"workload": c5_workload(world, emulate, len(sites) if sites else 0, L),
            "n_gpus": world, "scaling": "strong", "rank_elapsed_s": [round(x, 4) for x in rt] if rt else None,
            "units_per_step": units, "steps": steps, "ms_per_step": round(sec * 1e3, 1),
            "value": round(rate, 2), "unit": "patched prompts/s", "gflop_per_site": round(f_alg / 1e9, 2),
            "site_tflops": round(rate * f_alg / 1e12, 2), "site_frac": round(rate * f_alg / 1e12 / peak_all, 4),
            "exact16_gemms": x16, "model_build_s": round(build_s, 1), **extra}


def rank_times(el, dev):
    """Every rank's elapsed seconds (all_gather), for the max-over-ranks timing of the config legs."""
    t = torch.tensor([el], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [x.item() for x in out]


def c4_workload(world: int) -> str:
    base = ("pythia-6.9b bf16 FV suite per 50-pair task (answers: the model's zero-shot 2nd / 6th-10th choice, clean "
            "top-5 accuracy 0.5): extraction 512 x 5-shot, CIE 32x32 over 12 prompts, top-10-head FV added at every "
            "layer over 50 zero-shot prompts (top-5)")
    if world > 1:
        base += (f"; {world} GPUs: extraction prompts contiguous per rank (1 all-reduce), CIE sites in balanced "
                 "layer-pair blocks per rank (1 all-reduce), injection sites round-robin (1 all-gather)")
    return base


def c5_workload(world: int, emulate: int = 0, n_sites_rank: int = 0, layers: int = 36) -> str:
    cut = "" if layers == 36 else f" (REHEARSAL: the first {layers} of 36 layers)"
    base = f"pythia-12b CIE sweep {layers}x40 sites, 12 prompts/step, 10-shot, T=33{cut}"
    if emulate:
        return (f"pythia-12b CIE sweep, rank 0's share of a {emulate}-GPU split (sites in balanced layer-pair blocks "
                f"per rank: {n_sites_rank} of {layers * 40} sites), 12 prompts/step, 10-shot, T=33{cut} (planning "
                "emulation on one GPU)")
    if world > 1:
        base += ", sites in balanced layer-pair blocks per rank"
    return base


def config_c4(args, dev, n_tasks=3, world=1):
    """C4: Pythia-6.9B in the north star's bf16 configuration,
    the function-vector suite per synthetic 50-pair task — extraction over 512
    five-shot prompts (a1), the 32 x 32 CIE over 12 shuffled prompts (a7), the
    function vector of the top-10 heads (a10) added at every layer over the 50
    zero-shot prompts, top-5 accuracy (a11) — through the sharded entry points
    (one process: the plain functions).  One warm task, then ``n_tasks`` timed
    (tools/bench_configs.py --configs C4 runs the 20-task suite).  Roofline of
    the CIE sweep (95 % of a task's GEMM work): SURVEY §8d's F_alg per site
    (at the task's prompt length, T = 23) x CIE sites/s against the bf16 dense
    peak (``site_frac``), and
    the bf16 GEMM family's executed TFLOP/s from a separate profiled CIE pass
    (HIP events on the engine stream), with the committed rocprofv3 PMC
    summary of the same sweep (profiles/pmc_gemm_bf16.json) when its
    workload matches."""
    import random
    import tvr_amd
    from tvr_amd import distributed as D
    from tvr_amd import experiments as E
    t0 = time.time()
    model = tvr_amd.Model.from_pretrained("pythia-6.9b", device=dev, seed=0, gemm="bf16",
                                          fp16_weights=args.weights == "fp16")
    build_s = time.time() - t0
    arrow = tvr_amd.tasks.ARROW
    cie_in = {}

    def one(ti):
        # a model-consistent task whose FV accuracy can move both ways: after "x:" the answer is the
        # model's own zero-shot 2nd choice for even pairs (inside the clean top 5) and its 6th..10th choice for odd
        # ones (outside it) -- clean top-5 accuracy 0.5; random pairs on synthetic weights would leave it at 0 and
        # the zero-shot top-1 at 1
        xs = [x for x, _ in tvr_amd.tasks.synthetic_task(50, model.cfg.d_vocab, seed=100 + ti)]
        top = model.forward_clean([model.to_tokens(x + ":")[0].tolist() for x in xs], topk=10)["topk"].tolist()
        task = [(x, model.to_string(int(t[1] if i % 2 == 0 else t[5 + (i // 2) % 5])))
                for i, (x, t) in enumerate(zip(xs, top))]
        random.seed(ti)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t = time.perf_counter()
        ex_prompts = tvr_amd.prompts.sample_icl_prompts(model, task, arrow, ",", 512, 5)
        mean = D.mean_activation_sharded(ex_prompts, model)
        prompts, answers = E.generate_shuffled_prompts(task, model, 12, 5, arrow)
        torch.cuda.synchronize()
        tc = time.perf_counter()
        cie = D.cie_sharded(mean, prompts, answers, model)
        torch.cuda.synchronize()
        tc = time.perf_counter() - tc
        fv = E.assemble_task_vector(mean, cie, 10, 10)
        acc = D.check_accuracy_of_added_task_vector_by_layer_sharded(fv, task, 5, model)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        if world > 1:  # the max over ranks (every rank ends with the same all_gather, so they end together)
            rt = rank_times(el, dev)
            cie_in["rank_times"] = [round(x, 4) for x in rt]
            el, tc = max(rt), max(rank_times(tc, dev))
        cie_in.update(mean=mean, prompts=prompts, answers=answers, task=task)
        return el, tc, acc

    one(0)  # warm: trace / workspace sizing
    runs = [one(ti) for ti in range(1, n_tasks + 1)]
    clean_acc = E.check_accuracy_of_task_vector(torch.zeros(model.cfg.d_model, device=dev), 0, cie_in["task"], 5,
                                                model=model)[0]
    cfg = model.cfg
    L, H, d, V = cfg.n_layers, cfg.n_heads, cfg.d_model, cfg.d_vocab
    # the CIE sweep's roofline: a profiled pass of the last task's sweep (this rank's sites)
    model.profile(True)
    D.cie_sharded(cie_in["mean"], cie_in["prompts"], cie_in["answers"], model)
    torch.cuda.synchronize()
    st = model.profile_stats()
    model.profile(False)
    T = len(model.to_tokens(cie_in["prompts"][0])[0])
    P_l = 4 * d * d + 2 * d * cfg.d_mlp
    f_alg = sum((L - 1 - l) * (2 * P_l * T + 2 * T * (T + 1) * d) + 2 * d * V for l in range(L)) / L
    cie_rate = sum(12 * L * H / r[1] for r in runs) / n_tasks  # whole-job rate (all ranks' sites / max time)
    peak = PEAKS["bf16"] * world
    fam = st["all"]
    gemm_tf = fam["flops"] / (fam["ms"] * 1e-3) / 1e12 if fam["ms"] else None
    workload = f"pythia-6.9b CIE sweep {L}x{H} sites, 12 prompts/step, 5-shot, T={T}"
    # the committed PMC pass is the bench's own sweep at C4's model / sites / shots on synthetic prompts
    # (T = 18; the task's string prompts tokenise to T = 23): the counters' ratios carry over
    pmc, pmc_src = pmc_summary("bf16", workload, any_len=True)
    variants = {k: round(st[k]["flops"] / (st[k]["ms"] * 1e-3) / 1e12, 2) for k in ("qkv_mlpin", "o_mlpout", "unembed")
                if st[k]["ms"]}
    del model
    torch.cuda.empty_cache()
    return {"workload": c4_workload(world),
            "n_gpus": world, "rank_elapsed_s_last_task": cie_in.get("rank_times"),
            "gemm": "bf16", "tasks_timed": n_tasks, "s_per_task": round(sum(r[0] for r in runs) / n_tasks, 3),
            "clean_top5_acc_last_task": clean_acc,
            "cie_patched_prompts_per_s": round(cie_rate, 1),
            "cie_roofline": {"workload": workload, "gflop_per_site": round(f_alg / 1e9, 2),
                             "site_tflops": round(cie_rate * f_alg / 1e12, 2),
                             "site_frac": round(cie_rate * f_alg / 1e12 / peak, 4), "peak_tflops": peak,
                             "peak_basis": f"bf16 MFMA dense peak (v_mfma_f32_16x16x32_bf16 / _f16, one product) x "
                                           f"{world} GPU(s)",
                             "gemm_achieved_tflops": round(gemm_tf, 2) if gemm_tf else None,
                             "gemm_frac": round(gemm_tf / PEAKS["bf16"], 4) if gemm_tf else None,
                             "gemm_variants_tflops": variants,
                             "mfma_util_rocprof": (pmc.get("mfma") or {}).get("all") if pmc else None,
                             "mfma_util_variants": {k: v.get("mfma_util") for k, v in
                                                    ((pmc.get("mfma") or {}).get("variants") or {}).items()}
                                                   if pmc else None,
                             "traffic_ratio_to_alg": (pmc or {}).get("ratio_hbm_to_alg"),
                             "pmc_source": pmc_src},
            "fv_top5_acc_by_layer_last_task": runs[-1][2], "model_build_s": round(build_s, 1)}


def cpu_baseline(args, cfg, prompts, answers, mean, model):
    """the oracle (fp32 CPU, TransformerLens semantics, one
    batch-1 hooked forward per site — the reference loop scratch2.py:181-194)
    on prompt 0 at layers {0, L/2, L-1} x ALL heads, on every host core this
    process may use; rate = sites / wall time (per-forward time extrapolates
    linearly to the full sweep).  Also returns ``parity``: the engine's values
    for the same sites (same prompt, mean, layers, heads) against the oracle's."""
    import tvr_amd
    from oracle.hooked_pythia import HookedPythiaOracle, OracleConfig
    from oracle import reference_experiments as R
    from tvr_amd.experiments import causal_indirect_effect_sums

    # every core this process may use.  On the GPU box the
    # affinity mask shows the whole machine while the job's CPU share is
    # OMP_NUM_THREADS (16 per GPU): more threads than that only oversubscribe.
    affinity = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS") or affinity)
    cores = max(1, min(affinity, share))
    torch.set_num_threads(cores)
    t0 = time.time()
    # the engine's weights: the same seeded generator on the same device (synth_engine_weights),
    # processed there by the oracle's own TransformerLens restatement, then moved to the CPU
    shapes = tvr_amd.weights.hf_param_shapes(cfg)
    sd = {n: tvr_amd.weights.synth_param(cfg, n, s, 0, model.device, fp16=args.weights == "fp16")
          for n, s in shapes.items()}
    oracle = HookedPythiaOracle(OracleConfig(cfg.n_layers, cfg.d_model, cfg.n_heads, cfg.d_mlp, cfg.d_vocab,
                                             cfg.rotary_dim, cfg.n_ctx), sd, tokenizer=None)
    del sd
    torch.cuda.empty_cache()
    log(f"cpu baseline: oracle weights ready in {time.time() - t0:.1f}s")
    layers = sorted({0, cfg.n_layers // 2, cfg.n_layers - 1})
    heads = list(range(cfg.n_heads))
    mean_cpu = mean.detach().cpu()
    cie_ref = torch.zeros(cfg.n_layers, cfg.n_heads)
    t0 = time.perf_counter()
    for l in layers:  # the reference loop, one layer at a time for progress lines
        cie_ref += R.calculate_average_causal_indirect_effect(mean_cpu, [prompts[0]], [[answers[0]]], oracle,
                                                              layers=[l], heads=heads)
        log(f"cpu baseline: layer {l} x {len(heads)} heads done at {time.perf_counter() - t0:.1f}s")
    dt = time.perf_counter() - t0
    n_sites = len(layers) * len(heads)
    out = {"value": n_sites / dt, "unit": "patched prompts/s", "cores": cores, "kind": "port",
           "sample": (f"oracle fp32 CPU (TransformerLens semantics, batch-1 hooked forward per site, reference loop "
                      f"scratch2.py:181-194): prompt 0 (T={len(prompts[0])}), layers {layers} x all {len(heads)} "
                      f"heads = {n_sites} sites + {len(layers)} clean forwards in {dt:.1f}s on {cores} threads "
                      f"(torch.set_num_threads(min(len(os.sched_getaffinity(0)) = {affinity}, OMP_NUM_THREADS = {share})))")}
    # parity on the same sites: engine vs oracle
    logits_ref = oracle.forward(torch.tensor([prompts[0]]))[0, -1]
    clean = model.forward_clean([prompts[0]], targets=[answers[0]], topk=1, return_logits=True)
    ours = causal_indirect_effect_sums(mean, [prompts[0]], [answers[0]], model, layers=layers).cpu().double()
    ref = cie_ref.double()
    idx = torch.tensor(layers)
    d_cie = (ours[idx] - ref[idx]).abs().max().item()
    p_ref = torch.softmax(logits_ref.double(), 0)
    parity = {"sites": n_sites, "prompt": 0, "layers": layers, "heads": "all",
              "max_abs_cie_err": d_cie, "max_abs_cie_ref": ref[idx].abs().max().item(),
              "max_rel_cie_err": d_cie / max(ref[idx].abs().max().item(), 1e-30),
              "clean_logits_max_rel_err": ((clean["logits"][0].cpu().double() - logits_ref.double()).abs().max()
                                           / logits_ref.double().abs().max()).item(),
              "clean_prob_abs_err": abs(clean["prob"][0].item() - p_ref[answers[0]].item()),
              "top1_equal": int(clean["topk"][0, 0]) == int(logits_ref.argmax()),
              "tolerance": "CIE |err| <= 1e-4 max|CIE| + 1e-7, logits 1e-4 relative, top-1 identical"}
    parity["ok"] = bool(d_cie <= 1e-4 * ref[idx].abs().max().item() + 1e-7 and
                        parity["clean_logits_max_rel_err"] < 1e-4 and parity["top1_equal"])
    return out, parity


def parity_informative(args, dev, cores):
    """The driver-observed parity number on INFORMATIVE weights:
    the headline's bench weights (std 0.02) leave |CIE| ~ 1e-6, so ``parity``
    is measured on a 4-layer Pythia-2.8B-width copy with std-0.05 weights,
    where one head moves the answer's probability by percents: the CPU oracle
    (fp32, the reference's loops: scratch2.py:81-100 extraction over 16
    five-shot prompts, :171-197 CIE over every site of one prompt, answer = the
    oracle's clean top-1) against the engine on the same seeded weights, prompts
    and means, on the bench's GEMM path.  Bars as the full-depth tests: CIE
    |err| <= 1e-4 max|CIE| + 1e-7, extraction / logits 1e-4 relative, top-1
    identical."""
    import random
    import tvr_amd
    from oracle.hooked_pythia import HookedPythiaOracle, OracleConfig
    from oracle import reference_experiments as R
    from tvr_amd.experiments import causal_indirect_effect_sums
    torch.set_num_threads(cores)
    t0 = time.time()
    cfg = tvr_amd.get_config(args.model).with_(n_layers=4)
    shapes = tvr_amd.weights.hf_param_shapes(cfg)
    sd = {n: tvr_amd.weights.synth_param(cfg, n, s, 0, dev, 0.05, fp16=args.weights == "fp16")
          for n, s in shapes.items()}
    model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device=dev, gemm=args.gemm)
    oracle = HookedPythiaOracle(OracleConfig(cfg.n_layers, cfg.d_model, cfg.n_heads, cfg.d_mlp, cfg.d_vocab,
                                             cfg.rotary_dim, cfg.n_ctx), sd, tokenizer=model.tokenizer)
    del sd
    torch.cuda.empty_cache()
    task = tvr_amd.tasks.synthetic_task(52, cfg.d_vocab, seed=7)
    random.seed(11)
    mean_ref = R.generate_mean_activation(task, tvr_amd.tasks.ARROW, ",", oracle, 16, 5)
    random.seed(11)
    mean = tvr_amd.generate_mean_activation(task, tvr_amd.tasks.ARROW, ",", model=model, num_contexts=16,
                                            len_contexts=5)
    prompts, _ = tvr_amd.prompts.synthetic_cie_prompts(model, 1, args.kshot, seed=1234)
    logits_ref = oracle.forward(torch.tensor([prompts[0]]))[0, -1].double()
    answer = int(logits_ref.argmax())
    cie_ref = R.calculate_average_causal_indirect_effect(mean_ref, prompts, [[answer]], oracle).double()
    clean = model.forward_clean(prompts, targets=[answer], topk=1, return_logits=True)
    cie = causal_indirect_effect_sums(mean_ref.to(dev), prompts, [answer], model).cpu().double()
    model._check_range("bench parity")
    cmax = cie_ref.abs().max().item()
    d_cie = (cie - cie_ref).abs().max().item()
    out = {"weights": f"{args.model} width, 4 layers, seeded std-0.05 weights (informative: max |CIE| {cmax:.3e})",
           "sites": cfg.n_layers * cfg.n_heads, "prompt_T": len(prompts[0]), "gemm": args.gemm,
           "max_abs_cie_err": d_cie, "max_abs_cie_ref": cmax, "max_rel_cie_err": d_cie / max(cmax, 1e-30),
           "extraction_max_rel_err": ((mean.cpu().double() - mean_ref.double()).abs().max()
                                      / mean_ref.double().abs().max()).item(),
           "clean_logits_max_rel_err": ((clean["logits"][0].cpu().double() - logits_ref).abs().max()
                                        / logits_ref.abs().max()).item(),
           "top1_equal": int(clean["topk"][0, 0]) == answer,
           "tolerance": "CIE |err| <= 1e-4 max|CIE| + 1e-7, extraction and logits 1e-4 relative, top-1 identical",
           "seconds": round(time.time() - t0, 1)}
    out["ok"] = bool(d_cie <= 1e-4 * cmax + 1e-7 and out["extraction_max_rel_err"] < 1e-4 and
                     out["clean_logits_max_rel_err"] < 1e-4 and out["top1_equal"] and cmax > 1e-3)
    del model
    torch.cuda.empty_cache()
    return out


DTYPE_X16 = ("f32 (x2f16 emulation: fp32 activations as 2 fp16 planes against the checkpoint's exact fp16 weights, "
             "2 MFMA products, fp32 accumulate)")
DTYPES = {"x2f16": "f32 (x2f16 emulation: fp32 operands as 2 fp16 planes, 3 MFMA products, fp32 accumulate)",
          "x3bf16": "f32 (x3bf16 emulation: fp32 operands as 3 bf16 planes, 6 MFMA products, fp32 accumulate)",
          "f32": "f32 (v_mfma_f32_32x32x2_f32)",
          "bf16": "bf16 (bf16 GEMM operands, fp32 accumulate; LayerNorm / attention / softmax fp32)"}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if args.launch_check:
        launch_check(rank, world, "gloo" if args.dist_backend == "nccl" else args.dist_backend)
        return
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    if world > 1:
        # a rank that fails inside a config leg must not leave the others blocked in a collective forever
        from datetime import timedelta
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=timedelta(minutes=10))
        else:
            dist.init_process_group(args.dist_backend, timeout=timedelta(minutes=10))

    import tvr_amd
    from tvr_amd.distributed import balanced_site_shard, strided_shard
    from tvr_amd.experiments import causal_indirect_effect_sums, sum_last_z

    cfg = tvr_amd.get_config(args.model)
    t0 = time.time()
    model = tvr_amd.Model.from_pretrained(args.model, device=dev, seed=0, gemm=args.gemm,
                                          fp16_weights=args.weights == "fp16")
    torch.cuda.synchronize()
    log(f"[rank {rank}] {args.model} synthetic {args.weights}-valued weights on {dev} in {time.time() - t0:.1f}s "
        f"(exact-fp16 GEMMs: {model.exact16})")

    # --- mean head activations [L, H, d]: a real extraction (a1) or seeded random
    te, n_ex, hbm_ex = None, 0, None
    if args.extract > 0:
        import random
        random.seed(4321)
        pairs = tvr_amd.tasks.synthetic_task(52, cfg.d_vocab, seed=7)
        ex_prompts = tvr_amd.prompts.sample_icl_prompts(model, pairs, "→", ",", args.extract, 6)
        sum_last_z(model, ex_prompts[:64])  # workspace sizing outside the timed extraction
        torch.cuda.synchronize()
        te = time.perf_counter()
        zsum = sum_last_z(model, ex_prompts)
        torch.cuda.synchronize()
        te = time.perf_counter() - te
        model.profile(True)  # kernel timings of the capture from a separate profiled pass
        sum_last_z(model, ex_prompts)
        hbm_ex = model.profile_hbm_stats()
        model.profile(False)
        n_ex = len(ex_prompts)
        mean = model.project_heads(zsum) / n_ex
    else:
        g = torch.Generator(device=dev).manual_seed(4321)
        mean = torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, device=dev, generator=g) * 0.5

    emulate = args.emulate_world if world == 1 and args.emulate_world > 1 else 0
    shard = args.shard if (world > 1 or emulate) else "sites"
    if emulate and shard == "prompts":
        raise SystemExit("--emulate-world times a strong split: --shard sites or heads")
    everything = [(l, h) for l in range(cfg.n_layers) for h in range(cfg.n_heads)]
    if args.c4_prompts:  # C4's CIE prompts (config_c4): shuffled string prompts of a synthetic task, tokenised
        import random
        random.seed(1)
        task = tvr_amd.tasks.synthetic_task(50, cfg.d_vocab, seed=101)
        sp, sa = tvr_amd.experiments.generate_shuffled_prompts(task, model, args.prompts, args.kshot,
                                                               tvr_amd.tasks.ARROW)
        c4_prompts = [model.to_tokens(p)[0].tolist() for p in sp], [a[0] for a in sa]
    if shard in ("sites", "heads"):  # C3: the same prompts everywhere, this rank's share of the sites
        prompts, answers = (c4_prompts if args.c4_prompts else
                            tvr_amd.prompts.synthetic_cie_prompts(model, args.prompts, args.kshot, seed=1234))
        n_split = emulate or world
        sites = (balanced_site_shard(cfg.n_layers, cfg.n_heads, rank, n_split) if shard == "sites" else
                 [(l, h) for l in range(cfg.n_layers) for h in strided_shard(cfg.n_heads, rank, n_split)])
        units_total = len(prompts) * (len(sites) if emulate else cfg.n_layers * cfg.n_heads)
    else:  # weak scaling: per-rank prompts, every site
        prompts, answers = tvr_amd.prompts.synthetic_cie_prompts(model, args.prompts, args.kshot, seed=1234 + rank)
        sites = everything
        units_total = len(prompts) * cfg.n_layers * cfg.n_heads * world
    units_rank = len(prompts) * len(sites)

    def step():
        cie = causal_indirect_effect_sums(mean, prompts, answers, model, sites=sites)
        if world > 1:
            dist.all_reduce(cie)
        return cie

    rank_times = []

    def timed(warmup, steps, profile):
        for i in range(warmup):
            step()
            log(f"[rank {rank}] warmup step {i + 1}/{warmup}")
        if profile:
            model.profile(True)  # HIP events around every launch (separate pass: not the timed value)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        # one x2f16 range check when the steps end (Model.range_scope: the sticky device flag, inside the
        # timed region) instead of a synchronising check after every sweep, so step i + 1's host-side
        # preparation overlaps step i on the GPU
        with model.range_scope("bench steps"):
            for i in range(steps):
                cie = step()
                log(f"[rank {rank}] {'profiled ' if profile else ''}step {i + 1}/{steps}")  # host-side progress only
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        t = torch.tensor([el], device=dev if args.dist_backend == "nccl" else "cpu", dtype=torch.float64)
        if world > 1:
            times = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(times, t)
            rank_times[:] = [x.item() for x in times]
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.item(), cie

    elapsed, cie = timed(args.warmup, args.steps, False)
    rank_elapsed = list(rank_times)
    value = units_total * args.steps / elapsed

    # --- roofline of the dominant kernel + HBM-bound kernels: a separate profiled pass
    psteps = max(1, args.profile_steps)
    el_prof, _ = timed(0, psteps, True)
    st = model.profile_stats()
    hbm = model.profile_hbm_stats()
    model.profile(False)
    fam = st["all"]
    achieved = fam["flops"] / (fam["ms"] * 1e-3) / 1e12
    T = len(prompts[0])
    workload, scaling = describe_workload(args.model, cfg.n_layers, cfg.n_heads, args.prompts, args.kshot, T, world,
                                          shard, emulate, len(sites))
    if model.exact16 and args.gemm == "x2f16":  # another kernel instruction mix: 3-product counters do not apply
        workload += ", fp16-valued weights (exact-fp16 GEMMs, 2 products)"
    pmc, traffic_src = pmc_summary(args.gemm, workload)
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    products = 2 if (args.gemm == "x2f16" and model.exact16) else PRODUCTS.get(args.gemm)
    peak = BF16_MFMA_PEAK_TFLOPS / products if products else PEAKS[args.gemm]
    L, d, V = cfg.n_layers, cfg.d_model, cfg.d_vocab
    P_l = 4 * d * d + 2 * d * cfg.d_mlp
    # F_alg(site at layer l) = (L-1-l)(2 P_l T + 2 T(T+1) d) + 2 d V
    f_alg = sum((L - 1 - l) * (2 * P_l * T + 2 * T * (T + 1) * d) + 2 * d * V for l in range(L)) / L
    variants = {}
    for name in ("qkv_mlpin", "o_mlpout", "unembed"):
        v = st[name]
        if v["launches"]:
            variants[name] = {"launches": v["launches"],
                              "achieved_tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 2),
                              "avg_launch_ms": round(v["ms"] / v["launches"], 4),
                              "alg_bytes_per_launch": round(v["bytes"] / v["launches"]),
                              "share_of_gemm_time": round(v["ms"] / fam["ms"], 4)}
    parallelism = ("single GPU" if world == 1 else
                   f"{SPLITS[shard].format(n=world)} (same {args.prompts} prompts on every GPU), weights replicated, "
                   f"1 all-reduce of [L,H] per step" if shard in SPLITS else
                   f"prompt-sharded x{world}, weights replicated, 1 all-reduce of [L,H] per step")
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "patched prompts/s",
        "n_gpus": dist.get_world_size() if world > 1 else 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": DTYPE_X16 if (args.gemm == "x2f16" and model.exact16) else DTYPES[args.gemm],
        "data": f"synthetic (seeded {args.model}-shaped weights, "
                f"{'fp16-valued as the released checkpoints' if args.weights == 'fp16' else 'fp32-valued'}; "
                f"{'C4 shuffled string prompts of a synthetic task' if args.c4_prompts else 'seeded single-token shuffled-label prompts'})",
        "config": {
            "workload": workload,
            "sites_per_step": units_total,
            "sites_per_step_per_gpu": units_rank,
            "parallelism": parallelism,
            "shard": shard,
            "dist_backend": args.dist_backend if world > 1 else None,
            "rank_elapsed_s": [round(x, 4) for x in rank_elapsed] if world > 1 else None,
        },
        "roofline": {
            "bound": "mfma",
            "kernel": KERNELS["x2f16-exact16" if (args.gemm == "x2f16" and model.exact16) else args.gemm],
            "achieved": round(achieved, 2),
            "peak": round(peak, 1),
            "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            "flops_basis": "algorithmic fp32 2*M*N*K per launch / HIP-event launch time (separate profiled pass)",
            "peak_basis": ("fp32 MFMA dense peak" if args.gemm == "f32" else
                           f"fp16/bf16 MFMA dense peak {BF16_MFMA_PEAK_TFLOPS} / {products} products "
                           f"(= fp32-equivalent ceiling of the split; fp32 MFMA peak {FP32_MFMA_PEAK_TFLOPS})"),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "traffic_basis": (pmc or {}).get("basis"),
            "traffic_ratio_to_alg": (pmc or {}).get("ratio_hbm_to_alg"),
            "mfma_util_rocprof": (pmc.get("mfma") or {}).get("all") if pmc else None,
            "algorithmic_bytes_per_launch": round(fam["bytes"] / max(fam["launches"], 1)),
            "launches_per_step": fam["launches"] // psteps,
            "avg_launch_gflop": round(fam["flops"] / max(fam["launches"], 1) / 1e9, 3),
            "avg_launch_ms": round(fam["ms"] / max(fam["launches"], 1), 4),
            "gemm_share_of_step": round(fam["ms"] / (el_prof * 1e3), 4),
            "variants": variants,
        },
        "hbm_kernels": hbm_kernels(hbm, hbm_ex, psteps, workload),
        "algorithmic": {
            "gflop_per_site": round(f_alg / 1e9, 2),
            "site_tflops": round(value * f_alg / 1e12, 2),
            # BASELINE.md section 3's roofline fraction: the reference's algorithmic work per site
            #  x sites/s over the whole timed step, against the same peak
            # (work the engine skips -- shared prefixes, the trimmed last layer, the linearised
            # entry layer -- counts as done, as in the reference's loop)
            "site_frac": round(value * f_alg / 1e12 / peak, 4),
            "extraction_prompts_per_s": round(n_ex / te, 1) if te else None,
        },
    }
    out["config"]["gemm"] = args.gemm
    out["config"]["weights"] = args.weights
    out["config"]["exact16_gemms"] = bool(model.exact16 and args.gemm == "x2f16")  # (bf16 mode leaves them unused)
    if world == 1 and model.exact16 and args.gemm == "x2f16" and not emulate and args.processed_leg:
        # the same sweep on the TL-processed weights (3 products: the path of fp32-valued checkpoints)
        model.set_exact16(False)
        npw = max(1, min(args.steps, 2))
        el_pw, cie_pw = timed(1, npw, False)
        model.set_exact16(True)
        out["processed_weights_leg"] = {
            "gemm": "x2f16, 3 products on the processed (folded / centred) weights", "steps": npw,
            "value": round(units_rank * npw / el_pw, 2),
            "max_abs_cie_diff_vs_exact16": float((cie - cie_pw).abs().max()),
            "max_abs_cie": float(cie_pw.abs().max())}
    if world == 1 and args.f32_leg and args.gemm != "f32":
        model.set_gemm("f32")
        n32 = max(1, min(args.steps, 2))
        el32, cie32 = timed(1, n32, False)
        model.set_gemm(args.gemm)
        out["f32_leg"] = {
            "gemm": "f32", "steps": n32,
            "value": round(units_rank * n32 / el32, 2),
            "max_abs_cie_diff_vs_f32": float((cie - cie32).abs().max()),
            "max_abs_cie": float(cie32.abs().max()),
        }
    if emulate:
        out["emulated_world"] = emulate
    if world > 1 and shard in SPLITS and args.weak_leg:
        # the weak form (own prompts per rank, every site): reported beside the strong headline, never as `value`
        prompts, answers = tvr_amd.prompts.synthetic_cie_prompts(model, args.prompts, args.kshot, seed=1234 + rank)
        sites = everything
        nw = max(1, min(args.steps, 2))
        el_w, _ = timed(1, nw, False)
        out["weak_prompt_partition"] = {
            "workload": describe_workload(args.model, cfg.n_layers, cfg.n_heads, args.prompts, args.kshot, T, world,
                                          "prompts")[0],
            "steps": nw, "value": round(len(prompts) * cfg.n_layers * cfg.n_heads * world * nw / el_w, 2),
            "unit": "patched prompts/s", "scaling": "weak", "rank_elapsed_s": [round(x, 4) for x in rank_times]}
    if rank == 0 and world == 1 and args.cpu_baseline and not emulate:
        out["cpu_baseline"], out["parity_bench_weights"] = cpu_baseline(args, cfg, prompts, answers, mean, model)
        try:
            out["parity"] = parity_informative(args, dev, out["cpu_baseline"]["cores"])
        except Exception as e:
            out["parity"] = {"error": f"{type(e).__name__}: {e}", "ok": False}
    # the other BASELINE.json configs, timed after the headline (never part of `value`): C2 is a one-GPU config
    # (N = 1 only); C4 and C5 are BASELINE's 8-GPU configs, sharded over the ranks at N > 1;
    # --emulate-world times C5's rank-0 share
    which = {c for c in args.configs.split(",") if c} if args.model == "pythia-2.8b" else set()
    if world > 1:
        which -= {"C2"}
    if emulate:
        which &= {"C5"}
    if which:
        out["configs"] = {}
        if "C2" in which:
            try:
                out["configs"]["C2"] = config_c2(model, mean, peak)
                log(f"C2: {out['configs']['C2']['accuracy']['sites_per_s']} / {out['configs']['C2']['dprob']['sites_per_s']} sites/s")
            except Exception as e:  # a config leg never voids the headline line
                out["configs"]["C2"] = {"error": f"{type(e).__name__}: {e}"}
                log(f"[rank {rank}] C2 failed: {out['configs']['C2']['error']}")
        if which & {"C4", "C5"}:
            del model
            torch.cuda.empty_cache()
            model = None
        if "C4" in which:
            try:
                out["configs"]["C4"] = config_c4(args, dev, world=world)
                log(f"C4: {out['configs']['C4']['s_per_task']} s/task")
            except Exception as e:
                out["configs"]["C4"] = {"error": f"{type(e).__name__}: {e}"}
                log(f"[rank {rank}] C4 failed: {out['configs']['C4']['error']}")
        if "C5" in which:
            try:
                out["configs"]["C5"] = config_c5(args, dev, peak, world, rank, emulate)
                log(f"C5: {out['configs']['C5']['value']} patched prompts/s")
            except Exception as e:
                out["configs"]["C5"] = {"error": f"{type(e).__name__}: {e}"}
                log(f"[rank {rank}] C5 failed: {out['configs']['C5']['error']}")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""GPU, multi-process: the sharded entry points of distributed.py on the HIP
engine itself (not an oracle stand-in), 2 ranks with the gloo backend, both
on cuda:0 (one GPU per box here; the driver's 8-GPU runs use RCCL).  Each
rank builds the same seeded tiny model; the sharded results must equal the
single-process engine results:

* cie_sharded (balanced layer-pair sites, one all-reduce)  == calculate_average_causal_indirect_effect
* mean_activation_sharded (contiguous prompt split, all-reduce) == sum_last_z / n, projected
* the layer sweeps and the FV layer sweep with (prompt, layer) sites
  round-robin + all_gather                                      == the unsharded sweeps
* bench.py's C5 leg (Pythia-12B shape, 10-shot, depth cut to 6 of 36 layers so
  two replicas share one GPU): the 2-rank balanced site split (one whole layer
  pair per rank + the third pair split by head, one all-reduce) == the same
  sweep in one process.

Rendezvous through a file in pytest's tmp dir (no probed port that another
process could take between the probe and the bind).
"""
import os
import random
import types

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2


def _setup():
    import tvr_amd
    from conftest import TINY_STD
    cfg = tvr_amd.get_config("tiny")
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0, std=TINY_STD)
    tok = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
    model = tvr_amd.Model.from_hf_state_dict(cfg, sd, device="cuda", tokenizer=tok, gemm="x2f16")
    task = tvr_amd.tasks.synthetic_task(12, cfg.d_vocab, seed=3, lo=10)
    random.seed(11)
    ex = tvr_amd.prompts.sample_icl_prompts(model, task, tvr_amd.tasks.ARROW, ",", 9, 3)
    prompts, answers = tvr_amd.experiments.generate_shuffled_prompts(task, model, 3, 3, tvr_amd.tasks.ARROW)
    mean = torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, generator=torch.Generator().manual_seed(5)).cuda()
    return tvr_amd, model, task, ex, prompts, answers, mean


def _run(sharded: bool):
    tvr_amd, model, task, ex, prompts, answers, mean = _setup()
    E, D = tvr_amd.experiments, tvr_amd.distributed
    arrow = tvr_amd.tasks.ARROW
    lv = E.gather_head_activations_to_layers(mean)
    fv = mean[0, :2].sum(0)
    if sharded:
        return {"cie": D.cie_sharded(mean, prompts, answers, model).cpu(),
                "mean": D.mean_activation_sharded(ex, model).cpu(),
                "acc": D.apply_layered_vectors_to_zero_shot_sharded(lv, task, arrow, model),
                "dprob": D.apply_layered_vectors_to_zero_shot_by_probability_sharded(lv, task, arrow, model).cpu(),
                "fv": D.check_accuracy_of_added_task_vector_by_layer_sharded(fv, task, 5, model)}
    return {"cie": E.calculate_average_causal_indirect_effect(mean, prompts, answers, model).cpu(),
            "mean": (model.project_heads(E.sum_last_z(model, ex)) / len(ex)).cpu(),
            "acc": E.apply_layered_vectors_to_zero_shot(lv, task, arrow, model),
            "dprob": E.apply_layered_vectors_to_zero_shot_by_probability(lv, task, arrow, model).cpu(),
            "fv": E.check_accuracy_of_added_task_vector_by_layer(fv, task, 5, model)}


def _worker(rank, init, job, q):
    import torch.distributed as dist
    os.environ.update(HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=WORLD)
    try:
        q.put((rank, job(rank)))
    except Exception as e:  # surface the failure in the parent instead of hanging it
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _ranks(tmp_path, job, timeout=180):
    """job(rank) on WORLD spawned gloo ranks (file rendezvous); their results by rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = f"file://{tmp_path / 'rendezvous'}"
    procs = [ctx.Process(target=_worker, args=(r, init, job, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        return dict(q.get(timeout=timeout) for _ in range(WORLD))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()


def _sharded(rank):
    return _run(True)


def test_sharded_entry_points_on_the_engine(tmp_path):
    results = _ranks(tmp_path, _sharded)
    for r in range(WORLD):
        assert isinstance(results[r], dict), results[r]
    ref = _run(False)
    assert ref["cie"].abs().max() > 0 and ref["mean"].abs().max() > 0 and ref["dprob"].abs().max() > 0
    for r in range(WORLD):
        got = results[r]
        assert torch.allclose(got["cie"], ref["cie"], rtol=0, atol=1e-6 * ref["cie"].abs().max().item() + 1e-9)
        assert torch.allclose(got["mean"], ref["mean"], rtol=1e-5, atol=1e-6 * ref["mean"].abs().max().item())
        assert got["acc"] == ref["acc"]
        assert torch.allclose(got["dprob"], ref["dprob"], rtol=0, atol=1e-6)
        assert got["fv"] == ref["fv"]


C5_ARGS = types.SimpleNamespace(gemm="x2f16", weights="fp16", prompts=4, steps=1, c5_layers=6)


def _c5_rank(rank):
    import bench
    res = bench.config_c5(C5_ARGS, "cuda:0", 1.0, world=WORLD, rank=rank, return_cie=True)
    return {k: res[k] for k in ("cie", "workload", "units_per_step", "rank_elapsed_s")}


@pytest.mark.timeout(600)
def test_c5_leg_two_ranks_equals_one_process(tmp_path):
    """bench.config_c5 at world 2 (the sharded C5 leg had never completed): Pythia-12B's
    width / 40 heads / 10-shot T = 33 prompts, 6 layers, fp16-valued weights (exact-fp16 GEMMs, sliced
    accumulation, linearised entry).  balanced_site_shard gives each rank one whole layer pair and half the
    heads of the third; one all-reduce; the result must equal the single-process sweep's CIE sums."""
    import bench
    results = _ranks(tmp_path, _c5_rank, timeout=540)
    for r in range(WORLD):
        assert isinstance(results[r], dict), results[r]
    ref = bench.config_c5(C5_ARGS, "cuda:0", 1.0, world=1, return_cie=True)
    cie1 = ref["cie"].double()
    big = cie1.abs().max().item()
    assert big > 0 and (cie1 != 0).double().mean().item() > 0.9
    for r in range(WORLD):
        got = results[r]
        assert "REHEARSAL" in got["workload"] and got["units_per_step"] == 4 * 6 * 40
        assert len(got["rank_elapsed_s"]) == WORLD
        err = (got["cie"].double() - cie1).abs().max().item()
        print(f"C5 rehearsal rank {r}: |sharded - one process| {err:.2e} of max |CIE sum| {big:.3e}")
        assert err <= 1e-5 * big + 1e-9, (r, err, big)


def _rccl_worker(init, q):
    """One rank on the RCCL backend (torch's "nccl" is RCCL on ROCm), bound to cuda:0 as bench.py binds its
    ranks (device_id): the sharded CIE and extraction, whose collectives then run on device tensors through
    RCCL, plus an explicit all_reduce / all_gather / broadcast."""
    import torch.distributed as dist
    os.environ.update(HSA_ENABLE_IPC_MODE_LEGACY="0")
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=init, rank=0, world_size=1, device_id=torch.device("cuda", 0))
        assert dist.get_backend() == "nccl"
        out = _run(True)
        t = torch.arange(8, dtype=torch.float32, device="cuda") + 1
        dist.all_reduce(t)
        g = [torch.empty_like(t)]
        dist.all_gather(g, t)
        dist.broadcast(t, 0)
        torch.cuda.synchronize()
        out["coll"] = (t.cpu(), g[0].cpu())
        q.put(out)
    except Exception as e:
        q.put(repr(e))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_one_rank_on_the_engine(tmp_path):
    """The `nccl` (RCCL) branch bench.py takes on a multi-GPU node, executed on this box's one GPU at world
    size 1: init with device_id, the sharded entry points' collectives on device tensors, and the results
    equal the unsharded engine's."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(f"file://{tmp_path / 'rccl'}", q))
    p.start()
    try:
        got = q.get(timeout=240)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert isinstance(got, dict), got
    ref = _run(False)
    # (the same sites, possibly batched and split-K-planned differently: fp32 rounding only, as the 2-rank test)
    assert torch.allclose(got["cie"], ref["cie"], rtol=0, atol=1e-6 * ref["cie"].abs().max().item() + 1e-9)
    assert torch.allclose(got["mean"], ref["mean"], rtol=1e-5, atol=1e-6 * ref["mean"].abs().max().item())
    assert got["acc"] == ref["acc"] and got["fv"] == ref["fv"]
    assert torch.allclose(got["dprob"], ref["dprob"], rtol=0, atol=1e-6)
    t, g = got["coll"]
    assert torch.equal(t, torch.arange(8, dtype=torch.float32) + 1) and torch.equal(g, t)

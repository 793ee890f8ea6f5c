"""GPU, multi-process: the sharded entry points of distributed.py on the HIP
engine itself (not an oracle stand-in), 2 ranks with the gloo backend, both
on cuda:0 (one GPU per box here; the driver's 8-GPU runs use RCCL).  Each
rank builds the same seeded tiny model; the sharded results must equal the
single-process engine results:

* cie_sharded (balanced layer-pair sites, one all-reduce)  == calculate_average_causal_indirect_effect
* mean_activation_sharded (contiguous prompt split, all-reduce) == sum_last_z / n, projected
* the layer sweeps and the FV layer sweep with (prompt, layer) sites
  round-robin + all_gather                                      == the unsharded sweeps
"""
import os
import random
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


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


def _worker(rank, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        q.put((rank, _run(True)))
    except Exception as e:  # surface the failure in the parent instead of hanging it
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_sharded_entry_points_on_the_engine():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        results = dict(q.get(timeout=180) for _ in range(WORLD))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
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

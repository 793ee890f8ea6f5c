"""CPU, multi-process (gloo): the multi-GPU partition + reduction logic of
distributed.py, with the oracle standing in for each rank's GPU sweep.

* head-sharded CIE (head ≡ rank mod world, one SUM all-reduce) == the full
  single-process oracle CIE;
* prompt-sharded mean extraction (contiguous split, SUM all-reduce, one
  division by the global count) == the unsharded mean.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import tvr_amd
        from tvr_amd import distributed as D
        from conftest import TINY_STD, make_oracle
        from oracle import reference_experiments as R

        cfg = tvr_amd.get_config("tiny")
        sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0, std=TINY_STD)
        tok = tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab)
        oracle = make_oracle(cfg, sd, tok, torch.float64)
        g = torch.Generator().manual_seed(0)
        mean = torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, generator=g, dtype=torch.float64)
        prompts = [[0, 5, 1, 9, 44, 1, 7], [0, 3, 1, 8, 1, 12, 19, 1, 6]]
        answers = [[9], [12]]

        def local(heads):
            return R.calculate_average_causal_indirect_effect(mean, prompts, answers, oracle,
                                                              heads=heads) * len(prompts)

        cie = D.sharded_cie(cfg.n_layers, cfg.n_heads, len(prompts), local)
        # prompt-sharded extraction with a stand-in "Σ z" and projection
        vecs = torch.randn(10, 3, 4, generator=torch.Generator().manual_seed(1), dtype=torch.float64)
        ids = list(range(10))
        mean_x = D.sharded_mean_activation(ids, lambda ps: vecs[list(ps)].sum(0) if ps else torch.zeros(3, 4,
                                                                                                   dtype=torch.float64),
                                           lambda z: z * 2)
        q.put((rank, cie, mean_x, D.strided_shard(cfg.n_heads, rank, world),
               D.contiguous_shard(10, rank, world)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_sweeps_match_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    results.sort(key=lambda r: r[0])

    import tvr_amd
    from conftest import TINY_STD, make_oracle
    from oracle import reference_experiments as R
    cfg = tvr_amd.get_config("tiny")
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0, std=TINY_STD)
    oracle = make_oracle(cfg, sd, tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab), torch.float64)
    mean = torch.randn(cfg.n_layers, cfg.n_heads, cfg.d_model, generator=torch.Generator().manual_seed(0),
                       dtype=torch.float64)
    full = R.calculate_average_causal_indirect_effect(mean, [[0, 5, 1, 9, 44, 1, 7], [0, 3, 1, 8, 1, 12, 19, 1, 6]],
                                                      [[9], [12]], oracle)
    vecs = torch.randn(10, 3, 4, generator=torch.Generator().manual_seed(1), dtype=torch.float64)
    heads_seen, items_seen = [], []
    for rank, cie, mean_x, heads, (a, b) in results:
        torch.testing.assert_close(cie, full, rtol=0, atol=1e-15)
        torch.testing.assert_close(mean_x, vecs.sum(0) * 2 / 10, rtol=1e-14, atol=0)
        heads_seen += heads
        items_seen += list(range(a, b))
    assert sorted(heads_seen) == list(range(cfg.n_heads))   # every head exactly once
    assert sorted(items_seen) == list(range(10))            # every prompt exactly once

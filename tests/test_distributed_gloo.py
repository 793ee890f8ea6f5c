"""CPU, multi-process (gloo): the multi-GPU partition + reduction logic of
distributed.py, with the oracle standing in for each rank's GPU sweep.

* site-sharded CIE (balanced layer-pair blocks, one SUM all-reduce) == the
  full single-process oracle CIE;
* prompt-sharded mean extraction (contiguous split, SUM all-reduce, one
  division by the global count) == the unsharded mean.
"""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, store_file, q):
    # a file rendezvous: no port to race for with other processes on the machine
    dist.init_process_group("gloo", init_method=f"file://{store_file}", rank=rank, world_size=world)
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

        def local(sites):  # the reference loop over this rank's (layer, head) sites only
            out = torch.zeros(cfg.n_layers, cfg.n_heads, dtype=torch.float64)
            for l in sorted({l for l, _ in sites}):
                out += R.calculate_average_causal_indirect_effect(
                    mean, prompts, answers, oracle, layers=[l], heads=[h for ll, h in sites if ll == l])
            return out * len(prompts)

        cie = D.sharded_cie(cfg.n_layers, cfg.n_heads, len(prompts), local,
                            lambda: torch.zeros(cfg.n_layers, cfg.n_heads, dtype=torch.float64))
        # prompt-sharded extraction with a stand-in "Σ z" and projection
        vecs = torch.randn(10, 3, 4, generator=torch.Generator().manual_seed(1), dtype=torch.float64)
        ids = list(range(10))
        mean_x = D.sharded_mean_activation(ids, lambda ps: vecs[list(ps)].sum(0), lambda z: z * 2,
                                           lambda: torch.zeros(3, 4, dtype=torch.float64))
        q.put((rank, cie, mean_x, D.balanced_site_shard(cfg.n_layers, cfg.n_heads, rank, world),
               D.contiguous_shard(10, rank, world)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_sweeps_match_single_process(world, tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = tmp_path / "gloo_store"
    procs = [ctx.Process(target=_worker, args=(r, world, str(store), q)) for r in range(world)]
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
    sites_seen, items_seen = [], []
    for rank, cie, mean_x, sites, (a, b) in results:
        torch.testing.assert_close(cie, full, rtol=0, atol=1e-15)
        torch.testing.assert_close(mean_x, vecs.sum(0) * 2 / 10, rtol=1e-14, atol=0)
        sites_seen += sites
        items_seen += list(range(a, b))
    assert sorted(sites_seen) == [(l, h) for l in range(cfg.n_layers) for h in range(cfg.n_heads)]  # each once
    assert sorted(items_seen) == list(range(10))            # every prompt exactly once


@pytest.mark.parametrize("L,H,world", [(32, 32, 1), (32, 32, 2), (32, 32, 4), (32, 32, 8), (36, 40, 8),
                                       (36, 40, 2), (12, 12, 3), (5, 4, 2), (2, 4, 4), (3, 2, 4)])
def test_balanced_site_shard(L, H, world):
    """Every (layer, head) site on exactly one rank; the staircase work
    (Σ over a rank's sites of the L - 1 - l blocks after the site) equal on
    every rank when world divides H; whole layers per rank where the pairs
    divide evenly (C3: 2.8B on 8 GPUs = 2 layer pairs per rank, every head)."""
    from tvr_amd import distributed as D
    shares = [D.balanced_site_shard(L, H, r, world) for r in range(world)]
    allsites = sorted(s for sh in shares for s in sh)
    assert allsites == [(l, h) for l in range(L) for h in range(H)]
    work = [sum(L - 1 - l for l, _ in sh) for sh in shares]
    if H % world == 0:
        assert len(set(work)) == 1, work
    if (L // 2) % world == 0 and L % 2 == 0:
        for sh in shares:  # whole layers: every head of each of the rank's layers
            layers = {l for l, _ in sh}
            assert len(sh) == len(layers) * H


# ----------------------------------------------------------- site-sharded sweeps
class OracleEngine:
    """Stands in for ``tvr_amd.Model`` on CPU ranks: the three engine entry
    points the experiment layer calls (``_sweep_trace``, ``forward_clean``,
    ``patch_sweep`` with ADD_ATTN_OUT_LASTPOS sites) computed by the oracle
    one prompt / site at a time, so experiments.py's own site partition and
    gather code runs unchanged under gloo."""

    def __init__(self, oracle):
        self.o, self.cfg, self.tokenizer = oracle, oracle.cfg, oracle.tokenizer
        self.device = torch.device("cpu")

    def to_single_token(self, s):
        return self.o.to_single_token(s)

    def to_string(self, t):
        return self.o.to_string(t)

    def to_tokens(self, s, prepend_bos=True):
        return self.o.to_tokens(s, prepend_bos)

    def _sweep_trace(self, n, t):
        return {}

    @staticmethod
    def _outs(logits, targets, topk):
        out = {}
        if targets is not None:
            out["prob"] = torch.stack([torch.softmax(l, 0)[t] for l, t in zip(logits, targets)]).float()
        if topk:
            out["topk"] = torch.stack([torch.topk(l, topk).indices for l in logits]).int()
        return out

    def forward_clean(self, seqs, targets=None, topk=0, trace=None, **kw):
        trace["seqs"] = seqs
        return self._outs([self.o.forward(torch.tensor([s]))[0, -1] for s in seqs], targets, topk)

    def patch_sweep(self, trace, sites, vectors, topk=0, want_prob=True, **kw):
        from oracle import reference_experiments as R
        logits = []
        for s in sites:
            v = vectors[int(s["vec"])].to(self.o.dtype)
            logits.append(self.o.run_with_hooks(torch.tensor([trace["seqs"][int(s["seq"])]]), fwd_hooks=[
                (f"blocks.{int(s['layer'])}.hook_attn_out", lambda hv, hook, v=v: R.layer_addition_hook(hv, hook, v))])[0, -1])
        return self._outs(logits, [int(s["target"]) for s in sites] if want_prob else None, topk)


def _site_worker(rank, world, store_file, q):
    dist.init_process_group("gloo", init_method=f"file://{store_file}", rank=rank, world_size=world)
    try:
        from tvr_amd import distributed as D
        out = _site_sweeps(dist.group.WORLD)
        # uneven shares (5 items, world 2/3): every rank joins the gather with its padded share
        part = torch.tensor([[i, 10 * i] for i in D.strided_shard(5, rank, world)], dtype=torch.int32).view(-1, 2)
        out["gather"] = D.gather_strided(part, 5)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _site_sweeps(group):
    import tvr_amd
    from tvr_amd import distributed as D
    from conftest import TINY_STD, make_oracle
    cfg = tvr_amd.get_config("tiny")
    sd = tvr_amd.weights.synth_hf_state_dict(cfg, seed=0, std=TINY_STD)
    eng = OracleEngine(make_oracle(cfg, sd, tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab), torch.float64))
    g = torch.Generator().manual_seed(3)
    layered = torch.randn(cfg.n_layers, cfg.d_model, generator=g)
    fv = torch.randn(cfg.d_model, generator=g) * 3
    ctx = tvr_amd.tasks.letter_to_caps[:9]
    kw = {} if group is None else {"group": group}
    if group is None:
        from tvr_amd import experiments as E
        return {"acc": E.apply_layered_vectors_to_zero_shot(layered, ctx, "→", eng),
                "acc_pl": E.apply_layered_vectors_to_zero_shot(layered, ctx, "→", eng, reference_late_binding=False),
                "dp": E.apply_layered_vectors_to_zero_shot_by_probability(layered, ctx, "→", eng),
                "fv": E.check_accuracy_of_added_task_vector_by_layer(fv, ctx, 3, eng)}
    return {"acc": D.apply_layered_vectors_to_zero_shot_sharded(layered, ctx, "→", eng, **kw),
            "acc_pl": D.apply_layered_vectors_to_zero_shot_sharded(layered, ctx, "→", eng, False, **kw),
            "dp": D.apply_layered_vectors_to_zero_shot_by_probability_sharded(layered, ctx, "→", eng, **kw),
            "fv": D.check_accuracy_of_added_task_vector_by_layer_sharded(fv, ctx, 3, eng, **kw)}


@pytest.mark.parametrize("world", [2, 3])
def test_site_sharded_injection_sweeps_match_single_process(world, tmp_path):
    """The layer sweeps (a4 accuracy, a5 Δprob) and the per-layer FV top-k
    accuracy with (prompt, layer) sites round-robin over gloo ranks + one
    all_gather == the same experiment code in one process == the reference
    loop restated by the oracle."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = tmp_path / "gloo_store"
    procs = [ctx.Process(target=_site_worker, args=(r, world, str(store), q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = _site_sweeps(None)
    import tvr_amd
    from conftest import TINY_STD, make_oracle
    from oracle import reference_experiments as R
    cfg = tvr_amd.get_config("tiny")
    oracle = make_oracle(cfg, tvr_amd.weights.synth_hf_state_dict(cfg, seed=0, std=TINY_STD),
                         tvr_amd.tokenizer.SyntheticTokenizer(cfg.d_vocab), torch.float64)
    g = torch.Generator().manual_seed(3)
    layered = torch.randn(cfg.n_layers, cfg.d_model, generator=g).double()
    assert single["acc"] == R.apply_layered_vectors_to_zero_shot(layered, tvr_amd.tasks.letter_to_caps[:9], "→",
                                                                 oracle)
    for rank, out in results:
        assert out["acc"] == single["acc"] and out["acc_pl"] == single["acc_pl"] and out["fv"] == single["fv"]
        torch.testing.assert_close(out["dp"], single["dp"], rtol=0, atol=0)
        assert out["gather"].tolist() == [[i, 10 * i] for i in range(5)]

"""bench.py's JSON helpers on CPU: the HBM-kernel block and the PMC summary
lookup (keyed on GEMM family and workload, so counters of another workload
never leak into a bench line)."""
import json

import bench


def _kinds(ms, nbytes, launches):
    return {k: {"launches": launches, "ms": ms, "bytes": nbytes, "gbps": nbytes / (ms * 1e-3) / 1e9 if ms else None}
            for k in ("entry", "capture", "lnpre", "attention", "row_stats")}


def test_hbm_kernels_block():
    hbm = _kinds(2.0, 8e9, 4)  # 4 launches, 8 GB in 2 ms -> 4000 GB/s
    ex = _kinds(1.0, 1e9, 2)
    out = bench.hbm_kernels(hbm, ex, steps=2)
    assert out["peak_gbps"] == bench.HBM_PEAK_GBPS
    for k in ("entry", "lnpre", "attention", "row_stats"):
        row = out[k]
        assert row["launches_per_step"] == 2.0
        assert row["avg_launch_us"] == 500.0
        assert row["achieved_gbps"] == 4000.0 and row["frac"] == 0.5
    assert out["capture"]["launches"] == 2 and out["capture"]["achieved_gbps"] == 1000.0
    json.dumps(out)


def test_hbm_kernels_absent_kinds():
    hbm = _kinds(0.0, 0.0, 0)
    out = bench.hbm_kernels(hbm, None, steps=1)
    assert all(out[k] is None for k in ("entry", "lnpre", "attention", "row_stats", "capture"))


def test_pmc_summary_keyed_on_family_and_workload():
    p = bench.ROOT / "profiles" / "pmc_gemm_x2f16.json"
    d = json.loads(p.read_text())
    pmc, src = bench.pmc_summary("x2f16", d["workload"])
    assert pmc is not None and pmc["hbm_bytes_per_launch"] > 0 and src
    assert bench.pmc_summary("x2f16", "another workload") == (None, None)


def test_pmc_summary_c4_any_prompt_length():
    """The C4 block reads the bf16 counters of the same sweep (model, sites,
    prompts, shots) at another prompt length; another model never matches."""
    p = bench.ROOT / "profiles" / "pmc_gemm_bf16.json"
    d = json.loads(p.read_text())
    base = d["workload"].rsplit(", T=", 1)[0]
    assert bench.pmc_summary("bf16", base + ", T=999") == (None, None)  # exact match by default
    pmc, src = bench.pmc_summary("bf16", base + ", T=999", any_len=True)
    assert pmc is not None and d["workload"] in src
    assert bench.pmc_summary("bf16", base.replace("6.9b", "2.8b") + ", T=18", any_len=True) == (None, None)
    assert bench.pmc_summary("x2f16", base + ", T=18", any_len=True) == (None, None)  # another family


def test_hbm_kernels_pmc_traffic_keyed_on_workload():
    """profiles/pmc_hbm_kernels.json (tools/prof_summary.py) attaches memory-side
    bytes per launch to the matching workload's rows only."""
    p = bench.ROOT / "profiles" / "pmc_hbm_kernels.json"
    if not p.exists():
        return
    d = json.loads(p.read_text())
    hbm = _kinds(2.0, 8e9, 4)
    out = bench.hbm_kernels(hbm, None, steps=2, workload=d["workload"])
    for k, v in d["kernels"].items():
        if k in ("entry", "lnpre", "attention", "row_stats"):
            assert out[k]["traffic"] == v["fetch_bytes_x2_per_launch"] + v["write_bytes_per_launch"]
    other = bench.hbm_kernels(hbm, None, steps=2, workload="another workload")
    assert all("traffic" not in (other[k] or {}) for k in ("entry", "lnpre", "attention", "row_stats"))


def test_gpus_flag_launches_ranks_itself():
    """``bench.py --gpus 2`` without torchrun starts 2 ranks of itself (the
    parent never touches a GPU) and rank 0 reports the world size the process
    group saw (--gpus was parsed and ignored)."""
    import os
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, str(bench.ROOT / "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--launch-check"], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    out = lines[0]
    assert out["n_gpus"] == 2 and out["launch_check"]
    assert len(out["rank_elapsed_s"]) == 2 and out["max_elapsed_s"] == max(out["rank_elapsed_s"])


def test_headline_workload_is_the_strong_c3_sweep():
    """VERDICT r3 / ADVICE r3: the N > 1 headline is BASELINE's C3 — ONE 12-prompt
    32 x 32 sweep split by head across the ranks (strong scaling), the default;
    the prompt-partitioned weak form is opt-in (--shard prompts) or a side leg."""
    import sys
    argv = sys.argv
    try:
        sys.argv = ["bench.py"]
        assert bench.parse().shard == "sites"
    finally:
        sys.argv = argv
    for world in (1, 2, 8):
        for shard in ("sites", "heads"):
            w, scaling = bench.describe_workload("pythia-2.8b", 32, 32, 12, 4, 15, world, shard)
            assert scaling == "strong"
            assert w.startswith("pythia-2.8b CIE sweep 32x32 sites, 12 prompts/step, 4-shot, T=15")
            if world > 1:
                assert w.endswith("sites in balanced layer-pair blocks per rank" if shard == "sites" else
                                  f"sites h = rank (mod {world})")
    w, scaling = bench.describe_workload("pythia-2.8b", 32, 32, 12, 4, 15, 8, "prompts")
    assert scaling == "weak" and "prompts/GPU/step" in w
    # N = 1: the same string whichever --shard was given (the PMC summaries key on it)
    assert bench.describe_workload("pythia-2.8b", 32, 32, 12, 4, 15, 1, "prompts") == \
        bench.describe_workload("pythia-2.8b", 32, 32, 12, 4, 15, 1, "heads")


def test_launch_check_at_8_ranks_names_every_8gpu_config():
    """at N = 8 the bench times BASELINE's three multi-GPU configs —
    C3 (the headline, strong site split), C4 (extraction prompt-sharded, CIE
    site-sharded, injection round-robin) and C5 (the 12B sweep, strong site
    split) — and rank 0's launch check reports exactly those workloads."""
    import os
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, str(bench.ROOT / "bench.py"), "--gpus", "8", "--dist-backend", "gloo",
                        "--launch-check"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][0]
    assert out["n_gpus"] == 8 and len(out["rank_elapsed_s"]) == 8
    w = out["workloads"]
    assert set(w) == {"C3", "C4", "C5"}
    assert w["C3"] == ("pythia-2.8b CIE sweep 32x32 sites, 12 prompts/step, 4-shot, T=15, "
                       "sites in balanced layer-pair blocks per rank")
    assert w["C5"] == "pythia-12b CIE sweep 36x40 sites, 12 prompts/step, 10-shot, T=33, " \
                      "sites in balanced layer-pair blocks per rank"
    assert w["C4"].startswith("pythia-6.9b bf16 FV suite") and "8 GPUs" in w["C4"] and "round-robin" in w["C4"]
    assert bench.c5_workload(1) == "pythia-12b CIE sweep 36x40 sites, 12 prompts/step, 10-shot, T=33"

#!/usr/bin/env python3
"""Summarise rocprofv3 output of a bench.py run into profiles/.

  python tools/prof_summary.py --tag r01 --stats gpurun_out/prof_r1 \
      --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write

* kernel stats (--kernel-trace --stats): per kernel calls / total / avg ms
* PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs, as the MI355X guide
  prescribes): HBM bytes per GEMM launch = 2 x FETCH_SIZE x 1024 (gfx950
  reports half the bytes of 16-B/lane streaming reads) + WRITE_SIZE x 1024,
  next to the launch's algorithmic bytes (A + W + C, fp32).
Writes profiles/rocprof_<tag>.json, profiles/kernel_stats_<tag>.csv and
profiles/pmc_gemm_<family>.json (read by bench.py for roofline.traffic;
family = f32 | x3bf16, the GEMM kernel the profiled command ran).
"""
import argparse
import csv
import glob
import json
import shutil
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
# epilogue template argument -> variant; EPI_BIAS dispatches are the split-K partial
# launches of every GEMM (the reduce applies the real epilogue) and the
# linearised entry layer's G GEMMs; the unembed is EPI_STATS
VARIANTS = {"0": "bias_partials", "1": "qkv_mlpin", "2": "o_mlpout", "3": "qkv_mlpin", "4": "unembed"}
MAIN = ("qkv_mlpin", "o_mlpout")  # the step's two big GEMMs (95 % of its time): traffic / ratio basis
SIMDS = 1024  # 256 CUs x 4


def one(d, pattern):
    hits = glob.glob(str(Path(d) / "**" / pattern), recursive=True)
    if not hits:
        raise SystemExit(f"no {pattern} under {d}")
    return hits[0]


def short(name):
    return name.split("(")[0].replace("void ", "")


FAMILIES = {"gemm_f32_nt_kernel": "f32", "gemm_x3bf16_nt_kernel": "x3bf16", "gemm_planar_kernel": "planar",
            "gemm_pingpong_kernel": "pingpong"}
PLANAR_FMT = {"1": "x2f16", "2": "bf16"}  # gemm_planar_kernel<EPI, Tile, FMT, ...>, gemm_pingpong_kernel<EPI, FMT, ...>
FMT_ARG = {"planar": 2, "pingpong": 1}


def gemm_variant(name):
    """(family, epilogue variant) of a GEMM kernel name, or None."""
    for k, fam in FAMILIES.items():
        if k + "<" in name:
            args = name.split(k + "<")[1]
            if fam in FMT_ARG:  # the activation-format template argument
                depth, parts, cur = 0, [], ""
                for ch in args:
                    if ch == "<":
                        depth += 1
                    elif ch == ">":
                        if depth == 0:
                            break
                        depth -= 1
                    if ch == "," and depth == 0:
                        parts.append(cur.strip())
                        cur = ""
                    else:
                        cur += ch
                parts.append(cur.strip())
                fam = PLANAR_FMT.get(parts[FMT_ARG[fam]], fam)
            return fam, args[0]
    return None


# the HBM-bound kernels (bench.py hbm_kernels names)
HBM_KERNELS = {"lin_entry_kernel": "lin_entry", "entry_replace_mfma_kernel": "entry", "entry_kernel": "entry", "lnpre_kernel": "lnpre", "attention_mfma_kernel": "attention",
               "stats_merge_kernel": "row_stats", "row_stats_kernel": "row_stats", "capture_partial_kernel": "capture",
               "capture_finish_kernel": "capture"}


def hbm_kind(name):
    for k, v in HBM_KERNELS.items():
        if k in name:
            return v
    return None


def hbm_kernel_traffic(f, w, bench):
    """Memory-side bytes of the HBM-bound kernels from the same FETCH_SIZE /
    WRITE_SIZE passes: per kind, launches and bytes per launch.  FETCH_SIZE is
    given raw (x 1024) and doubled (the gfx950 correction, calibrated for
    16-B-per-lane reads only: MI355X_MICROARCH.md HBM); next to bench.py's
    algorithmic bytes per launch of the same kind."""
    def per_kind(rows):
        out = {}
        for r in rows:
            k = hbm_kind(r["Kernel_Name"])
            if k:
                o = out.setdefault(k, [0, 0.0])
                o[0] += 1
                o[1] += float(r["Counter_Value"]) * 1024
        return out
    fk, wk = per_kind(f), per_kind(w)
    alg = {k: v.get("bytes_per_launch") for k, v in ((bench or {}).get("hbm_kernels") or {}).items()
           if isinstance(v, dict)}
    res = {}
    for k, (n, fb) in fk.items():
        wn, wb = wk.get(k, (n, 0.0))
        r = {"launches": n, "fetch_bytes_raw_per_launch": round(fb / n), "fetch_bytes_x2_per_launch": round(2 * fb / n),
             "write_bytes_per_launch": round(wb / max(wn, 1))}
        if alg.get(k):
            r["alg_bytes_per_launch"] = alg[k]
            r["ratio_x2_to_alg"] = round((2 * fb / n + wb / max(wn, 1)) / alg[k], 2)
        res[k] = r
    return res


def pmc(d):
    rows = []
    for r in csv.DictReader(open(one(d, "*counter_collection.csv"))):
        rows.append(r)
    return rows


def mfma_util(rows, fam_only=None):
    """MFMA utilisation of the GEMM dispatches: SQ_VALU_MFMA_BUSY_CYCLES (summed
    over every SIMD) / (SIMDs x shader cycles), shader cycles = GRBM_GUI_ACTIVE / 8
    (rocprofv3 sums it over the 8 XCDs; MI355X_MICROARCH.md DVFS note); the
    effective clock is those cycles over the dispatch's wall time.  SQ wave
    states (quad-cycles) as fractions of SQ_WAVE_CYCLES."""
    by = {}
    for r in rows:
        gv = gemm_variant(r["Kernel_Name"])
        if not gv or (fam_only and gv[0] != fam_only):
            continue
        d = by.setdefault((r["Dispatch_Id"], gv), {"ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    per = {}
    for (_, (fam, v)), d in by.items():
        p = per.setdefault(VARIANTS[v], {"launches": 0, "busy": 0.0, "grbm": 0.0, "ns": 0,
                                         "wave": 0.0, "wait": 0.0, "wait_inst": 0.0, "active": 0.0})
        p["launches"] += 1
        p["busy"] += d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        p["grbm"] += d.get("GRBM_GUI_ACTIVE", 0.0)
        p["ns"] += d["ns"]
        p["wave"] += d.get("SQ_WAVE_CYCLES", 0.0)
        p["wait"] += d.get("SQ_WAIT_ANY", 0.0)
        p["wait_inst"] += d.get("SQ_WAIT_INST_ANY", 0.0)
        p["active"] += d.get("SQ_ACTIVE_INST_ANY", 0.0)
    def fmt(p):
        cyc = p["grbm"] / 8
        out = {"launches": p["launches"], "mfma_util": round(p["busy"] / (SIMDS * cyc), 4) if cyc else None,
               "clock_mhz": round(cyc / (p["ns"] * 1e-9) / 1e6) if p["ns"] else None}
        if p["wave"]:
            out.update({"wave_wait_any": round(p["wait"] / p["wave"], 3),
                        "wave_wait_inst": round(p["wait_inst"] / p["wave"], 3),
                        "wave_active_inst": round(p["active"] / p["wave"], 3)})
        return out
    tot = {k: sum(p[k] for p in per.values()) for k in ("launches", "busy", "grbm", "ns", "wave", "wait",
                                                          "wait_inst", "active")}
    res = {"basis": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8); clock = "
                    "GRBM_GUI_ACTIVE / 8 / dispatch time", "all": fmt(tot)}
    res["variants"] = {k: fmt(p) for k, p in per.items()}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--stats", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--mfma", help="PMC pass with SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE and the SQ wave states")
    ap.add_argument("--bench", help="bench.py JSON of the same command (algorithmic bytes per launch)")
    ap.add_argument("--cmd", default="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32-leg")
    ap.add_argument("--out", default=str(ROOT / "profiles"), help="summary directory")
    a = ap.parse_args()
    out_dir = Path(a.out)
    out_dir.mkdir(exist_ok=True)
    stats_csv = one(a.stats, "*kernel_stats.csv")
    shutil.copy(stats_csv, out_dir / f"kernel_stats_{a.tag}.csv")
    kernels = []
    for r in csv.DictReader(open(stats_csv)):
        kernels.append({"kernel": short(r["Name"]), "calls": int(r["Calls"]),
                        "total_ms": round(int(r["TotalDurationNs"]) / 1e6, 3),
                        "avg_ms": round(float(r["AverageNs"]) / 1e6, 4), "pct": round(float(r["Percentage"]), 2)})
    summary = {"command": a.cmd, "kernels": kernels[:20]}
    # the profiled family: the GEMM kernel with the most time (a planar-mode run
    # also launches the fp32 GEMM once per layer while it builds the linearised
    # entry layer's W1 W_O constants, csrc/lin_entry.hpp: model set-up, excluded)
    fam_ms = {}
    for r in csv.DictReader(open(stats_csv)):
        gv = gemm_variant(r["Name"])
        if gv:
            fam_ms[gv[0]] = fam_ms.get(gv[0], 0.0) + int(r["TotalDurationNs"]) / 1e6
    main_fam = max(fam_ms, key=fam_ms.get) if fam_ms else None
    summary["excluded_gemm_families_ms"] = {k: round(v, 3) for k, v in fam_ms.items() if k != main_fam}
    gemm = [k for k, r in zip(kernels, csv.DictReader(open(stats_csv)))
            if (gemm_variant(r["Name"]) or (None,))[0] == main_fam]
    tot_calls = sum(k["calls"] for k in gemm)
    summary["gemm_family"] = {"calls": tot_calls, "total_ms": round(sum(k["total_ms"] for k in gemm), 3),
                              "avg_ms": round(sum(k["total_ms"] for k in gemm) / max(tot_calls, 1), 4)}
    if a.fetch and a.write:
        f, w = pmc(a.fetch), pmc(a.write)
        # the two passes are separate runs of the same deterministic command:
        # pair the i-th GEMM dispatch of one with the i-th of the other
        fg = [r for r in f if (gemm_variant(r["Kernel_Name"]) or (None,))[0] == main_fam]
        wg = [r for r in w if (gemm_variant(r["Kernel_Name"]) or (None,))[0] == main_fam]
        if len(fg) != len(wg):
            raise SystemExit(f"PMC passes saw {len(fg)} vs {len(wg)} GEMM dispatches")
        per, fams = {}, set()
        for rf, rw in zip(fg, wg):
            fam, v = gemm_variant(rf["Kernel_Name"])
            if gemm_variant(rw["Kernel_Name"]) != (fam, v):
                raise SystemExit("PMC passes disagree on the GEMM dispatch order")
            fams.add(fam)
            hbm = 2.0 * float(rf["Counter_Value"]) * 1024 + float(rw["Counter_Value"]) * 1024
            p = per.setdefault(VARIANTS[v], {"launches": 0, "hbm_bytes": 0.0})
            p["launches"] += 1
            p["hbm_bytes"] += hbm
        n = sum(per[k]["launches"] for k in MAIN if k in per)
        hbm = sum(per[k]["hbm_bytes"] for k in MAIN if k in per)
        if len(fams) != 1:
            raise SystemExit(f"profiled command ran GEMM families {sorted(fams)}; profile one at a time")
        fam = fams.pop()
        pm = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, tag {a.tag}", "family": fam,
              "correction": "HBM bytes = 2 x FETCH_SIZE x 1024 (gfx950 half-count of 16-B/lane reads) + WRITE_SIZE x 1024",
              "basis": "qkv_mlpin + o_mlpout dispatches (split-K partial dispatches and the unembed listed apart)",
              "hbm_bytes_per_launch": round(hbm / n), "launches": n,
              "variants": {k: {"launches": p["launches"], "hbm_bytes_per_launch": round(p["hbm_bytes"] / p["launches"])}
                           for k, p in per.items()}}
        if a.bench:
            b = json.loads(Path(a.bench).read_text())
            bv = b["roofline"].get("variants", {})
            if all(k in bv and "alg_bytes_per_launch" in bv[k] for k in MAIN if k in per):
                alg = sum(bv[k]["alg_bytes_per_launch"] * per[k]["launches"] for k in MAIN if k in per) / n
                for k in MAIN:
                    if k in per:
                        pm["variants"][k]["alg_bytes_per_launch"] = bv[k]["alg_bytes_per_launch"]
                        pm["variants"][k]["ratio_hbm_to_alg"] = round(
                            per[k]["hbm_bytes"] / per[k]["launches"] / bv[k]["alg_bytes_per_launch"], 2)
            else:
                alg = b["roofline"]["algorithmic_bytes_per_launch"]
            pm["alg_bytes_per_launch"] = round(alg)
            pm["workload"] = b["config"]["workload"]
            pm["ratio_hbm_to_alg"] = round(hbm / n / alg, 2)
        if a.mfma:
            pm["mfma"] = mfma_util(pmc(a.mfma), main_fam)
        summary["pmc_gemm"] = pm
        (out_dir / f"pmc_gemm_{fam}.json").write_text(json.dumps(pm, indent=1) + "\n")
        hk = hbm_kernel_traffic(f, w, json.loads(Path(a.bench).read_text()) if a.bench else None)
        if hk:
            hk = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, tag {a.tag}",
                  "workload": json.loads(Path(a.bench).read_text())["config"]["workload"] if a.bench else None,
                  "note": "FETCH_SIZE doubling is calibrated for 16-B/lane reads; the attention kernel's V loads are "
                          "4 B/lane, so its x2 figure is an upper bound",
                  "kernels": hk}
            summary["pmc_hbm_kernels"] = hk
            (out_dir / "pmc_hbm_kernels.json").write_text(json.dumps(hk, indent=1) + "\n")
    (out_dir / f"rocprof_{a.tag}.json").write_text(json.dumps(summary, indent=1) + "\n")
    print(json.dumps(summary, indent=1)[:3000])


if __name__ == "__main__":
    main()

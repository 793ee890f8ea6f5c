"""Per-dispatch GEMM efficiency from a rocprofv3 kernel-trace CSV.

    python tools/dispatch_table.py <kernel_trace.csv> [N-of-qkv,...]

Groups the engine GEMM dispatches (gemm_pingpong / gemm_planar kernels) by
workgroup count and prints, per group: dispatches, blocks, block rounds on
256 CUs (ceil), mean duration, and microseconds per round — the number that
exposes partial last rounds (tail) and per-launch overhead at small M.
Diagnostic only.
"""
import csv
import json
import math
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    groups = defaultdict(list)
    for r in rows:
        name = r.get("Kernel_Name", "")
        if not any(k in name for k in ("gemm_pingpong", "gemm_planar", "splitk_reduce")):
            continue
        kind = "pp" if "gemm_pingpong" in name else "pl" if "gemm_planar" in name else "red"
        wg = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 0)) or 0)
        grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        blocks = grid // wg if wg else 0
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # us
        epi = name.split("kernel<")[1].split(",")[0] if "kernel<" in name else "?"
        groups[(kind, epi, blocks)].append(dur)
    out = []
    for (kind, epi, blocks), durs in sorted(groups.items()):
        rounds = math.ceil(blocks / 256) if blocks else 0
        mean = sum(durs) / len(durs)
        out.append({"kernel": kind, "epi": epi, "blocks": blocks, "dispatches": len(durs), "rounds": rounds,
                    "fill_last_round": round(blocks / 256 - (rounds - 1), 3) if rounds else 0,
                    "mean_us": round(mean, 1), "us_per_round": round(mean / rounds, 1) if rounds else 0,
                    "total_ms": round(sum(durs) / 1e3, 2)})
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()

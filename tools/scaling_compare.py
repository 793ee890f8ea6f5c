#!/usr/bin/env python3
"""Per-kernel-family time of the emulated rank share vs 1/N of the one-GPU run
(rocprofv3 --kernel-trace CSVs under two directories; tools/scaling_profile.sh).
Both runs time 1 warmup + 2 steps + 1 profiled step of the same sweep, so the
totals compare as (em) against (n1) / N.  Diagnostic only."""
import csv
import glob
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    out = defaultdict(float)
    cnt = defaultdict(int)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        fam = name.split("<")[0].replace("tvr::", "")
        if "gemm_pingpong" in name:
            fam += "<" + name.split("<")[1].split(",")[0] + ">"
        out[fam] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        cnt[fam] += 1
    return out, cnt


n1, c1 = load(sys.argv[1])
em, ce = load(sys.argv[2])
N = int(sys.argv[3])
print(f"{'kernel family':48s} {'n1/N ms':>9s} {'rank ms':>9s} {'excess':>8s} {'n1 launches':>11s} {'rank launches':>13s}")
tot1 = tote = 0.0
for k in sorted(set(n1) | set(em), key=lambda k: -(em.get(k, 0) - n1.get(k, 0) / N)):
    a, b = n1.get(k, 0) / N, em.get(k, 0)
    tot1 += a
    tote += b
    print(f"{k[:48]:48s} {a:9.2f} {b:9.2f} {b - a:8.2f} {c1.get(k, 0):11d} {ce.get(k, 0):13d}")
print(f"{'total':48s} {tot1:9.2f} {tote:9.2f} {tote - tot1:8.2f}   (kernel time only; ratio {tot1 / tote:.4f})")

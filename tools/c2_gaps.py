"""Dispatch gaps of the C2 layer sweeps from a rocprofv3 kernel-trace CSV.

    python tools/c2_gaps.py <kernel_trace.csv> [--split-us 300]

Dispatches are sorted by start time and cut into bursts wherever the device
idles longer than --split-us (a host synchronisation: the end of one
experiment call).  Per burst: dispatches, span (first start to last end),
summed kernel time, and the idle time between consecutive dispatches inside
it (the per-launch dispatch cost plus any host work that does not sync).
Diagnostic only.
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--split-us", type=float, default=300.0)
    ap.add_argument("--min-dispatches", type=int, default=100)
    a = ap.parse_args()
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", ""))
                for r in csv.DictReader(open(a.trace)))
    bursts, cur = [], [ks[0]]
    for k in ks[1:]:
        if (k[0] - max(e for _, e, _ in cur)) / 1e3 > a.split_us:
            bursts.append(cur)
            cur = []
        cur.append(k)
    bursts.append(cur)
    for b in bursts:
        if len(b) < a.min_dispatches:
            continue
        span = (max(e for _, e, _ in b) - b[0][0]) / 1e3
        busy = sum(e - s for s, e, _ in b) / 1e3
        gaps, end = [], b[0][1]
        for s, e, _ in b[1:]:
            gaps.append(max(0, s - end) / 1e3)
            end = max(end, e)
        print(json.dumps({"dispatches": len(b), "span_ms": round(span / 1e3, 3), "kernel_ms": round(busy / 1e3, 3),
                          "gap_ms": round(sum(gaps) / 1e3, 3),
                          "gap_us_median": round(sorted(gaps)[len(gaps) // 2], 2) if gaps else None,
                          "gaps_over_20us": sum(g > 20 for g in gaps)}))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-kernel means of a rocprofv3 --pmc counter_collection.csv (tools/pmc_probe.sh): wave-cycle split
(quad-cycles, MI355X_MICROARCH.md 'rocprofv3 PMC slots'), MFMA busy per SIMD-cycle, the clock from
GRBM_GUI_ACTIVE / 8 XCDs over the dispatch time."""
import csv
import glob
import sys
from collections import defaultdict

path = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
agg = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
times = {}
for row in csv.DictReader(open(path)):
    k = row["Kernel_Name"].split("(")[0].replace("void ", "")
    key = (k, row["Dispatch_Id"])
    agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
    disp[k].add(row["Dispatch_Id"])
    if "Start_Timestamp" in row:
        times[key] = (int(row["Start_Timestamp"]), int(row["End_Timestamp"]))
for k, c in agg.items():
    n = len(disp[k])
    ns = sum(times[(k, d)][1] - times[(k, d)][0] for d in disp[k] if (k, d) in times)
    wc = c["SQ_WAVE_CYCLES"] or 1
    gui = c["GRBM_GUI_ACTIVE"] / 8
    out = {"dispatches": n,
           "wait_any": c["SQ_WAIT_ANY"] / wc, "wait_inst_any": c["SQ_WAIT_INST_ANY"] / wc,
           "active_inst": c["SQ_ACTIVE_INST_ANY"] / wc, "wait_inst_lds": c["SQ_WAIT_INST_LDS"] / wc,
           "lds_bank_conflict_per_lds_inst": c["SQ_LDS_BANK_CONFLICT"] / max(1.0, c["SQ_INSTS_LDS"]),
           "mfma_busy": c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1.0, gui * 1024),
           "clock_ghz": gui / ns if ns else None}
    print(k[-90:], {a: (round(b, 4) if isinstance(b, float) else b) for a, b in out.items()})

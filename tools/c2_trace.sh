# Per-dispatch kernel trace of the C2 accuracy sweep (tools/c2_probe.py under rocprofv3 --kernel-trace):
# the last sweep's dispatches (the profiled one) in order, with durations, to gpurun_out/c2_trace_<tag>.txt.
#   gpurun -- 'bash tools/c2_trace.sh <tag>'
set -o pipefail
TAG=${1:?tag}
R=$PWD
export TMPDIR=/tmp
RAW=/tmp/c2trace_$TAG
mkdir -p $RAW gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $RAW -o run -- python3 $R/tools/c2_probe.py --reps 2 \
    > $R/gpurun_out/c2_probe_$TAG.json 2> $R/gpurun_out/c2_probe_$TAG.err && \
python3 - "$RAW" > $R/gpurun_out/c2_trace_$TAG.txt <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# every layer sweep starts with embed_kernel (the clean rows' embedding): split there; the last one is the
# profiled sweep (HIP events between launches), the one before it the last timed sweep
starts = [i for i, r in enumerate(rows) if "embed_kernel" in r["Kernel_Name"]]
sweeps = [rows[a:b] for a, b in zip(starts, starts[1:] + [len(rows)])]
sw = sweeps[-2]
t0 = int(sw[0]["Start_Timestamp"])
tot = {}
for r in sw:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("tvr::", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    g = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0) // max(1, int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1))
    print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {d:8.1f}  {name[:70]:70s} grid={g}")
    tot[name] = tot.get(name, 0) + d
span = (int(sw[-1]["End_Timestamp"]) - t0) / 1e3
print(f"# sweep span {span:.1f} us, {len(sw)} dispatches, busy {sum(tot.values()):.1f} us")
for k, v in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"# {v:9.1f} us  {k}")
PY
rc=$?
rm -rf $RAW
tail -25 $R/gpurun_out/c2_trace_$TAG.txt
exit $rc

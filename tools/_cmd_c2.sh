export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/c2_probe.py > gpurun_out/c2_probe.json 2> gpurun_out/c2_probe.err || { tail -5 gpurun_out/c2_probe.err; exit 1; }
cat gpurun_out/c2_probe.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/c2 -o run -- python3 $GRAFT_REPO_ROOT/tools/c2_probe.py --reps 1 > /dev/null 2>&1
cp /tmp/c2/run_kernel_stats.csv $GRAFT_REPO_ROOT/gpurun_out/c2_kstats.csv

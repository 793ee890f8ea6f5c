export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/lin_probe.py --reps 2 > gpurun_out/lin_probe_28.json 2> gpurun_out/lin_probe_28.err || { tail -20 gpurun_out/lin_probe_28.err; exit 1; }
cat gpurun_out/lin_probe_28.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lp -o run -- python3 $GRAFT_REPO_ROOT/tools/lin_probe.py --reps 1 > /dev/null 2>&1
cp /tmp/lp/run_kernel_stats.csv $GRAFT_REPO_ROOT/gpurun_out/lin_kstats.csv
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_lin_entry.py -v --timeout 900 --timeout-method thread > gpurun_out/lin_tests.log 2>&1; rc=$?
tail -3 gpurun_out/lin_tests.log
exit $rc

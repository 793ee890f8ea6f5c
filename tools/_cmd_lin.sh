export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_lin_entry.py -v --timeout 900 --timeout-method thread > gpurun_out/lin_tests.log 2>&1; rc=$?
tail -12 gpurun_out/lin_tests.log
grep -E "^E  .*assert|Error" gpurun_out/lin_tests.log | head
exit $rc

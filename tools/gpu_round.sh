# GPU-box session: the -m gpu suite, then the default bench, each under its own
# time limit.  The bench runs only if pytest ended normally (pass or ordinary
# test failures); after a timeout / abort / signal nothing else touches the GPU.
#   gpurun --timeout 1200 -- 'bash tools/gpu_round.sh r02a [extra pytest args]'
TAG=${1:?tag}; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread "$@" \
    > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_tests_$TAG.log
grep -E "FAILED|ERROR" gpurun_out/gpu_tests_$TAG.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
brc=$?
cut -c1-400 gpurun_out/bench_$TAG.json
tail -2 gpurun_out/bench_$TAG.err
[ $brc -ne 0 ] && exit $brc
exit $rc

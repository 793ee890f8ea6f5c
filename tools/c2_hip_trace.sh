# HIP API + kernel trace of the C2 probe (no counters): the host timeline of
# a sweep (engine prep before the first launch, launch rate).
#   gpurun -- 'bash tools/c2_hip_trace.sh <tag>'
TAG=${1:?tag}
R=$PWD
export TMPDIR=/tmp
OUT=$R/gpurun_out/c2hip_$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $OUT/raw -o run -- python3 $R/tools/c2_probe.py --reps 2 \
    > $OUT/probe.json 2> $OUT/probe.err
rc=$?
find $OUT/raw -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
find $OUT/raw -name "*hip_api_trace.csv" -exec cp {} $OUT/hip_api_trace.csv \;
rm -rf $OUT/raw
exit $rc

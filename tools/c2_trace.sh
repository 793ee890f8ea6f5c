# Per-dispatch kernel trace of the C2 accuracy sweep (tools/c2_probe.py) under
# rocprofv3 (kernel trace only), for the per-layer launch anatomy.
#   gpurun -- 'bash tools/c2_trace.sh <tag> [ENV=val ...]'
TAG=${1:?tag}; shift
R=$PWD
export TMPDIR=/tmp
OUT=$R/gpurun_out/c2trace_$TAG
mkdir -p $OUT
cd /tmp
env "$@" timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/raw -o run -- python3 $R/tools/c2_probe.py --reps 1 \
    > $OUT/probe.json 2> $OUT/probe.err
rc=$?
find $OUT/raw -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
rm -rf $OUT/raw
exit $rc

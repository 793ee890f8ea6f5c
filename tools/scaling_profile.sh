# Where rank 0's share of an N-way strong split loses time against 1/N of the
# one-GPU sweep: rocprofv3 kernel stats of the N = 1 bench and of the
# --emulate-world N bench (same box, same call), summarised per kernel family
# by tools/scaling_compare.py.   gpurun -- 'bash tools/scaling_profile.sh <tag> <N> [sites|heads]'
TAG=${1:?tag}; N=${2:-8}; SH=${3:-sites}
R=$PWD
export TMPDIR=/tmp
OUT=$R/gpurun_out/scaling_$TAG
RAW=/tmp/scal_raw
mkdir -p $OUT $RAW
cd /tmp
B="$R/bench.py --steps 2 --warmup 1 --profile-steps 1 --no-cpu-baseline --no-f32-leg --extract 0 --configs="
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $RAW/n1 -o run -- python3 $B > $OUT/n1.json 2> $OUT/n1.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $RAW/em -o run -- python3 $B --emulate-world $N --shard $SH > $OUT/em.json 2> $OUT/em.err && \
python3 $R/tools/scaling_compare.py $RAW/n1 $RAW/em $N > $OUT/compare.txt
rc=$?
rm -rf $RAW
cat $OUT/compare.txt
exit $rc

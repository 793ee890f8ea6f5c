# Same-box A/B of in-tree engine builds, interleaved (A B C A B C ...), reporting the bench value and the
# HBM-bound kernels' launch times (hbm_kernels: entry / lnpre / attention / lin_entry); lines to
# gpurun_out/ab_<tag>/summary.txt.
#   gpurun -- 'bash tools/ab_hbm.sh <tag> <rounds> <libA.so,libB.so[,...]> [extra bench args]'
# A variant may carry env knobs: VAR=v+VAR2=w:lib.so
set -o pipefail
TAG=${1:?tag}; ROUNDS=${2:?rounds}; LIBS=${3:?libs}; shift 3
export TMPDIR=/tmp
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for var in ${LIBS//,/ }; do
    lib=${var##*:}; ev=""; [ "$lib" != "$var" ] && ev=${var%:*}
    n=$(basename $(dirname $lib))_$(basename $lib .so)${ev:+_${ev//[=+]/_}}_$r
    env ${ev//+/ } TVR_LIB=$lib timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32-leg \
        --no-processed-leg --extract 0 --configs= "$@" > $OUT/$n.json 2> $OUT/$n.err || { tail -5 $OUT/$n.err; exit 1; }
    python3 -c "
import json, sys
d = json.load(open(sys.argv[1])); h = d.get('hbm_kernels') or {}
ks = {k: (v['avg_launch_us'], v['frac']) for k, v in h.items() if isinstance(v, dict) and 'avg_launch_us' in v}
print(sys.argv[2], d['value'], d['ms_per_step'], ks)" $OUT/$n.json $n | tee -a $OUT/summary.txt
  done
done

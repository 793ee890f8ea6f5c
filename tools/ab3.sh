# Same-box interleaved A/B/C of up to three in-tree engine builds on the default bench (tools/ab_libs.sh form).
#   gpurun -- 'bash tools/ab3.sh <tag> <rounds> <libA.so> <libB.so> [<libC.so>] -- [extra bench args]'
set -o pipefail
TAG=${1:?tag}; ROUNDS=${2:?rounds}; shift 2
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" == "--" ] && shift
export TMPDIR=/tmp
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for lib in "${LIBS[@]}"; do
    n=$(basename $(dirname $lib))_$r
    TVR_LIB=$lib timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-f32-leg --extract 0 "$@" \
        > $OUT/$n.json 2> $OUT/$n.err || { tail -5 $OUT/$n.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['achieved'], {k: v['achieved_tflops'] for k, v in r['variants'].items()})" $OUT/$n.json $n | tee -a $OUT/summary.txt
  done
done

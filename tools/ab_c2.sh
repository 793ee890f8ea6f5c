# Same-box A/B of two engine builds on the C2 accuracy sweep (tools/c2_probe.py),
# interleaved, one process per run; lines to gpurun_out/ab_c2_<tag>/summary.txt.
#   gpurun -- 'bash tools/ab_c2.sh <tag> <rounds> <libA.so> <libB.so>'
set -o pipefail
TAG=${1:?tag}; ROUNDS=${2:?rounds}; LA=${3:?libA}; LB=${4:?libB}
export TMPDIR=/tmp
OUT=gpurun_out/ab_c2_$TAG
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for lib in $LA $LB; do
    n=$(basename $lib .so)_$r
    TVR_LIB=$lib timeout -k 10 240 python3 tools/c2_probe.py --reps 5 > $OUT/$n.json 2> $OUT/$n.err || { tail -5 $OUT/$n.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], min(d['accuracy_sweep_ms']), {k: (v['ms'], v['tflops']) for k, v in d['gemm'].items()})" $OUT/$n.json $n | tee -a $OUT/summary.txt
  done
done

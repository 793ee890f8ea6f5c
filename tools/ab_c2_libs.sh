# Same-box A/B of two in-tree engine builds on the C2 layer sweeps
# (tools/c2_probe.py), interleaved A B A B ..., summary to gpurun_out/abc2_<tag>/.
#   gpurun -- 'bash tools/ab_c2_libs.sh <tag> <rounds> <libA.so> <libB.so>'
set -o pipefail
TAG=${1:?tag}; ROUNDS=${2:?rounds}; LA=${3:?libA}; LB=${4:?libB}
OUT=gpurun_out/abc2_$TAG
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for lib in $LA $LB; do
    n=$(basename $(dirname $lib))_$r
    TVR_LIB=$lib timeout -k 10 200 python3 tools/c2_probe.py --reps 5 > $OUT/$n.json 2> $OUT/$n.err || { tail -5 $OUT/$n.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); g=d['gemm']; print(sys.argv[2], min(d['accuracy_sweep_ms']), {k: v['ms'] for k, v in g.items()})" $OUT/$n.json $n | tee -a $OUT/summary.txt
  done
done

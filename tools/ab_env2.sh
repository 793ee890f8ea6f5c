# Same-box A/B of engine env knobs with extra bench arguments, interleaved over rounds.
#   gpurun -- 'bash tools/ab_env2.sh <tag> <rounds> "<bench args>" "VAR=a" "VAR=b" ...'
set -o pipefail
TAG=${1:?tag}; ROUNDS=${2:?rounds}; ARGS=$3; shift 3
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    env $v timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-f32-leg --extract 0 --configs= $ARGS \
        > $OUT/run${i}_$r.json 2> $OUT/run${i}_$r.err || { tail -5 $OUT/run${i}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['achieved'], {k: v['achieved_tflops'] for k, v in r['variants'].items()})" $OUT/run${i}_$r.json "$v" | tee -a $OUT/summary.txt
  done
done

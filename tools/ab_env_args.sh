# Same-box A/B of engine env knobs on bench.py with extra bench arguments, interleaved rounds:
#   gpurun -- 'bash tools/ab_env_args.sh <tag> <rounds> "<bench args>" "VAR=a" "VAR=b" ...'
# ("-" as a variant: no env change).  One line per run in gpurun_out/ab_<tag>/summary.txt.
set -o pipefail
TAG=${1:?tag}; ROUNDS=${2:?rounds}; ARGS=${3:?bench args}; shift 3
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    e=$v; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-f32-leg --extract 0 $ARGS \
        > $OUT/run${i}_$r.json 2> $OUT/run${i}_$r.err || { tail -5 $OUT/run${i}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['achieved'], {k: (v['achieved_tflops'], v['avg_launch_ms']) for k, v in r['variants'].items()})" $OUT/run${i}_$r.json "$v round $r" | tee -a $OUT/summary.txt
  done
done

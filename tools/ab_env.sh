# Same-box A/B of engine env knobs on the default bench: one bench process per
# variant (the knobs are read once per process), value lines to gpurun_out/.
#   gpurun -- 'bash tools/ab_env.sh <tag> "VAR=a" "VAR=b VAR2=c" ...'
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
i=0
for v in "$@"; do
  i=$((i + 1))
  echo "== $i $v" | tee -a $OUT/summary.txt
  env $v timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-f32-leg --configs= > $OUT/run$i.json 2> $OUT/run$i.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; h=d.get('hbm_kernels') or {}; print(d['value'], d['ms_per_step'], r['achieved'], {k: v['achieved_tflops'] for k, v in r['variants'].items()}, {k: (v['avg_launch_us'], v['achieved_gbps']) for k, v in h.items() if isinstance(v, dict)})" $OUT/run$i.json | tee -a $OUT/summary.txt
done

# C2 accuracy-sweep time (tools/c2_probe.py) under environment A/B settings, interleaved in one call.
#   gpurun -- 'bash tools/c2_ab_env.sh <rounds> "TVR_STREAM_K=0" "TVR_STREAM_K=1" ...'
set -o pipefail
ROUNDS=${1:?rounds}; shift
mkdir -p gpurun_out
for r in $(seq 1 $ROUNDS); do
  for e in "$@"; do
    out=$(env $e timeout -k 10 200 python3 tools/c2_probe.py --reps 3) || exit 1
    echo "$e round $r $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["accuracy_sweep_ms"], {k: (v["ms"], v["tflops"]) for k, v in d["gemm"].items()})')"
  done
done

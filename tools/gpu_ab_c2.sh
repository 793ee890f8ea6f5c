# C2 layer-sweep anatomy under the small-M switches (same box, interleaved):
# TVR_STREAM_K (stream-K GEMM launches) x TVR_ROW_ATTN (single-query attention).
#   gpurun -- 'bash tools/gpu_ab_c2.sh <tag>'
TAG=${1:?tag}
mkdir -p gpurun_out
for i in 1 2; do
  for v in "1 1" "0 0" "1 0" "0 1"; do
    set -- $v
    TVR_STREAM_K=$1 TVR_ROW_ATTN=$2 timeout -k 10 200 python -u tools/c2_probe.py --reps 3 \
      > gpurun_out/c2_${TAG}_sk$1_ra$2_$i.json 2> gpurun_out/c2_${TAG}_sk$1_ra$2_$i.err || exit $?
    echo "sk=$1 ra=$2: $(cut -c1-120 gpurun_out/c2_${TAG}_sk$1_ra$2_$i.json)"
  done
done

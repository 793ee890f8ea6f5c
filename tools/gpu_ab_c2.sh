# C2 layer-sweep anatomy with stream-K on and off (same box, interleaved):
#   gpurun -- 'bash tools/gpu_ab_c2.sh <tag>'
TAG=${1:?tag}
mkdir -p gpurun_out
for i in 1 2; do
  for sk in 1 0; do
    TVR_STREAM_K=$sk timeout -k 10 200 python -u tools/c2_probe.py --reps 3 > gpurun_out/c2_${TAG}_sk${sk}_$i.json 2> gpurun_out/c2_${TAG}_sk${sk}_$i.err || exit $?
    echo "sk=$sk: $(cut -c1-200 gpurun_out/c2_${TAG}_sk${sk}_$i.json)"
  done
done

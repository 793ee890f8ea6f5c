# Strong-scaling planning on ONE GPU (the driver measures real N = 2/4/8):
# rank 0's share of a --shard heads run at G = 2, 4, 8 (bench --emulate-world),
# then a 2-rank gloo rehearsal of --shard heads with both ranks on this GPU.
#   gpurun --timeout 900 -- 'bash tools/gpu_scaling.sh r02'
TAG=${1:?tag}
export TMPDIR=/tmp
OUT=gpurun_out/scaling_$TAG
mkdir -p $OUT
for G in 2 4 8; do
  timeout -k 10 300 python -u bench.py --emulate-world $G --steps 5 --warmup 2 --no-cpu-baseline --no-f32-leg \
      --extract 0 > $OUT/emulate_$G.json 2> $OUT/emulate_$G.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['achieved'])" $OUT/emulate_$G.json $G
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --extract 0 --no-f32-leg \
    > $OUT/rehearsal_2rank_gloo_1gpu.json 2> $OUT/rehearsal_2rank.err || exit $?
cut -c1-300 $OUT/rehearsal_2rank_gloo_1gpu.json

# The SURVEY §8(d) configurations on one GPU (C2, C3, C4 via tools/bench_configs.py;
# C5 = bench.py on Pythia-12B, 10-shot), then a 2-rank gloo rehearsal of the C4
# driver's sharded entry points with both ranks on this GPU.
#   gpurun --timeout 1200 -- 'bash tools/gpu_configs.sh r02'
TAG=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/bench_configs.py --configs C2,C3,C4 > gpurun_out/configs_$TAG.json \
    2> gpurun_out/configs_$TAG.err || exit $?
cut -c1-300 gpurun_out/configs_$TAG.json
timeout -k 10 400 python -u bench.py --model pythia-12b --kshot 10 --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit $?
cut -c1-300 gpurun_out/bench_c5_$TAG.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 tools/bench_configs.py --configs C4 --c4-tasks 2 --dist-backend gloo \
    > gpurun_out/configs_c4_2rank_gloo_$TAG.json 2> gpurun_out/configs_c4_2rank_gloo_$TAG.err || exit $?
cut -c1-300 gpurun_out/configs_c4_2rank_gloo_$TAG.json

#!/bin/bash
# bench (with CPU baseline) + 2-rank gloo rehearsal of the multi-GPU path + profile passes
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo bench failed; tail gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
MINISCHED_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 \
    > gpurun_out/bench2_gloo_${TAG}.json 2> gpurun_out/bench2_gloo_${TAG}.err || { echo 2-rank rehearsal failed; tail -20 gpurun_out/bench2_gloo_${TAG}.err; exit 1; }
cat gpurun_out/bench2_gloo_${TAG}.json
bash tools/profile.sh ${TAG}

#!/bin/bash
# Full round-end rehearsal: GPU tests, smoke, bench (+ CPU baseline), rocprof stats + PMC passes,
# secondary config timings and a 2-rank gloo rehearsal of the multi-GPU bench path.
set -o pipefail
TAG=${1:-r01}
bash tools/gpu_check.sh ${TAG} && bash tools/profile.sh ${TAG} || exit 1
timeout -k 10 300 python tools/bench_configs.py > gpurun_out/configs_${TAG}.jsonl 2> gpurun_out/configs_${TAG}.err || { echo configs failed; tail gpurun_out/configs_${TAG}.err; exit 1; }
cat gpurun_out/configs_${TAG}.jsonl
MINISCHED_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 \
    > gpurun_out/bench2_gloo_${TAG}.json 2> gpurun_out/bench2_gloo_${TAG}.err || { echo 2-rank rehearsal failed; tail -20 gpurun_out/bench2_gloo_${TAG}.err; exit 1; }
cat gpurun_out/bench2_gloo_${TAG}.json

#!/bin/bash
# Sharded parity tests, bench (with CPU baselines) and the 2-rank gloo rehearsal of the N>1 path.
set -o pipefail
TAG=${1:-r01q}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -v --timeout 120 --timeout-method thread \
    > gpurun_out/sharded_${TAG}.log 2>&1 || { tail -30 gpurun_out/sharded_${TAG}.log; exit 1; }
tail -2 gpurun_out/sharded_${TAG}.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo bench failed; tail gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
MINISCHED_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 \
    > gpurun_out/bench2_gloo_${TAG}.json 2> gpurun_out/bench2_gloo_${TAG}.err || { echo 2-rank rehearsal failed; tail -20 gpurun_out/bench2_gloo_${TAG}.err; exit 1; }
cat gpurun_out/bench2_gloo_${TAG}.json

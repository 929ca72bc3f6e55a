#!/bin/bash
# bench (with CPU baseline) + profile passes for the current production kernel
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo bench failed; tail gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
bash tools/profile.sh ${TAG}

#!/bin/bash
# K1 per-8-pod group test: A/B (interleaved, one process) at 100k / 50k / 12.5k rows, then the GPU
# parity suite with the default (group test on) and the parity file with it off.
set -o pipefail
TAG=${1:-r01w}
mkdir -p gpurun_out
for n in 100000 50000 12500; do
  AB_NODES=$n AB_ROUNDS=12 AB_VARIANTS="MINISCHED_K1_GROUP=1,MINISCHED_K1_GROUP=0" timeout -k 10 120 python tools/ab_k1.py \
      >> gpurun_out/k1_group_ab_${TAG}.jsonl 2> gpurun_out/k1_group_ab_${TAG}.err || { tail gpurun_out/k1_group_ab_${TAG}.err; exit 1; }
done
cat gpurun_out/k1_group_ab_${TAG}.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_${TAG}.log
MINISCHED_K1_GROUP=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread \
    > gpurun_out/pytest_gpu_nogroup_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_nogroup_${TAG}.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_nogroup_${TAG}.log

#!/bin/bash
# Spare key buffers of the decode-stream pipeline (host flow-control slack), N>1 step probe on one GPU.
set -o pipefail
TAG=${1:-r01r}
mkdir -p gpurun_out
for sp in 2 4 8; do
  MINISCHED_PIPE_SPARE=$sp timeout -k 10 200 python tools/step_probe.py --worlds 2,4,8 --steps 400 \
      > gpurun_out/probe_sp${sp}_${TAG}.jsonl 2> gpurun_out/probe_sp${sp}_${TAG}.err || { tail gpurun_out/probe_sp${sp}_${TAG}.err; exit 1; }
  grep '^{' gpurun_out/probe_sp${sp}_${TAG}.jsonl | sed "s/^{/{\"spare\": $sp, /"
done

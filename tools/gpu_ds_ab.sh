#!/bin/bash
# Interleaved A/B (twice) of the decode stream in the N>1 step probe on one GPU.
set -o pipefail
TAG=${1:-r01s}
mkdir -p gpurun_out
for rep in 1 2; do
for ds in 0 1; do
  MINISCHED_DECODE_STREAM=$ds timeout -k 10 200 python tools/step_probe.py --worlds 2,4,8 --steps 400 \
      > gpurun_out/probe_ds${ds}_${rep}_${TAG}.jsonl 2> gpurun_out/probe_ds${ds}_${rep}_${TAG}.err || { tail gpurun_out/probe_ds${ds}_${rep}_${TAG}.err; exit 1; }
  grep '^{' gpurun_out/probe_ds${ds}_${rep}_${TAG}.jsonl | sed "s/^{/{\"rep\": $rep, \"decode_stream\": $ds, /"
done
done

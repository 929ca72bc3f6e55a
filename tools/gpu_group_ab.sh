#!/bin/bash
# Pipeline forms of the N>1 step, interleaved A/B on one GPU (1-rank RCCL group): decode stream,
# depth and drain group; plus the sharded/RCCL parity tests.
set -o pipefail
TAG=${1:-r01t}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -v --timeout 120 --timeout-method thread \
    > gpurun_out/sharded_${TAG}.log 2>&1 || { tail -30 gpurun_out/sharded_${TAG}.log; exit 1; }
tail -2 gpurun_out/sharded_${TAG}.log
for rep in 1 2; do
for cfg in "0 1 1" "0 2 2" "0 3 3" "1 1 1" "1 2 2"; do
  set -- $cfg
  MINISCHED_DECODE_STREAM=$1 MINISCHED_PIPE_DEPTH=$2 MINISCHED_PIPE_GROUP=$3 timeout -k 10 200 python tools/step_probe.py --worlds 2,4,8 --steps 400 \
      > gpurun_out/probe_g_${1}_${2}_${3}_${rep}.jsonl 2> gpurun_out/probe_g_${TAG}.err || { tail gpurun_out/probe_g_${TAG}.err; exit 1; }
  grep '^{' gpurun_out/probe_g_${1}_${2}_${3}_${rep}.jsonl | sed "s/^{/{\"rep\": $rep, \"decode_stream\": $1, \"depth\": $2, \"group\": $3, /"
done
done

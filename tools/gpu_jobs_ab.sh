#!/bin/bash
# Grouped decode in one launch (ms_decode_device_jobs): sharded/RCCL parity tests, then the
# N>1 step probe at depth 3 / group 3 (default) and the per-step form, interleaved twice.
set -o pipefail
TAG=${1:-r01v}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -v --timeout 120 --timeout-method thread \
    > gpurun_out/sharded_${TAG}.log 2>&1 || { tail -30 gpurun_out/sharded_${TAG}.log; exit 1; }
tail -2 gpurun_out/sharded_${TAG}.log
for rep in 1 2; do
for cfg in "1 1" "3 3" "4 4"; do
  set -- $cfg
  MINISCHED_PIPE_DEPTH=$1 MINISCHED_PIPE_GROUP=$2 timeout -k 10 200 python tools/step_probe.py --worlds 2,4,8 --steps 400 \
      > gpurun_out/probe_j_${1}_${2}_${rep}.jsonl 2> gpurun_out/probe_j_${TAG}.err || { tail gpurun_out/probe_j_${TAG}.err; exit 1; }
  grep '^{' gpurun_out/probe_j_${1}_${2}_${rep}.jsonl | sed "s/^{/{\"rep\": $rep, \"depth\": $1, \"group\": $2, /"
done
done

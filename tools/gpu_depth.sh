#!/bin/bash
# Pipeline A/B of the N>1 step (one GPU, 1-rank RCCL group per shard size): decode stream
# off/on x depth, the sharded parity tests, and a kernel-trace timeline of the chosen form.
set -o pipefail
TAG=${1:-r01o}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -v --timeout 120 --timeout-method thread \
    > gpurun_out/sharded_${TAG}.log 2>&1 || { tail -30 gpurun_out/sharded_${TAG}.log; exit 1; }
tail -3 gpurun_out/sharded_${TAG}.log
for cfg in "0 1" "1 1" "1 2"; do
  set -- $cfg
  MINISCHED_DECODE_STREAM=$1 MINISCHED_PIPE_DEPTH=$2 timeout -k 10 200 python tools/step_probe.py --worlds 1,2,4,8 --steps 300 \
      > gpurun_out/probe_${1}_${2}_${TAG}.jsonl 2> gpurun_out/probe_${1}_${2}_${TAG}.err || { tail gpurun_out/probe_${1}_${2}_${TAG}.err; exit 1; }
  grep '^{' gpurun_out/probe_${1}_${2}_${TAG}.jsonl | sed "s/^{/{\"decode_stream\": $1, \"depth\": $2, /"
done
MINISCHED_DECODE_STREAM=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_${TAG} -o run -- \
    python tools/step_probe.py --worlds 8 --steps 200 > /dev/null 2> gpurun_out/tl_${TAG}.err || { tail gpurun_out/tl_${TAG}.err; exit 1; }
python tools/timeline.py gpurun_out/tl_${TAG}/run_kernel_trace.csv 1200 > gpurun_out/tl_${TAG}.json

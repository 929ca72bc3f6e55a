#!/bin/bash
# K1 pp at the G=8 strong-scaling shard (12.5k rows x 100k pods): per-rank pipelined step and sweep-only
# under geometry overrides (MINISCHED_PP_WAVES / MINISCHED_PP_CHUNK / MINISCHED_PP_WORDS)
set -o pipefail
TAG=${1:-r03n}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp PROBE_G=8 PROBE_STREAMS=1 PROBE_STEPS=100
T="timeout -k 10"
for v in "default" "MINISCHED_PP_WAVES=2" "MINISCHED_PP_WAVES=8" "MINISCHED_PP_WAVES=2 MINISCHED_PP_CHUNK=48" "MINISCHED_PP_WAVES=4 MINISCHED_PP_CHUNK=48" "default"; do
  if [ "$v" = default ]; then E=""; else E="$v"; fi
  env $E $T 120 python -u tools/step_probe_lib.py > gpurun_out/$TAG/probe.json 2> gpurun_out/$TAG/probe.err || exit 1
  echo "$v" $(tail -n 1 gpurun_out/$TAG/probe.json)
done

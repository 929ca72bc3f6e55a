#!/bin/bash
# Which HW queue each stream's kernels land on in the per-rank pipelined step (G=8 shard,
# 1-rank communicator): rocprofv3 kernel trace (queue_id, stream_id per dispatch).
set -o pipefail
TAG=${1:-r03zb}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp PROBE_G=8 PROBE_STREAMS=1 PROBE_STEPS=50
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/step_probe_lib.py > $GRAFT_REPO_ROOT/gpurun_out/$TAG/probe.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && tail -2 gpurun_out/$TAG/probe.log

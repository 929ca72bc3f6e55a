#!/bin/bash
# per-rank pipelined step: collective/decode streams at high priority (default) vs normal (MINISCHED_COMM_PRIO=0)
set -o pipefail
TAG=${1:-r03zc}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp PROBE_G=2,4,8 PROBE_STREAMS=1
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_sharded.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/sharded_tests.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/sharded_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  MINISCHED_COMM_PRIO=$v $T 200 python -u tools/step_probe_lib.py > gpurun_out/$TAG/probe_$v.log 2>&1 || exit 1
  echo prio=$v $(tail -1 gpurun_out/$TAG/probe_$v.log)
done

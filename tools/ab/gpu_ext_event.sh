#!/bin/bash
# completion events recorded by the K1 dispatch (hipExtLaunchKernel) instead of separate event packets:
# GPU parity (parity + sharded suites), the caller-stream sweep probe and the per-rank pipelined step
set -o pipefail
TAG=${1:-r03x}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
$T 200 python -u tools/probe_fixed.py > gpurun_out/$TAG/fixed.json 2> gpurun_out/$TAG/fixed.err || exit 1
tail -n 1 gpurun_out/$TAG/fixed.json
PROBE_G=8,4,2 PROBE_STREAMS=1 PROBE_STEPS=100 $T 150 python -u tools/step_probe_lib.py > gpurun_out/$TAG/step.json 2> gpurun_out/$TAG/step.err || exit 1
tail -n 1 gpurun_out/$TAG/step.json

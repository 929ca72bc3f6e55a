#!/bin/bash
# sweep stream waits for older collectives once per several submissions: sharded GPU tests, per-rank step probe
set -o pipefail
TAG=${1:-r03y}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_sharded.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
for d in 4 2 6; do
  MINISCHED_PIPE_DEPTH=$d PROBE_G=8,4 PROBE_STREAMS=1 PROBE_STEPS=100 $T 150 python -u tools/step_probe_lib.py > gpurun_out/$TAG/step_d$d.json 2> gpurun_out/$TAG/step_d$d.err || exit 1
  echo depth=$d $(tail -n 1 gpurun_out/$TAG/step_d$d.json)
done

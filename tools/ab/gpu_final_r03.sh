#!/bin/bash
# round-3 closing check: full GPU suite, smoke, compact cycle (one launch over coherent pinned memory vs staged)
set -o pipefail
TAG=${1:-r03zq}
mkdir -p gpurun_out/$TAG
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="timeout -k 10"
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
$T 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -5 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
for v in 1 0 1 0; do
  MINISCHED_COMPACT_ZC=$v $T 120 python -u tools/probe_compact.py >> gpurun_out/$TAG/probe.jsonl 2>> gpurun_out/$TAG/probe.err || exit 1
  tail -1 gpurun_out/$TAG/probe.jsonl
done
